"""A/B the persistent-kernel variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Usage:
    python scripts/sweep.py [--config sponza] [--spp 8] [--rounds 3] [--variants 0,1,2]
Prints one JSON line per variant: median / min ms and Mray/s.
"""
import argparse
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "chiaroscuro-raytracer_amd"))
os.environ.setdefault("CHIARO_QUIET", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sponza")
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="")
    ap.add_argument("--waves", default="0", help="comma list of waves_per_cu values (0 = default)")
    ap.add_argument("--refill", default="16", help="comma list of refill thresholds (dynamic variants)")
    args = ap.parse_args()
    import torch
    import chiaroscuro_amd as ca
    from chiaroscuro_amd import scenes

    sc = ca.Scene(scenes.config_rtc(args.config))
    info = sc.info
    m = ca.Model(sc)
    kd = ca.KDTree(m, sc)
    dev = ca.Device(0)
    dev.upload(kd.describe())
    xres, yres, k, seed = info["xres"], info["yres"], info["k"], info["seed"]
    cam = ca.camera(info["VP"], info["LA"], info["UP"], info["yview"], xres, yres)
    frame = torch.zeros((yres, xres, 3), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    dev.set_option("counters", 0)
    variants = [int(v) for v in args.variants.split(",")] if args.variants else list(range(64))
    ok = []
    for v in variants:
        try:
            dev.set_option("variant", v)
            ok.append(v)
        except RuntimeError:
            break
    waves = [int(w) for w in args.waves.split(",")]
    refills = [int(f) for f in args.refill.split(",")]
    res = {}
    ref = None
    for r in range(args.rounds):
        for v in ok:
            for w, f in [(w, f) for w in waves for f in refills]:
                dev.set_option("variant", v)
                dev.set_option("waves_per_cu", w)
                dev.set_option("refill", f)
                p = ca.render_params(xres, yres, args.spp, k, seed, layer=1)
                dev.render_device(cam, p, frame.data_ptr(), stream)
                torch.cuda.synchronize()
                c = dev.counters()
                if ref is None:
                    ref = frame.clone()
                else:
                    assert torch.equal(frame, ref), "variant %d changed the image" % v
                res.setdefault((v, w, f), []).append((dev.last_kernel_ms(), c["closest"] + c["shadow"]))
        print("round %d done" % r, file=sys.stderr, flush=True)
    for (v, w, f), xs in sorted(res.items()):
        ms = [x[0] for x in xs]
        rays = xs[0][1]
        med = statistics.median(ms)
        print(json.dumps({"variant": v, "waves_per_cu": w, "refill": f, "median_ms": round(med, 2), "min_ms": round(min(ms), 2),
                          "mray_s": round(rays / med / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
