"""A/B the render kernels / variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Usage:
    python scripts/sweep.py [--config sponza] [--spp 8] [--rounds 3] [--kernel 0,2]
                            [--variants 0,1,2] [--waves 0] [--refill 16] [--wf-paths 0]
Prints one JSON line per configuration: median / min ms and Mray/s, and checks
that every configuration renders the identical image.
"""
import argparse
import itertools
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "chiaroscuro-raytracer_amd"))
os.environ.setdefault("CHIARO_QUIET", "1")


def ints(s):
    return [int(x) for x in s.split(",")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sponza")
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--kernel", default="2", help="0 persistent megakernel, 2 wavefront (default)")
    ap.add_argument("--variants", default="-1", help="-1 = the kernel's default build")
    ap.add_argument("--waves", default="0", help="waves_per_cu (persistent kernel; 0 = default)")
    ap.add_argument("--refill", default="0", help="refill thresholds (0 = the kernel's default)")
    ap.add_argument("--wf-paths", default="0", help="wavefront paths per chunk (0 = default)")
    ap.add_argument("--refill-shadow", default="0", help="wavefront shadow-trace thresholds (0 = refill)")
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
    configs = list(itertools.product(ints(args.kernel), ints(args.variants), ints(args.waves), ints(args.refill),
                                     ints(args.wf_paths), ints(args.refill_shadow)))
    res = {}
    ref = None
    for r in range(args.rounds):
        for cfg in configs:
            kern, v, w, f, wp, fs = cfg
            dev.set_option("kernel", kern)
            dev.set_option("variant", v)
            dev.set_option("waves_per_cu", w)
            dev.set_option("refill", f)
            dev.set_option("refill_shadow", fs)
            dev.set_option("wf_paths", wp or (256 << 20))
            p = ca.render_params(xres, yres, args.spp, k, seed, layer=1)
            dev.render_device(cam, p, frame.data_ptr(), stream)
            torch.cuda.synchronize()
            c = dev.counters()
            if ref is None:
                ref = frame.clone()
            else:
                assert torch.equal(frame, ref), "configuration %s changed the image" % (cfg,)
            res.setdefault(cfg, []).append((dev.last_kernel_ms(), c["closest"] + c["shadow"]))
        print("round %d done" % r, file=sys.stderr, flush=True)
    for cfg, xs in res.items():
        ms = [x[0] for x in xs]
        rays = xs[0][1]
        med = statistics.median(ms)
        kern, v, w, f, wp, fs = cfg
        print(json.dumps({"kernel": kern, "variant": v, "waves_per_cu": w, "refill": f, "refill_shadow": fs,
                          "wf_paths": wp,
                          "median_ms": round(med, 2), "min_ms": round(min(ms), 2),
                          "mray_s": round(rays / med / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
