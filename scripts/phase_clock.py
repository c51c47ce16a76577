"""Phase clock of the wavefront trace kernels (measurement builds 23 / 24 of
wavefront.hip): shader-clock cycles per wave spent in trav_round's kd descent, leaf
cull, leaf tests and stack pop, against the persistent loop's total, for the
shadow-ray or the secondary closest-ray trace of one lean render.

    python scripts/phase_clock.py [--config sponza] [--variants 23,24] [--kind shadow]
"""
import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "chiaroscuro-raytracer_amd"))
os.environ.setdefault("CHIARO_QUIET", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sponza")
    ap.add_argument("--spp", type=int, default=128)
    ap.add_argument("--variants", default="23,24")
    ap.add_argument("--kinds", default="shadow,closest")
    args = ap.parse_args()
    import torch
    import chiaroscuro_amd as ca
    from chiaroscuro_amd import scenes

    sc = ca.Scene(scenes.config_rtc(args.config))
    i = sc.info
    kd = ca.KDTree(ca.Model(sc), sc)
    dev = ca.Device(0)
    dev.upload(kd.describe())
    cam = ca.camera(i["VP"], i["LA"], i["UP"], i["yview"], i["xres"], i["yres"])
    frame = torch.zeros((i["yres"], i["xres"], 3), dtype=torch.float32, device="cuda")
    dev.set_option("counters", 0)
    out = {}
    for v in args.variants.split(","):
        dev.set_option("variant", int(v))
        for kind in args.kinds.split(","):
            dev.set_option("diag_kinds", {"closest": 2, "shadow": 4}[kind])
            p = ca.render_params(i["xres"], i["yres"], args.spp, i["k"], i["seed"])
            dev.render_device(cam, p, frame.data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            g = dev.diag()
            vals = list(g.values())[:8]
            names = ("descent", "cull", "tests", "pop", "calls", "loop_total", "refill", "refills")
            r = dict(zip(names, vals))
            frac = {k: round(r[k] / max(r["loop_total"], 1), 3) for k in ("descent", "cull", "tests", "pop", "refill")}
            frac["rest"] = round(1 - sum(frac.values()), 3)
            frac["calls_per_refill"] = round(r["calls"] / max(r["refills"], 1), 2)
            frac["cycles_per_refill"] = round(r["refill"] / max(r["refills"], 1), 1)
            ts = dev.trace_stats()[kind]
            out["%s/%s" % (v, kind)] = {"frac": frac, "cycles_per_call": {k: round(r[k] / max(r["calls"], 1), 1)
                                                                          for k in ("descent", "cull", "tests", "pop")},
                                        "ms": round(ts["ms"], 2), "launches": ts["launches"]}
            print(v, kind, json.dumps(out["%s/%s" % (v, kind)]), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
