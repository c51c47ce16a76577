"""A/B render options in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Usage:
    python scripts/sweep.py [--config sponza] [--spp 8] [--rounds 3] \
        --grid kernel=0,2 --grid refill=16,48 --grid wf_dir_res=4,8 ...
Every --grid names a cr_set_option key and its values; the cartesian product is
swept (defaults for everything not named).  Prints one JSON line per
configuration (median / min ms and Mray/s) and checks that every configuration
renders the identical image.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sponza")
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--grid", action="append", default=[], help="option=v1,v2,...")
    ap.add_argument("--nranks", type=int, default=1, help="render rank 0's tiles of an N-way tile split")
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
    if args.nranks > 1:
        p0 = ca.render_params(xres, yres, args.spp, k, seed, layer=1, rank=0, nranks=args.nranks)
        frame = torch.zeros((ca.Device.tiles_for_rank(p0, 0), 32, 32, 3), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    dev.set_option("counters", 0)
    keys, values = [], []
    for g in args.grid:
        key, vals = g.split("=")
        keys.append(key)
        values.append([int(v) for v in vals.split(",")])
    configs = list(itertools.product(*values)) if keys else [()]
    res = {}
    ref = None
    for r in range(args.rounds):
        for cfg in configs:
            for key, v in zip(keys, cfg):
                dev.set_option(key, v)
            p = ca.render_params(xres, yres, args.spp, k, seed, layer=1, rank=0, nranks=args.nranks)
            if args.nranks > 1:
                dev.render_tiles_device(cam, p, frame.data_ptr(), stream)
            else:
                dev.render_device(cam, p, frame.data_ptr(), stream)
            torch.cuda.synchronize()
            c = dev.counters()
            if ref is None:
                ref = frame.clone()
            else:
                assert torch.equal(frame, ref), "configuration %s changed the image" % (dict(zip(keys, cfg)),)
            res.setdefault(cfg, []).append((dev.last_kernel_ms(), c["closest"] + c["shadow"]))
        print("round %d done" % r, file=sys.stderr, flush=True)
    for cfg, xs in res.items():
        ms = [x[0] for x in xs]
        rays = xs[0][1]
        med = statistics.median(ms)
        out = dict(zip(keys, cfg))
        out.update({"median_ms": round(med, 2), "min_ms": round(min(ms), 2), "mray_s": round(rays / med / 1e3, 1)})
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
