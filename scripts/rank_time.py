"""Per-rank render time of the tile split on ONE GPU (rehearses N-GPU scaling
without N GPUs): renders rank 0's tiles of an N-way split and reports the pass
time and Mray/s, for N in --nranks.
    python scripts/rank_time.py [--config sponza] [--nranks 1,2,4,8] [--rounds 2]
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
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--nranks", default="1,2,4,8")
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    import torch
    import chiaroscuro_amd as ca
    from chiaroscuro_amd import scenes

    sc = ca.Scene(scenes.config_rtc(args.config))
    i = sc.info
    m = ca.Model(sc)
    dev = ca.Device(0)
    dev.upload(ca.KDTree(m, sc).describe())
    dev.set_option("counters", 0)
    spp = args.spp or i["samples"]
    cam = ca.camera(i["VP"], i["LA"], i["UP"], i["yview"], i["xres"], i["yres"])
    res = {}
    for r in range(args.rounds):
        for n in (int(x) for x in args.nranks.split(",")):
            p = ca.render_params(i["xres"], i["yres"], spp, i["k"], i["seed"], rank=0, nranks=n)
            tiles = torch.zeros((ca.Device.tiles_for_rank(p, 0), 32, 32, 3), dtype=torch.float32, device="cuda")
            dev.render_tiles_device(cam, p, tiles.data_ptr())
            torch.cuda.synchronize()
            c = dev.counters()
            res.setdefault(n, []).append((dev.last_kernel_ms(), c["closest"] + c["shadow"]))
    base = None
    for n, xs in sorted(res.items()):
        ms = statistics.median(x[0] for x in xs)
        rays = xs[0][1]
        base = base or ms
        print(json.dumps({"nranks": n, "rank0_ms": round(ms, 2), "rank0_mray_s": round(rays / ms / 1e3, 1),
                          "ideal_ms": round(base / n, 2), "projected_speedup": round(base / ms, 2)}), flush=True)


if __name__ == "__main__":
    main()
