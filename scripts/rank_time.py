"""Per-rank render time of the tile split on ONE GPU (rehearses N-GPU scaling
without N GPUs): renders EVERY rank's tiles of an N-way split one after another
and reports each rank's pass time; a strong-scaling step ends with the slowest
rank, so the projected speedup is t(1) / max over ranks of t(rank), for N in
--nranks.  --layers L renders up to L progressive layers per pass (what fits one path
chunk: cr_layers_per_pass, 1 for the whole frame), as bench.py does; times are per layer.
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
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE", help="cr_set_option (experiments)")
    ap.add_argument("--tile", type=int, default=32, help="tile edge of the split (bench.py: 32)")
    ap.add_argument("--layers", type=int, default=32, help="layers per pass group (bench.py --layers-per-pass)")
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
    for kv in args.opt:
        key, val = kv.split("=", 1)
        dev.set_option(key, int(val, 0))
    spp = args.spp or i["samples"]
    cam = ca.camera(i["VP"], i["LA"], i["UP"], i["yview"], i["xres"], i["yres"])
    res = {}
    for r in range(args.rounds):
        for n in (int(x) for x in args.nranks.split(",")):
            for rank in range(n):
                p = ca.render_params(i["xres"], i["yres"], spp, i["k"], i["seed"], rank=rank, nranks=n,
                                     tile=args.tile)
                if n == 1:  # one GPU: the frame in pieces, as DistributedFrame.plan_layers / bench.py
                    from chiaroscuro_amd.tiles import DistributedFrame
                    fr = DistributedFrame(dev, i["xres"], i["yres"], 0, 1, args.tile)
                    nl, pieces = fr.plan_layers(p, args.layers)
                    fr.render_layers(cam, p, nl, pieces=pieces)
                    torch.cuda.synchronize()
                    st = fr.last_stats()
                    ms, c = st["kernel_ms"], st["counters"]
                else:
                    nl, pieces = dev.layers_per_group(p, args.layers), 1  # (pieces inside the library)
                    tiles = torch.zeros((nl, ca.Device.tiles_for_rank(p, 0), args.tile, args.tile, 3),
                                        dtype=torch.float32, device="cuda")
                    dev.render_tiles_layers_device(cam, p, nl, tiles.data_ptr())
                    torch.cuda.synchronize()
                    ms, c = dev.last_kernel_ms(), dev.counters()
                res.setdefault(n, {}).setdefault(rank, []).append(
                    (ms / nl, (c["closest"] + c["shadow"]) / nl, nl, pieces))
    base = None
    for n, ranks in sorted(res.items()):
        ms = {rk: statistics.median(x[0] for x in xs) for rk, xs in ranks.items()}
        rays = sum(xs[0][1] for xs in ranks.values())
        slow = max(ms, key=ms.get)
        base = base or ms[0]
        print(json.dumps({"nranks": n, "rank_ms": [round(ms[rk], 2) for rk in sorted(ms)], "max_rank_ms":
                          round(ms[slow], 2), "slowest_rank": slow, "rank0_ms": round(ms[0], 2),
                          "imbalance": round(ms[slow] / (sum(ms.values()) / n), 3),
                          "projected_mray_s": round(rays / ms[slow] / 1e3, 1), "ideal_ms": round(base / n, 2),
                          "projected_speedup": round(base / ms[slow], 2),
                          "layers_per_pass": ranks[0][0][2], "pieces": ranks[0][0][3],
                          "rank_mrays": [round(ranks[rk][0][1] / 1e6, 2) for rk in sorted(ranks)]}), flush=True)


if __name__ == "__main__":
    main()
