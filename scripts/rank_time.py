"""Per-rank render time of the tile split on ONE GPU (rehearses N-GPU scaling
without N GPUs): renders EVERY rank's tiles of an N-way split one after another
and reports each rank's pass time; a strong-scaling step ends with the slowest
rank, so the projected speedup is t(1) / max over ranks of t(rank), for N in
--nranks.  --layers L renders up to L progressive layers per pass (what fits one path
chunk: cr_layers_per_pass, 1 for the whole frame), as bench.py does; times are per layer.
For N > 1 the root's side of a group is timed too: ONE blend of the group's layers from the
gathered [N][layers][tiles] buffers (cr_blend_tiles_layers_device, what cr_group_render_layers /
cr_render_dist_layers_device / DistributedFrame run), and the gather priced at one xGMI link per
peer (each peer's buffer over its own ~153 GB/s link to the root, all in parallel:
MI355X_MICROARCH.md); `step_ms` = slowest rank + gather + blend, per layer.
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
    root = {}  # n -> [(blend ms of a group, gather bytes per peer, layers)]
    XGMI_GBS = 153.0
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
                if n > 1 and rank == 0:  # the root's blend of the group, from gathered buffers of this size
                    frame = torch.zeros((i["yres"], i["xres"], 3), dtype=torch.float32, device="cuda")
                    gathered = torch.rand((n,) + tuple(tiles.shape), dtype=torch.float32, device="cuda")
                    q = ca.render_params(i["xres"], i["yres"], spp, i["k"], i["seed"], layer=1, nranks=n,
                                         tile=args.tile)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    dev.blend_tiles_layers_device(q, nl, gathered.data_ptr(), frame.data_ptr())  # (warm)
                    e0.record()
                    dev.blend_tiles_layers_device(q, nl, gathered.data_ptr(), frame.data_ptr())
                    e1.record()
                    torch.cuda.synchronize()
                    root.setdefault(n, []).append((e0.elapsed_time(e1), tiles.numel() * 4, nl))
                    del gathered, frame
    base = None
    for n, ranks in sorted(res.items()):
        ms = {rk: statistics.median(x[0] for x in xs) for rk, xs in ranks.items()}
        extra = {}
        if n in root:
            nl = root[n][0][2]
            blend = statistics.median(x[0] for x in root[n]) / nl
            gather = root[n][0][1] / (XGMI_GBS * 1e9) * 1e3 / nl  # ms per layer, peers in parallel
            extra = {"root_blend_ms": round(blend, 3), "gather_ms_xgmi_model": round(gather, 3),
                     "gather_bytes_per_peer_per_group": root[n][0][1]}
        rays = sum(xs[0][1] for xs in ranks.values())
        slow = max(ms, key=ms.get)
        base = base or ms[0]
        print(json.dumps({"nranks": n, "rank_ms": [round(ms[rk], 2) for rk in sorted(ms)], "max_rank_ms":
                          round(ms[slow], 2), "slowest_rank": slow, "rank0_ms": round(ms[0], 2),
                          "imbalance": round(ms[slow] / (sum(ms.values()) / n), 3),
                          "projected_mray_s": round(rays / ms[slow] / 1e3, 1), "ideal_ms": round(base / n, 2),
                          "projected_speedup": round(base / ms[slow], 2),
                          "layers_per_pass": ranks[0][0][2], "pieces": ranks[0][0][3],
                          "rank_mrays": [round(ranks[rk][0][1] / 1e6, 2) for rk in sorted(ranks)], **extra,
                          **({"step_ms": round(ms[slow] + extra["root_blend_ms"] + extra["gather_ms_xgmi_model"], 2),
                              "projected_speedup_with_gather": round(base / (ms[slow] + extra["root_blend_ms"] +
                                                                             extra["gather_ms_xgmi_model"]), 2)}
                             if extra else {})}), flush=True)


if __name__ == "__main__":
    main()
