"""Config C5 (BASELINE.json configs[4]): sponza stand-in 3840x2160, 3000 spp as
30 progressive layers of 100 spp (src/rayTracer.cpp:18-33, 64), each layer
tile-split over the ranks and gathered to rank 0 (chiaroscuro_amd.tiles.
DistributedFrame), on 1 GPU or under torch.distributed.run on N.

Layers run in pass groups of up to --layers-per-pass layers (DistributedFrame.plan_layers /
render_layers; 1 = one layer per pass).  Reports per-group device time and wall
time, the whole-run Mray/s, and checks
the finished frame against the oracle on every --check-ystep-th full row (all 30
layers rendered and blended by the oracle the same way; bit-exact), plus that
the frame stays finite and non-negative.

    python scripts/c5_progressive.py [--layers 30] [--spp 100] [--check-ystep 135]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "chiaroscuro-raytracer_amd", ROOT / "oracle"):
    sys.path.insert(0, str(p))
os.environ.setdefault("CHIARO_QUIET", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="sponza_4k")
    ap.add_argument("--layers", type=int, default=30)
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--check-ystep", type=int, default=135,
                    help="oracle check on rows 0, ystep, 2 ystep, ... (0: no check; one oracle thread per row)")
    ap.add_argument("--gather", default="torch")
    ap.add_argument("--layers-per-pass", type=int, default=32)
    args = ap.parse_args()
    import torch
    import chiaroscuro_amd as ca
    from chiaroscuro_amd import scenes
    from chiaroscuro_amd.tiles import DistributedFrame

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    sc = ca.Scene(scenes.config_rtc(args.config))
    i = sc.info
    m = ca.Model(sc)
    kd = ca.KDTree(m, sc)
    dev = ca.Device(local)
    dev.upload(kd.describe())
    dev.set_option("counters", 0)
    xres, yres, k, seed = i["xres"], i["yres"], i["k"], i["seed"]
    spp = args.spp or i["samples"]
    cam = ca.camera(i["VP"], i["LA"], i["UP"], i["yview"], xres, yres)
    stream = torch.cuda.current_stream().cuda_stream
    fr = DistributedFrame(dev, xres, yres, rank, world, 32, dist, gather=args.gather)
    layers, rays = [], 0
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    L = 1
    while L <= args.layers:
        p = ca.render_params(xres, yres, spp, k, seed, layer=L, rank=rank, nranks=world, tile=32)
        n, pieces = fr.plan_layers(p, min(args.layers_per_pass, args.layers - L + 1))
        tl = time.perf_counter()
        fr.render_layers(cam, p, n, stream, pieces)
        torch.cuda.synchronize()
        st = fr.last_stats()
        c = st["counters"]
        rays += c["closest"] + c["shadow"]
        layers.append({"layers": [L, L + n - 1], "pieces": pieces, "passes": st["passes"],
                       "wall_ms": round((time.perf_counter() - tl) * 1e3, 2),
                       "render_ms": round(st["kernel_ms"], 2)})
        if rank == 0:
            print("group %s" % (layers[-1],), file=sys.stderr, flush=True)
        L += n
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    wall = time.perf_counter() - t0
    if dist:
        t = torch.tensor([rays], dtype=torch.float64, device="cuda")
        dist.all_reduce(t)
        rays = float(t.item())
    out = {"config": "C5 %s %dx%d, %d layers x %d spp, %d rank(s), gather %s, up to %d layers per pass" % (
        args.config, xres, yres, args.layers, spp, world, args.gather if world > 1 else "-", args.layers_per_pass),
        "wall_s": round(wall, 3), "rays": int(rays), "mray_s": round(rays / wall / 1e6, 2),
        "ms_per_layer": round(wall * 1e3 / args.layers, 2), "trace_build": dev.last_trace_build(),
        "groups": layers}
    if rank == 0:
        f = fr.frame.cpu().numpy()
        out["frame_finite_nonneg"] = bool(np.isfinite(f).all() and (f >= 0).all())
        out["frame_mean"] = float(f.mean())
        if args.check_ystep:
            import pyoracle as po
            osc = po.OracleScene(m.triangles(), leaf_size=i["leaf_size"], textures=m.textures(),
                                 build_threads=int(os.environ.get("OMP_NUM_THREADS", "16")))
            t1 = time.time()
            o = np.zeros((yres, xres, 3), np.float32)
            rows = list(range(0, yres, args.check_ystep))
            for L in range(1, args.layers + 1):
                osc.render(cam.as_array(), xres, yres, spp, k, seed, layer=L, pixels=o, ystep=args.check_ystep)
            bad = int((f[rows].view(np.uint32) != o[rows].view(np.uint32)).sum())
            out["oracle_rows"] = rows
            out["oracle_row_mismatches"] = bad
            out["oracle_s"] = round(time.time() - t1, 1)
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
