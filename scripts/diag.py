"""SIMD-efficiency diagnostics of the wavefront kernel's counting build (one counting render).
    python scripts/diag.py [--config sponza] [--spp 8]
lane efficiency of a phase = lane work / (64 x wave iterations of that phase)."""
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
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--kernel", type=int, default=2)
    ap.add_argument("--variant", type=int, default=-1)
    ap.add_argument("--refill", type=int, default=0)
    ap.add_argument("--k", type=int, default=0, help="path depth override (1: camera + first shadow rays only)")
    args = ap.parse_args()
    import torch
    import chiaroscuro_amd as ca
    from chiaroscuro_amd import scenes

    sc = ca.Scene(scenes.config_rtc(args.config))
    i = sc.info
    m = ca.Model(sc)
    kd = ca.KDTree(m, sc)
    dev = ca.Device(0)
    dev.upload(kd.describe())
    cam = ca.camera(i["VP"], i["LA"], i["UP"], i["yview"], i["xres"], i["yres"])
    frame = torch.zeros((i["yres"], i["xres"], 3), dtype=torch.float32, device="cuda")
    dev.set_option("counters", 1)
    dev.set_option("kernel", args.kernel)
    dev.set_option("variant", args.variant)
    dev.set_option("refill", args.refill)
    p = ca.render_params(i["xres"], i["yres"], args.spp, args.k or i["k"], i["seed"])
    dev.render_device(cam, p, frame.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    c = dev.counters()
    rays = c["closest"] + c["shadow"]
    out = dict(c)
    out.update({
        "ms": round(dev.last_kernel_ms(), 2),
        "per_ray": {"inner": round(c["inner"] / rays, 1), "leaf": round(c["leaf"] / rays, 1),
                    "tritest": round(c["tritest"] / rays, 1)},
        "eff_desc": round(c["inner"] / (64 * max(c["wave_desc"], 1)), 3),
        "eff_tri": round(c["tritest"] / (64 * max(c["wave_tri"], 1)), 3),
        "eff_round": round(c["leaf"] / (64 * max(c["wave_round"], 1)), 3),
        "eff_query": round(rays / (64 * max(c["wave_query"], 1)), 3),
        "rounds_per_query_wave": round(c["wave_round"] / max(c["wave_query"], 1), 1),
        "leaves_per_query_lane": round(c["leaf"] / rays, 1),
        "uniform_desc": round(c["wave_desc_uniform"] / max(c["wave_desc"], 1), 3),
        "uniform_tri": round(c["wave_tri_uniform"] / max(c["wave_tri"], 1), 3),
        "lines_per_desc": round(c["wave_desc_lines"] / max(c["wave_desc"], 1), 2),
        "lines_per_tri": round(c["wave_tri_lines"] / max(c["wave_tri"], 1), 2),
        "nonuniform_leaf_rounds": round(c["leaf_rounds"] / max(c["wave_round"], 1), 3),
        "distinct_leaves_per_round": round(c["leaf_distinct"] / max(c["leaf_rounds"], 1), 2),
        "records_per_round": round(c["leaf_records"] / max(c["leaf_rounds"], 1), 1),
        "rounds_fit21": round(c["leaf_fit21"] / max(c["leaf_rounds"], 1), 3),
        "rounds_fit56": round(c["leaf_fit56"] / max(c["leaf_rounds"], 1), 3),
    })
    ts = dev.trace_stats()  # wavefront: per-kind inner / leaf / tritest (counting build)
    ncam = i["xres"] * i["yres"] * args.spp
    if args.kernel == 2 and "camera" in ts:
        out["camera_per_ray"] = {k: round(ts["camera"][k] / ncam, 1) for k in ("inner", "leaf", "tritest")}
        out["trace_stats"] = ts
    print(json.dumps(out))


if __name__ == "__main__":
    main()
