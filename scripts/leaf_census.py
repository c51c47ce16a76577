"""Leaf-round shapes and the repeated-miss census of the trace kernels (one counting
render per trace kind, cr_get_diag):

  staging   what loading a divergent round's distinct leaves into LDS once per wave
            would take (records, distinct leaves, lanes per leaf) against the
            per-lane loads of the leaf loop (wave iterations = the round's largest leaf)
  mailbox   the lane tests that reject for any segment (det, u, v, t < 0) and repeat
            such a miss of the lane's last 1 / 4 / 8 in the same query -- exact to skip

    python scripts/leaf_census.py [--config sponza] [--spp 128] [--kinds shadow,closest,camera]
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
    ap.add_argument("--kinds", default="shadow,closest,camera")
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
    dev.set_option("counters", 1)
    out = {"config": args.config, "spp": args.spp}
    for kind in args.kinds.split(","):
        bit = {"camera": 1, "closest": 2, "shadow": 4}[kind]
        dev.set_option("diag_kinds", bit)
        p = ca.render_params(i["xres"], i["yres"], args.spp, i["k"], i["seed"])
        dev.render_device(cam, p, frame.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        g = dev.diag()
        ts = dev.trace_stats()[kind]
        r = max(g["rounds"], 1)
        out[kind] = {
            "raw": g, "trace": ts,
            "uniform_round_frac": round(g["urounds"] / max(g["urounds"] + g["rounds"], 1), 3),
            "lanes_per_round": round(g["lanes"] / r, 1),
            "distinct_per_round": round(g["distinct"] / r, 2),
            "lanes_per_leaf": round(g["lanes"] / max(g["distinct"], 1), 2),
            "records_per_round": round(g["records"] / r, 1),
            "maxcount_per_round": round(g["maxcount"] / r, 2),
            "loop_lane_eff": round(g["lanetests"] / max(64 * g["maxcount"], 1), 3),
            "fit21": None, "fit64": round(g["fit64"] / r, 3), "fit128": round(g["fit128"] / r, 3),
            "geomiss_frac": round(g["geomiss"] / max(g["tests"], 1), 3),
            "rep1_frac": round(g["rep1"] / max(g["tests"], 1), 3),
            "rep4_frac": round(g["rep4"] / max(g["tests"], 1), 3),
            "rep8_frac": round(g["rep8"] / max(g["tests"], 1), 3),
        }
        c = dev.counters()
        out[kind]["fit21"] = round(c["leaf_fit21"] / max(c["leaf_rounds"], 1), 3)
        out[kind]["fit56"] = round(c["leaf_fit56"] / max(c["leaf_rounds"], 1), 3)
        print(kind, json.dumps({k: v for k, v in out[kind].items() if k not in ("raw", "trace")}), file=sys.stderr,
              flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
