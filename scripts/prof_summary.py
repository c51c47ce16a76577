"""Summarise a scripts/profile.sh output directory into profiles/.

    python scripts/prof_summary.py gpurun_out/prof_r01 r01 [--config sponza]

The profiled command is bench.py: `warmup + steps` timed render passes plus ONE
counting pass (the FULL-counter trace build), each pass ending with one
sum_samples dispatch.  A render pass is the unit of `roofline` in bench.py.

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_pmc.json           per-kernel PMC sums / averages + per-pass totals
  profiles/pmc_<config>.json        fabric bytes per render pass (timed kernels only),
                                    read by bench.py for roofline.traffic
Derived (MI355X_MICROARCH.md, HBM section): FETCH_SIZE/WRITE_SIZE are KiB of
L2 memory-side requests; gfx950 tallies 128-B read requests at 64 B, so reads
are doubled.  Infinity-Cache hits are included in those counters, so the
figure is L2-miss (fabric) traffic, an upper bound on HBM bytes.
"""
import collections
import csv
import re
import json
import shutil
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from kernel_names import is_counting, trace_info  # noqa: E402

ROOT = Path(__file__).resolve().parents[1]


def main():
    src, tag = Path(sys.argv[1]), sys.argv[2]
    config = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "sponza"
    prof = ROOT / "profiles"
    prof.mkdir(exist_ok=True)
    stats = next(src.glob("trace/*kernel_stats.csv"))
    shutil.copy(stats, prof / ("%s_kernel_stats.csv" % tag))
    rows = {r["Name"]: r for r in csv.DictReader(open(stats))}
    # passes: the timed (lean) renders and ONE counting render.  A render of a large frame runs in
    # several sample chunks (one sum_samples each), so the lean renders are counted by the cull-box
    # kernel, which runs once per lean render of a culling build
    calls = {n: int(r["Calls"]) for n, r in rows.items()}
    cull = [c for n, c in calls.items() if "cam_cull_kernel" in n]
    lean = cull[0] if cull else calls[next(n for n in rows if "sum_samples" in n)] - 1
    passes = lean + 1
    # PMC: sum per kernel over its dispatches (one pass per counter group)
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in src.glob("*/pmc_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            sums[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
    summary, per_pass = {}, collections.defaultdict(float)
    for name, r in rows.items():
        if not any(k in name for k in ("render_", "wf_", "sum_samples", "rocprim", "cam_cull")):  # rocprim: queue sorts
            continue
        counting = is_counting(name)
        # counting-build kernels run in the counting render only, the lean trace / tail / cull kernels in
        # the timed renders only, the rest (camera, shade, resolve, sorts, sum_samples) in both
        lean_only = any(k in name for k in ("wf_trace", "wf_tail", "render_dynamic", "cam_cull"))
        frames = 1 if counting else (lean if lean_only else passes)
        e = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "total_ns": float(r["TotalDurationNs"]),
             "counting_build": counting, "passes": frames}
        c = sums.get(name, {})
        e.update({k: v for k, v in c.items()})
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["fabric_bytes_total"] = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            e["l2_hit_rate"] = c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1.0)
        if "SQ_WAVE_CYCLES" in c:
            w = c["SQ_WAVE_CYCLES"]
            e["wave_time_split"] = {k: c.get(k, 0.0) / w for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY",
                                                                   "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU")}
        summary[name] = e
        if not counting:
            per_pass["duration_ns"] += e["total_ns"] / frames
            if "fabric_bytes_total" in e:
                per_pass["fabric_bytes"] += e["fabric_bytes_total"] / frames
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "TCC_HIT_sum", "TCC_MISS_sum"):
                if k in c:
                    per_pass[k] += c[k] / frames
    per_pass["fabric_GBps"] = per_pass["fabric_bytes"] / max(per_pass["duration_ns"], 1.0)
    out = {"render_pass": dict(per_pass), "kernels": summary, "passes_profiled": passes, "timed_passes": lean}
    (prof / ("%s_pmc.json" % tag)).write_text(json.dumps(out, indent=1, sort_keys=True))
    spp = int(sys.argv[sys.argv.index("--spp") + 1]) if "--spp" in sys.argv else 128
    # the trace kernel's lean instantiations (bench.py roofline): fabric bytes per launch
    trace = {}
    for n, e in summary.items():
        info = trace_info(n)
        if not info or info[0] == "tail" or "fabric_bytes_total" not in e:
            continue
        kind, mode = info
        if mode == "lean":  # the timed builds
            trace[kind] = {
                "kernel": n, "calls": e["calls"], "avg_ns": e["avg_ns"],
                "fabric_bytes_per_launch": e["fabric_bytes_total"] / e["calls"]}
    (prof / ("pmc_%s.json" % config)).write_text(json.dumps({
        "source": "profiles/%s_pmc.json" % tag, "spp": spp, "n_gpus": 1,
        "hbm_bytes_per_launch": per_pass["fabric_bytes"],
        "trace": trace,
        "unit": "one render pass (all timed kernels of one layer); trace: per launch of that kernel",
        "note": "2*FETCH_SIZE+WRITE_SIZE (KiB) summed over the pass's dispatches; includes Infinity-Cache hits "
                "(upper bound on HBM bytes)",
    }, indent=1))
    print(json.dumps(out["render_pass"], indent=1))
    for n, e in summary.items():
        print("%-70s calls %3d avg %10.3f ms%s" % (n[:70], e["calls"], e["avg_ns"] / 1e6,
                                                   "  (counting)" if e["counting_build"] else ""))


if __name__ == "__main__":
    main()
