"""Summarise a scripts/profile.sh output directory into profiles/.

    python scripts/prof_summary.py gpurun_out/prof_r01 r01 [--config sponza]

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_pmc.json           per-kernel PMC averages per dispatch + derived figures
  profiles/pmc_<config>.json        fabric bytes per launch of the timed render kernel,
                                    read by bench.py for roofline.traffic
Derived (MI355X_MICROARCH.md, HBM section): FETCH_SIZE/WRITE_SIZE are KiB of
L2 memory-side requests; gfx950 tallies 128-B read requests at 64 B, so reads
are doubled.  Infinity-Cache hits are included in those counters, so the
figure is L2-miss (fabric) traffic, an upper bound on HBM bytes.
"""
import collections
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def pmc(dirpath):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in Path(dirpath).glob("*/pmc_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            out[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in out.items()}


def main():
    src, tag = Path(sys.argv[1]), sys.argv[2]
    config = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "sponza"
    prof = ROOT / "profiles"
    prof.mkdir(exist_ok=True)
    stats = next(src.glob("trace/*kernel_stats.csv"))
    shutil.copy(stats, prof / ("%s_kernel_stats.csv" % tag))
    rows = list(csv.DictReader(open(stats)))
    durations = {r["Name"]: float(r["AverageNs"]) for r in rows}
    counters = pmc(src)
    summary = {}
    for name, c in counters.items():
        if "render_" not in name and "sum_samples" not in name:
            continue
        e = dict(c)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["fabric_bytes_per_launch"] = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            e["l2_hit_rate"] = c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1.0)
        if "SQ_WAVE_CYCLES" in c:
            w = c["SQ_WAVE_CYCLES"]
            e["wave_time_split"] = {k: c.get(k, 0.0) / w for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY",
                                                                   "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU")}
        d = durations.get(name)
        if d:
            e["avg_duration_ns"] = d
            if "fabric_bytes_per_launch" in e:
                e["fabric_GBps"] = e["fabric_bytes_per_launch"] / d
        summary[name] = e
    (prof / ("%s_pmc.json" % tag)).write_text(json.dumps(summary, indent=1, sort_keys=True))
    timed = [n for n in summary if "render_dynamic" in n and "true, true, 1" not in n]
    if timed:
        t = summary[timed[0]]
        (prof / ("pmc_%s.json" % config)).write_text(json.dumps({
            "kernel": timed[0], "source": "profiles/%s_pmc.json" % tag,
            "hbm_bytes_per_launch": t.get("fabric_bytes_per_launch"),
            "note": "2*FETCH_SIZE+WRITE_SIZE (KiB) per dispatch; includes Infinity-Cache hits (upper bound on HBM)",
        }, indent=1))
    for n, e in summary.items():
        print(n[:70], {k: (round(v, 4) if isinstance(v, float) else v) for k, v in e.items()
                       if k in ("avg_duration_ns", "fabric_bytes_per_launch", "fabric_GBps", "l2_hit_rate")})


if __name__ == "__main__":
    main()
