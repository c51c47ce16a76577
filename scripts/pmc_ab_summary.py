"""Summarise scripts/pmc_ab.sh: per variant and lean trace kind, counters per launch and the mean
launch time.   python3 scripts/pmc_ab_summary.py gpurun_out/pmc_ab 43 49"""
import collections
import csv
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from kernel_names import trace_info  # noqa: E402


def summary(src, v):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    ns = collections.defaultdict(dict)
    for p in ("a", "b"):
        f = Path(src) / ("v%s_%s" % (v, p))
        for r in csv.DictReader(open(next(f.rglob("*counter_collection.csv")))):
            info = trace_info(r["Kernel_Name"])
            if not info or info[1] != "lean":
                continue
            agg[info[0]][r["Counter_Name"]] += float(r["Counter_Value"])
            if p == "a":
                ns[info[0]][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {}
    for k, c in agg.items():
        n = max(len(ns[k]), 1)
        out[k] = {"launches": n, "avg_ms": round(sum(ns[k].values()) / n / 1e6, 3)}
        for name, val in sorted(c.items()):
            out[k][name] = val / n if not name.endswith("_avr") else val / n
        if c.get("SQ_WAVE_CYCLES"):
            out[k]["wait_share"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
    return out


def main(src, *vs):
    res = {v: summary(src, v) for v in vs}
    json.dump(res, open(Path(src) / "summary.json", "w"), indent=1)
    kinds = sorted({k for r in res.values() for k in r})
    for k in kinds:
        print("==", k)
        names = sorted({n for r in res.values() for n in r.get(k, {})})
        for n in names:
            print("  %-32s" % n, "  ".join("%14.4g" % res[v].get(k, {}).get(n, float("nan")) for v in vs))


if __name__ == "__main__":
    main(*sys.argv[1:])
