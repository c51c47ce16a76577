"""Summarise scripts/pmc_mem.sh (memory path of the trace kernels) into a JSON file, per lean trace kind,
per launch: L1 (TCP) tag lookups and their rate per CU-cycle, L1 miss rate (TCP->TCC read requests over
lookups), mean L2 read latency, L2 hit rate, the address unit's stall on the L1, the waves' wait share.
    python scripts/pmc_mem_summary.py gpurun_out/pmc_mem profiles/r05_pmc_mem_sponza.json
"""
import collections
import csv
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from kernel_names import trace_info  # noqa: E402


def main(src, dst):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    ns = collections.defaultdict(dict)
    for p in ("c", "d"):
        for r in csv.DictReader(open(Path(src) / p / "pmc_counter_collection.csv")):
            info = trace_info(r["Kernel_Name"])
            if not info or info[1] != "lean":
                continue
            agg[info[0]][r["Counter_Name"]] += float(r["Counter_Value"])
            if p == "c":
                ns[info[0]][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {}
    for k, v in agg.items():
        n = len(ns[k])
        cyc = v["GRBM_GUI_ACTIVE"] / 8  # per XCD: the kernels' cycles
        acc = v["TCP_TOTAL_CACHE_ACCESSES_sum"]
        out[k] = {"launches": n, "avg_launch_ms": round(sum(ns[k].values()) / n / 1e6, 3),
                  "l1_lookups_per_launch": acc / n,
                  "l1_lookups_per_cu_cycle": round(acc / 256 / cyc, 3),
                  "l1_miss_rate": round(v["TCP_TCC_READ_REQ_sum"] / acc, 4),
                  "l2_read_latency_cycles": round(v["TCP_TCC_READ_REQ_LATENCY_sum"] / v["TCP_TCC_READ_REQ_sum"], 1),
                  "l2_hit_rate": round(v["TCC_HIT_sum"] / (v["TCC_HIT_sum"] + v["TCC_MISS_sum"]), 4),
                  "ta_addr_stalled_by_l1": round(v["TA_ADDR_STALLED_BY_TC_CYCLES_sum"] / 256 / cyc, 4),
                  "vmem_rd_insts_per_launch": v["SQ_INSTS_VMEM_RD"] / n,
                  "l1_lookups_per_vmem_inst": round(acc / max(v["SQ_INSTS_VMEM_RD"], 1), 2),
                  "wave_wait_share": round(v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"], 4)}
    json.dump({"source": "scripts/pmc_mem.sh (rocprofv3 --pmc, two passes, no trace domains)", "kinds": out},
              open(dst, "w"), indent=1)
    for k, v in out.items():
        print(k, v)


if __name__ == "__main__":
    main(*sys.argv[1:3])
