"""Summarise scripts/pmc_issue.sh (instruction mix per trace kernel) into a JSON file:
per dispatch-averaged instruction counts and the issue utilisation they imply,
    VALU busy = SQ_INSTS_VALU x 2 cycles (wave64 f32 throughput, MI355X_MICROARCH.md)
                / (1024 SIMDs x shader clock x kernel time)
    SALU busy = SQ_INSTS_SALU / (256 CUs x shader clock x kernel time)  (one scalar
                unit per CU, one instruction per cycle)
with the shader clock from SQ_BUSY_CYCLES / (32 shader engines x kernel time), and
    TA busy   = TA_BUSY_avr / (GRBM_GUI_ACTIVE / 8 XCDs)  (vector-memory address path)
    VALU lanes = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU)  (rocprofv3's VALUUtilization:
                the active lanes of an issued VALU instruction, pass c)
    python scripts/pmc_issue_summary.py gpurun_out/pmc_issue/a/pmc_counter_collection.csv \
        profiles/pmc_issue_sponza.json [spp]
"""
import collections
import csv
import json
import re
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from kernel_names import trace_info  # noqa: E402


def main(src, dst, spp=128):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    ns = collections.defaultdict(dict)
    srcb = src.replace("/a/", "/b/")  # pass b: TA busy (vector-memory address path)
    srcc = src.replace("/a/", "/c/")  # pass c: VALU lane utilisation
    for f in (src, srcb, srcc):
        try:
            rows = list(csv.DictReader(open(f)))
        except FileNotFoundError:
            continue
        for r in rows:
            k = r["Kernel_Name"]
            if "wf_trace" not in k and "wf_tail" not in k:
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if f == src:
                ns[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {}
    for k, v in agg.items():
        t = sum(ns[k].values()) * 1e-9
        clk = v["SQ_BUSY_CYCLES"] / 32 / t
        cyc = clk * t
        out[k] = {
            "dispatches": len(ns[k]), "seconds": round(t, 4), "shader_clock_ghz": round(clk / 1e9, 3),
            **{c: v[c] for c in sorted(v)},
            "valu_issue_busy": round(v["SQ_INSTS_VALU"] * 2 / (1024 * cyc), 3),
            "salu_issue_busy": round(v["SQ_INSTS_SALU"] / (256 * cyc), 3),
            "branch_per_cu_cycle": round(v["SQ_INSTS_BRANCH"] / (256 * cyc), 3),
            "salu_per_valu": round(v["SQ_INSTS_SALU"] / v["SQ_INSTS_VALU"], 3),
        }
        if v.get("GRBM_GUI_ACTIVE"):  # TA busy cycles (average TA) over the kernel's cycles per XCD
            out[k]["ta_busy"] = round(v["TA_BUSY_avr"] / (v["GRBM_GUI_ACTIVE"] / 8), 3)
        if v.get("SQ_ACTIVE_INST_VALU"):
            out[k]["valu_lane_util"] = round(v["SQ_THREAD_CYCLES_VALU"] / (64 * v["SQ_ACTIVE_INST_VALU"]), 3)
    # per lean trace kind (bench.py roofline.issue): SHADOW, FULL, ..., CAM[, BF] template args
    kinds = {}
    for k, v in out.items():
        info = trace_info(k)
        if not info or info[0] == "tail" or info[1] != "lean":
            continue  # the counting and performed-work instances, the tail kernel
        kind = info[0]
        d = v["dispatches"]
        kinds[kind] = {"kernel": k, "valu_issue_busy": v["valu_issue_busy"], "salu_issue_busy": v["salu_issue_busy"],
                       "ta_busy": v.get("ta_busy"), "valu_lane_util": v.get("valu_lane_util"),
                       "shader_clock_ghz": v["shader_clock_ghz"],
                       "salu_per_valu": v["salu_per_valu"], "dispatches": d,
                       "avg_launch_ms": round(v["seconds"] * 1e3 / d, 3),
                       # per-launch instruction counts: bench.py roofline (issue ceilings) divides
                       # them by its own live HIP-event launch time
                       "valu_insts_per_launch": v["SQ_INSTS_VALU"] / d,
                       "salu_insts_per_launch": v["SQ_INSTS_SALU"] / d,
                       "vmem_rd_insts_per_launch": v["SQ_INSTS_VMEM_RD"] / d}
    json.dump({"spp": spp, "note": __doc__.strip().split("\n\n")[0], "kinds": kinds, "kernels": out},
              open(dst, "w"), indent=1)
    for k, v in out.items():
        print(k[:70], v["valu_issue_busy"], v["salu_issue_busy"], v["shader_clock_ghz"])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 128)
