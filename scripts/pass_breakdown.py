"""Per-phase time of each wavefront render pass from a rocprofv3 kernel trace.
    python scripts/pass_breakdown.py gpurun_out/prof_r01/trace/trace_kernel_trace.csv
A pass starts at wf_camera, or at the packet camera trace when no wf_camera precedes it (the
fused camera, WfArgs::cam_fused); trace launches are numbered by generation (closest and
shadow separately: shadow g runs beside closest g + 1).  pass_ms sums kernel
times, busy_ms is the union of their intervals, overlap_ms the difference.  The
counting launch (FULL build) is marked "counting" and is not a timed pass.
"""
import csv
import json
import re
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from kernel_names import trace_info  # noqa: E402


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    passes, cur, prev = [], None, ""
    for r in rows:
        n = r["Kernel_Name"]
        if "wf_camera" in n or ("wf_trace_packet" in n and "wf_camera" not in prev):
            cur = []
            passes.append(cur)
        if cur is not None:
            cur.append(r)
        prev = n
    for p in passes:
        g, gs, acc, tot, counting = 0, 0, {}, 0.0, False
        for r in p:
            n = r["Kernel_Name"]
            ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            tot += ms
            info = trace_info(n)
            if info and info[0] in ("camera", "closest"):
                g += 1
                k = "g%d closest" % g
                counting |= info[1] != "lean"
            elif info and info[0] == "shadow":
                gs += 1
                k = "g%d shadow" % gs
            elif info and info[0] == "tail":
                k = "tail (g%d..)" % (gs + 1)
                counting |= info[1] != "lean"
            elif "rocprim" in n or "rs_upsweep" in n or "rs_downsweep" in n or "rs_scan" in n:
                k = "sort"
            elif "wf_shade" in n or "wf_bounce" in n or "wf_resolve" in n:
                k = "shade+resolve"
            elif "__amd_rocclr" in n:
                k = "copies/fills"
            else:
                k = n.split("(")[0].split("::")[-1]
            acc[k] = acc.get(k, 0.0) + ms
        wall = (max(int(r["End_Timestamp"]) for r in p) - int(p[0]["Start_Timestamp"])) / 1e6
        busy, end = 0, None  # union of the kernel intervals (kernels on two streams overlap)
        for a, b in sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in p):
            if end is None or a > end:
                busy += b - a
                end = b
            elif b > end:
                busy += b - end
                end = b
        busy /= 1e6
        print(json.dumps({"pass_ms": round(tot, 1), "wall_ms": round(wall, 1), "busy_ms": round(busy, 1),
                          "overlap_ms": round(tot - busy, 1), "gaps_ms": round(wall - busy, 1),
                          "counting": counting,
                          "phases_ms": {k: round(v, 1) for k, v in acc.items()}}))


if __name__ == "__main__":
    main()
