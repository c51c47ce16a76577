"""Per-phase time of each wavefront render pass from a rocprofv3 kernel trace.
    python scripts/pass_breakdown.py gpurun_out/prof_r01/trace/trace_kernel_trace.csv
A pass starts at wf_camera; trace launches are numbered by generation.  The
counting launch (FULL build) is marked "counting" and is not a timed pass.
"""
import csv
import json
import re
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    passes, cur = [], None
    for r in rows:
        if "wf_camera" in r["Kernel_Name"]:
            cur = []
            passes.append(cur)
        if cur is not None:
            cur.append(r)
    for p in passes:
        g, acc, tot, counting = 0, {}, 0.0, False
        for r in p:
            n = r["Kernel_Name"]
            ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            tot += ms
            if "wf_trace<false" in n:
                g += 1
                k = "g%d closest" % g
                counting |= re.search(r"wf_trace<false, true,", n) is not None
            elif "wf_trace<true" in n:
                k = "g%d shadow" % g
            elif "wf_tail" in n:
                k = "tail (g%d..)" % (g + 1)
                counting |= "wf_tail<true" in n
            elif "rocprim" in n:
                k = "sort"
            elif "wf_shade" in n or "wf_bounce" in n:
                k = "shade+bounce"
            elif "__amd_rocclr" in n:
                k = "copies/fills"
            else:
                k = n.split("(")[0].split("::")[-1]
            acc[k] = acc.get(k, 0.0) + ms
        wall = (max(int(r["End_Timestamp"]) for r in p) - int(p[0]["Start_Timestamp"])) / 1e6
        print(json.dumps({"pass_ms": round(tot, 1), "wall_ms": round(wall, 1), "gaps_ms": round(wall - tot, 1),
                          "counting": counting,
                          "phases_ms": {k: round(v, 1) for k, v in acc.items()}}))


if __name__ == "__main__":
    main()
