"""Timeline of the first timed wavefront pass from a rocprofv3 kernel trace:
    python scripts/timeline.py <kernel_trace.csv> [pass index]
One line per kernel: start offset and duration (ms), queue id, short name."""
import csv
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from kernel_names import short  # noqa: E402


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    want = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    passes, cur = [], None
    for r in rows:
        if "wf_camera" in r["Kernel_Name"]:
            cur = []
            passes.append(cur)
        if cur is not None:
            cur.append(r)
    p = passes[min(want, len(passes) - 1)]
    t0 = int(p[0]["Start_Timestamp"])
    for r in p:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print("%9.3f %9.3f  q%-3s %s" % ((s - t0) / 1e6, (e - s) / 1e6, r.get("Queue_Id", r.get("Stream_Id", "?")),
                                         short(r["Kernel_Name"])))


if __name__ == "__main__":
    main()
