#!/bin/bash
# Kernel trace of one default bench pass, hand-written queue sort vs hipcub's: per-kernel totals of the sort.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sortprof
for lib in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sortprof/lib$lib -o trace --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --opt wf_sort_lib=$lib > gpurun_out/sortprof/lib$lib.log 2>&1 || { echo "lib $lib failed"; tail gpurun_out/sortprof/lib$lib.log; exit 1; }
  f=$(find gpurun_out/sortprof/lib$lib -name "*kernel_stats.csv")
  echo "== wf_sort_lib $lib"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = 0.0
for r in rows:
    n = r["Name"]
    if any(k in n for k in ("rs_", "rocprim", "onesweep", "radix", "hipcub")):
        ms = float(r["TotalDurationNs"]) / 1e6
        tot += ms
        print("%-90s calls %4s total %8.3f ms" % (n[:90], r["Calls"], ms))
print("sort total %.3f ms (2 passes: 1 timed + 1 counting)" % tot)
PY
done
