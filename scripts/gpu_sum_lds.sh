#!/bin/bash
# sum_samples occupancy cap (option sum_lds): its kernel time per launch from a rocprofv3 kernel trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for CFG in cornell_box sponza; do
  for L in "sum_lds=0 --opt sum_staged=0" "sum_lds=65536 --opt sum_staged=0" "sum_staged=1" "sum_staged=1 --opt sum_lds=65536"; do
    rm -rf gpurun_out/sl
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sl -o t --output-format csv -- python3 bench.py --config $CFG \
        --no-cpu-baseline --parity-rows 0 --single-layer-steps 0 --no-perf-pass --steps 4 --warmup 1 --opt $L \
        > gpurun_out/sl.json 2> gpurun_out/sl.err || { tail -5 gpurun_out/sl.err; exit 1; }
    python - "$CFG" "$L" <<'PY'
import csv, glob, sys
f = glob.glob('gpurun_out/sl/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'sum_samples' in r['Name'] and int(r['Calls']) > 0:
        print(sys.argv[1], sys.argv[2], 'calls', r['Calls'], 'avg_ms', round(float(r['AverageNs']) / 1e6, 3))
PY
  done
done
rm -rf gpurun_out/sl
