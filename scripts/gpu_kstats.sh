#!/bin/bash
# Kernel-time summary (rocprofv3 kernel trace) of the bench on each given config -> gpurun_out/kstats_<cfg>.txt
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for CFG in "$@"; do
  rm -rf gpurun_out/ks
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ks -o t --output-format csv -- python3 bench.py --config $CFG \
      --no-cpu-baseline --parity-rows 0 --single-layer-steps 0 --no-perf-pass --steps 8 --warmup 1 \
      > gpurun_out/ks.json 2> gpurun_out/ks.err || { tail -5 gpurun_out/ks.err; exit 1; }
  python - "$CFG" > gpurun_out/kstats_$CFG.txt <<'PY'
import csv, glob, json, sys
f = glob.glob('gpurun_out/ks/**/*kernel_stats.csv', recursive=True)[0]
d = json.load(open('gpurun_out/ks.json'))
print(sys.argv[1], 'ms_per_step', d['ms_per_step'], 'value', d['value'])
for r in csv.DictReader(open(f)):
    print('%-70s calls %5s total_ms %9.1f avg_ms %8.3f' % (r['Name'][:70], r['Calls'], float(r['TotalDurationNs']) / 1e6, float(r['AverageNs']) / 1e6))
PY
  cat gpurun_out/kstats_$CFG.txt | head -14
done
rm -rf gpurun_out/ks
