#!/bin/bash
# Parity of the listed tests, then an interleaved sweep of bench argument sets (sponza 1080p x 128).
#   bash scripts/gpu_sweep_keys.sh ROUNDS "pytest -k expr" "args A" "args B" ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
R=$1; K=$2; shift 2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pytest_sweep.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_sweep.log
[ $rc -eq 0 ] || exit $rc
for r in $(seq 1 $R); do
  i=0
  for a in "$@"; do
    i=$((i+1))
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-perf-pass $a > gpurun_out/sweep/$i.$r.json 2> gpurun_out/sweep/$i.$r.err || { echo "failed: $a"; tail -5 gpurun_out/sweep/$i.$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/sweep/$i.$r.json')); r=d['roofline']; o=r.get('other_traces',{}); print('%-45s %8.2f ms  shadow %6.2f closest %6.2f camera %6.2f' % (sys.argv[1], d['ms_per_step'], r.get('avg_launch_ms',0), (o.get('closest') or {}).get('avg_launch_ms',0), (o.get('camera') or {}).get('avg_launch_ms',0)))" "$a"
  done
done
