#!/bin/bash
# Interleaved sweep of bench option sets (each string passed to bench.py as-is; "" = the defaults), the
# timed frame checked against the oracle on 2 full rows:
#   bash scripts/gpu_sweep_opts.sh "pytest -k expr" rounds "bench args" "optsA" "optsB" ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K=$1; N=$2; BA=$3; shift 3
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > gpurun_out/pytest_sweep.txt 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_sweep.txt
  [ $rc -eq 0 ] || exit $rc
fi
i=0
for r in $(seq $N); do
  for O in "$@"; do
    i=$((i+1))
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-rows 2 --single-layer-steps 0 --steps 20 --warmup 5 \
        $BA $O > gpurun_out/sw_$i.json 2> gpurun_out/sw_$i.err || { tail -5 gpurun_out/sw_$i.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/sw_$i.json')); r=d['roofline']
print('[$O]', d['value'], d['ms_per_step'], 'parity', d['parity']['differing'], r.get('avg_launch_ms'), {k: (v or {}).get('avg_launch_ms') for k, v in r.get('other_traces', {}).items()})"
  done
done
