#!/bin/bash
# A/B of bench options, interleaved rounds: bash scripts/gpu_ab.sh "pytest -k expr" "optsA" "optsB" [rounds]
# (each opts string is passed to bench.py as-is, e.g. "--opt wf_fold=0"; "" = the defaults)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K=$1; A=$2; B=$3; N=${4:-2}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > gpurun_out/pytest_ab.txt 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab.txt
  [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq $N); do
  for tag in A B; do
    if [ $tag = A ]; then O=$A; else O=$B; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-rows 0 --steps 20 --warmup 5 $O > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { tail -5 gpurun_out/ab_$tag.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/ab_$tag.json')); r=d['roofline']
print('$tag', '$O', d['value'], d['ms_per_step'], r.get('avg_launch_ms'), {k: (v or {}).get('avg_launch_ms') for k, v in r.get('other_traces', {}).items()})"
  done
done
