#!/bin/bash
# Tests selected by -k, then the default bench line twice (sponza 1080p x 128).
#   bash scripts/gpu_quick_r03.sh "pytest -k expr" [bench args]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K=$1; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_quick.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -5 gpurun_out/bench_quick.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_quick.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r.get('avg_launch_ms'), {k: (v or {}).get('avg_launch_ms') for k, v in r.get('other_traces', {}).items()})"
done
