#!/bin/bash
# Parity of the trace builds, then interleaved bench A/B of builds given as arguments.
#   bash scripts/gpu_ab_builds.sh ROUNDS "pytest -k expr" v1 v2 ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$1; K=$2; shift 2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || exit $rc
for r in $(seq 1 $R); do
  for v in "$@"; do
    timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --variant $v > gpurun_out/bench_v$v.json 2> gpurun_out/bench_v$v.err || { tail -5 gpurun_out/bench_v$v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/bench_v$v.json')); r=d['roofline']; print($v, d['value'], d['ms_per_step'], {k: (v or {}).get('avg_launch_ms') for k, v in r.get('other_traces', {}).items()}, r.get('kernel','')[:15], r.get('avg_launch_ms'))"
  done
done
