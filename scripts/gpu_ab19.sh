#!/bin/bash
# Leaf-cull build (19) against the default (18): parity tests of the new build, then an A/B bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "19 or triangle_less or shift" > gpurun_out/pytest_19.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_19.log
[ $rc -eq 0 ] || exit $rc
for v in 18 19 18 19; do
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --variant $v > gpurun_out/bench_v$v.json 2> gpurun_out/bench_v$v.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/bench_v$v.json')); r=d['roofline']; print($v, d['value'], d['ms_per_step'], {k: (v or {}).get('avg_launch_ms') for k, v in r.get('other_traces', {}).items()}, r.get('avg_launch_ms'))"
done
