#!/bin/bash
# Full GPU suite on the default compile, then the default bench line and a cornell_box A/B
# with the new build first (order check).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print(d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'), {k: (v or {}).get('avg_launch_ms') for k, v in d['roofline'].get('other_traces', {}).items()})"
for r in 1 2; do
  for v in 44 18; do
    timeout -k 10 300 python -u bench.py --config cornell_box --steps 3 --warmup 1 --no-cpu-baseline --no-perf-pass --variant $v > gpurun_out/cb_$v.json 2> gpurun_out/cb_$v.err || { tail -5 gpurun_out/cb_$v.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/cb_$v.json')); r=d['roofline']; o=r.get('other_traces',{}); print($v, d['ms_per_step'], r.get('avg_launch_ms'), {k: (v or {}).get('avg_launch_ms') for k, v in o.items()})"
  done
done
