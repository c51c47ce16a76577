#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "25" > gpurun_out/pytest_lc2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_lc2.log
[ $rc -eq 0 ] || exit $rc
run() {
  tag=$1; shift
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/lc_$tag.json 2> gpurun_out/lc_$tag.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/lc_$tag.json')); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], {k: (v or {}).get('avg_launch_ms') for k, v in r.get('other_traces', {}).items()}, r.get('avg_launch_ms'))"
}
run v18 --variant 18
run v19 --variant 19
run v25 --variant 25
run v19m8 --variant 19 --opt lc_min=8
run v25m8 --variant 25 --opt lc_min=8
run v25m6 --variant 25 --opt lc_min=6
run v18b --variant 18
run v25b --variant 25
