#!/bin/bash
# Leaf-cull builds: parity of builds 19-22, then one bench per configuration (sponza 1080p x 128).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "19 or 20 or 21 or 22" > gpurun_out/pytest_lc.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_lc.log
[ $rc -eq 0 ] || exit $rc
run() { # tag, bench args
  tag=$1; shift
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/lc_$tag.json 2> gpurun_out/lc_$tag.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/lc_$tag.json')); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], {k: (v or {}).get('avg_launch_ms') for k, v in r.get('other_traces', {}).items()}, r.get('avg_launch_ms'))"
}
run v18 --variant 18
run v19 --variant 19
run v19_all --variant 19 --opt lc_debug=1
run v19_none --variant 19 --opt lc_debug=2
run v20 --variant 20
run v21 --variant 21
run v22 --variant 22
run v18b --variant 18
run v20b --variant 20
run v22b --variant 22
