#!/bin/bash
# Full GPU parity suite, the smoke, then the default bench (with the CPU baseline).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; grep -v amdgpu.ids gpurun_out/smoke.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-600 gpurun_out/bench.json
exit $rc
