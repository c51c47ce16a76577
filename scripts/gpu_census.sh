#!/bin/bash
# Parity tests, the leaf / repeated-miss census of the trace kinds, then the default bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/leaf_census.py ${CENSUS_ARGS} > gpurun_out/census.json 2> gpurun_out/census.err
rc=$?; echo "census rc=$rc"; grep -v amdgpu.ids gpurun_out/census.err | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --cpu-budget 6 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/bench.json
exit $rc
