#!/bin/bash
# Quick GPU iteration: parity tests then the variant sweep.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python scripts/sweep.py ${@} > gpurun_out/sweep.txt 2>&1
echo "sweep rc=$?"; grep -v amdgpu.ids gpurun_out/sweep.txt
