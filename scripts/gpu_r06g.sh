#!/bin/bash
# The leaf-exchange tie / multi-window parity test, then the C5 (sponza 4K x 100 spp) profiles of build 54.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "leaf_exchange" > gpurun_out/pytest_lx.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_lx.txt
[ $rc -eq 0 ] || exit $rc
TAG=r06b bash scripts/gpu_profile_cfgs_r06.sh "sponza_4k:100"
