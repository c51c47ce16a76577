#!/bin/bash
# The camera packet's speculative grandchild fetch (lib) against HEAD (ab_h): exactness, then A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "camera_cull or packet_camera or trace_builds or camera_fused" > gpurun_out/pytest_exp.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_exp.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_dirs.sh ab_h lib || exit 1
