#!/bin/bash
# The descent quorum leaving through the loop's own exit (lib) against HEAD (ab_h): exactness, then A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "desc_quorum or trace_builds or camera_fused or tail" > gpurun_out/pytest_exp.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_exp.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_dirs.sh ab_h lib || exit 1
