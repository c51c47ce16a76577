#!/bin/bash
# The descent loop with one exit (lib) against HEAD (ab_h): exactness, then A/B on sponza and cornell_box.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "desc_quorum or trace_builds or camera_fused or tail or leaf or xcd" > gpurun_out/pytest_exp.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_exp.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_dirs.sh ab_h lib || exit 1
BA="--config nanobox" bash scripts/gpu_ab_dirs.sh ab_h lib || exit 1
