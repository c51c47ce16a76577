#!/bin/bash
# Round-4 experiments in one call: exactness of the changed builds, library A/B, desc_quorum sweep.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "desc_quorum or camera_cull or packet_camera or trace_builds or camera_fused" > gpurun_out/pytest_exp.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_exp.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_dirs.sh ab_base ab_p lib || exit 1
bash scripts/gpu_sweep_opts.sh "" 2 "" "--opt desc_quorum=16" "--opt desc_quorum=32" "--opt desc_quorum=48" || exit 1
