#!/bin/bash
# The divergent leaf loop of the leaf-cull traces: occluded lanes leaving through the loop's own exit
# (ab_v1), and that with two records in flight in alternating roles (lib), against HEAD (ab_h).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "desc_quorum or trace_builds or camera_fused or tail or leaf" > gpurun_out/pytest_exp.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_exp.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_dirs.sh ab_h ab_v1 lib || exit 1
