#!/bin/bash
# The camera packet's shared-origin triangle test (lib) against the committed build (ab_q), its exactness
# first; then the refill thresholds re-swept with desc_quorum 16.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "camera_cull or packet_camera or trace_builds or camera_fused" > gpurun_out/pytest_exp.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_exp.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_dirs.sh ab_q lib || exit 1
Q="--opt desc_quorum=16"
bash scripts/gpu_sweep_opts.sh "" 2 "" "$Q" "$Q --opt refill_shadow=48" "$Q --opt refill_shadow=64" "$Q --opt refill=40" "$Q --opt refill=56" || exit 1
