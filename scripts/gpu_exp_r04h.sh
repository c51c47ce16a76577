#!/bin/bash
# The descent quorum in the tail kernel too (lib) against HEAD (ab_h), then refill thresholds on HEAD's defaults.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "desc_quorum or tail or camera_fused" > gpurun_out/pytest_exp.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_exp.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_dirs.sh ab_h lib || exit 1
export CHIARO_LIB_DIR=$GRAFT_REPO_ROOT/ab_h
bash scripts/gpu_sweep_opts.sh "" 2 "" "" "--opt refill_shadow=64" "--opt refill_shadow=60" || exit 1
