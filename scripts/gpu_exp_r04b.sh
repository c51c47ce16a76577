#!/bin/bash
# desc_quorum: a finer sweep on sponza, then the candidate against 0 on cornell_box and the nanobox stand-in.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/gpu_sweep_opts.sh "" 2 "" "" "--opt desc_quorum=4" "--opt desc_quorum=8" "--opt desc_quorum=12" "--opt desc_quorum=16" "--opt desc_quorum=20" || exit 1
bash scripts/gpu_sweep_opts.sh "" 2 "--config cornell_box" "" "--opt desc_quorum=8" "--opt desc_quorum=16" || exit 1
bash scripts/gpu_sweep_opts.sh "" 2 "--config nanobox" "" "--opt desc_quorum=8" "--opt desc_quorum=16" || exit 1
