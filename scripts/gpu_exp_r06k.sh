#!/bin/bash
# Round-6: the leaf cull against the leaf exchange -- leaves below lc_min references tested without their
# cull record (33: no leaf culls), build 54, two interleaved rounds at the driver's command.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 bash scripts/gpu_sweep_opts.sh "" 2 "" "" "--opt lc_min=3" "--opt lc_min=6" "--opt lc_min=12" "--opt lc_min=33"
