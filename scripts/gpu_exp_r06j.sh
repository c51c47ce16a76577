#!/bin/bash
# Round-6 re-sweep of the queue-order knobs on the leaf-exchange build 54 (sponza stand-in, driver
# command, two interleaved rounds, 2 full rows of parity per run).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1100 bash scripts/gpu_sweep_opts.sh "" 2 "" "" "--opt wf_dir_res_shadow=64" "--opt wf_dir_res_shadow=256" \
    "--opt refill_shadow=62" "--opt refill_shadow=64" "--opt desc_quorum=12"
