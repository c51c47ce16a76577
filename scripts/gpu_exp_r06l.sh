#!/bin/bash
# Round-6: the tail-kernel and queue-sort cut-offs re-swept on the leaf-exchange build 54 (sponza
# stand-in, driver command, two interleaved rounds, 2 full rows of parity per run).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 bash scripts/gpu_sweep_opts.sh "" 2 "" "" "--opt wf_tail_min=524288" "--opt wf_tail_min=2097152" \
    "--opt wf_sort_min=524288" "--opt wf_sort_min=2097152"
