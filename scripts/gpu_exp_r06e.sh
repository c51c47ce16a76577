#!/bin/bash
# Round-6 knob re-sweep on the leaf-exchange build 54 (sponza stand-in, driver command, 2 full rows of
# parity per run): the exchange's per-lane fallback (lx_min), descent quorum, shadow / closest refill
# thresholds, leaf-record minimum.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1150 bash scripts/gpu_sweep_opts.sh "trace_builds_bitexact" 2 "" "" "--opt lx_min=2" "--opt lx_min=3" "--opt lx_min=4" \
    "--opt desc_quorum=4" "--opt desc_quorum=16" "--opt refill_shadow=56" "--opt refill=56"
