#!/bin/bash
# Round-6: the leaf exchange's prefix by a DPP scan (build 59) against the ballot prefix (54): parity
# tests, then two interleaved rounds at the driver's command (2 full rows of parity per run).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 bash scripts/gpu_sweep_opts.sh "trace_builds_bitexact or leaf_exchange" 3 "" "--variant 54" "--variant 59"
