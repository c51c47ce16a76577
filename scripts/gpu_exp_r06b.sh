#!/bin/bash
# Round-6 leaf exchange: the trace-build parity tests, then builds 49 / 53 / 54 / 55 interleaved at the
# driver's command (sponza stand-in), each timed frame checked against the oracle on 2 full rows.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 bash scripts/gpu_sweep_opts.sh "trace_builds_bitexact" 2 "" "--variant 49" "--variant 53" "--variant 54" "--variant 55"
