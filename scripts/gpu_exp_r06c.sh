#!/bin/bash
# Round-6 leaf exchange, spill-free at 8 waves (lane ids re-derived, owner data staged): the trace-build,
# tail, quorum and XCD parity tests, then builds 49 / 53 / 54 interleaved at the driver's command.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 bash scripts/gpu_sweep_opts.sh "trace_builds_bitexact or tail or desc_quorum or xcd_partition" 2 "" "--variant 49" "--variant 53" "--variant 54"
