#!/bin/bash
# Option sweeps under the leaf-keyed queues (round-2 end): refill thresholds, sort and
# tail cut-offs, full frame and one rank's share of the 8-way split (sweep.py checks that
# every configuration renders the identical image).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/leaf_sweep
S="timeout -k 10 240 python -u scripts/sweep.py --spp 128 --rounds 2"
$S --grid refill_shadow=40,48,56,64 --grid refill=48,56,64 > gpurun_out/leaf_sweep/refill.jsonl 2> gpurun_out/leaf_sweep/refill.err || exit 1
cat gpurun_out/leaf_sweep/refill.jsonl
$S --grid wf_sort_min=262144,1048576,4194304 --grid wf_tail_min=262144,1048576,4194304 > gpurun_out/leaf_sweep/cut.jsonl 2> gpurun_out/leaf_sweep/cut.err || exit 1
cat gpurun_out/leaf_sweep/cut.jsonl
$S --nranks 8 --grid wf_sort_min=65536,262144,1048576 --grid wf_tail_min=262144,1048576 > gpurun_out/leaf_sweep/cut8.jsonl 2> gpurun_out/leaf_sweep/cut8.err || exit 1
cat gpurun_out/leaf_sweep/cut8.jsonl
$S --nranks 8 --grid refill_shadow=40,48,56 --grid refill=48,56,64 > gpurun_out/leaf_sweep/refill8.jsonl 2> gpurun_out/leaf_sweep/refill8.err || exit 1
cat gpurun_out/leaf_sweep/refill8.jsonl
