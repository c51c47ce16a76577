#!/bin/bash
# Option sweep under pass groups (16 layers in 16 pieces): refill thresholds and queue-key grids,
# two interleaved rounds; ms per layer (bench.py --steps 16, no CPU leg).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for o in "" "--opt refill_shadow=48" "--opt refill_shadow=64" "--opt refill=40" "--opt refill=56" "--opt wf_leaf_shift=0" "--opt wf_leaf_shift=2" "--opt wf_dir_res=64" "--opt wf_tail_min=524288" "--opt wf_tail_min=2097152"; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-perf-pass $o > gpurun_out/go.json 2> gpurun_out/go.err || { tail -3 gpurun_out/go.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/go.json')); print('round $r', '${o:-default}', d['value'], d['ms_per_step'])"
  done
done
