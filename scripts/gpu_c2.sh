#!/bin/bash
# C2 (cornell_box 1024^2 x 500 spp) options, two interleaved rounds.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for O in "" "--opt wf_tail_min=2147483647" "--kernel 0" "--opt wf_sort=0" "--opt wf_leaf_keys=0"; do
    timeout -k 10 300 python -u bench.py --config cornell_box --no-cpu-baseline --parity-rows 0 --single-layer-steps 0 \
        --steps 8 --warmup 2 --no-perf-pass $O > gpurun_out/c2.json 2> gpurun_out/c2.err || { tail -5 gpurun_out/c2.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/c2.json'))
print('$O', d['value'], d['ms_per_step'])"
  done
done
