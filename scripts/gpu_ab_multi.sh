#!/bin/bash
# Interleaved A/B of several bench option sets on the default config (two rounds):
#   bash scripts/gpu_ab_multi.sh "" "--opt wf_shade_waves=8" "--opt lc_min=2" ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for O in "$@"; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-rows 0 --single-layer-steps 0 --steps 20 --warmup 5 \
        $O > gpurun_out/abm.json 2> gpurun_out/abm.err || { tail -5 gpurun_out/abm.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/abm.json')); r=d['roofline']
print('[$O]', d['value'], d['ms_per_step'], r.get('avg_launch_ms'), {k: (v or {}).get('avg_launch_ms') for k, v in r.get('other_traces', {}).items()})"
  done
done
