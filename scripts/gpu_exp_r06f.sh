#!/bin/bash
# Interleaved A/B: ab_base/ (the library without the lx_min fallback) vs the tree's library at lx_min
# 0 / 3 and build 58 (the exchange's pair-list form) at lx_min 0 / 3 (sponza stand-in, driver command,
# 2 full rows of parity per run).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
for r in 1 2; do
  for LV in "base 0 -1" "new 0 -1" "new 3 -1" "new 0 58" "new 3 58"; do
    set -- $LV; i=$((i+1))
    if [ $1 = base ]; then export CHIARO_LIB_DIR=$GRAFT_REPO_ROOT/ab_base; O=""; else unset CHIARO_LIB_DIR; O="--opt lx_min=$2 --variant $3"; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-rows 2 --single-layer-steps 0 --steps 20 --warmup 5 \
        $O > gpurun_out/f_$i.json 2> gpurun_out/f_$i.err || { tail -5 gpurun_out/f_$i.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/f_$i.json')); r=d['roofline']
print('$1 lx_min=$2 variant $3', d['value'], d['ms_per_step'], 'parity', d['parity']['differing'], r.get('avg_launch_ms'), {k: (v or {}).get('avg_launch_ms') for k, v in r.get('other_traces', {}).items()})"
  done
done
