#!/bin/bash
# Interleaved A/B of two BUILDS (ab_base/: the libraries of the base commit, copied there by
# `bash scripts/ab_base_build.sh <commit>`; default: the tree's own lib/) over bench option sets:
#   bash scripts/gpu_ab_libs.sh "" "--config cornell_box"
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for O in "$@"; do
    for L in base new; do
      if [ $L = base ]; then export CHIARO_LIB_DIR=$GRAFT_REPO_ROOT/ab_base; else unset CHIARO_LIB_DIR; fi
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-rows 0 --single-layer-steps 0 --steps 20 --warmup 5 \
          $O > gpurun_out/abl.json 2> gpurun_out/abl.err || { tail -5 gpurun_out/abl.err; exit 1; }
      python -c "
import json; d=json.load(open('gpurun_out/abl.json')); r=d['roofline']
print('$L [$O]', d['value'], d['ms_per_step'], r.get('avg_launch_ms'), {k: (v or {}).get('avg_launch_ms') for k, v in r.get('other_traces', {}).items()})"
    done
  done
done
