#!/bin/bash
# Interleaved bench of several builds of the libraries (directories holding libchiaro_hip.so and
# libchiaroscuro.so; "tree" = the in-tree lib/), two rounds, the driver's command otherwise:
#   bash scripts/gpu_ab_dirs.sh tree ab_pad1 ab_pad2 [-- bench args]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DIRS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do DIRS+=("$1"); shift; done
[ "$1" = "--" ] && shift
for r in 1 2; do
  for L in "${DIRS[@]}"; do
    if [ $L = tree ]; then unset CHIARO_LIB_DIR; else export CHIARO_LIB_DIR=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-rows 0 --single-layer-steps 0 --steps 20 --warmup 5 \
        "$@" > gpurun_out/abd.json 2> gpurun_out/abd.err || { tail -5 gpurun_out/abd.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/abd.json')); r=d['roofline']
print('$L', d['value'], d['ms_per_step'], r.get('avg_launch_ms'), {k: (v or {}).get('avg_launch_ms') for k, v in r.get('other_traces', {}).items()})"
  done
done
