#!/bin/bash
# Interleaved A/B/... of library builds: each argument a directory holding libchiaro_hip.so +
# libchiaroscuro.so ("lib": the tree's own chiaroscuro-raytracer_amd/lib), bench args in $BA:
#   BA="--config cornell_box" bash scripts/gpu_ab_dirs.sh ab_base ab_p lib
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for L in "$@"; do
    if [ $L = lib ]; then unset CHIARO_LIB_DIR; else export CHIARO_LIB_DIR=$GRAFT_REPO_ROOT/$L; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-rows 2 --single-layer-steps 0 --steps 20 --warmup 5 \
        $BA > gpurun_out/abd.json 2> gpurun_out/abd.err || { tail -5 gpurun_out/abd.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/abd.json')); r=d['roofline']
print('$L', d['value'], d['ms_per_step'], 'parity', d['parity']['differing'], r.get('avg_launch_ms'), {k: (v or {}).get('avg_launch_ms') for k, v in r.get('other_traces', {}).items()})"
  done
done
