#!/bin/bash
# Layers-per-pass check: its parity tests, then the one-GPU rehearsal of the N-way split with
# one and with two progressive layers per render pass.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "layers_per_pass" > gpurun_out/pytest_layers.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_layers.log
[ $rc -eq 0 ] || exit $rc
for L in 1 2; do
  timeout -k 10 300 python -u scripts/rank_time.py --nranks 1,2,4,8 --rounds 2 --layers $L > gpurun_out/rank_time_l$L.txt 2> gpurun_out/rank_time_l$L.err || { tail -5 gpurun_out/rank_time_l$L.err; exit 1; }
  cat gpurun_out/rank_time_l$L.txt
done
