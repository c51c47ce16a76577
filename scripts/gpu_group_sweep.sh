#!/bin/bash
# Pass-group sweep on one GPU: layers per group x tile edge (rank_time.py at N = 1: the frame in
# the fewest pieces whose paths fill one chunk); ms per layer.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "8 32" "16 32" "4 32" "8 64" "8 128" "16 64"; do
  set -- $cfg
  timeout -k 10 300 python -u scripts/rank_time.py --nranks 1 --rounds 2 --layers $1 --tile $2 > gpurun_out/gs_$1_$2.txt 2> gpurun_out/gs_$1_$2.err || { tail -5 gpurun_out/gs_$1_$2.err; exit 1; }
  echo "layers $1 tile $2: $(cat gpurun_out/gs_$1_$2.txt)"
done
