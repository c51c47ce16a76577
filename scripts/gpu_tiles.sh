#!/bin/bash
# Tile edge of the N-way split: per-rank times and rays of the one-GPU rehearsal.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for t in 32 16 8; do
  timeout -k 10 300 python scripts/rank_time.py --nranks 1,8 --rounds 2 --tile $t > gpurun_out/rank_tile$t.txt 2> gpurun_out/rank_tile$t.err || { echo "rank_time failed"; tail -5 gpurun_out/rank_tile$t.err; exit 1; }
  echo "tile $t"; cat gpurun_out/rank_tile$t.txt
done
