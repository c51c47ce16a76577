#!/bin/bash
cd $GRAFT_REPO_ROOT
bash scripts/gpu_sweep_keys.sh 2 "trace_builds" "--variant 26" "--variant 33" "--variant 34" "--opt wf_side_priority=1" || exit 1
for pr in 0 1; do
  timeout -k 10 300 python scripts/rank_time.py --nranks 8 --rounds 2 --opt wf_side_priority=$pr > gpurun_out/rank_pr$pr.txt 2> gpurun_out/rank_pr$pr.err || { echo "rank_time failed"; tail -5 gpurun_out/rank_pr$pr.err; exit 1; }
  echo "side priority $pr"; cat gpurun_out/rank_pr$pr.txt
done
