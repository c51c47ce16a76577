#!/bin/bash
# Overlapped tail (wf_tail_overlap): parity, bench A/B and the 8-way rehearsal with and without it.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/gpu_sweep_keys.sh 2 "tail or perf_counters or c5 or two_lanes or default_build" "--opt wf_tail_overlap=1" "--opt wf_tail_overlap=0" || exit 1
for ov in 1 0; do
  timeout -k 10 300 python scripts/rank_time.py --nranks 1,8 --rounds 2 --opt wf_tail_overlap=$ov > gpurun_out/rank_ov$ov.txt 2> gpurun_out/rank_ov$ov.err || { echo "rank_time failed"; tail -5 gpurun_out/rank_ov$ov.err; exit 1; }
  echo "overlap $ov"; cat gpurun_out/rank_ov$ov.txt
done
