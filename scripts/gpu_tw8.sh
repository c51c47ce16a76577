#!/bin/bash
cd $GRAFT_REPO_ROOT
bash scripts/gpu_sweep_keys.sh 2 "sorted_queues" "--opt wf_leaf_shift=1 --opt wf_dir_res=128" "--opt wf_leaf_shift=2 --opt wf_dir_res=128" "--opt wf_leaf_shift=3 --opt wf_dir_res=256" "--opt wf_leaf_shift=2 --opt wf_dir_res=64 --opt wf_dir_res_shadow=128" || exit 1
for tw in 4 5; do
  timeout -k 10 300 python scripts/rank_time.py --nranks 8 --rounds 2 --opt wf_tail_waves=$tw > gpurun_out/rank_tw$tw.txt 2> gpurun_out/rank_tw$tw.err || { echo "rank_time failed"; tail -5 gpurun_out/rank_tw$tw.err; exit 1; }
  echo "tail waves $tw"; cat gpurun_out/rank_tw$tw.txt
done
