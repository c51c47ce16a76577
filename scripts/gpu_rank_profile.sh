#!/bin/bash
# Kernel trace of the N-way tile split rehearsal (rank 0's tiles only, one GPU),
# per-pass phase breakdown for each N.  Usage: bash scripts/gpu_rank_profile.sh [nranks]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rank_prof
for n in ${@:-1 8}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/rank_prof/n$n -o trace --output-format csv -- python3 scripts/rank_time.py --nranks $n --rounds 2 > gpurun_out/rank_prof/n$n.log 2>&1 || { echo "n=$n failed"; tail gpurun_out/rank_prof/n$n.log; exit 1; }
  echo "== nranks $n"; grep nranks gpurun_out/rank_prof/n$n.log
  python3 scripts/pass_breakdown.py $(find gpurun_out/rank_prof/n$n -name "*kernel_trace.csv") || exit 1
done
