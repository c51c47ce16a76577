#!/bin/bash
# One sweep.py run per argument group (separated by ';' in $1 ... each arg is one sweep's args).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  echo "== sweep $i: $a"
  timeout -k 10 400 python scripts/sweep.py $a > gpurun_out/sweep_$i.txt 2>&1 || { echo "sweep $i failed"; tail -5 gpurun_out/sweep_$i.txt; exit 1; }
  grep '^{' gpurun_out/sweep_$i.txt
done
