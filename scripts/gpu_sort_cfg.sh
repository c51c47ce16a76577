#!/bin/bash
# Sorting on / off per configuration (two interleaved rounds), after the sort tests.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "sort_choice or sorted_queues" > gpurun_out/pytest_sort.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_sort.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in "nanobox --steps 8 --warmup 2" "cornell --steps 16 --warmup 2" "cornell_box --steps 8 --warmup 2"; do
    for O in "--opt wf_sort=1" "--opt wf_sort=0"; do
      timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --parity-rows 0 --single-layer-steps 0 \
          --no-perf-pass $O > gpurun_out/sc.json 2> gpurun_out/sc.err || { tail -5 gpurun_out/sc.err; exit 1; }
      python -c "
import json; d=json.load(open('gpurun_out/sc.json'))
print('$cfg', '$O', d['value'], d['ms_per_step'])"
    done
  done
done
