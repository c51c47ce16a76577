#!/bin/bash
# Round-6 leaf exchange: the trace-build parity tests, then two interleaved rounds of the round's base
# library (ab_base/, commit f1f302f) on build 49 and the tree's library on builds 49 / 53 / 54 / 56 / 57,
# sponza stand-in at the driver's command (no parity rows: the tests above hold them).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "trace_builds_bitexact" > gpurun_out/pytest_d.txt 2>&1
rc=$?; tail -2 gpurun_out/pytest_d.txt; [ $rc -eq 0 ] || exit $rc
i=0
for r in 1 2; do
  for LV in "base 49" "new 49" "new 53" "new 54" "new 56" "new 57"; do
    set -- $LV; i=$((i+1))
    if [ $1 = base ]; then export CHIARO_LIB_DIR=$GRAFT_REPO_ROOT/ab_base; else unset CHIARO_LIB_DIR; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --parity-rows 2 --single-layer-steps 0 --steps 20 --warmup 5 \
        --variant $2 > gpurun_out/d_$i.json 2> gpurun_out/d_$i.err || { tail -5 gpurun_out/d_$i.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/d_$i.json')); r=d['roofline']
print('$1 $2', d['value'], d['ms_per_step'], 'parity', d['parity']['differing'], r.get('avg_launch_ms'), {k: (v or {}).get('avg_launch_ms') for k, v in r.get('other_traces', {}).items()})"
  done
done
