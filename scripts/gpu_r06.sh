#!/bin/bash
# Round-6 check on one MI355X: the GPU suite (optionally a -k subset: $1), smoke(), then bench lines of
# the configurations in $2 (default "sponza": the driver's command, --steps 20 --warmup 5, parity of the
# timed frame included; the others at --steps 16 --warmup 1).  Every step under its own limit; the script
# stops at the first failure.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K=${1:-}
CFGS=${2:-sponza}
if [ "$K" != "none" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${K:+-k "$K"} \
    > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.txt
[ $rc -eq 0 ] || exit $rc
fi
for CFG in $CFGS; do
  if [ "$CFG" = sponza ]; then A="--steps 20 --warmup 5"; else A="--steps 16 --warmup 1"; fi
  timeout -k 10 600 python -u bench.py --config $CFG $A > gpurun_out/bench_$CFG.json 2> gpurun_out/bench_$CFG.err
  rc=$?; echo "bench $CFG rc=$rc"; tail -2 gpurun_out/bench_$CFG.err
  [ $rc -eq 0 ] || exit $rc
  python -c "
import json; d=json.load(open('gpurun_out/bench_$CFG.json'))
print('$CFG', d['value'], d['value_traced'], d['single_layer_mray_s'], d['ms_per_step'], d['parity']['differing'], d['vs_cpu'])"
done
