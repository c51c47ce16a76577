#!/bin/bash
# Round-5 check on one MI355X: the GPU suite (optionally a -k subset: $1), smoke(), then the driver's
# bench command (--steps 20 --warmup 5, parity of the timed frame included).  Every step under its own
# limit; the script stops at the first failure.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${K:+-k "$K"} \
    > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
python -c "
import json; d=json.load(open('gpurun_out/bench.json'))
print(d['value'], d['value_traced'], d['single_layer_mray_s'], d['ms_per_step'], d['parity']['differing'], d['vs_cpu'], d['cpu_baseline']['value_1t'])"
