#!/bin/bash
# GPU check: parity tests, smoke, then a short bench.  Usage: bash scripts/gpu_check.sh [bench args]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
BENCH_ARGS=${@:-"--config sponza --spp 8 --steps 2 --warmup 1 --cpu-budget 8"}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -5 gpurun_out/smoke.log
[ $rc2 -eq 0 ] || exit $rc2
timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
rc3=$?; echo "bench rc=$rc3"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
[ $rc3 -eq 0 ] || exit $rc3
timeout -k 10 600 python bench.py $BENCH_ARGS --kernel 1 --no-cpu-baseline > gpurun_out/bench_k1.json 2> gpurun_out/bench_k1.err
echo "bench k1 rc=$?"; cat gpurun_out/bench_k1.json
