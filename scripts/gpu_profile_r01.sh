#!/bin/bash
# Round-1 evidence run: GPU parity, the default bench line, and the rocprofv3
# passes of the same bench command (kernel trace + separate PMC passes).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 1; }
cat gpurun_out/bench_default.json
bash scripts/profile.sh r01 --steps 2 --warmup 1 --no-cpu-baseline
