#!/bin/bash
# Round evidence run: GPU parity, the rocprofv3 passes of the default bench
# command (kernel trace + separate PMC passes), their summary into profiles/
# (pmc_sponza.json feeds roofline.traffic), then the default bench line.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash scripts/profile.sh $TAG --steps 2 --warmup 1 --no-cpu-baseline || exit 1
python scripts/prof_summary.py gpurun_out/prof_$TAG $TAG > gpurun_out/prof_summary.txt || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 1; }
cat gpurun_out/bench_default.json
