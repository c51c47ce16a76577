#!/bin/bash
# Round evidence run: GPU parity, the rocprofv3 passes of the default bench command
# (kernel trace + separate PMC passes), their summaries into profiles/ (pmc_sponza.json
# feeds roofline.traffic, pmc_issue_sponza.json roofline.issue), the per-pass phase
# breakdown, the one-GPU rehearsal of the N-way tile split, then the default bench
# line.  profiles/ written on the GPU box is copied to gpurun_out/profiles (merged back).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/profiles
TAG=${1:?tag, e.g. r02}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
bash scripts/profile.sh $TAG --steps 16 --warmup 0 --no-cpu-baseline || exit 1
python scripts/prof_summary.py gpurun_out/prof_$TAG $TAG > gpurun_out/prof_summary.txt || exit 1
# instruction-issue and address-path utilisation of the trace kernels (roofline.issue)
bash scripts/pmc_issue.sh || exit 1
python scripts/pmc_issue_summary.py gpurun_out/pmc_issue/a/pmc_counter_collection.csv profiles/pmc_issue_sponza.json 128 || exit 1
cp profiles/pmc_issue_sponza.json profiles/${TAG}_pmc_issue.json
# per-pass phase breakdown (default trace) and the one-GPU rehearsal of the N-way split
python scripts/pass_breakdown.py $(find gpurun_out/prof_$TAG/trace -name "*kernel_trace.csv") > profiles/${TAG}_pass_breakdown.jsonl || exit 1
timeout -k 10 300 python scripts/rank_time.py --nranks 1,2,4,8 --rounds 2 > profiles/${TAG}_rank_time.txt 2> gpurun_out/rank_time.err || { echo "rank_time failed"; exit 1; }
cat profiles/${TAG}_rank_time.txt
# the bench line with this run's PMC summaries (traffic, issue)
timeout -k 10 600 python bench.py > profiles/${TAG}_bench_default.json 2> gpurun_out/bench_default.log || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 1; }
cat profiles/${TAG}_bench_default.json
cp -r profiles/. gpurun_out/profiles/
