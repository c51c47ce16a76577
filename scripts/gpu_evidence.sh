#!/bin/bash
# One-call round evidence on one MI355X: the GPU suite, smoke(), the driver's default bench line, then
# the rocprofv3 trace + PMC passes (profiles/<tag>_*, pmc_sponza.json, pmc_issue_sponza.json) and the
# one-GPU rank rehearsal.  Every GPU step under its own limit; the script stops at the first failure.
cd $GRAFT_REPO_ROOT
TAG=${1:?tag, e.g. r04}
mkdir -p gpurun_out/profiles
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh $TAG --steps 16 --warmup 0 --no-cpu-baseline || exit 1
python scripts/prof_summary.py gpurun_out/prof_$TAG $TAG > profiles/${TAG}_prof_summary.txt || exit 1
bash scripts/pmc_issue.sh || exit 1
python scripts/pmc_issue_summary.py gpurun_out/pmc_issue/a/pmc_counter_collection.csv profiles/pmc_issue_sponza.json 128 || exit 1
cp profiles/pmc_issue_sponza.json profiles/${TAG}_pmc_issue.json
python scripts/pass_breakdown.py $(find gpurun_out/prof_$TAG/trace -name "*kernel_trace.csv") > profiles/${TAG}_pass_breakdown.jsonl || exit 1
# the driver's bench command, with this run's PMC summaries (traffic, issue)
timeout -k 10 600 python -u bench.py > profiles/${TAG}_bench_default.json 2> gpurun_out/bench_default.log
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_default.log
[ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('profiles/${TAG}_bench_default.json')); print(d['value'], d['ms_per_step'], d['single_layer_ms'], d['parity']['differing'], d['roofline']['frac'])"
cp -r profiles/. gpurun_out/profiles/
timeout -k 10 300 python scripts/rank_time.py --nranks 1,2,4,8 --rounds 2 > profiles/${TAG}_rank_time.txt 2> gpurun_out/rank_time.err || { echo "rank_time failed"; exit 1; }
tail -5 profiles/${TAG}_rank_time.txt
cp -r profiles/. gpurun_out/profiles/
