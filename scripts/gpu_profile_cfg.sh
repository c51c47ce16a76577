#!/bin/bash
# rocprofv3 evidence of one non-headline configuration (BASELINE configs C2 cornell_box,
# C3 nanobox, C5 sponza_4k): kernel trace + PMC passes -> profiles/pmc_<cfg>.json and
# <tag>_<cfg>_*, the instruction-issue pass -> profiles/pmc_issue_<cfg>.json, then the
# bench line of that configuration (with its cpu_baseline) -> profiles/<tag>_bench_<cfg>.json.
#   bash scripts/gpu_profile_cfg.sh <tag> <cfg> <spp>
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}; CFG=${2:?config}; SPP=${3:?spp of the config}
mkdir -p gpurun_out/profiles
bash scripts/profile.sh ${TAG}_$CFG --config $CFG --steps 16 --warmup 0 --no-cpu-baseline || exit 1
python scripts/prof_summary.py gpurun_out/prof_${TAG}_$CFG ${TAG}_$CFG --config $CFG --spp $SPP > gpurun_out/prof_summary_$CFG.txt || exit 1
rm -rf gpurun_out/pmc_issue
bash scripts/pmc_issue.sh --config $CFG --steps 16 --warmup 0 --no-cpu-baseline || exit 1
python scripts/pmc_issue_summary.py gpurun_out/pmc_issue/a/pmc_counter_collection.csv profiles/pmc_issue_$CFG.json $SPP || exit 1
timeout -k 10 600 python bench.py --config $CFG --steps 16 --warmup 1 > profiles/${TAG}_bench_$CFG.json 2> gpurun_out/bench_$CFG.log || { echo "bench $CFG failed"; tail -20 gpurun_out/bench_$CFG.log; exit 1; }
cat profiles/${TAG}_bench_$CFG.json
cp -r profiles/. gpurun_out/profiles/
# the raw rocprofv3 csvs stay on the box (their summaries are in profiles/): gpurun returns at most 64 MiB
rm -rf gpurun_out/prof_${TAG}_$CFG gpurun_out/pmc_issue
