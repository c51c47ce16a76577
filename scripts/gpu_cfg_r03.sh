#!/bin/bash
# Round-3 config evidence on the final default: optionally the headline bench line with its CPU
# baseline, then scripts/gpu_profile_cfg.sh for each "config:spp" argument.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/profiles
if [ "$HEADLINE" = 1 ]; then
  timeout -k 10 600 python bench.py > profiles/r03_bench_default.json 2> gpurun_out/bench_default.log || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 1; }
  cut -c1-300 profiles/r03_bench_default.json
  cp profiles/r03_bench_default.json gpurun_out/profiles/
fi
for cs in "$@"; do
  bash scripts/gpu_profile_cfg.sh r03 ${cs%%:*} ${cs##*:} > gpurun_out/cfg_${cs%%:*}.log 2>&1 || { echo "config $cs failed"; tail -20 gpurun_out/cfg_${cs%%:*}.log; exit 1; }
  tail -1 gpurun_out/cfg_${cs%%:*}.log | cut -c1-300
  rm -rf gpurun_out/prof_r03_${cs%%:*} gpurun_out/pmc_issue  # raw CSVs (summaries are in profiles/): stay under the 64 MiB pull
done
