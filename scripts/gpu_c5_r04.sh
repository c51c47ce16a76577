#!/bin/bash
# C1 profile + bench line, then the whole C5 schedule (30 layers x 100 spp at 4K in pass groups) with
# its oracle rows -> profiles/r04_c5_progressive_n1.json.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/profiles
bash scripts/gpu_profile_cfg.sh r04 cornell 4 > gpurun_out/cfg_c1.log 2>&1 || { echo "C1 failed"; tail -20 gpurun_out/cfg_c1.log; exit 1; }
tail -1 gpurun_out/cfg_c1.log | cut -c1-300
timeout -k 10 600 python -u scripts/c5_progressive.py --layers 30 > profiles/r04_c5_progressive_n1.json 2> gpurun_out/c5.log || { echo "C5 failed"; tail -20 gpurun_out/c5.log; exit 1; }
cat profiles/r04_c5_progressive_n1.json | cut -c1-600
cp profiles/r04_c5_progressive_n1.json gpurun_out/profiles/
