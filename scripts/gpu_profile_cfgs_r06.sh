#!/bin/bash
# Round-6 profiles of the non-headline configurations (kernel trace + PMC + issue passes with the lane
# utilisation pass, then each configuration's bench line): bash scripts/gpu_profile_cfgs_r06.sh "cfg:spp ..."
# (TAG: the profiles' name prefix, default r06)
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r06}
for CS in ${1:-"nanobox:64 cornell_box:500 sponza_4k:100 cornell:4"}; do
  CFG=${CS%%:*}; SPP=${CS##*:}
  bash scripts/gpu_profile_cfg.sh $TAG $CFG $SPP > gpurun_out/prof_cfg_$CFG.log 2>&1 || { echo "$CFG failed"; tail -20 gpurun_out/prof_cfg_$CFG.log; exit 1; }
  echo "$CFG ok"; tail -c 400 profiles/${TAG}_bench_$CFG.json; echo
done
