#!/bin/bash
# Round-6: the C5 (sponza 4K x 100 spp) profiles and bench line on the final default build 59.
cd $GRAFT_REPO_ROOT
TAG=r06e bash scripts/gpu_profile_cfgs_r06.sh "sponza_4k:100"
