#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/phase_clock.py ${PHASE_ARGS} > gpurun_out/phase.json 2> gpurun_out/phase.err
rc=$?; echo "phase rc=$rc"; grep -v amdgpu.ids gpurun_out/phase.err | tail -8
exit $rc
