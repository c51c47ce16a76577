#!/bin/bash
# Round-6 validation of the DPP-prefix default (build 59): GPU suite, smoke, the driver's sponza bench,
# then the profile refresh of the default bench command (kernel trace, PMC, issue passes, pass breakdown,
# rehearsal, bench line with this run's PMC summaries).
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r06.sh "" "sponza" || exit $?
SKIP_TESTS=1 bash scripts/gpu_profile.sh r06e
