#!/bin/bash
# Round-6 final validation on HEAD (GPU suite, smoke, the driver's sponza bench), then the secondary
# closest trace's refill threshold re-swept on the leaf-exchange build (40 / 44 vs the default 48).
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r06.sh "" "sponza" || exit $?
timeout -k 10 600 bash scripts/gpu_sweep_opts.sh "" 2 "" "" "--opt refill=40" "--opt refill=44"
