#!/bin/bash
# refill_shadow around 60 on sponza, then 60 against the default (56) on cornell_box and the nanobox stand-in.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/gpu_sweep_opts.sh "" 2 "" "" "--opt refill_shadow=58" "--opt refill_shadow=60" "--opt refill_shadow=62" || exit 1
bash scripts/gpu_sweep_opts.sh "" 2 "--config cornell_box" "" "--opt refill_shadow=60" || exit 1
bash scripts/gpu_sweep_opts.sh "" 2 "--config nanobox" "" "--opt refill_shadow=60" || exit 1
