#!/bin/bash
# Chunked-append check: the GPU tests that touch wf_shade's appends, then interleaved A/B of the base libraries
# (ab_base/) against the tree on sponza and cornell_box.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "chunked_appends or shade_waves or tail or sorted_queues or resolve or fold or multi_chunk or layer_groups" \
    > gpurun_out/pytest_chunk.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_chunk.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_libs.sh "" "--config cornell_box"
