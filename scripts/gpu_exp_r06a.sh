cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/perf_shape.py > gpurun_out/perf_shape.txt 2>&1 || { tail -5 gpurun_out/perf_shape.txt; exit 1; }
cat gpurun_out/perf_shape.txt
timeout -k 10 900 bash scripts/gpu_sweep_opts.sh "" 2 "" "" "--opt wf_measure_skip=1"
