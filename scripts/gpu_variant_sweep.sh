cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_pytest_tile.log 2>&1 || { tail -30 gpurun_out/r02_pytest_tile.log; exit 1; }
tail -2 gpurun_out/r02_pytest_tile.log
for r in 1 2; do for v in 9 10 11 12; do
  timeout -k 10 300 python bench.py --variant $v --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/v$v.r$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/v$v.r$r.json'));print($v, d['ms_per_step'], d['roofline']['avg_launch_ms'], {k:v['avg_launch_ms'] for k,v in d['roofline']['other_traces'].items()})"
done; done
