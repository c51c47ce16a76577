cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc2=$?; echo "smoke rc=$rc2"; tail -5 gpurun_out/smoke.log
  if [ $rc2 -eq 0 ]; then
    timeout -k 10 600 python bench.py --config sponza --spp 8 --steps 2 --warmup 1 --cpu-budget 8 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
    echo "bench rc=$?"; cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err
  fi
fi
