#!/bin/bash
# Pass-group check: the layer-group parity tests, the default bench line (8 layers per pass
# group) against one layer per pass, and the one-GPU rehearsal of the N-way split.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "layers_per_pass or layer_groups" > gpurun_out/pytest_groups.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_groups.log
[ $rc -eq 0 ] || exit $rc
for L in 8 1 8; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --layers-per-pass $L --steps 8 --warmup 1 > gpurun_out/bench_l$L.json 2> gpurun_out/bench_l$L.err || { tail -5 gpurun_out/bench_l$L.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_l$L.json')); r=d['roofline']; print($L, d['value'], d['ms_per_step'], d['config']['pass_groups'], r.get('avg_launch_ms'), {k: (v or {}).get('avg_launch_ms') for k, v in r.get('other_traces', {}).items()})"
done
timeout -k 10 300 python -u scripts/rank_time.py --nranks 1,2,4,8 --rounds 2 --layers 8 > gpurun_out/rank_time_g8.txt 2> gpurun_out/rank_time_g8.err || { tail -5 gpurun_out/rank_time_g8.err; exit 1; }
cat gpurun_out/rank_time_g8.txt
