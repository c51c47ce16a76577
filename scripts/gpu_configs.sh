#!/bin/bash
# One bench line per BASELINE config besides the headline (C2 cornell_box, C3 nanobox, C5-per-batch sponza_4k).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in ${@:-cornell_box nanobox sponza_4k}; do
  timeout -k 10 400 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { echo "$cfg failed"; tail -5 gpurun_out/bench_$cfg.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_$cfg.json')); print('$cfg', d['value'], d['unit'], d['ms_per_step'], 'ms/step', d['config']['workload'], d['config']['spp_per_step'], 'spp')"
done
