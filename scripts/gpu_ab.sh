#!/bin/bash
# Interleaved A/B timing of bench.py argument sets (default sponza config, no CPU leg).
#   bash scripts/gpu_ab.sh ROUNDS "args A" "args B" ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
R=$1; shift
for r in $(seq 1 $R); do
  i=0
  for a in "$@"; do
    i=$((i+1))
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 $a > gpurun_out/ab/$i.$r.json 2>gpurun_out/ab/$i.$r.log || { echo "failed: $a"; tail -5 gpurun_out/ab/$i.$r.log; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/ab/$i.$r.json'));r=d['roofline'];o=r.get('other_traces',{});print('%-40s %8.2f ms  %s %7.2f  camera %7.2f' % (sys.argv[1], d['ms_per_step'], r['kernel'][9:15], r['avg_launch_ms'], o.get('camera',{}).get('avg_launch_ms',r['avg_launch_ms'])))" "$a"
  done
done
