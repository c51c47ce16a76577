#!/bin/bash
# round-3 evidence: C1 cornell bench line (with cpu_baseline), the chunked configs' bench lines on the
# corrected pass accounting, and the kernel trace of the 8-way split rehearsal
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/profiles
for cfg in cornell cornell_box sponza_4k; do
  timeout -k 10 400 python bench.py --config $cfg --steps 3 --warmup 1 > gpurun_out/profiles/r03_bench_$cfg.json 2> gpurun_out/bench_$cfg.log || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_$cfg.log; exit 1; }
  echo "$cfg: $(head -c 400 gpurun_out/profiles/r03_bench_$cfg.json)"
done
bash scripts/gpu_rank_profile.sh 1 8 > gpurun_out/rank_prof.txt 2>&1 || { echo "rank profile failed"; tail -20 gpurun_out/rank_prof.txt; exit 1; }
cat gpurun_out/rank_prof.txt
python3 scripts/timeline.py $(find gpurun_out/rank_prof/n8 -name "*kernel_trace.csv") 3 > gpurun_out/timeline_n8.txt
