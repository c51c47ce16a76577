#!/bin/bash
# C2 without sorting: kernel breakdown (rocprofv3 kernel trace) and an option sweep.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c2prof -o c2 -- python3 bench.py --config cornell_box \
    --no-cpu-baseline --parity-rows 0 --single-layer-steps 0 --no-perf-pass --steps 4 --warmup 1 > gpurun_out/c2prof.json 2> gpurun_out/c2prof.err || { tail -5 gpurun_out/c2prof.err; exit 1; }
find gpurun_out/c2prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/c2_kernel_stats.csv
python - <<'PY'
import csv
rows = list(csv.reader(open('gpurun_out/c2_kernel_stats.csv')))
for r in rows[1:16]:
    print(r[0][:60], r[1], round(float(r[2]) / 1e6, 1), round(float(r[3]) / 1e6, 3))
PY
for r in 1 2; do
  for O in "" "--opt wf_xcd=0" "--opt refill=64 --opt refill_shadow=64" "--opt wf_tail_min=4194304" "--opt wf_tail_min=262144" "--opt wf_resolve_paths=0"; do
    timeout -k 10 300 python -u bench.py --config cornell_box --no-cpu-baseline --parity-rows 0 --single-layer-steps 0 \
        --steps 8 --warmup 2 --no-perf-pass $O > gpurun_out/c2.json 2> gpurun_out/c2.err || { tail -5 gpurun_out/c2.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/c2.json'))
print('$O', d['value'], d['ms_per_step'])"
  done
done
