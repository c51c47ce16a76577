#!/bin/bash
# PMC comparison of trace builds: per variant two rocprofv3 --pmc passes (instruction mix; address
# path and L1), each its own run, no trace domains; summarised per lean trace kind and launch by
# scripts/pmc_ab_summary.py.   bash scripts/pmc_ab.sh 43 49 [-- bench args]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ab
mkdir -p $OUT
VS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do VS+=("$1"); shift; done
[ "$1" = "--" ] && shift
ARGS="--config sponza --steps 8 --warmup 0 --no-cpu-baseline --no-perf-pass --parity-rows 0 --single-layer-steps 0 $*"
for V in "${VS[@]}"; do
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d $OUT/v${V}_a -o pmc --output-format csv -- python3 bench.py $ARGS --variant $V > $OUT/v${V}_a.log 2>&1 || { echo "pass a $V failed"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE -d $OUT/v${V}_b -o pmc --output-format csv -- python3 bench.py $ARGS --variant $V > $OUT/v${V}_b.log 2>&1 || { echo "pass b $V failed"; exit 1; }
  echo "variant $V ok"
done
python3 scripts/pmc_ab_summary.py $OUT "${VS[@]}"
