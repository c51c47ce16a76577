#!/bin/bash
# Instruction-mix PMC pass over one bench configuration (issue-bound analysis of the
# trace kernels): counts per instruction class, its own rocprofv3 --pmc run.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc_issue
mkdir -p $OUT
ARGS="${@:-"--config sponza --steps 16 --warmup 0 --no-cpu-baseline"} --no-perf-pass --parity-rows 0 --single-layer-steps 0"
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/a -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/a.log 2>&1 || { echo "pass a failed"; exit 1; }
echo "pass a ok"
timeout -s KILL 300 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE -d $OUT/b -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/b.log 2>&1 || { echo "pass b failed"; exit 1; }
echo "pass b ok"
# lane utilisation of the VALU (rocprofv3's VALUUtilization: thread-cycles / (64 x active VALU cycles))
timeout -s KILL 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU -d $OUT/c -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/c.log 2>&1 || { echo "pass c failed"; exit 1; }
echo "pass c ok"
find $OUT -name "*.csv"
