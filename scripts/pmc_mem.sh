#!/bin/bash
# Memory-path PMC passes over one bench configuration: where the trace kernels' vector loads
# spend their time -- the address unit (TA) stalled by the L1 (TCP), L1 hit rate, L1->L2 requests
# and their latency, L2 hit rate.  One rocprofv3 --pmc run per pass, no trace domains.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc_mem
mkdir -p $OUT
ARGS="${@:-"--config sponza --steps 8 --warmup 0 --no-cpu-baseline"} --no-perf-pass --parity-rows 0 --single-layer-steps 0"
timeout -s KILL 300 rocprofv3 --pmc TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE -d $OUT/c -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/c.log 2>&1 || { echo "pass c failed"; exit 1; }
echo "pass c ok"
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TD_TD_BUSY_sum SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAVE_CYCLES -d $OUT/d -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/d.log 2>&1 || { echo "pass d failed"; exit 1; }
echo "pass d ok"
find $OUT -name "*.csv"
