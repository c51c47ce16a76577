#!/bin/bash
# rocprofv3 passes over one bench configuration (kernel trace + separate PMC passes,
# as MI355X_MICROARCH.md's rocprofv3 section prescribes).  Usage:
#   bash scripts/profile.sh <tag> [bench args...]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}; shift
ARGS="${@:-"--config sponza --spp 8 --steps 2 --warmup 1 --no-cpu-baseline"} --no-perf-pass --parity-rows 0 --single-layer-steps 0"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
echo "trace ok"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
echo "fetch ok"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || { echo "write pass failed"; exit 1; }
echo "write ok"
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $OUT/sq -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/sq.log 2>&1 || { echo "sq pass failed"; exit 1; }
echo "sq ok"
timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $OUT/tcc -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/tcc.log 2>&1 || { echo "tcc pass failed"; exit 1; }
echo "tcc ok"
find $OUT -name "*.csv" | head -50
