#!/bin/bash
# Memory-pipeline PMC passes over one sweep configuration (one pass per counter
# group, never combined with trace domains).  Usage:
#   bash scripts/profile_mem.sh <tag> [sweep args...]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-mem}; shift
ARGS=${@:-"--grid kernel=2 --rounds 1"}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for grp in "GRBM_GUI_ACTIVE TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS" \
           "TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES" \
           "SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY" \
           "TCP_PENDING_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/p$i -o pmc --output-format csv -- python3 scripts/sweep.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok"
done
