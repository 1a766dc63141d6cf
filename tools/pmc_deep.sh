#!/bin/bash
# Issue/memory-pipe PMC passes (one group per rocprofv3 run, kernel-trace only).
# usage (GPU box): bash tools/pmc_deep.sh <outdir> <config> [more bench args]
set -e
OUT=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
export HK_BENCH_OPTS=channel_streams=0,gbuffer_pipeline=0,tail_pipeline=0
i=0
for group in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" \
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
  "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $group --output-format csv -d $R/$OUT/deep$i -o run -- \
    python $R/bench.py --config $CFG --steps 8 --warmup 2 --cpu-budget 0 "$@" > $R/$OUT/deep$i.log 2>&1
  echo "pass $i ok"
done
