#!/bin/bash
# PMC passes (one counter group per pass, kernel-trace only; never combined with sys/runtime traces)
# usage: tools/pmc.sh <outdir> <bench args...>
set -e
OUT=$1; shift
mkdir -p $GRAFT_REPO_ROOT/$OUT
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $group --output-format csv -d $R/$OUT/pmc$i -o run -- python $R/bench.py --steps 10 --warmup 2 --cpu-budget 0 "$@" > $R/$OUT/pmc$i.log 2>&1
done
