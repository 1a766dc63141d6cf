#!/bin/bash
# HBM traffic passes (FETCH_SIZE, WRITE_SIZE; one counter group per rocprofv3 run, kernel-trace only)
# for the bench configs, every kernel on its own (channel fork and frame pipelining off), so each
# launch's bytes are its own; summarise with tools/pmc_summary.py --skip 2 (steady-state dispatches).
# usage (GPU box): [PMC_OPTS=key=v,...] bash tools/pmc_traffic.sh <outdir> [configs...]
set -e
OUT=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
export HK_BENCH_OPTS=channel_streams=0,gbuffer_pipeline=0,tail_pipeline=0${PMC_OPTS:+,$PMC_OPTS}
for cfg in "$@"; do
  for group in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $group --output-format csv -d $R/$OUT/$cfg/$group -o run -- \
      python $R/bench.py --config $cfg --steps ${PMC_STEPS:-8} --warmup 2 --cpu-budget 0 > $R/$OUT/$cfg.$group.log 2>&1
    echo "$cfg $group ok"
  done
done
