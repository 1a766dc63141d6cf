#!/bin/bash
# Kernel-trace stats pass + PMC passes of one bench config.
# usage: tools/profile.sh <config> [extra bench args]   -> gpurun_out/prof_<config>/
set -e
CFG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/prof_$CFG
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/stats -o run -- \
  python $R/bench.py --config $CFG --steps 20 --warmup 3 --cpu-budget 0 "$@" > $R/$OUT/stats.log 2>&1
cd $R && bash tools/pmc.sh $OUT --config $CFG "$@"
