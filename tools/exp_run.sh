#!/bin/bash
# Timing experiments: serial per-kernel times (HK_CHANNEL_STREAMS=0) of bench configs for the
# in-tree library and experiment builds under exp_build/.  usage: tools/exp_run.sh <tag> <lib|-> [configs...]
set -e
TAG=$1; LIB=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/exp
for c in ${@:-cornell-1080p-nee}; do
  if [ "$LIB" = "-" ]; then unset HK_LIB; else export HK_LIB=$R/$LIB; fi
  HK_CHANNEL_STREAMS=0 timeout -k 10 120 python -u $R/bench.py --config $c --steps 20 --warmup 5 --cpu-budget 0 > $R/gpurun_out/exp/${TAG}_$c.json 2> $R/gpurun_out/exp/${TAG}_$c.log
done
