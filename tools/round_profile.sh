#!/bin/bash
# Round evidence on one GPU: bench lines, rocprofv3 kernel stats and PMC passes per config.
# usage (on the GPU box): bash tools/round_profile.sh <out dir under gpurun_out> [configs...]
set -e
OUT=${1:-gpurun_out/round}; shift || true
CONFIGS=${@:-cornell-1080p-nee scene-1080p-full city-4k}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/$OUT
cd $R
timeout -k 10 600 python bench.py > $R/$OUT/bench_default.json 2> $R/$OUT/bench_default.err
for CFG in $CONFIGS; do
  timeout -k 10 600 python bench.py --config $CFG --steps 30 --warmup 5 --cpu-budget 0 > $R/$OUT/bench_$CFG.json 2> $R/$OUT/bench_$CFG.err
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $R/$OUT/stats_$CFG -o run -- python $R/bench.py --config $CFG --steps 20 --warmup 3 --cpu-budget 0 \
     > $R/$OUT/stats_$CFG.log 2>&1)
  bash tools/pmc.sh $OUT/pmc_$CFG --config $CFG
done
