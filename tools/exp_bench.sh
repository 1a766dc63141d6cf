#!/bin/bash
# bench.py (default config, fork-join streams) per experiment library. usage: tools/exp_bench.sh tag=lib ...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/exp
for tl in "$@"; do
  tag=${tl%%=*}; lib=${tl#*=}
  if [ "$lib" = "-" ]; then unset HK_LIB; else export HK_LIB=$R/$lib; fi
  timeout -k 10 120 python -u $R/bench.py --steps 60 --warmup 10 --cpu-budget 0 ${BENCH_ARGS} > $R/gpurun_out/exp/bench_$tag.json 2> $R/gpurun_out/exp/bench_$tag.log
  unset HK_LIB
done
