#!/bin/bash
# Run exp_run.sh + trace_bench for several experiment libraries. usage: tools/exp_multi.sh tag=lib ...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
for tl in "$@"; do
  tag=${tl%%=*}; lib=${tl#*=}
  bash $R/tools/exp_run.sh $tag $lib cornell-1080p-nee
  if [ "$lib" = "-" ]; then unset HK_LIB; else export HK_LIB=$R/$lib; fi
  timeout -k 10 120 python -u $R/tools/trace_bench.py > $R/gpurun_out/exp/tb_$tag.log 2>&1
  unset HK_LIB
done
