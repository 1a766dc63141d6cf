#!/bin/bash
# FETCH_SIZE of one kernel family per experiment library. usage: tools/pmc_fetch.sh <config> tag=lib ...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=$1; shift
cd /tmp && export TMPDIR=/tmp
for tl in "$@"; do
  tag=${tl%%=*}; lib=${tl#*=}
  if [ "$lib" = "-" ]; then unset HK_LIB; else export HK_LIB=$R/$lib; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcf_$tag -o run -- python $R/bench.py --config $CFG --steps 4 --warmup 2 --cpu-budget 0 > $R/gpurun_out/pmcf_$tag.log 2>&1
  unset HK_LIB
done
