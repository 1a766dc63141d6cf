#!/bin/bash
# One GPU call: the GPU parity suite, smoke(), the default bench line and a rocprofv3 kernel-stats
# pass of the same command.  usage (on the GPU box): bash tools/gpu_check.sh <tag>
set -e
TAG=${1:-check}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
   -d $R/$OUT/stats -o run -- python $R/bench.py --steps 20 --warmup 3 --cpu-budget 0 > $R/$OUT/stats.log 2>&1)
echo done
