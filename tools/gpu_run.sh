#!/bin/bash
# One GPU call: a test selection, then bench lines.  usage (on the GPU box):
#   bash tools/gpu_run.sh <tag> "<pytest args>" [bench configs...]
# every GPU step has its own time limit; the script stops at the first failing step.
set -e
TAG=$1
TESTS=$2
shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest $TESTS -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
fi
for spec in "$@"; do
  # spec: name:config[:ENV=V,ENV2=V2]
  IFS=: read -r name cfg envs <<< "$spec"
  ENVS=""
  [ -n "$envs" ] && ENVS=$(echo $envs | tr ',' ' ')
  env $ENVS timeout -k 10 300 python bench.py --config $cfg $BENCH_ARGS > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail -20 $OUT/bench_$name.err; exit 1; }
  echo "$name: $(python -c "import json;d=json.load(open('$OUT/bench_$name.json'));print(d['value'], d['ms_per_step'], d.get('latency_ms'), d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['duration_ms'], d['kernel_ms'])")"
done
echo done
