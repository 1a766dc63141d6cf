#!/bin/bash
# Round-4 GPU call: the committed tree as the driver runs it at round end — the GPU suite, smoke() and the default
# bench line.  usage (GPU box): bash profiles/r04/scripts/c21.sh <tag>
set -e
TAG=${1:-c21}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
python -c "import json;d=json.load(open('$OUT/bench_default.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['duration_ms'], d['roofline']['traffic'], d['cpu_baseline']['value'])"
echo c21-done
