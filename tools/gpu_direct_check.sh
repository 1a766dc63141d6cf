#!/bin/bash
# GPU suite + default bench + serialised cornell / city benches (direct-pass changes).
set -e
TAG=${1:-dc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/$TAG
S=HK_CHANNEL_STREAMS=0,HK_GB_PIPELINE=0,HK_DN_PIPELINE=0
BENCH_ARGS='--steps 20 --warmup 4 --cpu-budget 0' bash tools/gpu_round2.sh $TAG 'tests -m gpu -x' \
  cornell5:cornell-1080p-nee:$S scene5:scene-1080p-full:$S city5:city-4k:$S
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench_default.json 2> gpurun_out/$TAG/bench_default.err
python -c "import json;d=json.load(open('gpurun_out/$TAG/bench_default.json'));print(d['value'], d['ms_per_step'], d['latency_ms'], d['roofline'])"
