#!/bin/bash
# Bench lines of every BASELINE config plus the one-GPU band/stripe projections.
# usage (GPU box): bash tools/gpu_benches.sh <tag>
set -e
TAG=${1:-benches}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/bench_cornell-1080p-nee.json 2> $OUT/bench_cornell.err
echo "cornell $(python -c "import json;d=json.load(open('$OUT/bench_cornell-1080p-nee.json'));print(d['value'], d['ms_per_step'], d['latency_ms'])")"
BENCH_ARGS='--steps 20 --warmup 4 --cpu-budget 0' bash tools/gpu_round2.sh $TAG '' \
  cornell256:cornell-256-all city-dynamic:city-4k-dynamic
BENCH_ARGS='--steps 2 --warmup 1 --cpu-budget 0' bash tools/gpu_round2.sh $TAG '' \
  city16-wavefront:city-4k-16spp city16-megakernel:city-4k-16spp:HK_BENCH_WAVEFRONT=0
timeout -k 10 300 python tools/band_scaling.py cornell-1080p-nee 50 > $OUT/bands_cornell.log 2> $OUT/bands_cornell.err
timeout -k 10 300 python tools/band_scaling.py scene-1080p-full 30 --bands > $OUT/bands_scene.log 2> $OUT/bands_scene.err
echo all-done
