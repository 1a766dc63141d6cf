#!/bin/bash
# GPU suite + serial and pipelined scene / city benches.  usage (GPU box): bash tools/gpu_quick_sp.sh <tag>
set -e
TAG=${1:-spq}
S=HK_CHANNEL_STREAMS=0,HK_GB_PIPELINE=0,HK_DN_PIPELINE=0
BENCH_ARGS='--steps 20 --warmup 4 --cpu-budget 0' bash tools/gpu_round2.sh $TAG 'tests -m gpu -x' \
  scene5:scene-1080p-full:$S city5:city-4k:$S scene:scene-1080p-full city:city-4k
