#!/bin/bash
# spatial-reuse + band-window round: GPU suite, serial spatial benches (5 / 6 waves), pipelined
# scene / city benches, band scaling projection.  usage (GPU box): bash tools/gpu_sp.sh <tag>
set -e
TAG=${1:-sp}
S=HK_CHANNEL_STREAMS=0,HK_GB_PIPELINE=0,HK_DN_PIPELINE=0
BENCH_ARGS='--steps 20 --warmup 4 --cpu-budget 0' bash tools/gpu_round2.sh $TAG 'tests -m gpu -x' \
  scene5:scene-1080p-full:$S city5:city-4k:$S \
  scene6:scene-1080p-full:$S,HK_LIB=exp_sp6/libhikari_amd.so city6:city-4k:$S,HK_LIB=exp_sp6/libhikari_amd.so \
  scene:scene-1080p-full city:city-4k
timeout -k 10 300 python tools/band_scaling.py city-4k 20 --bands > gpurun_out/$TAG/bands_city-4k.json 2> gpurun_out/$TAG/bands_city-4k.err
echo bands-done
