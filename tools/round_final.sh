#!/bin/bash
# Round-end measurement set on one GPU: tools/final_check.sh (GPU suite, smoke, default bench,
# rocprofv3 kernel statistics, 2-rank rehearsal; SKIP_CHECK=1 skips it), then bench lines of the other BASELINE configs
# and the one-GPU stripe / band projections.  usage (GPU box): bash tools/round_final.sh <tag>
set -e
TAG=${1:-round_final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
[ -z "$SKIP_CHECK" ] && bash tools/final_check.sh $TAG
BENCH_ARGS='--steps 20 --warmup 4 --cpu-budget 0' bash tools/gpu_run.sh $TAG '' \
  scene:scene-1080p-full city:city-4k cornell256:cornell-256-all city-dynamic:city-4k-dynamic \
  cornell-orbit:cornell-1080p-nee-orbit city-orbit:city-4k-orbit
BENCH_ARGS='--steps 2 --warmup 1 --cpu-budget 0' bash tools/gpu_run.sh $TAG '' \
  city16-wavefront:city-4k-16spp city16-megakernel:city-4k-16spp:HK_BENCH_WAVEFRONT=0
timeout -k 10 300 python tools/band_scaling.py cornell-1080p-nee 50 > gpurun_out/$TAG/bands_cornell.log 2>&1
timeout -k 10 300 python tools/band_scaling.py scene-1080p-full 30 --bands > gpurun_out/$TAG/bands_scene.log 2>&1
timeout -k 10 300 python tools/band_scaling.py city-4k 20 --bands > gpurun_out/$TAG/bands_city-4k.log 2>&1
echo round-final-done
