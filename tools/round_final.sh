#!/bin/bash
# Round-end measurement set on one GPU, in two calls (each under gpurun's 20-minute limit):
#   part a: tools/final_check.sh (GPU suite, smoke, default bench, rocprofv3 kernel statistics pipelined and
#           isolated, the RCCL path at world size 1, a 2-rank rehearsal), then the PMC HBM-traffic passes
#           (FETCH_SIZE / WRITE_SIZE, every kernel alone) of the three 1-spp configs;
#   part b: bench lines of the other BASELINE configs and the balanced one-GPU band projections with the
#           measured world-1 collective-path overheads.
# usage (GPU box): bash tools/round_final.sh <tag> a|b
set -e
TAG=${1:-round_final}
PART=${2:-a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
if [ "$PART" = "a" ]; then
  bash tools/final_check.sh $TAG
  bash tools/pmc_traffic.sh gpurun_out/$TAG/pmc cornell-1080p-nee scene-1080p-full city-4k
  echo round-final-a-done
else
  BENCH_ARGS='--steps 20 --warmup 4 --cpu-budget 0' bash tools/gpu_run.sh $TAG '' \
    scene:scene-1080p-full city:city-4k cornell256:cornell-256-all city-dynamic:city-4k-dynamic \
    cornell-orbit:cornell-1080p-nee-orbit city-orbit:city-4k-orbit
  BENCH_ARGS='--steps 2 --warmup 1 --cpu-budget 0' bash tools/gpu_run.sh $TAG '' \
    city16-wavefront:city-4k-16spp city16-megakernel:city-4k-16spp:HK_BENCH_WAVEFRONT=0
  # overheads: the world-1 collective path with the per-peer exchange's RCCL self send / receive (profiles/r06/c3)
  timeout -k 10 300 python tools/band_scaling.py cornell-1080p-nee 50 --overhead-ms 0.012 > gpurun_out/$TAG/bands_cornell.log 2>&1
  timeout -k 10 400 python tools/band_scaling.py scene-1080p-full 30 --overhead-ms 0.014 > gpurun_out/$TAG/bands_scene.log 2>&1
  timeout -k 10 600 python tools/band_scaling.py city-4k 30 --overhead-ms 0.057 > gpurun_out/$TAG/bands_city-4k.log 2>&1
  for f in gpurun_out/$TAG/bands_*.log; do tail -n 2 $f; done
  echo round-final-b-done
fi
