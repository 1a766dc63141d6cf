#!/bin/bash
# Round-4 GPU call: the RCCL path at world size 1 against the single-GPU line at the bench's default step count
# (cornell, city), and the city 4K band projection with 5 balancing rounds.  usage (GPU box): bash profiles/r04/scripts/c18.sh <tag>
set -e
TAG=${1:-c18}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/check_run.sh $TAG cornell:cornell-1080p-nee cornell_dist:cornell-1080p-nee::dist city:city-4k city_dist:city-4k::dist \
    scene:scene-1080p-full scene_dist:scene-1080p-full::dist
timeout -k 10 700 python -u tools/band_scaling.py city-4k 30 --balance 5 --overhead-ms 0.037 > gpurun_out/$TAG/bands_city-4k.log 2>&1
tail -n 4 gpurun_out/$TAG/bands_city-4k.log
echo c18-done
