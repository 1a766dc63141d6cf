#!/bin/bash
# Round-4 GPU call: the separate direct_lit / emissive launches (orbiting camera: the fused launch needs identity
# reprojection) with the scene staged in LDS (option lds_scene = 2) against the default.  usage: bash profiles/r04/scripts/c22.sh <tag>
set -e
TAG=${1:-c22}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/check_run.sh $TAG orbit:cornell-1080p-nee-orbit orbit_lds2:cornell-1080p-nee-orbit:HK_BENCH_OPTS=lds_scene=2 \
    orbit2:cornell-1080p-nee-orbit orbit_lds22:cornell-1080p-nee-orbit:HK_BENCH_OPTS=lds_scene=2
echo c22-done
