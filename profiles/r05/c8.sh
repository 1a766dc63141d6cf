#!/bin/bash
# Round-5 GPU call 8: branch-free hk_sincos (same bits), spatial reuse reading its depth window without bounds tests
# and its planes through the row-band index (no stripe map) — the whole GPU suite, bench lines against the previous
# commit (exp_lib/libhk_prev.so) alternated on one box.  usage (GPU box): bash profiles/r05/c8.sh <tag>
set -e
TAG=${1:-c8}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
PREV=$R/exp_lib/libhk_prev.so
TESTS="tests -m gpu" bash tools/check_run.sh $TAG city:city-4k city_prev:city-4k:HK_LIB=$PREV scene:scene-1080p-full \
    scene_prev:scene-1080p-full:HK_LIB=$PREV cornell:cornell-1080p-nee cornell_prev:cornell-1080p-nee:HK_LIB=$PREV \
    city2:city-4k city_prev2:city-4k:HK_LIB=$PREV
echo c8-done
