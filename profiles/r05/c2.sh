#!/bin/bash
# Round-5 GPU call 2: branch-free hk_exp2 / hk_log2 (same bits) and the a-trous levels' per-pixel work cut (luminance
# denominators from demodulation, class tests, no stripe index) — the whole GPU suite on the default build, then bench
# lines of the round-start build (exp_lib/libhk_base.so), the default build and its batched-tap-load variant
# (exp_lib/libhk_pf.so, -DHK_DENOISE_PF=1) on one box.  usage (GPU box): bash profiles/r05/c2.sh <tag>
set -e
TAG=${1:-c2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
BASE=$R/exp_lib/libhk_base.so
PF=$R/exp_lib/libhk_pf.so
TESTS="tests -m gpu" bash tools/check_run.sh $TAG \
    scene_base:scene-1080p-full:HK_LIB=$BASE scene:scene-1080p-full scene_pf:scene-1080p-full:HK_LIB=$PF \
    city_base:city-4k:HK_LIB=$BASE city:city-4k city_pf:city-4k:HK_LIB=$PF \
    cornell_base:cornell-1080p-nee:HK_LIB=$BASE cornell:cornell-1080p-nee \
    scene_base2:scene-1080p-full:HK_LIB=$BASE scene2:scene-1080p-full city_base2:city-4k:HK_LIB=$BASE city2:city-4k
echo c2-done
