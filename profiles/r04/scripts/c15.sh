#!/bin/bash
# Round-4 GPU call: spatial reuse at 6 waves per SIMD (exp_lib/libhk_sp6.so, -DHK_SPATIAL_WAVES=6: 78 VGPRs, no
# spills) against the default 5, and LDS scene staging in every traversal kernel (option lds_scene = 2) on cornell
# now that staging is cheap.  usage (GPU box): bash profiles/r04/scripts/c15.sh <tag>
set -e
TAG=${1:-c15}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LIB=$R/exp_lib/libhk_sp6.so
bash tools/check_run.sh $TAG scene:scene-1080p-full scene_sp6:scene-1080p-full:HK_LIB=$LIB \
    city:city-4k city_sp6:city-4k:HK_LIB=$LIB cornell:cornell-1080p-nee cornell_lds2:cornell-1080p-nee:HK_BENCH_OPTS=lds_scene=2 \
    scene2:scene-1080p-full scene_sp62:scene-1080p-full:HK_LIB=$LIB cornell2:cornell-1080p-nee cornell_lds22:cornell-1080p-nee:HK_BENCH_OPTS=lds_scene=2
echo c15-done
