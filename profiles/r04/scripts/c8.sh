#!/bin/bash
# Round-4 GPU call: k_indirect forced to 6 waves per SIMD (exp_lib/libhk_w6.so, -DHK_INDIRECT_WAVES=6: 80 VGPRs
# with 25 spilled) against the default 5-wave build.  usage (GPU box): bash profiles/r04/scripts/c8.sh <tag>
set -e
TAG=${1:-c8}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LIB=$R/exp_lib/libhk_w6.so
bash tools/check_run.sh $TAG cornell:cornell-1080p-nee cornell_w6:cornell-1080p-nee:HK_LIB=$LIB \
    city:city-4k city_w6:city-4k:HK_LIB=$LIB cornell2:cornell-1080p-nee cornell_w62:cornell-1080p-nee:HK_LIB=$LIB
echo c8-done
