#!/bin/bash
# Round-5 GPU call 3: the a-trous levels with their tile + step region staged in LDS (k_denoise3s, default build)
# against the per-tap loads (exp_lib/libhk_unstaged.so) and the batched per-tap loads (exp_lib/libhk_pf.so): the
# parity suites on the default build, then bench lines alternated on one box.  usage: bash profiles/r05/c3.sh <tag>
set -e
TAG=${1:-c3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
UN=$R/exp_lib/libhk_unstaged.so
PF=$R/exp_lib/libhk_pf.so
TESTS="tests/test_gpu_parity.py tests/test_gpu_motion.py -m gpu" bash tools/check_run.sh $TAG \
    city:city-4k city_un:city-4k:HK_LIB=$UN city_pf:city-4k:HK_LIB=$PF \
    scene:scene-1080p-full scene_un:scene-1080p-full:HK_LIB=$UN scene_pf:scene-1080p-full:HK_LIB=$PF \
    city2:city-4k city_pf2:city-4k:HK_LIB=$PF
echo c3-done
