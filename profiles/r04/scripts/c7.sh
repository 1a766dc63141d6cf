#!/bin/bash
# Round-4 GPU call: k_indirect's temporal tail with the previous record read in two steps (default build) and,
# in the experiment build exp_lib/libhk_reload.so (-DHK_EXP_RELOAD=2), the pixel's G-buffer / noise fields read
# again after the walks (105 -> 94 VGPRs, 5 waves per SIMD): parity suites on the experiment build, bench lines
# of both.  usage (GPU box): bash profiles/r04/scripts/c7.sh <tag>
set -e
TAG=${1:-c7}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$TAG
mkdir -p $OUT
LIB=$R/exp_lib/libhk_reload.so
HK_LIB=$LIB timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_motion.py tests/test_gpu_wavefront.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > $OUT/tests_reload.log 2>&1 || { tail -40 $OUT/tests_reload.log; exit 1; }
tail -1 $OUT/tests_reload.log
bash tools/check_run.sh $TAG cornell:cornell-1080p-nee cornell_reload:cornell-1080p-nee:HK_LIB=$LIB \
    scene:scene-1080p-full scene_reload:scene-1080p-full:HK_LIB=$LIB city:city-4k city_reload:city-4k:HK_LIB=$LIB \
    cornell2:cornell-1080p-nee cornell_reload2:cornell-1080p-nee:HK_LIB=$LIB
echo c7-done
