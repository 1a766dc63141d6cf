#!/bin/bash
# Round-4 GPU call: LDS scene staging in 16-byte copies (default build) against the word-by-word staging
# (exp_lib/libhk_base.so): parity
# suites, bench lines of both on one box.  usage (GPU box): bash profiles/r04/scripts/c12.sh <tag>
set -e
TAG=${1:-c12}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LIB=$R/exp_lib/libhk_base.so
TESTS="tests/test_gpu_parity.py tests/test_gpu_motion.py tests/test_gpu_wavefront.py tests/test_gpu_runtime.py -m gpu" \
  bash tools/check_run.sh $TAG cornell:cornell-1080p-nee cornell_base:cornell-1080p-nee:HK_LIB=$LIB \
    city:city-4k city_base:city-4k:HK_LIB=$LIB scene:scene-1080p-full scene_base:scene-1080p-full:HK_LIB=$LIB \
    cornell2:cornell-1080p-nee cornell_base2:cornell-1080p-nee:HK_LIB=$LIB
echo c12-done
