#!/bin/bash
# Round-4 GPU call: spatial reuse's depth window staged with all of a thread's 15 loads in flight (default build)
# against one load -> wait -> store round trip per texel (exp_lib/libhk_base.so): parity suites, bench lines of both
# on one box.  usage (GPU box): bash profiles/r04/scripts/c14.sh <tag>
set -e
TAG=${1:-c14}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LIB=$R/exp_lib/libhk_base.so
TESTS="tests/test_gpu_parity.py tests/test_gpu_motion.py tests/test_gpu_wavefront.py tests/test_gpu_runtime.py -m gpu" \
  bash tools/check_run.sh $TAG scene:scene-1080p-full scene_base:scene-1080p-full:HK_LIB=$LIB \
    city:city-4k city_base:city-4k:HK_LIB=$LIB scene2:scene-1080p-full scene_base2:scene-1080p-full:HK_LIB=$LIB \
    cornell:cornell-1080p-nee
echo c14-done
