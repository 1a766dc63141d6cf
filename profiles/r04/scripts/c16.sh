#!/bin/bash
# Round-4 GPU call: the à-trous taps without branches (all 8 taps' loads in flight; default build) against the
# branchy taps (exp_lib/libhk_base.so, -DHK_DENOISE_BRANCHY=1); the default build also carries spatial reuse's
# window variant at 6 waves and the fused direct launch's scene staging (measured in c15).  Parity suites, bench
# lines.  usage (GPU box): bash profiles/r04/scripts/c16.sh <tag>
set -e
TAG=${1:-c16}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LIB=$R/exp_lib/libhk_base.so
TESTS="tests/test_gpu_parity.py tests/test_gpu_motion.py tests/test_gpu_wavefront.py tests/test_gpu_runtime.py -m gpu" \
  bash tools/check_run.sh $TAG scene:scene-1080p-full scene_base:scene-1080p-full:HK_LIB=$LIB \
    city:city-4k city_base:city-4k:HK_LIB=$LIB cornell:cornell-1080p-nee scene2:scene-1080p-full \
    scene_base2:scene-1080p-full:HK_LIB=$LIB cornell256:cornell-256-all
echo c16-done
