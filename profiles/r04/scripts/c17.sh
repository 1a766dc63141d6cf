#!/bin/bash
# Round-4 GPU call: demodulation with its G-buffer texels read directly and its variance taps selected (default
# build) against the branchy form (exp_lib/libhk_base.so, -DHK_DEMOD_BRANCHY=1); the default build also carries
# the c16 build's changes.  Parity suites, bench
# lines.  usage (GPU box): bash profiles/r04/scripts/c17.sh <tag>
set -e
TAG=${1:-c17}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LIB=$R/exp_lib/libhk_base.so
TESTS="tests/test_gpu_parity.py tests/test_gpu_motion.py tests/test_gpu_wavefront.py tests/test_gpu_runtime.py -m gpu" \
  bash tools/check_run.sh $TAG scene:scene-1080p-full scene_base:scene-1080p-full:HK_LIB=$LIB \
    city:city-4k city_base:city-4k:HK_LIB=$LIB cornell:cornell-1080p-nee scene2:scene-1080p-full \
    scene_base2:scene-1080p-full:HK_LIB=$LIB cornell256:cornell-256-all
echo c17-done
