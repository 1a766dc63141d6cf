#!/bin/bash
# Round-4 GPU call: the direct passes' previous reservoir read in two steps (default build: fused w4 113/115 -> 97/99
# VGPRs) and, in exp_lib/libhk_resurf.so (-DHK_EXP_RESURF=1), the emissive pass fetching its surface itself instead
# of holding the direct pass's through its walks (93/95 VGPRs: 5 waves per SIMD).  Parity suites on the experiment
# build (it contains both changes), bench lines of both.  usage (GPU box): bash profiles/r04/scripts/c9.sh <tag>
set -e
TAG=${1:-c9}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$TAG
mkdir -p $OUT
LIB=$R/exp_lib/libhk_resurf.so
HK_LIB=$LIB timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_motion.py tests/test_gpu_wavefront.py tests/test_gpu_runtime.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > $OUT/tests_resurf.log 2>&1 || { tail -40 $OUT/tests_resurf.log; exit 1; }
tail -1 $OUT/tests_resurf.log
bash tools/check_run.sh $TAG cornell:cornell-1080p-nee cornell_resurf:cornell-1080p-nee:HK_LIB=$LIB \
    scene:scene-1080p-full scene_resurf:scene-1080p-full:HK_LIB=$LIB city:city-4k city_resurf:city-4k:HK_LIB=$LIB \
    cornell2:cornell-1080p-nee cornell_resurf2:cornell-1080p-nee:HK_LIB=$LIB
echo c9-done
