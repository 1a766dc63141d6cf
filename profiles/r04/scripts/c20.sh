#!/bin/bash
# Round-4 GPU call: the à-trous taps in two batches of four with all of a batch's texel loads issued before the
# first wait (exp_lib/libhk_pf.so, -DHK_DENOISE_PF=1; branches kept) against the default per-tap loads: parity
# suites on the experiment build, bench lines of both.  usage (GPU box): bash profiles/r04/scripts/c20.sh <tag>
set -e
TAG=${1:-c20}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LIB=$R/exp_lib/libhk_pf.so
OUT=gpurun_out/$TAG
mkdir -p $OUT
HK_LIB=$LIB timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_motion.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > $OUT/tests_pf.log 2>&1 || { tail -40 $OUT/tests_pf.log; exit 1; }
tail -1 $OUT/tests_pf.log
bash tools/check_run.sh $TAG scene:scene-1080p-full scene_pf:scene-1080p-full:HK_LIB=$LIB \
    city:city-4k city_pf:city-4k:HK_LIB=$LIB scene2:scene-1080p-full scene_pf2:scene-1080p-full:HK_LIB=$LIB
echo c20-done
