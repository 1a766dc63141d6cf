#!/bin/bash
# Round-5 GPU call 1: the indirect bounce walk with the ordered closest-hit rule (exp_lib/libhk_ordered.so,
# -DHK_ORDERED_WALKS=1) — the whole GPU suite on it (the oracle checks every bounce ray both ways), then bench lines
# of the default build and the experiment build alternated on one box.  usage (GPU box): bash profiles/r05/c1.sh <tag>
set -e
TAG=${1:-c1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LIB=$R/exp_lib/libhk_ordered.so
OUT=gpurun_out/$TAG
mkdir -p $OUT
HK_LIB=$LIB timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/tests_ordered.log 2>&1 || { tail -40 $OUT/tests_ordered.log; exit 1; }
tail -1 $OUT/tests_ordered.log
bash tools/check_run.sh $TAG cornell:cornell-1080p-nee cornell_ord:cornell-1080p-nee:HK_LIB=$LIB \
    cornell2:cornell-1080p-nee cornell_ord2:cornell-1080p-nee:HK_LIB=$LIB \
    scene:scene-1080p-full scene_ord:scene-1080p-full:HK_LIB=$LIB city:city-4k city_ord:city-4k:HK_LIB=$LIB
echo c1-done
