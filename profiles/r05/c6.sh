#!/bin/bash
# Round-5 GPU call 6: issue / memory-pipe PMC passes (tools/pmc_deep.sh) of the LDS-staged a-trous levels (city 4K),
# and the transcendentals' Horner steps fused (exp_lib/libhk_fma.so, -DHK_MATH_FMA=1; other bits than the oracle's,
# timing only) against the default build.  usage (GPU box): bash profiles/r05/c6.sh <tag>
set -e
TAG=${1:-c6}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
FMA=$R/exp_lib/libhk_fma.so
bash tools/check_run.sh $TAG city:city-4k city_fma:city-4k:HK_LIB=$FMA scene:scene-1080p-full \
    scene_fma:scene-1080p-full:HK_LIB=$FMA cornell:cornell-1080p-nee cornell_fma:cornell-1080p-nee:HK_LIB=$FMA \
    city2:city-4k city_fma2:city-4k:HK_LIB=$FMA
bash tools/pmc_deep.sh gpurun_out/$TAG/pmc_city city-4k
python3 tools/pmc_summary.py gpurun_out/$TAG/pmc_city city-4k --skip 2 --levels --deep-json gpurun_out/$TAG/pmc_deep_city-4k.json "round-5 LDS-staged a-trous levels (tools/pmc_deep.sh)" > gpurun_out/$TAG/pmc_city_summary.txt 2>&1
echo c6-done
