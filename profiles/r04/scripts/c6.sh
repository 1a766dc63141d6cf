#!/bin/bash
# Round-4 GPU call: per-channel band windows (direct / emissive launch on core +-16 without emissive spatial
# reuse) — band parity tests, then the balanced band projections with the measured world-1 collective-path
# overheads of c5; scene spatial reuse HBM traffic with and without the view planes.
# usage (GPU box): bash profiles/r04/scripts/c6.sh <tag>
set -e
TAG=${1:-c6}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "row_bands or full_size_bench" -x -v --timeout 300 \
    --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 600 python -u tools/band_scaling.py city-4k 30 --overhead-ms 0.037 > $OUT/bands_city-4k.log 2>&1
tail -5 $OUT/bands_city-4k.log
timeout -k 10 400 python -u tools/band_scaling.py scene-1080p-full 30 --overhead-ms 0.015 > $OUT/bands_scene.log 2>&1
tail -5 $OUT/bands_scene.log
timeout -k 10 300 python -u tools/band_scaling.py cornell-1080p-nee 50 --overhead-ms 0.008 > $OUT/bands_cornell.log 2>&1
tail -5 $OUT/bands_cornell.log
bash tools/pmc_traffic.sh $OUT/pmc_view scene-1080p-full
PMC_OPTS=spatial_view_planes=0 bash tools/pmc_traffic.sh $OUT/pmc_noview scene-1080p-full
for d in pmc_view pmc_noview; do
  python tools/pmc_summary.py $OUT/$d scene-1080p-full --skip 2 > $OUT/$d.txt 2>&1 || true
  grep -i spatial $OUT/$d.txt || true
done
echo c6-done
