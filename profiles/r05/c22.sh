#!/bin/bash
# c22: frames with spatial reuse or the denoiser pipelined at every size (GPU suite), then the band projections, G-buffer
# rendered every frame.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05/c22; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/band_scaling.py cornell-1080p-nee 50 --overhead-ms 0.003 > $O/bands_cornell.log 2>&1
timeout -k 10 400 python tools/band_scaling.py scene-1080p-full 30 --overhead-ms 0.008 > $O/bands_scene.log 2>&1
timeout -k 10 600 python tools/band_scaling.py city-4k 30 --overhead-ms 0.044 > $O/bands_city-4k.log 2>&1
for f in $O/bands_*.log; do grep "^N=" $f | grep speedup; done
echo c22-done
