#!/bin/bash
# c6: 2-D tiles (hk_resize_tile) — the tile parity tests (cornell 2x2 / 4x2 tiles against the whole-frame oracle, the
# 8-tile city 4K decomposition, the rectangle copy), then the band tests and the whole GPU suite.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c6; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "tile or rect" -v --timeout 400 --timeout-method thread > $O/tiles.log 2>&1 || { tail -40 $O/tiles.log; exit 1; }
grep -E "PASSED|FAILED" $O/tiles.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log

# spatial reuse's lane efficiency per neighbour-loop stage (the lane-stats build), scene and city 4K
HK_LIB=exp_lanestats/lanestats.so timeout -k 10 400 python tools/lane_stats.py $O/lane_stats.json scene-1080p-full,city-4k > $O/lane_stats.log 2>&1 || { tail -20 $O/lane_stats.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/lane_stats.json'))
for c, v in d['configs'].items():
    for k, x in v['megakernel'].items(): print(c, k, x['efficiency'], x['iterations'])
"
echo c6-lanes-done
