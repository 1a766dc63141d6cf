#!/bin/bash
# Round-5 GPU call 9: sticky band windows (a setting that widens a band's light-pass window zeroes the
# rows it brings in and keeps the window wide) — the band tests with the new settings-toggle test, then the whole
# GPU suite.  usage (GPU box): bash profiles/r05/c9.sh <tag>
set -e
TAG=${1:-c9}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s -k "row_bands" --timeout 200 \
    --timeout-method thread > $OUT/bands.log 2>&1 || { tail -40 $OUT/bands.log; exit 1; }
grep -E "toggle:|passed|failed" $OUT/bands.log | tail -3
TESTS="tests -m gpu" bash tools/check_run.sh $TAG cornell:cornell-1080p-nee
echo c9-done
