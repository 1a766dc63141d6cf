#!/bin/bash
# c19: tone-mapping run length — the GPU parity suite on the in-tree build (runs of TONE_RUN = 4, the loop form), then
# A/B: prev (the committed 4-pixel kernel), tone8 / tone2 (runs of 8 / 2 pixels): cornell (3 rounds), city (2).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c19; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=3 bash tools/ab.sh r06c19 prev:exp_lib/libhk_prev.so tone8:exp_lib/libhk_tone8.so tone2:exp_lib/libhk_tone2.so
REPS=2 CONFIG=city-4k STEPS=20 bash tools/ab.sh r06c19c prev:exp_lib/libhk_prev.so tone8:exp_lib/libhk_tone8.so tone2:exp_lib/libhk_tone2.so
echo c19-done
