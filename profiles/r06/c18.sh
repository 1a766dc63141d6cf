#!/bin/bash
# c18: tone mapping as 4-pixel row runs (k_tone4: 16-byte loads, a wave on 2 KiB of contiguous plane) instead of 8x8
# tiles; demodulation and the a-trous levels issue their pixel's own global loads before their LDS staging;
# the GPU parity suite, then A/B against the committed build (exp_lib/libhk_prev.so): cornell (3 rounds),
# scene and city (2 rounds).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c18; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=3 bash tools/ab.sh r06c18 prev:exp_lib/libhk_prev.so new:-
REPS=2 CONFIG=scene-1080p-full STEPS=30 bash tools/ab.sh r06c18s prev:exp_lib/libhk_prev.so new:-
REPS=2 CONFIG=city-4k STEPS=20 bash tools/ab.sh r06c18c prev:exp_lib/libhk_prev.so new:-
echo c18-done
