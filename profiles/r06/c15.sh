#!/bin/bash
# c15: the texel preload moved to the indirect variant scene and city run (one bounce, no LDS staging) — the GPU
# parity suite, then A/B against the committed build (exp_lib/libhk_prev.so: preload in the multi-bounce variants):
# scene, city, cornell (2 rounds each).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c15; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=2 CONFIG=scene-1080p-full STEPS=30 bash tools/ab.sh r06c15s prev:exp_lib/libhk_prev.so new:-
REPS=2 CONFIG=city-4k STEPS=20 bash tools/ab.sh r06c15c prev:exp_lib/libhk_prev.so new:-
REPS=2 bash tools/ab.sh r06c15 prev:exp_lib/libhk_prev.so new:-
echo c15-done
