#!/bin/bash
# c11: the light passes load their pixel's G-buffer and noise texels before the scene staging (PixelTexels) — the GPU
# parity suite, then A/B against the previous build (exp_lib/libhk_prev.so): cornell (3 rounds), scene, city.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c11; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=3 bash tools/ab.sh r06c11 prev:exp_lib/libhk_prev.so new:-
REPS=2 CONFIG=scene-1080p-full STEPS=30 bash tools/ab.sh r06c11s prev:exp_lib/libhk_prev.so new:-
REPS=2 CONFIG=city-4k STEPS=20 bash tools/ab.sh r06c11c prev:exp_lib/libhk_prev.so new:-
echo c11-done
