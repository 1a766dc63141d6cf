#!/bin/bash
# c12: texel preload before the scene staging, one-light indirect variant limited to position + noise (PRE_POSITION,
# 95 VGPRs) — the GPU parity suite, then A/B: prev (exp_lib/libhk_prev.so, no preload), pnone (one-light indirect
# without preload, exp_lib/libhk_pnone.so), new (in-tree): cornell (3 rounds), scene, city.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c12; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=3 bash tools/ab.sh r06c12 prev:exp_lib/libhk_prev.so pnone:exp_lib/libhk_pnone.so new:-
REPS=2 CONFIG=scene-1080p-full STEPS=30 bash tools/ab.sh r06c12s prev:exp_lib/libhk_prev.so new:-
REPS=2 CONFIG=city-4k STEPS=20 bash tools/ab.sh r06c12c prev:exp_lib/libhk_prev.so new:-
echo c12-done
