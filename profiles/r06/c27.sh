#!/bin/bash
# c27: the G-buffer walk loads each 64-byte wide entry whole (the right child box no longer waits for the entry's kind)
# — the GPU parity suite, then A/B against the committed build: cornell (3 rounds), scene and city (2).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c27; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=3 bash tools/ab.sh r06c27 prev:exp_lib/libhk_prev.so new:-
REPS=2 CONFIG=scene-1080p-full STEPS=30 bash tools/ab.sh r06c27s prev:exp_lib/libhk_prev.so new:-
REPS=2 CONFIG=city-4k STEPS=20 bash tools/ab.sh r06c27c prev:exp_lib/libhk_prev.so new:-
echo c27-done
