#!/bin/bash
# c14: k_spatial issues its pixel's own loads (G-buffer texels; new: + its C.cur record) before the depth-window
# staging — the GPU parity suite on the in-tree build, then A/B on scene and city: prev (the committed build),
# spnores (G-buffer texels only, exp_lib/libhk_spnores.so), new (in-tree, + the record; 128 B of scratch in the
# indirect-channel variants).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c14; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=3 CONFIG=scene-1080p-full STEPS=30 bash tools/ab.sh r06c14s prev:exp_lib/libhk_prev.so spnores:exp_lib/libhk_spnores.so new:-
REPS=3 CONFIG=city-4k STEPS=20 bash tools/ab.sh r06c14c prev:exp_lib/libhk_prev.so spnores:exp_lib/libhk_spnores.so new:-
echo c14-done
