#!/bin/bash
# c29 (second build: flags per G-buffer slot, the LDS-typed scene pointers kept; the first build selected the global
# arrays in background tiles and made every scene access a flat load): background tiles skip the LDS scene copy —
# k_gbuffer writes one flag per 8x8 wave quad of a whole-plane
# launch (no geometry hit), the staged light kernels read their tile's four flags with one uniform load and walk the
# global scene arrays there instead (their pixels never read the scene) — the GPU parity suite, then A/B against the
# committed build: cornell (3 rounds), cornell orbiting camera (2).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c29; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=3 bash tools/ab.sh r06c29 prev:exp_lib/libhk_prev.so new:-
REPS=2 CONFIG=cornell-1080p-nee-orbit STEPS=40 bash tools/ab.sh r06c29o prev:exp_lib/libhk_prev.so new:-
echo c29-done
