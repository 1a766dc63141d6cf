#!/bin/bash
# c13: the multi-light indirect pass's texel preload in two compilations of the same code (c11r: the c11 sources,
# 119 VGPRs; pnone: the c12 sources with the one-light variant not preloading, 120 VGPRs) against prev, on one box:
# scene and city (3 rounds each), cornell (2 rounds).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
REPS=3 CONFIG=scene-1080p-full STEPS=30 bash tools/ab.sh r06c13s prev:exp_lib/libhk_prev.so c11r:exp_lib/libhk_c11r.so pnone:exp_lib/libhk_pnone.so
REPS=3 CONFIG=city-4k STEPS=20 bash tools/ab.sh r06c13c prev:exp_lib/libhk_prev.so c11r:exp_lib/libhk_c11r.so pnone:exp_lib/libhk_pnone.so
REPS=2 bash tools/ab.sh r06c13 prev:exp_lib/libhk_prev.so c11r:exp_lib/libhk_c11r.so pnone:exp_lib/libhk_pnone.so
echo c13-done
