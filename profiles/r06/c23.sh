#!/bin/bash
# c23: stream priorities on the current build — gbhi: the G-buffer stream at high priority (the next frame's G-buffer
# gates its light passes); sidehi: the indirect side stream at high priority (its end gates the next G-buffer, which
# shares its hardware queue) — against the product (prev): cornell (3 rounds), scene (2).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
REPS=3 bash tools/ab.sh r06c23 prev:exp_lib/libhk_prev.so gbhi:exp_lib/libhk_gbhi.so sidehi:exp_lib/libhk_sidehi.so
REPS=2 CONFIG=scene-1080p-full STEPS=30 bash tools/ab.sh r06c23s prev:exp_lib/libhk_prev.so gbhi:exp_lib/libhk_gbhi.so sidehi:exp_lib/libhk_sidehi.so
echo c23-done
