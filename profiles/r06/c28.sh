#!/bin/bash
# c28: wave issue priority (s_setprio) — gbprio: G-buffer waves at priority 2 (the next frame's G-buffer shares SIMDs
# with the direct pass's tail and gates the next light passes); iprio: indirect-pass waves at 1 (its end gates the
# next G-buffer) — against the product: cornell (3 rounds), scene (2).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
REPS=3 bash tools/ab.sh r06c28 prev:- gbprio:exp_lib/libhk_gbprio.so iprio:exp_lib/libhk_iprio.so
REPS=2 CONFIG=scene-1080p-full STEPS=30 bash tools/ab.sh r06c28s prev:- gbprio:exp_lib/libhk_gbprio.so iprio:exp_lib/libhk_iprio.so
echo c28-done
