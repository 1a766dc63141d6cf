#!/bin/bash
# c9: the walk step with both node loads issued before the first node's test (exp_lib/libhk_pre2.so: an asm barrier
# keeps the second load from sinking into the branch that uses it) against the product build: cornell, scene, city.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
REPS=3 bash tools/ab.sh r06c9 base:- pre2:exp_lib/libhk_pre2.so
REPS=2 CONFIG=scene-1080p-full STEPS=30 bash tools/ab.sh r06c9s base:- pre2:exp_lib/libhk_pre2.so
REPS=2 CONFIG=city-4k STEPS=20 bash tools/ab.sh r06c9c base:- pre2:exp_lib/libhk_pre2.so
echo c9-done
