#!/bin/bash
# Round-4 GPU call: the separate direct_lit / emissive launches staging the scene by default — the GPU suite, the
# orbiting-camera and 256x256 lines, the default line.  usage (GPU box): bash profiles/r04/scripts/c23.sh <tag>
set -e
TAG=${1:-c23}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TESTS="tests -m gpu" bash tools/check_run.sh $TAG orbit:cornell-1080p-nee-orbit cornell256:cornell-256-all cornell:cornell-1080p-nee \
    orbit2:cornell-1080p-nee-orbit
echo c23-done
