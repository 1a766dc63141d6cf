#!/bin/bash
# Round-4 GPU call: the separate direct launches staging the scene only on frames of >= direct_w4_min_px pixels —
# the orbiting-camera and 256x256 lines, the forced-variant and motion parity tests.  usage: bash profiles/r04/scripts/c24.sh <tag>
set -e
TAG=${1:-c24}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TESTS="tests/test_gpu_motion.py tests/test_gpu_parity.py -m gpu" \
  bash tools/check_run.sh $TAG orbit:cornell-1080p-nee-orbit cornell256:cornell-256-all
echo c24-done
