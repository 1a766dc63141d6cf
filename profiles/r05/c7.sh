#!/bin/bash
# Round-5 GPU call 7: the fused Horner steps of hk_exp2 / hk_log2 (oracle and kernels alike) and hk_exp_weight in the
# a-trous levels — the whole GPU suite, the default line and the scene / city lines.  usage: bash profiles/r05/c7.sh <tag>
set -e
TAG=${1:-c7}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TESTS="tests -m gpu" bash tools/check_run.sh $TAG cornell:cornell-1080p-nee scene:scene-1080p-full city:city-4k
echo c7-done
