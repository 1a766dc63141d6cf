#!/bin/bash
# Round-4 GPU call: post-change issue / memory-pipe PMC passes (tools/pmc_deep.sh) of the final build, city 4K
# (spatial reuse, the denoiser) and cornell 1080p (k_indirect).  usage (GPU box): bash profiles/r04/scripts/c19.sh <tag>
set -e
TAG=${1:-c19}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/pmc_deep.sh gpurun_out/$TAG/deep_city city-4k
bash tools/pmc_deep.sh gpurun_out/$TAG/deep_cornell cornell-1080p-nee
echo c19-done
