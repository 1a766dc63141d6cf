#!/bin/bash
# Round profile refresh (one GPU call): GPU suite + smoke + default bench + rocprofv3 stats, then the
# PMC passes of the default config.  usage (on the GPU box): bash tools/gpu_profiles.sh <tag>
set -e
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_check.sh $TAG
bash tools/pmc.sh gpurun_out/$TAG/pmc
echo profiles-done
