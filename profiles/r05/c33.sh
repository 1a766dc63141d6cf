#!/bin/bash
# c33: issue / memory-pipe PMC passes (tools/pmc_deep.sh, every kernel alone) of the final build on city 4K —
# spatial reuse, demodulation and the four a-trous levels after the round's changes.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/pmc_deep.sh gpurun_out/r05/c33/pmc city-4k
echo c33-done
