#!/bin/bash
# c37: the cornell stripe projection on the final build (k_light_merged with its dynamic-LDS stash), smoke().
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05/c37; mkdir -p $O
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python tools/band_scaling.py cornell-1080p-nee 50 --overhead-ms 0.003 > $O/bands_cornell.log 2>&1
grep "^N=" $O/bands_cornell.log
echo c37-done
