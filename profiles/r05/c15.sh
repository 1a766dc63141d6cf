#!/bin/bash
# c15: cornell 8-way stripe frame under option A/Bs (merge, lds_scene, fused_w4), and its kernel trace.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05/c15; mkdir -p $O
for o in "" merge=0 lds_scene=0 fused_w4=0 "merge=0,channel_streams=0"; do
  timeout -k 10 200 python tools/band_scaling.py cornell-1080p-nee 100 --only 8 --kernels --opts "$o" 2>&1 | grep -v amdgpu.ids | grep -v '^{' | sed "s/^/[$o] /"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/band_scaling.py cornell-1080p-nee 100 --only 8 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
cat $(find $GRAFT_REPO_ROOT/$O/prof -name '*kernel_stats.csv') | cut -d, -f1-8 | head -12
