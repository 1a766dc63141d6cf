#!/bin/bash
# c8: (1) the tiles' per-kernel times against the bands' at N = 4 (scene: band_scaling --kernels, the middle rank),
# after the schedule choices (fused direct launch, pipelining, w4 direct) weigh a tile's window pixels instead of its
# full-width planes; (2) k_indirect at 6 and 7 waves per SIMD (amdgpu_waves_per_eu) against the 5 of its 91 VGPRs.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
O=gpurun_out/r06/c8; mkdir -p $O
timeout -k 10 300 python tools/band_scaling.py scene-1080p-full 30 --tiles --only 4 --balance 3 --kernels --overhead-ms 0.014 > $O/tiles4_scene.log 2>&1
grep -E "kernel ms|N=4" $O/tiles4_scene.log | tail -4
timeout -k 10 300 python tools/band_scaling.py scene-1080p-full 30 --only 4 --balance 3 --kernels --overhead-ms 0.014 > $O/bands4_scene.log 2>&1
grep -E "kernel ms|N=4" $O/bands4_scene.log | tail -4
REPS=3 bash tools/ab.sh r06c8 base:- w6:exp_lib/libhk_ind6.so w7:exp_lib/libhk_ind7.so
echo c8-done
