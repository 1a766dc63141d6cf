#!/bin/bash
# c14: where the N=8 cornell stripe frame goes (per-kernel times + host enqueue per frame), N=1 beside it.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r05/c14
timeout -k 10 300 python tools/band_scaling.py cornell-1080p-nee 50 --kernels --only 8 > gpurun_out/r05/c14/bands8.log 2>&1
timeout -k 10 300 python tools/band_scaling.py cornell-1080p-nee 50 --kernels --only 1 > gpurun_out/r05/c14/bands1.log 2>&1
cat gpurun_out/r05/c14/bands8.log gpurun_out/r05/c14/bands1.log | grep -v amdgpu.ids
