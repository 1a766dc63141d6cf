#!/bin/bash
# Round-end check on one GPU: the GPU parity suite, smoke(), the default bench line and a
# 2-rank rehearsal of the multi-GPU bench path (both ranks on the one GPU, gloo collectives).
# usage (on the GPU box): bash tools/final_check.sh
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_final2.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final2.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_final2.json 2> gpurun_out/bench_final2.err
HK_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/rehearsal3.log 2>&1
