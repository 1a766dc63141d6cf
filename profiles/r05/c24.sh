#!/bin/bash
# c24: 2-rank rehearsals (gloo, both ranks on the one GPU) of the band path now that 2-way bands of scene / city
# pipeline (pipeline_heavy_min_px): balanced bands, per-peer gather, 20 frames.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05/c24; mkdir -p $O
for c in scene-1080p-full city-4k; do
  HK_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --config $c --steps 20 --warmup 5 --cpu-budget 0 > $O/rehearsal_$c.log 2>&1
  tail -1 $O/rehearsal_$c.log | cut -c1-400
done
echo c24-done
