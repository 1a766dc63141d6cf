#!/bin/bash
# c34: 4-rank rehearsals (gloo, all four ranks on the one GPU) of the bench's multi-GPU path on the final build:
# cornell stripes, scene / city balanced bands (pipelined), per-peer gather; 10 frames each.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05/c34; mkdir -p $O
port=29551
for c in cornell-1080p-nee scene-1080p-full city-4k; do
  port=$((port+1))
  HK_BENCH_REHEARSAL=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus 4 --config $c --steps 10 --warmup 3 --cpu-budget 0 > $O/rehearsal4_$c.log 2>&1
  tail -1 $O/rehearsal4_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['n_gpus'], d['ms_per_step'], d['config']['parallelism'])"
done
echo c34-done
