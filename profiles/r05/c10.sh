#!/bin/bash
# Round-5 GPU call 10: ADVICE r04 fixes (internal-variance copies waited for by hk_denoise, completed foreign-copy
# events pruned, integer-only option values) and the per-peer gather (HK_BENCH_GATHER=peer, the default) — the
# whole GPU suite; the RCCL path at world size 1 with the per-peer and the ring gather beside the single-GPU line
# (cornell stripes, scene / city bands); 2-rank gloo rehearsals of both decompositions on the one GPU.
set -e
TAG=${1:-c10}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$TAG
TESTS="tests -m gpu" bash tools/check_run.sh $TAG cornell:cornell-1080p-nee cornell_peer:cornell-1080p-nee::dist \
    cornell_ring:cornell-1080p-nee:HK_BENCH_GATHER=ring:dist scene:scene-1080p-full scene_peer:scene-1080p-full::dist \
    scene_ring:scene-1080p-full:HK_BENCH_GATHER=ring:dist city:city-4k city_peer:city-4k::dist
port=29640
for cfg in cornell-1080p-nee scene-1080p-full; do
  port=$((port+1))
  HK_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port $port bench.py --config $cfg --gpus 2 --steps 10 --warmup 3 --cpu-budget 0 \
      > $OUT/rehearsal_$cfg.json 2> $OUT/rehearsal_$cfg.err || { tail -20 $OUT/rehearsal_$cfg.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/rehearsal_$cfg.json')); print('$cfg rehearsal', d['value'], d['ms_per_step'], d['config']['parallelism'])"
done
echo c10-done
