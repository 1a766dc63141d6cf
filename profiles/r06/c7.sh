#!/bin/bash
# c7: one-GPU projections of the 2-D tiles against the row bands (tools/band_scaling.py --tiles, 5 balancing rounds, the
# collective-path overheads measured at world size 1 in c3: scene 0.014, city 0.057 ms), a 4-rank rehearsal of
# bench.py's tile path (gloo on one GPU: calibration, rect copies, padded-part gather, reassembly), and the VALU
# issue counters of the scene / city kernels (every kernel alone).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
O=gpurun_out/r06/c7; mkdir -p $O
HK_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 4 --config scene-1080p-full --steps 10 --warmup 3 > $O/rehearsal_tiles4.log 2>&1 || { tail -30 $O/rehearsal_tiles4.log; exit 1; }
grep '"metric"' $O/rehearsal_tiles4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rehearsal', d['config']['parallelism'], d['value'], d['config']['band_bounds'], d['config']['tile_col_bounds'])"
timeout -k 10 500 python tools/band_scaling.py scene-1080p-full 30 --tiles --overhead-ms 0.014 > $O/tiles_scene.log 2>&1
tail -3 $O/tiles_scene.log
timeout -k 10 700 python tools/band_scaling.py city-4k 20 --tiles --overhead-ms 0.057 > $O/tiles_city-4k.log 2>&1
tail -3 $O/tiles_city-4k.log
cd /tmp && export TMPDIR=/tmp
export HK_BENCH_OPTS=channel_streams=0,gbuffer_pipeline=0,tail_pipeline=0
for cfg in scene-1080p-full city-4k; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_WAVE_CYCLES \
    --output-format csv -d $R/$O/valu_$cfg -o run -- python $R/bench.py --config $cfg --steps 6 --warmup 2 --cpu-budget 0 > $R/$O/valu_$cfg.log 2>&1 && echo "valu $cfg ok"
done
echo c7-done
