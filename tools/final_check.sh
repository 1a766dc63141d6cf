#!/bin/bash
# Round-end check on one GPU: the GPU parity suite, smoke(), the default bench line, its rocprofv3
# kernel statistics and a 2-rank rehearsal of the multi-GPU bench path (both ranks on the one GPU,
# gloo collectives).  usage (on the GPU box): bash tools/final_check.sh [tag]
set -e
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
# the driver's own command (BENCH_rNN.json: --gpus 1 --steps 20 --warmup 5) beside the default 100 / 16 (VERDICT r05
# item 3): its 20 frames are frames 5-24, heavier than the steady state (ReSTIR history filling)
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_$i.json 2> $OUT/bench_driver_$i.err
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
   -d $R/$OUT/stats -o run -- python $R/bench.py --steps 20 --warmup 3 --cpu-budget 0 > $R/$OUT/stats.log 2>&1)
# the same with every kernel alone (channel fork and frame pipelining off): the isolated durations of the roofline
(cd /tmp && export TMPDIR=/tmp && HK_BENCH_OPTS=channel_streams=0,gbuffer_pipeline=0,tail_pipeline=0 timeout -k 10 300 rocprofv3 \
   --kernel-trace --stats --output-format csv -d $R/$OUT/stats_isolated -o run -- python $R/bench.py --steps 20 --warmup 3 \
   --cpu-budget 0 > $R/$OUT/stats_isolated.log 2>&1)
# the RCCL path itself at world size 1 (communicator, per-frame all-gather, reductions) on the one GPU
HK_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29534 bench.py --cpu-budget 0 > $OUT/rccl_world1.json 2> $OUT/rccl_world1.err
HK_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 > $OUT/rehearsal.log 2>&1
echo final-done
