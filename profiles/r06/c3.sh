#!/bin/bash
# c3: the world-1 RCCL line with the per-peer exchange's self send/recv (cornell stripes, scene and city bands) beside
# the single-GPU lines on the same box (the collective-path overheads of the N > 1 projections), a kernel trace of
# the world-1 cornell and scene lines (the RCCL point-to-point kernels), the self-send GPU test, and the driver's
# command with the cached camera view.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
O=gpurun_out/r06/c3; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_rccl.py -v --timeout 150 --timeout-method thread > $O/rccl_test.log 2>&1 || { tail -30 $O/rccl_test.log; exit 1; }
tail -1 $O/rccl_test.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-budget 0 > $O/drv_$i.json 2> $O/drv_$i.err
  python3 -c "import json; d=json.load(open('$O/drv_$i.json')); print('drv', d['value'], d['ms_per_step'])"
done
port=29541
for cfg in cornell-1080p-nee scene-1080p-full city-4k; do
  for i in 1 2; do
    timeout -k 10 300 python bench.py --config $cfg --cpu-budget 0 > $O/single_${cfg}_$i.json 2> $O/single_${cfg}_$i.err
    port=$((port+1))
    HK_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $port bench.py --config $cfg --cpu-budget 0 > $O/rccl_${cfg}_$i.json 2> $O/rccl_${cfg}_$i.err
    python3 -c "
import json; a=json.load(open('$O/single_${cfg}_$i.json')); b=json.load(open('$O/rccl_${cfg}_$i.json'))
print('$cfg', a['ms_per_step'], b['ms_per_step'], round(b['ms_per_step']-a['ms_per_step'],4), b['config']['parallelism'])"
  done
done
for cfg in cornell-1080p-nee scene-1080p-full; do
  port=$((port+1))
  (cd /tmp && export TMPDIR=/tmp && RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
   HK_BENCH_DIST=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace_$cfg -o run -- \
   python $R/bench.py --config $cfg --steps 20 --warmup 5 --cpu-budget 0 > $R/$O/trace_$cfg.json 2> $R/$O/trace_$cfg.err)
  python3 - <<PY
import csv, glob, collections
f = glob.glob("$O/trace_$cfg/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"].lower() for k in ("nccl", "rccl", "sendrecv", "copy")):
        print("$cfg", r["Name"][:90], r["Calls"], r["AverageNs"])
PY
done
echo c3-done
