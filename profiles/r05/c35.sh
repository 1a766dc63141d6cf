#!/bin/bash
# c35: bench.py after the rehearsal-label change: the default line and a 2-rank rehearsal line.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05/c35; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['ms_per_step'], d['config']['parallelism'])"
HK_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 3 > $O/rehearsal.log 2>&1
tail -1 $O/rehearsal.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['config']['parallelism'])"
echo c35-done
