#!/bin/bash
# c1: the driver's bench command (--gpus 1 --steps 20 --warmup 5) beside the builder's default (100 / 16) on one box,
# alternated, plus the two factors split: warm-up 16 with 20 steps, warm-up 5 with 100 steps, and the 20/5 command
# with the per-kernel timing events off (HK_BENCH_TIMING_EVERY above the step count).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c1; mkdir -p $O
run() {  # name, env, args
  env $2 timeout -k 10 200 python bench.py --cpu-budget 0 $3 > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('$1', d['value'], d['ms_per_step'], d['roofline']['duration_ms'])"
}
for i in 1 2 3; do
  run drv_$i "" "--gpus 1 --steps 20 --warmup 5"
  run def_$i "" "--gpus 1 --steps 100 --warmup 16"
  run s20w16_$i "" "--gpus 1 --steps 20 --warmup 16"
  run s100w5_$i "" "--gpus 1 --steps 100 --warmup 5"
  run drv_noev_$i "HK_BENCH_TIMING_EVERY=1000" "--gpus 1 --steps 20 --warmup 5"
done
echo c1-done
