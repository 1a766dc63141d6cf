#!/bin/bash
# Runtime-knob sweep of one bench config (each line: knobs -> value, ms/frame).
# usage (GPU box): bash tools/knob_sweep.sh <tag> <config> "<ENV=V,...>" ...
set -e
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for spec in "$@"; do
  i=$((i+1))
  ENVS=""
  [ "$spec" != "-" ] && ENVS=$(echo $spec | tr ',' ' ')
  env $ENVS timeout -k 10 200 python bench.py --config $CFG --steps 60 --warmup 10 --cpu-budget 0 > $OUT/k$i.json 2> $OUT/k$i.err
  echo "$spec: $(python -c "import json;d=json.load(open('$OUT/k$i.json'));print(d['value'], d['ms_per_step'], d['latency_ms'])")"
done
