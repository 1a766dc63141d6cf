#!/bin/bash
# direct/emissive cost breakdown: serialised benches with experiment builds (exp_direct/*.so)
set -e
OUT=gpurun_out/${1:-exp_direct}
mkdir -p $OUT
for lib in product exp_direct/NO_SHADOW.so exp_direct/NO_EMITTER_TRAVERSE.so exp_direct/BOTH.so; do
  n=$(basename $lib .so)
  for cfg in cornell-1080p-nee city-4k; do
    if [ $lib = product ]; then L=""; else L="HK_LIB=$lib"; fi
    env $L HK_CHANNEL_STREAMS=0 HK_GB_PIPELINE=0 HK_DN_PIPELINE=0 timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 4 --cpu-budget 0 > $OUT/${n}_$cfg.json
    echo "$n $cfg $(python -c "import json;d=json.load(open('$OUT/${n}_$cfg.json'));print(d['ms_per_step'], {k: v for k, v in d['kernel_ms'].items() if 'direct' in k})")"
  done
done
