#!/bin/bash
# spatial-reuse cost breakdown: the scene 1080p and city 4K benches with experiment builds that skip
# parts of the neighbour loop (exp_sp/*.so, -DHK_EXPERIMENT_SP_*), all kernels serialised
set -e
OUT=gpurun_out/${1:-exp_sp}
mkdir -p $OUT
for lib in product exp_sp/NO_MARCH.so exp_sp/NO_SHADE.so exp_sp/BOTH.so; do
  n=$(basename $lib .so)
  for cfg in scene-1080p-full city-4k; do
    if [ $lib = product ]; then L=""; else L="HK_LIB=$lib"; fi
    env $L HK_CHANNEL_STREAMS=0 HK_GB_PIPELINE=0 HK_DN_PIPELINE=0 timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 4 --cpu-budget 0 > $OUT/${n}_$cfg.json
    echo "$n $cfg $(python -c "import json;d=json.load(open('$OUT/${n}_$cfg.json'));print(d['ms_per_step'], {k: v for k, v in d['kernel_ms'].items() if 'spatial' in k})")"
  done
done
