#!/bin/bash
# c31: where spatial reuse's time goes — timing-only experiment builds (wrong results, never shipped): the neighbour
# merge without `shade` (sp_noshade), without the depth march (sp_nomarch), with fixed offsets instead of sincos
# (sp_nosincos), against the committed build; isolated spatial-reuse times of scene 1080p and city 4K.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$PWD
O=gpurun_out/r05/c31; mkdir -p $O
for v in prev sp_noshade sp_nomarch sp_nosincos; do
  for c in scene-1080p-full city-4k; do
    HK_LIB=$R/exp_lib/libhk_$v.so timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --cpu-budget 0 > $O/${v}_${c}.json 2> $O/${v}_${c}.err
    python3 -c "
import json; d=json.load(open('$O/${v}_${c}.json')); k=d.get('isolated_kernel_ms') or {}
print('$v $c', k.get('indirect_spatial_reuse'))"
  done
done
echo c31-done
