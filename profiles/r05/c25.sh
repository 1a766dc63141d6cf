#!/bin/bash
# c25: spatial reuse with the neighbour's view plane 0 gathered before the march (default build) and with all three
# view planes gathered there (exp_lib/libhk_p012.so), against the previous commit (exp_lib/libhk_prev.so): spatial
# parity tests, bench lines of scene / city alternated (isolated spatial-reuse times in the lines).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$PWD
O=gpurun_out/r05/c25; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in new prev p012; do
    L=""; [ $v != new ] && L="HK_LIB=$R/exp_lib/libhk_$v.so"
    for c in city-4k scene-1080p-full; do
      env $L timeout -k 10 300 python bench.py --config $c --steps 30 --warmup 5 --cpu-budget 0 > $O/${v}_${c}_$rep.json 2> $O/${v}_${c}_$rep.err
      python3 -c "
import json; d=json.load(open('$O/${v}_${c}_$rep.json')); k=d.get('isolated_kernel_ms') or {}
print('$v $c $rep', d['ms_per_step'], k.get('indirect_spatial_reuse'), k.get('indirect_lit_ambient'))"
    done
  done
done
echo c25-done
