#!/bin/bash
# c26: the indirect pass keeping the pixel's G-buffer / noise fields in an LDS slot through its walks (default build;
# its tail reads them from LDS instead of global memory) against the previous commit (exp_lib/libhk_prev.so): the
# GPU suite, then bench lines alternated (cornell default, scene, city; isolated k_indirect in the lines).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$PWD
O=gpurun_out/r05/c26; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in new prev; do
    L=""; [ $v != new ] && L="HK_LIB=$R/exp_lib/libhk_$v.so"
    for c in cornell-1080p-nee city-4k scene-1080p-full; do
      env $L timeout -k 10 300 python bench.py --config $c --steps 60 --warmup 10 --cpu-budget 0 > $O/${v}_${c}_$rep.json 2> $O/${v}_${c}_$rep.err
      python3 -c "
import json; d=json.load(open('$O/${v}_${c}_$rep.json')); k=d.get('isolated_kernel_ms') or {}
print('$v $c $rep', d['ms_per_step'], d['value'], k.get('indirect_lit_ambient'), k.get('direct_lit_emissive'))"
    done
  done
done
for n in 8 4; do
  for v in new prev; do
    L=""; [ $v != new ] && L="HK_LIB=$R/exp_lib/libhk_$v.so"
    env $L timeout -k 10 120 python tools/band_scaling.py cornell-1080p-nee 200 --only $n > $O/bands_${v}_$n.log 2>&1
    echo "$v N=$n $(grep -o 'slowest band [0-9.]*' $O/bands_${v}_$n.log)"
  done
done
echo c26-done
