#!/bin/bash
# c30: exact reciprocal rewrites (1 / sqrt in spatial reuse's march, 1 / depth_ratio, -1 / (s + n.z), 1 / count by
# rcp_exact; shade's 0.5 / (lambdaV + lambdaL) by half_over, checked on all 2^32 inputs) against the previous commit
# (exp_lib/libhk_prev.so): the GPU suite, bench lines alternated.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$PWD
O=gpurun_out/r05/c30; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in new prev; do
    L=""; [ $v != new ] && L="HK_LIB=$R/exp_lib/libhk_$v.so"
    for c in cornell-1080p-nee scene-1080p-full city-4k; do
      env $L timeout -k 10 300 python bench.py --config $c --steps 40 --warmup 8 --cpu-budget 0 > $O/${v}_${c}_$rep.json 2> $O/${v}_${c}_$rep.err
      python3 -c "
import json; d=json.load(open('$O/${v}_${c}_$rep.json')); k=d.get('isolated_kernel_ms') or {}
print('$v $c $rep', d['ms_per_step'], {a: round(b, 4) for a, b in k.items() if a in ('direct_lit_emissive', 'indirect_lit_ambient', 'indirect_spatial_reuse')})"
    done
  done
done
echo c30-done
