#!/bin/bash
# c28: k_indirect gathering the previous record's head words before its walks (held in registers through them;
# 5 waves per SIMD forced: 96 VGPRs, 20-24 B of scratch) — default build — against the previous commit
# (exp_lib/libhk_prev.so: the LDS stash alone): parity suite, bench lines alternated.  Then c27.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$PWD
O=gpurun_out/r05/c28; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in new prev; do
    L=""; [ $v != new ] && L="HK_LIB=$R/exp_lib/libhk_$v.so"
    for c in cornell-1080p-nee city-4k scene-1080p-full; do
      env $L timeout -k 10 300 python bench.py --config $c --steps 60 --warmup 10 --cpu-budget 0 > $O/${v}_${c}_$rep.json 2> $O/${v}_${c}_$rep.err
      python3 -c "
import json; d=json.load(open('$O/${v}_${c}_$rep.json')); k=d.get('isolated_kernel_ms') or {}
print('$v $c $rep', d['ms_per_step'], d['value'], k.get('indirect_lit_ambient'))"
    done
  done
done
echo c28-done
