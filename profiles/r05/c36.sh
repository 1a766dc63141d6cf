#!/bin/bash
# c36: k_light_merged's indirect role with the IndStash in the launch's dynamic LDS (after the staged scene, inside
# the park area's size on validation frames) against the previous commit: GPU suite, cornell stripes N = 2 / 4 / 8
# alternated.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$PWD
O=gpurun_out/r05/c36; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for n in 8 4 2; do
    for v in new prev; do
      L=""; [ $v != new ] && L="HK_LIB=$R/exp_lib/libhk_$v.so"
      env $L timeout -k 10 120 python tools/band_scaling.py cornell-1080p-nee 200 --only $n > $O/bands_${v}_${n}_$rep.log 2>&1
      echo "$v N=$n rep $rep $(grep -o 'slowest band [0-9.]*' $O/bands_${v}_${n}_$rep.log)"
    done
  done
done
echo c36-done
