#!/bin/bash
# c27: the LDS stash in k_indirect only (k_light_merged without it): the GPU suite, cornell stripes N = 8 / 4 against
# the previous commit, default line.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$PWD
O=gpurun_out/r05/c27; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for n in 8 4; do
  for v in new prev; do
    L=""; [ $v != new ] && L="HK_LIB=$R/exp_lib/libhk_$v.so"
    env $L timeout -k 10 120 python tools/band_scaling.py cornell-1080p-nee 200 --only $n > $O/bands_${v}_$n.log 2>&1
    echo "$v N=$n $(grep -o 'slowest band [0-9.]*' $O/bands_${v}_$n.log)"
  done
done
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
python3 -c "
import json; d=json.load(open('$O/bench_default.json')); print('default', d['ms_per_step'], d['value'], d['roofline']['duration_ms'], d['roofline']['frac'])"
echo c27-done
