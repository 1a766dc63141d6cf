#!/bin/bash
# c17: k_light_merged with the texel preload in its direct role only (c16: both roles, stripes 1-2 % slower) — the
# GPU parity suite, then the cornell 2-, 4- and 8-way stripes against the committed build (one-GPU band projection,
# tools/band_scaling.py --only N), two rounds.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c17; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for n in 2 4 8; do
    HK_LIB=$PWD/exp_lib/libhk_prev.so timeout -k 10 200 python tools/band_scaling.py cornell-1080p-nee 50 --only $n --balance 0 > $O/bands_prev_${n}_$rep.log 2>&1
    timeout -k 10 200 python tools/band_scaling.py cornell-1080p-nee 50 --only $n --balance 0 > $O/bands_new_${n}_$rep.log 2>&1
    echo "N=$n rep $rep prev: $(grep slowest $O/bands_prev_${n}_$rep.log)"
    echo "N=$n rep $rep new:  $(grep slowest $O/bands_new_${n}_$rep.log)"
  done
done
echo c17-done
