#!/bin/bash
# c16: the texel preload in the separate direct launches (k_direct, k_direct_lit_w4: moving camera, bands), the
# compacted fused kernel and both roles of k_light_merged (small stripes) — the GPU parity suite, then A/B against
# the committed build (exp_lib/libhk_prev.so): cornell and city orbiting cameras, and the cornell 4- and 8-way
# stripes (one-GPU band projection, tools/band_scaling.py --only N).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c16; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=2 CONFIG=cornell-1080p-nee-orbit STEPS=40 bash tools/ab.sh r06c16o prev:exp_lib/libhk_prev.so new:-
REPS=2 CONFIG=city-4k-orbit STEPS=20 bash tools/ab.sh r06c16co prev:exp_lib/libhk_prev.so new:-
for rep in 1 2; do
  for n in 4 8; do
    HK_LIB=$PWD/exp_lib/libhk_prev.so timeout -k 10 200 python tools/band_scaling.py cornell-1080p-nee 50 --only $n --balance 0 > $O/bands_prev_${n}_$rep.log 2>&1
    timeout -k 10 200 python tools/band_scaling.py cornell-1080p-nee 50 --only $n --balance 0 > $O/bands_new_${n}_$rep.log 2>&1
    echo "N=$n rep $rep prev: $(grep slowest $O/bands_prev_${n}_$rep.log)"
    echo "N=$n rep $rep new:  $(grep slowest $O/bands_new_${n}_$rep.log)"
  done
done
echo c16-done
