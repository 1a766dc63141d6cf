#!/bin/bash
# c19: the G-buffer with scene + stack in LDS on small frames (gbuffer_lds_max_px, default 6e5): GPU suite, then
# cornell stripes N = 8 / 4 / 2 / 1 with the threshold at its default, 0 (off) and 1e12 (every frame).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05/c19; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for n in 8 4 2 1; do
  for o in "" gbuffer_lds_max_px=0 gbuffer_lds_max_px=1e12; do
    timeout -k 10 120 python tools/band_scaling.py cornell-1080p-nee 200 --only $n --kernels --opts "$o" > $O/n${n}_$o.log 2>&1
    echo "N=$n [$o] $(grep -o 'slowest band [0-9.]*' $O/n${n}_$o.log) $(grep -o 'kernel ms: .*' $O/n${n}_$o.log)"
  done
done
echo c19-done
