#!/bin/bash
# c25: the cornell 2- and 4-way stripes (one-GPU band projection) with frame pipelining below the default 1.2 Mpx
# threshold (pipeline_min_px = 4e5 / 9e5): the 2-way stripe (1.04 Mpx) runs unpipelined by default.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c25; mkdir -p $O
for rep in 1 2; do
  for n in 2 4; do
    for opt in default pipeline_min_px=9e5 pipeline_min_px=4e5; do
      a=""; [ $opt != default ] && a="--opts $opt"
      timeout -k 10 200 python tools/band_scaling.py cornell-1080p-nee 50 --only $n --balance 0 $a > $O/b_${n}_${opt}_$rep.log 2>&1
      echo "N=$n $opt rep $rep: $(grep slowest $O/b_${n}_${opt}_$rep.log | cut -c1-40)"
    done
  done
done
echo c25-done
