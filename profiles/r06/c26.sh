#!/bin/bash
# c26: the cornell 2-, 4- and 8-way stripes with the G-buffer pipelined next to the merged light kernel
# (pipeline_min_px = 1e5 with merge = 1; with and without the tail pipeline) against the default (unpipelined, merged)
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c26; mkdir -p $O
for rep in 1 2; do
  for n in 2 4 8; do
    for opt in default pipeline_min_px=1e5+merge=1 pipeline_min_px=1e5+merge=1+tail_pipeline=0; do
      a=""; [ $opt != default ] && a="--opts $(echo $opt | tr '+' ',')"
      timeout -k 10 200 python tools/band_scaling.py cornell-1080p-nee 50 --only $n --balance 0 $a > $O/b_${n}_${opt}_$rep.log 2>&1
      echo "N=$n $opt rep $rep: $(grep slowest $O/b_${n}_${opt}_$rep.log | cut -c1-40)"
    done
  done
done
echo c26-done
