#!/bin/bash
# c16: k_light_merged variants on the cornell 4- and 8-way stripe frames (alternated, 2 reps):
#   base, w5 (waves_per_eu 5: 96 VGPRs + spills), dfirst (direct workgroups dispatched first), inter (even/odd interleave)
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05/c16; mkdir -p $O
for rep in 1 2; do
  for v in base w5 dfirst inter; do
    L=""; [ $v != base ] && L="HK_LIB=$PWD/exp_lib/libhk_$v.so"
    for n in 8 4; do
      env $L timeout -k 10 120 python tools/band_scaling.py cornell-1080p-nee 200 --only $n > $O/${v}_${n}_$rep.log 2>&1
      echo "$v N=$n rep $rep: $(grep -o 'slowest band [0-9.]*' $O/${v}_${n}_$rep.log)"
    done
  done
done
