#!/bin/bash
# c18: cornell stripes with the G-buffer rendered every frame (bench.py's gbuffer_reuse = 0 at 1 spp; band_scaling
# used the library default, which skips it on a static camera): N = 1 / 8, option variants, kernel trace at N = 8.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05/c18; mkdir -p $O
for n in 1 8 4; do
  for o in "" pipeline_min_px=0 "pipeline_min_px=0,merge=1" "merge=0"; do
    timeout -k 10 120 python tools/band_scaling.py cornell-1080p-nee 200 --only $n --kernels --opts "$o" > $O/n${n}_$o.log 2>&1
    echo "N=$n [$o] $(grep -o 'slowest band [0-9.]*' $O/n${n}_$o.log) $(grep -o 'kernel ms: .*' $O/n${n}_$o.log)"
  done
done
for v in dfirst inter; do
  for n in 8 4 2; do
    env HK_LIB=$PWD/exp_lib/libhk_$v.so timeout -k 10 120 python tools/band_scaling.py cornell-1080p-nee 200 --only $n > $O/${v}_$n.log 2>&1
    echo "$v N=$n $(grep -o 'slowest band [0-9.]*' $O/${v}_$n.log)"
  done
done
timeout -k 10 120 python tools/band_scaling.py cornell-1080p-nee 200 --only 2 > $O/base_2.log 2>&1
echo "base N=2 $(grep -o 'slowest band [0-9.]*' $O/base_2.log)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace8 -o run -- python3 $GRAFT_REPO_ROOT/tools/band_scaling.py cornell-1080p-nee 100 --only 8 > $GRAFT_REPO_ROOT/$O/trace8.log 2>&1
echo c18-done
