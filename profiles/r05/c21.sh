#!/bin/bash
# c21: frame pipelining (G-buffer of frame f+1 next to frame f's light passes) on the bands of scene / city, whose
# per-rank bands fall under pipeline_min_px (1.2e6) from N = 2 (scene) / 8 (city): default vs pipeline_min_px=0.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05/c21; mkdir -p $O
for n in 2 4 8; do
  for o in "" pipeline_min_px=0; do
    timeout -k 10 300 python tools/band_scaling.py scene-1080p-full 30 --only $n --balance 3 --kernels --opts "$o" > $O/scene_n${n}_$o.log 2>&1
    echo "scene N=$n [$o] $(grep -o 'slowest band [0-9.]*' $O/scene_n${n}_$o.log)"
  done
done
for o in "" pipeline_min_px=0; do
  timeout -k 10 400 python tools/band_scaling.py city-4k 20 --only 8 --balance 3 --opts "$o" > $O/city_n8_$o.log 2>&1
  echo "city N=8 [$o] $(grep -o 'slowest band [0-9.]*' $O/city_n8_$o.log)"
done
echo c21-done
