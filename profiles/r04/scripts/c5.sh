#!/bin/bash
# Round-4 GPU call: the collective path at world size 1 after the row-copy reassembly (cornell stripes,
# scene / city bands), against the single-GPU lines on the same box; 2-rank rehearsals (gloo, one GPU) of the
# stripe and balanced-band paths.  usage (GPU box): bash profiles/r04/scripts/c5.sh <tag>
set -e
TAG=${1:-c5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash tools/check_run.sh $TAG cornell:cornell-1080p-nee cornell_dist:cornell-1080p-nee::dist \
    scene:scene-1080p-full scene_dist:scene-1080p-full::dist city:city-4k city_dist:city-4k::dist \
    cornell2:cornell-1080p-nee cornell_dist2:cornell-1080p-nee::dist
for cfg in cornell-1080p-nee city-4k; do
  HK_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29565 bench.py --gpus 2 --config $cfg --steps 5 --warmup 3 --cpu-budget 0 \
      > $OUT/rehearsal_$cfg.json 2> $OUT/rehearsal_$cfg.err
  python -c "import json;d=json.load(open('$OUT/rehearsal_$cfg.json'));print('rehearsal $cfg', d['value'], d['config']['parallelism'], d['config']['band_bounds'])"
done
echo c5-done
