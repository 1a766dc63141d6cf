#!/bin/bash
# Round-4 GPU call: runtime tests, the default lines against this round's variants, the experiment libraries
# (spatial reuse: view plane 0 staged in LDS, view planes as one line per pixel), the balanced-band
# projection of city 4K and a 2-rank rehearsal of its balanced bands.  usage (GPU box): bash profiles/r04/scripts/c3.sh <tag>
set -e
TAG=${1:-c3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$TAG
mkdir -p $OUT
P0=HK_LIB=$R/exp_lib/libhk_p0win.so
AOS=HK_LIB=$R/exp_lib/libhk_viewaos.so
env $P0 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "scene-1080p or row_bands_match or spatial_reuse_without" > $OUT/tests_p0win.log 2>&1 || { tail -30 $OUT/tests_p0win.log; exit 1; }
tail -1 $OUT/tests_p0win.log
TESTS="tests/test_gpu_runtime.py -m gpu" bash tools/check_run.sh $TAG cornell:cornell-1080p-nee \
    cornell_cw:cornell-1080p-nee:HK_BENCH_OPTS=compact_emitter=1 cornell_dist:cornell-1080p-nee::dist \
    scene:scene-1080p-full scene_dist:scene-1080p-full::dist scene_p0:scene-1080p-full:$P0 scene_aos:scene-1080p-full:$AOS \
    city:city-4k city_p0:city-4k:$P0 city_aos:city-4k:$AOS
timeout -k 10 600 python -u tools/band_scaling.py city-4k 30 > $OUT/bands_city-4k.log 2>&1
tail -5 $OUT/bands_city-4k.log
HK_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --config city-4k --steps 5 --warmup 3 --cpu-budget 0 \
    > $OUT/rehearsal_city.json 2> $OUT/rehearsal_city.err
python -c "import json;d=json.load(open('$OUT/rehearsal_city.json'));print('rehearsal', d['config']['band_bounds'], d['config']['band_calibration'])"
echo c3-done
