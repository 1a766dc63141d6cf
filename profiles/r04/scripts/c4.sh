#!/bin/bash
# Round-4 GPU call: where the collective path's cost at world size 1 goes (cornell 1080p: the band copy, the
# all-gather, the stripe reorder, the hardware-queue count), a kernel trace of that run, and the balanced
# city 4K band projection with 3 calibration rounds.  usage (GPU box): bash profiles/r04/scripts/c4.sh <tag>
set -e
TAG=${1:-c4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$TAG
mkdir -p $OUT
TESTS="tests/test_gpu_runtime.py -m gpu" bash tools/check_run.sh $TAG cornell:cornell-1080p-nee \
    dist_full:cornell-1080p-nee::dist dist_copy:cornell-1080p-nee:HK_BENCH_COMM=copy:dist \
    dist_noreorder:cornell-1080p-nee:HK_BENCH_COMM=noreorder:dist dist_none:cornell-1080p-nee:HK_BENCH_COMM=none:dist \
    dist_q8:cornell-1080p-nee:GPU_MAX_HW_QUEUES=8:dist cornell_q8:cornell-1080p-nee:GPU_MAX_HW_QUEUES=8 \
    city:city-4k city_dist:city-4k::dist
(cd /tmp && export TMPDIR=/tmp && RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29641 HK_BENCH_DIST=1 \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace_dist -o run -- \
  python $R/bench.py --steps 30 --warmup 5 --cpu-budget 0 > $R/$OUT/trace_dist.log 2>&1)
echo trace-ok
timeout -k 10 600 python -u tools/band_scaling.py city-4k 30 > $OUT/bands_city-4k.log 2>&1
tail -4 $OUT/bands_city-4k.log
echo c4-done
