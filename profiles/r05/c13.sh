#!/bin/bash
# Round-5 GPU call 13: demodulation staging its variance taps in LDS (default build) against the previous commit (exp_lib/libhk_prev.so): parity suites, bench lines alternated, and
# serialised per-level times (rocprofv3).  usage (GPU box): bash profiles/r05/c13.sh <tag>
set -e
TAG=${1:-c13}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
PREV=$R/exp_lib/libhk_prev.so
OUT=$R/gpurun_out/$TAG
TESTS="tests/test_gpu_parity.py tests/test_gpu_motion.py -m gpu" bash tools/check_run.sh $TAG city:city-4k \
    city_prev:city-4k:HK_LIB=$PREV scene:scene-1080p-full scene_prev:scene-1080p-full:HK_LIB=$PREV \
    city2:city-4k city_prev2:city-4k:HK_LIB=$PREV
cd /tmp && export TMPDIR=/tmp
HK_BENCH_OPTS="gbuffer_pipeline=0,tail_pipeline=0,channel_streams=0" timeout -k 10 300 rocprofv3 --kernel-trace --stats \
  --output-format csv -d $OUT/serial_city -o run -- python $R/bench.py --config city-4k --steps 10 --warmup 3 --cpu-budget 0 \
  > $OUT/serial_city.log 2>&1
cd $R
python3 - $OUT/serial_city/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "denoise" in r["Name"] or "demod" in r["Name"]:
        print(f"  {r['Name'][:64]:64s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:9.1f} us")
PY
echo c13-done
