#!/bin/bash
# Round-5 GPU call 29: the a-trous weights from hk_exp_weight with a one-step scale (subnormal weights flushed to 0,
# no selects) against the previous commit (exp_lib/libhk_prev.so): the GPU suite, bench lines alternated, serialised
# per-level times (rocprofv3).
set -e
TAG=${1:-r05/c29}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
PREV=$R/exp_lib/libhk_prev.so
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
TESTS="tests -m gpu" bash tools/check_run.sh $TAG city:city-4k \
    city_prev:city-4k:HK_LIB=$PREV scene:scene-1080p-full scene_prev:scene-1080p-full:HK_LIB=$PREV \
    city2:city-4k city_prev2:city-4k:HK_LIB=$PREV scene2:scene-1080p-full scene_prev2:scene-1080p-full:HK_LIB=$PREV
cd /tmp && export TMPDIR=/tmp
for c in city-4k scene-1080p-full; do
  for v in new prev; do
    L=""; [ $v = prev ] && L="HK_LIB=$PREV"
    env $L HK_BENCH_OPTS="gbuffer_pipeline=0,tail_pipeline=0,channel_streams=0" timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d $OUT/serial_${c}_$v -o run -- python $R/bench.py --config $c --steps 10 --warmup 3 --cpu-budget 0 \
      > $OUT/serial_${c}_$v.log 2>&1
    echo "$c $v"
    python3 - $OUT/serial_${c}_$v/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "denoise" in r["Name"] or "demod" in r["Name"]:
        print(f"  {r['Name'][:64]:64s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:9.1f} us")
PY
  done
done
cd $R

echo c29-done
