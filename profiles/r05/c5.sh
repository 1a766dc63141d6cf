#!/bin/bash
# Round-5 GPU call 5: the a-trous levels on packed level planes (the 3 channels' RGB halves + instance in 24 B, 3
# staged loads per texel) — the whole GPU suite, bench lines against the round-start build (exp_lib/libhk_base.so),
# and rocprofv3 kernel statistics of serialised frames (pipelining and channel streams off: each kernel alone) for the
# per-level times.  usage (GPU box): bash profiles/r05/c5.sh <tag>
set -e
TAG=${1:-c5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
BASE=$R/exp_lib/libhk_base.so
OUT=$R/gpurun_out/$TAG
TESTS="tests -m gpu" bash tools/check_run.sh $TAG city:city-4k city_base:city-4k:HK_LIB=$BASE scene:scene-1080p-full \
    scene_base:scene-1080p-full:HK_LIB=$BASE cornell:cornell-1080p-nee cornell_base:cornell-1080p-nee:HK_LIB=$BASE
cd /tmp && export TMPDIR=/tmp
for cfg in city-4k scene-1080p-full; do
  HK_BENCH_OPTS="gbuffer_pipeline=0,tail_pipeline=0,channel_streams=0" timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $OUT/serial_$cfg -o run -- python $R/bench.py --config $cfg --steps 10 --warmup 3 --cpu-budget 0 \
    > $OUT/serial_$cfg.log 2>&1
done
cd $R
for f in $(find $OUT -name "run_kernel_stats.csv"); do echo $f; python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"  {r['Name'][:64]:64s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:9.1f} us")
PY
done
echo c5-done
