#!/bin/bash
# Round-5 GPU call 11: config 5's wavefront indirect pass, kernel by kernel — rocprofv3 kernel statistics of
# serialised sub-frames (channel fork and pipelining off) of city 4K 16 spp with the wavefront pass and with the
# megakernel, and the two bench lines.  usage (GPU box): bash profiles/r05/c11.sh <tag>
set -e
TAG=${1:-c11}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
BENCH_ARGS='--steps 2 --warmup 1' bash tools/check_run.sh $TAG city16-wavefront:city-4k-16spp \
    city16-megakernel:city-4k-16spp:HK_BENCH_WAVEFRONT=0
cd /tmp && export TMPDIR=/tmp
for mode in 1 0; do
  HK_BENCH_WAVEFRONT=$mode HK_BENCH_OPTS="gbuffer_pipeline=0,tail_pipeline=0,channel_streams=0" timeout -k 10 300 \
    rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/serial_wf$mode -o run -- \
    python $R/bench.py --config city-4k-16spp --steps 1 --warmup 1 --cpu-budget 0 > $OUT/serial_wf$mode.log 2>&1
done
cd $R
for f in $(find $OUT -name "run_kernel_stats.csv"); do echo $f; python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"  {r['Name'][:64]:64s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:9.1f} us  total {float(r['TotalDurationNs']) / 1e6:8.2f} ms")
PY
done
echo c11-done
