#!/bin/bash
# Round-5 GPU call 4: per-level times of the LDS-staged a-trous levels (rocprofv3 kernel statistics, city 4K and
# scene 1080p), and the levels computing their luminance denominators themselves (exp_lib/libhk_noden.so,
# -DHK_DN_DENOM=0: no denominator plane written by demodulation) against the default.  usage: bash profiles/r05/c4.sh <tag>
set -e
TAG=${1:-c4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
NODEN=$R/exp_lib/libhk_noden.so
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
bash tools/check_run.sh $TAG city:city-4k city_noden:city-4k:HK_LIB=$NODEN scene:scene-1080p-full \
    scene_noden:scene-1080p-full:HK_LIB=$NODEN city2:city-4k city_noden2:city-4k:HK_LIB=$NODEN
cd /tmp && export TMPDIR=/tmp
for cfg in city-4k scene-1080p-full; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$cfg -o run -- \
    python $R/bench.py --config $cfg --steps 10 --warmup 3 --cpu-budget 0 > $OUT/stats_$cfg.log 2>&1
done
cd $R
for f in $(find $OUT -name "*kernel_stats.csv"); do echo $f; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows:
    n=r['Name']
    if 'denoise' in n or 'demod' in n: print(n[:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"; done
echo c4-done
