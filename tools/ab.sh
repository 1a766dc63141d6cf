#!/bin/bash
# A/B timing of experiment libraries, alternated: bench.py's default config (pipelined frame time and
# the dominant kernel's isolated time) per library, REPS rounds.
# usage (GPU box): REPS=2 CONFIG=cornell-1080p-nee bash tools/ab.sh <tag> name=lib|- ...
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab_$TAG
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for tl in "$@"; do
    name=${tl%%=*}; lib=${tl#*=}
    if [ "$lib" = "-" ]; then unset HK_LIB; else export HK_LIB=$R/$lib; fi
    timeout -k 10 150 python -u $R/bench.py --config ${CONFIG:-cornell-1080p-nee} --steps 60 --warmup 10 --cpu-budget 0 \
        > $OUT/${name}_$rep.json 2> $OUT/${name}_$rep.log
    unset HK_LIB
    python - $OUT/${name}_$rep.json $name <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d.get("roofline", {})
print(sys.argv[2], d["value"], d["ms_per_step"], d.get("latency_ms"), r.get("kernel"), r.get("avg_ms"), r.get("isolated_avg_ms"))
PY
  done
done
