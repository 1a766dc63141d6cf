#!/bin/bash
# A/B timing of experiment libraries and runtime settings, alternated over REPS rounds: bench.py's
# pipelined frame time, latency and the dominant kernel's roofline duration (isolated), plus every
# kernel's isolated time.
# usage (GPU box): REPS=2 CONFIG=cornell-1080p-nee bash tools/ab.sh <tag> name:lib[:VAR=val,VAR2=val] ...
#   lib: a library path under the repo (HK_LIB) or '-' for the in-tree build
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab_$TAG
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for spec in "$@"; do
    IFS=: read -r name lib envs <<< "$spec"
    ENVARGS=()
    [ -n "$envs" ] && IFS=',' read -ra ENVARGS <<< "$envs"
    [ "$lib" != "-" ] && ENVARGS+=("HK_LIB=$R/$lib")
    timeout -k 10 200 env "${ENVARGS[@]}" python -u $R/bench.py --config ${CONFIG:-cornell-1080p-nee} --steps ${STEPS:-60} \
        --warmup 10 --cpu-budget 0 > $OUT/${name}_$rep.json 2> $OUT/${name}_$rep.log
    python - $OUT/${name}_$rep.json $name <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d.get("roofline", {})
print(sys.argv[2], d["value"], d["ms_per_step"], d.get("latency_ms"), r.get("kernel"), r.get("duration_ms"),
      d.get("isolated_kernel_ms"))
PY
  done
done
