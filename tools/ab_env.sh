#!/bin/bash
# A/B timing of runtime env settings, alternated: bench.py (pipelined frame time, latency and the
# dominant kernel's isolated time) per setting, REPS rounds.
# usage (GPU box): REPS=2 CONFIG=cornell-1080p-nee bash tools/ab_env.sh <tag> name=VAR=val,VAR2=val|- ...
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/abenv_$TAG
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for tl in "$@"; do
    name=${tl%%=*}; envs=${tl#*=}
    ENVARGS=()
    if [ "$envs" != "-" ]; then IFS=',' read -ra ENVARGS <<< "$envs"; fi
    timeout -k 10 150 env "${ENVARGS[@]}" python -u $R/bench.py --config ${CONFIG:-cornell-1080p-nee} --steps 60 --warmup 10 \
        --cpu-budget 0 > $OUT/${name}_$rep.json 2> $OUT/${name}_$rep.log
    python - $OUT/${name}_$rep.json $name <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d.get("roofline", {})
print(sys.argv[2], d["value"], d["ms_per_step"], d.get("latency_ms"), r.get("kernel"), r.get("avg_ms"), r.get("isolated_avg_ms"))
PY
  done
done
