#!/bin/bash
# One GPU call: the GPU suite (optional), then bench lines single-GPU and through the RCCL path at world
# size 1.  usage (GPU box): TESTS="<pytest args>|" bash tools/check_run.sh <tag> name:config[:ENV=V+ENV2=V2][:dist] ...
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
port=29600
for spec in "$@"; do
  IFS=: read -r name cfg envs mode <<< "$spec"
  ENVARGS=()
  [ -n "$envs" ] && IFS='+' read -ra ENVARGS <<< "$envs"
  port=$((port+1))
  if [ "$mode" = "dist" ]; then
    timeout -k 10 300 env "${ENVARGS[@]}" HK_BENCH_DIST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $port bench.py --config $cfg --cpu-budget 0 $BENCH_ARGS \
      > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail -20 $OUT/bench_$name.err; exit 1; }
  else
    timeout -k 10 300 env "${ENVARGS[@]}" python bench.py --config $cfg --cpu-budget 0 $BENCH_ARGS \
      > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail -20 $OUT/bench_$name.err; exit 1; }
  fi
  python - $OUT/bench_$name.json $name <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d.get("roofline", {})
print(sys.argv[2], d["value"], d["ms_per_step"], d.get("latency_ms"), r.get("kernel"), r.get("frac"), r.get("duration_ms"),
      {k: round(v, 3) for k, v in (d.get("isolated_kernel_ms") or d.get("kernel_ms") or {}).items()})
PY
done
echo done
