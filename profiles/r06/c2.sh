#!/bin/bash
# c2: band window refill (hk_band_window_grow / hk_reservoir_rows) — the settings-toggle band test with and without
# the refill, then the whole GPU suite; a kernel trace of the driver's bench command (--steps 20 --warmup 5) for the
# timed region's fill / drain (tools/timed_span.py).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
O=gpurun_out/r06/c2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k settings_toggle -v --timeout 200 --timeout-method thread > $O/toggle.log 2>&1 || true
tail -5 $O/toggle.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
   -d $R/$O/trace -o run -- python $R/bench.py --gpus 1 --steps 20 --warmup 5 --cpu-budget 0 > $R/$O/trace_bench.json 2> $R/$O/trace_bench.err)
python tools/timed_span.py $(find $O/trace -name '*kernel_trace.csv' | head -1) 5 20 > $O/timed_span.txt
cat $O/timed_span.txt
echo c2-done
