#!/bin/bash
# c5: (1) the short-timed-region transient: first_frame.py with and without hk_resize between repeats;
# (2) PC sampling (host trap) of the default workload with every kernel alone, for k_indirect's hot spots.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
O=gpurun_out/r06/c5; mkdir -p $O
timeout -k 10 120 python tools/first_frame.py 20 5 4 reset > $O/first_frame_reset.txt 2>&1
cat $O/first_frame_reset.txt
timeout -k 10 120 python tools/first_frame.py 20 30 3 > $O/first_frame_w30.txt 2>&1
cat $O/first_frame_w30.txt
cd /tmp && export TMPDIR=/tmp
HK_BENCH_OPTS=channel_streams=0,gbuffer_pipeline=0,tail_pipeline=0 timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled \
  --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 --kernel-trace --output-format csv \
  -d $R/$O/pcs -o run -- python $R/bench.py --steps 40 --warmup 3 --cpu-budget 0 > $R/$O/pcs.log 2>&1 && echo pcs-ok || echo pcs-failed
ls -la $R/$O/pcs 2>/dev/null | head
echo c5-done
