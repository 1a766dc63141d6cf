#!/bin/bash
# c4: k_indirect's issue cost on cornell 1080p: PMC instruction counts per wave and the
# instruction-cache counters (every kernel alone: channel fork and frame pipelining off), the walk iterations per wave
# from the lane-stats build, and the host side of the driver's short timed region (tools/first_frame.py).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
O=gpurun_out/r06/c4; mkdir -p $O
timeout -k 10 120 python tools/first_frame.py 20 5 4 > $O/first_frame.txt 2>&1
cat $O/first_frame.txt
HK_LIB=exp_lanestats/lanestats.so timeout -k 10 300 python tools/lane_stats.py $O/lane_stats.json cornell-1080p-nee > $O/lane_stats.log 2>&1
tail -2 $O/lane_stats.log
cd /tmp && export TMPDIR=/tmp
export HK_BENCH_OPTS=channel_streams=0,gbuffer_pipeline=0,tail_pipeline=0
i=0
for group in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
  "SQ_WAVES SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY" \
  "SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $group --output-format csv -d $R/$O/pmc$i -o run -- \
    python $R/bench.py --steps 8 --warmup 2 --cpu-budget 0 > $R/$O/pmc$i.log 2>&1 && echo "pass $i ok" || echo "pass $i failed"
done
echo c4-done
