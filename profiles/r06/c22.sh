#!/bin/bash
# c22: runtime-option sweep of the default config on the current build (after the tone-run change, which showed that
# what runs next to the light passes matters): defaults, merge=1, lds_scene=2, fused_w4=0, gbuffer_pipeline=0,
# tail_pipeline=0, direct staging off (lds_scene=0), two rounds.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for rep in 1 2; do
  bash tools/knob_sweep.sh r06c22_$rep cornell-1080p-nee - HK_BENCH_OPTS=merge=1 HK_BENCH_OPTS=lds_scene=2 \
      HK_BENCH_OPTS=fused_w4=0 HK_BENCH_OPTS=gbuffer_pipeline=0 HK_BENCH_OPTS=tail_pipeline=0 HK_BENCH_OPTS=lds_scene=0
done
echo c22-done
