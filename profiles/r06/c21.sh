#!/bin/bash
# c21: config 5's wavefront pass with the queued pixels' texels loaded before anything else in k_wf_trace / k_wf_shade
# — the GPU parity suite, then config 5 (city 4K 16 spp) A/B: prev (committed), new (in-tree), seg256 (new + 256 queue
# segments instead of 64: a quarter of the same-address atomics per counter in k_wf_gen / k_wf_trace / k_wf_scatter),
# mega (in-tree, megakernel indirect pass), 2 rounds.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c21; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=2 CONFIG=city-4k-16spp STEPS=2 bash tools/ab.sh r06c21 prev:exp_lib/libhk_prev.so new:- seg256:exp_lib/libhk_seg256.so mega:-:HK_BENCH_WAVEFRONT=0
echo c21-done
