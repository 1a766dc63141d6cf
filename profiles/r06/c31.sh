#!/bin/bash
# c31: demodulation as rows of pixels without LDS (k_demod_run, exp_lib/libhk_demodrun.so) — its parity (the cornell
# frames incl. 256x256 with the denoiser, the full-size scene / city workloads) through HK_LIB, then A/B against the
# product on scene and city (2 rounds each).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c31; mkdir -p $O
HK_LIB=$PWD/exp_lib/libhk_demodrun.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "cornell_frames or full_size" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=2 CONFIG=scene-1080p-full STEPS=30 bash tools/ab.sh r06c31s prev:- demodrun:exp_lib/libhk_demodrun.so
REPS=2 CONFIG=city-4k STEPS=20 bash tools/ab.sh r06c31c prev:- demodrun:exp_lib/libhk_demodrun.so
echo c31-done
