#!/bin/bash
# c24: the cornell parity test at an odd size (63x47: partial tiles, the k_tone fallback), every LDS mode
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r06/c24; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "test_cornell_frames_bit_exact" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -15 $O/tests.log
