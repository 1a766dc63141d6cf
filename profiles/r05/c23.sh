#!/bin/bash
# c23: GPU suite with the serial-heavy and schedule-switch parity tests.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r05/c23; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "pipelining or schedule" > $O/new_tests.log 2>&1 || { tail -40 $O/new_tests.log; exit 1; }
grep -E "PASS|FAIL" $O/new_tests.log | tail -6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
