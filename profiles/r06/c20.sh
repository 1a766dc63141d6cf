#!/bin/bash
# c20: the GPU parity suite on the in-tree build (tone runs of 2 pixels), then config 5 (city 4K 16 spp, wavefront
# indirect) under rocprofv3: kernel statistics, and the HBM traffic passes (FETCH_SIZE, WRITE_SIZE) of its kernels.
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$PWD
O=gpurun_out/r06/c20; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/stats -o run -- \
    python $R/bench.py --config city-4k-16spp --steps 1 --warmup 1 --cpu-budget 0 > $R/$O/stats.log 2>&1
echo stats-ok
for group in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $group --output-format csv -d $R/$O/pmc/$group -o run -- \
      python $R/bench.py --config city-4k-16spp --steps 1 --warmup 1 --cpu-budget 0 > $R/$O/pmc_$group.log 2>&1
  echo "$group ok"
done
echo c20-done
