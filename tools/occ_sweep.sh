# Occupancy sweep of the traversal kernels: rebuild with forced waves/SIMD, bench two configs.
set -e
run() {  # tag, EXTRA flags
  make -s -C bevy-hikari_amd -B -j16 EXTRA="$2" > /dev/null 2>&1
  timeout -k 10 100 python bench.py --steps 30 --warmup 5 --cpu-budget 0 > gpurun_out/occ_c_$1.log 2>&1
  timeout -k 10 150 python bench.py --config scene-1080p-full --steps 20 --warmup 3 --cpu-budget 0 > gpurun_out/occ_s_$1.log 2>&1
  timeout -k 10 150 python bench.py --config city-4k --steps 10 --warmup 2 --cpu-budget 0 > gpurun_out/occ_k_$1.log 2>&1
}
run base ""
run d5i5 "-DHK_DIRECT_WAVES=5 -DHK_INDIRECT_WAVES=5"
run i5 "-DHK_INDIRECT_WAVES=5"
run d5 "-DHK_DIRECT_WAVES=5"
