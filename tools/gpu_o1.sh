set -e
mkdir -p gpurun_out/o1
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_motion.py -x -q --timeout 300 --timeout-method thread -k "full_size or cornell_frames or golden or proxy or textured or forced or moving_camera_bit" > gpurun_out/o1/tests.log 2>&1 || { tail -30 gpurun_out/o1/tests.log; exit 1; }
tail -2 gpurun_out/o1/tests.log
for v in 0 1; do
  if [ $v = 1 ]; then E="HK_NO_FUSED_W4=1"; else E=""; fi
  env $E timeout -k 10 200 python bench.py --cpu-budget 0 > gpurun_out/o1/bench_w4off$v.json
  python -c "import json;d=json.load(open('gpurun_out/o1/bench_w4off$v.json'));print('w4off=$v', d['value'], d['ms_per_step'], d['latency_ms'], d['roofline']['avg_ms'], d['roofline']['isolated_avg_ms'])"
done
for cfg in scene-1080p-full city-4k; do
  HK_CHANNEL_STREAMS=0 HK_GB_PIPELINE=0 HK_DN_PIPELINE=0 timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 4 --cpu-budget 0 > gpurun_out/o1/serial_$cfg.json
  python -c "import json;d=json.load(open('gpurun_out/o1/serial_$cfg.json'));print('$cfg', d['ms_per_step'], d['kernel_ms'])"
done
