"""Quick GPU timing probe (development aid): cornell at WxH, config-2 settings."""
import sys, time
sys.path.insert(0, 'bevy-hikari_amd')
import numpy as np
from hikari_amd import HikariRenderer, HikariSettings, Upscale, examples, frame_inputs

W, H = int(sys.argv[1]) if len(sys.argv) > 1 else 1920, int(sys.argv[2]) if len(sys.argv) > 2 else 1080
scene, cam, lights = examples.cornell()
scene.build()
st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=False, denoise=False)
s = st.to_c()
r = HikariRenderer(0); r.set_noise(); r.upload_scene(scene); r.resize(W, H, 1.0)
fi0 = frame_inputs(0, cam, lights, W, H)
r.render_gbuffer(fi0)
r.enable_kernel_timing(True)
for f in range(20):
    fi = frame_inputs(f, cam, lights, W, H)
    r.render_frame(s, fi)
r.output(10)
print(r.kernel_timing())
r.enable_kernel_timing(False)
r.reset_counters()
t = time.time()
N = 30
for f in range(20, 20 + N):
    fi = frame_inputs(f, cam, lights, W, H)
    r.render_frame(s, fi)
r.output(10)
dt = (time.time() - t) / N
c = r.counters()
rays = (c['traverse_top'] + c['traverse_emitter']) / N
print(f"{W}x{H}: {dt*1e3:.3f} ms/frame, {rays/1e6:.2f} Mrays/frame, {rays/dt/1e6:.1f} Mrays/s", c)
