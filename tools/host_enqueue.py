"""Host enqueue rate vs GPU frame rate of bench.py's default loop (cornell 1080p NEE): the wall time of
enqueuing K frames (frame_inputs + hk_render_gbuffer + hk_render_frame + hk_tone_sum, no sync) against the
time until the GPU has finished them.  If the enqueue time approaches the total, the frame loop is host-bound.

usage (GPU box): python tools/host_enqueue.py [frames]"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "bevy-hikari_amd"))
import torch  # noqa: E402

from hikari_amd import HikariRenderer, HikariSettings, Upscale, Taa, examples, frame_inputs  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
scene, cam, lights = examples.cornell()
st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, taa=Taa.None_, indirect_spatial_reuse=False, denoise=False)
s = st.to_c()
r = HikariRenderer(0)
r.set_noise()
r.upload_scene(scene)
r.resize(1920, 1080, 1.0)
sp = torch.cuda.current_stream().cuda_stream
for f in range(20):
    fi = frame_inputs(f, cam, lights, 1920, 1080)
    r.render_gbuffer(fi, sp)
    r.render_frame(s, fi, sp)
    r.tone_sum(s, sp)
torch.cuda.synchronize()
t0 = time.perf_counter()
t_fi = 0.0
for f in range(20, 20 + K):
    a = time.perf_counter()
    fi = frame_inputs(f, cam, lights, 1920, 1080)
    t_fi += time.perf_counter() - a
    r.render_gbuffer(fi, sp)
    r.render_frame(s, fi, sp)
    r.tone_sum(s, sp)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"frames {K}: enqueue {1e3 * (t1 - t0) / K:.4f} ms/frame (frame_inputs {1e3 * t_fi / K:.4f}), "
      f"total {1e3 * (t2 - t0) / K:.4f} ms/frame")
r.close()
