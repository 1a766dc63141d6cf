"""Host side of a short timed region (the driver's bench command: 20 steps after 5 warm-up frames): how long each
frame's enqueue takes on the host (frame_inputs + hk_render_gbuffer + hk_render_frame + hk_tone_sum, no sync) after the
device sync that opens the timed region, and when the GPU finishes each frame (a HIP event on the frame stream after
the frame's calls), relative to t0.

usage (GPU box): python tools/first_frame.py [steps] [warmup] [repeats] [reset]
reset: every repeat after the first starts from hk_resize (reservoirs zero-filled, frame numbers from 0 again: the
ReSTIR history restarts as at the start of the process) — separates a transient of the workload (ReSTIR history
filling) from one of the process / GPU (clocks, first launches)."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "bevy-hikari_amd"))
import torch  # noqa: E402

from hikari_amd import HikariRenderer, HikariSettings, Taa, Upscale, examples, frame_inputs  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
Wm = int(sys.argv[2]) if len(sys.argv) > 2 else 5
REP = int(sys.argv[3]) if len(sys.argv) > 3 else 3
RESET = len(sys.argv) > 4 and sys.argv[4] == "reset"
r = HikariRenderer(0)
scene, cam, lights = examples.cornell()
st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, taa=Taa.None_, indirect_spatial_reuse=False, denoise=False)
s = st.to_c()
r.set_options({"gbuffer_reuse": 0})
r.set_noise()
r.upload_scene(scene)
r.resize(1920, 1080, 1.0)
stream = torch.cuda.current_stream()
sp = stream.cuda_stream


def step(f):
    fi = frame_inputs(f, cam, lights, 1920, 1080)
    r.render_gbuffer(fi, sp)
    r.render_frame(s, fi, sp)
    r.tone_sum(s, sp)


f = 0
for rep in range(REP):
    if RESET and rep > 0:
        torch.cuda.synchronize()
        r.resize(1920, 1080, 1.0)
        f = 0
    for _ in range(Wm):
        step(f)
        f += 1
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(K)]
    host = []
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(K):
        step(f)
        f += 1
        host.append(time.perf_counter() - t0)
        evs[k].record(stream)
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    gpu = [ev0.elapsed_time(e) for e in evs]
    print(f"rep {rep}: total {total * 1e3:.4f} ms ({total / K * 1e3:.4f} ms/frame); host enqueue done (ms): "
          + " ".join(f"{h * 1e3:.3f}" for h in host[:4]) + f" ... {host[-1] * 1e3:.3f}")
    print("   frame-stream events (ms from t0): " + " ".join(f"{g:.3f}" for g in gpu[:4]) + f" ... {gpu[-1]:.3f}; "
          f"steady {((gpu[-1] - gpu[4]) / (K - 5)):.4f} ms/frame")
