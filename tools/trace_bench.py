"""Throughput of the stand-alone reference-order ray query (hk_trace, k_trace) on device-resident
rays: how much of an integrator kernel's time is the walk itself.  usage: python tools/trace_bench.py [scene]"""
import sys
import time
from pathlib import Path

import torch  # noqa: F401  (import before the HIP library, see bench.py)

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "bevy-hikari_amd"))
import numpy as np  # noqa: E402

from hikari_amd import HikariRenderer, examples  # noqa: E402

scene_fn = sys.argv[1] if len(sys.argv) > 1 else "cornell"
scene, cam, lights = examples.SCENES[scene_fn]()
scene.build()
r = HikariRenderer(0)
r.set_noise()
r.upload_scene(scene)
n = 1920 * 1080
rng = np.random.default_rng(1)
lo, hi = (np.array([-0.9, 0.1, -0.9]), np.array([0.9, 1.9, 0.9])) if scene_fn == "cornell" else \
    (np.array([-20.0, 0.5, -20.0]), np.array([20.0, 10.0, 20.0]))
org = rng.uniform(lo, hi, (n, 3))
d = rng.normal(size=(n, 3))
d /= np.linalg.norm(d, axis=1, keepdims=True)
rays = torch.tensor(np.concatenate([org, d], axis=1).astype(np.float32), device="cuda")
hits = torch.empty((n, 5), dtype=torch.int32, device="cuda")
early = torch.full((n,), 65535.0, device="cuda")
L = r._L
for mode, e in (("closest", None), ("any-hit(early=65535)", early)):
    ep = e.data_ptr() if e is not None else None
    for _ in range(3):
        L.hk_trace(r.ctx, rays.data_ptr(), None, ep, None, n, hits.data_ptr(), 1, None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    K = 20
    for _ in range(K):
        L.hk_trace(r.ctx, rays.data_ptr(), None, ep, None, n, hits.data_ptr(), 1, None)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K
    print(f"{scene_fn} {mode}: {n} rays {dt * 1e3:.3f} ms  {n / dt / 1e6:.0f} Mrays/s")
r.close()
