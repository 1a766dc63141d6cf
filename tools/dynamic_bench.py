"""Cost of a dynamic-instance update (city.rs rotates its emissive sphere every frame,
city.rs:290-294): hk_update_instances on the GPU vs the host rebuild + upload it replaces."""
import sys
import time
from pathlib import Path

import torch  # noqa: F401  (import before the HIP library, see bench.py)

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "bevy-hikari_amd"))
import numpy as np  # noqa: E402

from hikari_amd import HikariRenderer, examples  # noqa: E402

scene_fn = sys.argv[1] if len(sys.argv) > 1 else "city"
scene, cam, lights = examples.SCENES[scene_fn]()
scene.build()
r = HikariRenderer(0)
r.set_noise()
r.upload_scene(scene)
models, aabbs = scene.instance_models(), scene.instance_local_aabbs()
K = 20
for _ in range(3):
    r.update_instances(models, aabbs)
t0 = time.perf_counter()
for k in range(K):
    models[-1, 12] += 0.001  # nudge the last instance
    r.update_instances(models, aabbs)
torch.cuda.synchronize()
gpu = (time.perf_counter() - t0) / K
t0 = time.perf_counter()
for k in range(3):
    scene.build()
    r.upload_scene(scene)
torch.cuda.synchronize()
host = (time.perf_counter() - t0) / 3
print(f"{scene_fn}: {len(scene.instances)} instances; hk_update_instances {gpu * 1e3:.2f} ms/update (incl. one "
      f"stream sync); host hks_build + hk_scene_upload {host * 1e3:.1f} ms")
r.close()
