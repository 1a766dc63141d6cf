"""The G-buffer's ordered primary walk selects the surfaces the reference-order walk selects (CPU).

The reference rasterises its G-buffer (prepass.wgsl:84-100); this build traces one primary ray per
pixel with an ordered closest-hit walk (nearer child first), which is the one rule
the build defines itself.  Here every primary ray of 1920x1080 frames — static, TAA-jittered
(prepass.wgsl:30-38) and orbiting cameras — is walked both ways by the oracle
(`hko_primary_hits`): the ordered walk and light.wgsl's reference-order `traverse_top` closest
hit (light.wgsl:400-486, no early exit).  Instance id, primitive id and hit distance must be
identical for every pixel.  The GPU's ordered walk equals the oracle's bit for bit
(test_gpu_parity.py::test_gbuffer_ordered_traversal_matches_oracle), so this closes the chain.
"""
import math

import numpy as np
import pytest

W, H = 1920, 1080


def _cameras(cam):
    from hikari_amd import Camera, Transform
    yield 0, cam, 0
    yield 3, cam, 1  # HK_JITTER_TAA
    t = np.asarray(cam.transform.translation, np.float64)
    r = math.hypot(t[0], t[2])
    for k, a in enumerate((0.15, -0.3)):
        p = (r * math.sin(a), float(t[1]) + 0.2 * k, r * math.cos(a))
        yield 5 + k, Camera(Transform.from_xyz(*p).looking_at((0.0, float(t[1]) * 0.5, 0.0))), 2  # TAA_SMAA


@pytest.mark.parametrize("scene_fn", ["cornell", "scene", "city"])
def test_ordered_primary_walk_matches_reference_order(scene_fn):
    from hikari_amd import examples, frame_inputs, load_noise
    from oracle import Oracle
    scene, cam, lights = examples.SCENES[scene_fn]()
    o = Oracle(scene.build(), load_noise(), W, H, 1.0)
    for f, c, jitter in _cameras(cam):
        hits = o.primary_hits(frame_inputs(f, c, lights, W, H, jitter=jitter))
        ordered, reference = hits[:, :, 0], hits[:, :, 1]
        covered = float((reference[..., 0] != 0xFFFFFFFF).mean())
        assert covered > 0.2, (scene_fn, f, covered)
        bad = np.argwhere((ordered != reference).any(-1))
        assert len(bad) == 0, (scene_fn, f, len(bad), bad[:3].tolist())
