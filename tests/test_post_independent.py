"""SMAA TU4x + TAA Jasmine pinned by an independent restatement (CPU).

include/hk_post.h holds the per-pixel post-process code that both the oracle and the GPU kernels
compile (test_gpu_parity.py::test_post_process_smaa_taa_bit_exact shows GPU == oracle), so that
comparison alone cannot catch a misreading of smaa.wgsl / taa.wgsl made in the header.  Here the
oracle's outputs are compared with tests/post_numpy.py, a vectorised float32 restatement written
from the WGSL and the WGSL texture rules, fed the same frame data (a moving camera, so reprojection,
the clipping branches and the extrapolation all run).  Tolerance: >= 99.5 % of output texels
bit-identical and every texel within 2e-3 (the restatement takes cos from numpy, the oracle from
include/hk_math.h; everything else is the same IEEE float32 arithmetic).
"""
import copy

import numpy as np
import pytest

import post_numpy as pn


def _f16(raw):
    return raw.view(np.float16).astype(np.float32)


def _close(got, want_f32, label):
    want = want_f32.astype(np.float16)
    a, b = got.view(np.uint16), want.view(np.uint16)
    exact = float((a == b).all(axis=-1).mean())
    diff = float(np.abs(got.view(np.float16).astype(np.float32) - want.astype(np.float32)).max())
    assert exact >= 0.995 and diff <= 2e-3, f"{label}: {exact:.4f} of texels exact, max |diff| {diff}"


@pytest.mark.parametrize("ratio_setting", ["SMAA_TU_2_0", "SMAA_TU_1_0"])
def test_smaa_taa_match_independent_restatement(ratio_setting):
    from hikari_amd import Camera, HikariSettings, Taa, Transform, Upscale, examples, frame_inputs, load_noise
    from oracle import Oracle
    W, H = 33, 21
    st = HikariSettings(upscale=getattr(Upscale, ratio_setting), taa=Taa.Jasmine)
    scene, cam, lights = examples.cornell()
    o = Oracle(scene.build(), load_noise(), W, H, st.upscale.ratio(), threads=4)
    s = st.to_c()
    prev, prev_cam = None, None
    t0 = cam.transform.translation
    for f in range(5):
        c = Camera(Transform.from_xyz(float(t0[0]) + 0.03 * f, float(t0[1]), float(t0[2]) - 0.05 * f)
                   .looking_at((0.0, 1.0, 0.0)))
        fi = frame_inputs(f, c, lights, W, H, previous_camera=prev_cam)
        prev_cam = copy.deepcopy(c)
        o.render_gbuffer(fi)
        o.render_frame(s, fi)
        o.denoise(s, fi)
        o.tone_sum(s)
        o.post_process(s, fi)
        cur = {k: o.output(k) for k in (10, 11, 14, 15, 18, 19)}
        if prev is not None:
            position, previous_position = cur[11].view(np.float32), prev[11].view(np.float32)
            velocity, previous_velocity = cur[15].view(np.float32), prev[15].view(np.float32)
            upscaled = _f16(cur[18])
            out = np.zeros_like(upscaled)
            tone = _f16(cur[10])
            pn.smaa_tu4x(f, tone, _f16(prev[10]), position, previous_position, velocity, previous_velocity,
                         cur[14].view(np.float32), out)
            pn.smaa_extrapolate(out, tone.shape[0], tone.shape[1])
            _close(cur[18], out, f"frame {f} SMAA TU4x")
            taa = pn.taa(st.upscale.ratio(), list(s.clear_color), upscaled, _f16(prev[19]), position,
                         previous_position, velocity, previous_velocity, upscaled.shape[0], upscaled.shape[1])
            _close(cur[19], taa, f"frame {f} TAA")
            assert (velocity[..., :2] != 0).any()
        prev = cur
