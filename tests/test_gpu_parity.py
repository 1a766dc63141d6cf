"""GPU parity: the HIP path (libhikari_amd.so, via the C ABI) against the CPU oracle,
bit-exact on every output plane and reservoir buffer (NaN payloads canonicalised).

Scenes: cornell (examples/cornell.rs) at small sizes; frames 0..N so that validation frames
(number % 3 == 0 and % 5 == 0), temporal reuse and the spatial pass are all exercised.
"""
import numpy as np
import pytest

from parity import canon_plane, canon_reservoirs, mismatch_report

pytestmark = pytest.mark.gpu

OUTPUTS = list(range(0, 17))


def _setup(width, height, settings, scene_fn="cornell"):
    from hikari_amd import HikariRenderer, examples, load_noise
    from oracle import Oracle
    scene, cam, lights = examples.SCENES[scene_fn]()
    desc = scene.build()
    r = HikariRenderer(0)
    r.set_noise()
    r.upload_scene(scene)
    r.resize(width, height, settings.upscale.ratio())
    o = Oracle(desc, load_noise(), width, height, settings.upscale.ratio())
    return scene, cam, lights, r, o


def _compare_frame(r, o, frame, errors):
    for oid in OUTPUTS:
        a = canon_plane(oid, r.output(oid))
        b = canon_plane(oid, o.output(oid))
        m = mismatch_report(a, b, f"frame {frame} output {oid}")
        if m:
            errors.append(m)
    for rid in range(10):
        m = mismatch_report(canon_reservoirs(r.reservoirs(rid)), canon_reservoirs(o.reservoirs(rid)),
                            f"frame {frame} reservoir {rid}")
        if m:
            errors.append(m)


@pytest.mark.parametrize("size", [(64, 64), (96, 72)])
def test_cornell_frames_bit_exact(size):
    from hikari_amd import HikariSettings, Upscale, frame_inputs
    w, h = size
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0)
    scene, cam, lights, r, o = _setup(w, h, st)
    s = st.to_c()
    errors = []
    for f in range(7):
        fi = frame_inputs(f, cam, lights, w, h)
        r.render_gbuffer(fi)
        o.render_gbuffer(fi)
        r.render_frame(s, fi)
        o.render_frame(s, fi)
        r.denoise(s, fi)
        o.denoise(s, fi)
        r.tone_sum(s)
        o.tone_sum(s)
        _compare_frame(r, o, f, errors)
        if errors:
            break
    assert not errors, "\n".join(errors[:20])
    assert r.counters() == o.counters()


def test_trace_matches_oracle():
    from hikari_amd import HikariSettings, Upscale
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0)
    scene, cam, lights, r, o = _setup(16, 16, st)
    rng = np.random.default_rng(7)
    n = 20000
    org = rng.uniform([-1.2, -0.2, -1.2], [1.2, 2.2, 1.2], (n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d[:100, 0] = 0.0  # axis-parallel rays: 1/0 = inf in the slab test
    rays = np.concatenate([org, d], axis=1).astype(np.float32)
    early = np.where(rng.random(n) < 0.5, 0.0, 65535.0).astype(np.float32)
    excl = rng.integers(0, 9, n).astype(np.uint32)
    a = r.trace(rays, None, early, excl)
    b = o.trace(rays, None, early, excl)
    assert (a == b).all(), f"{int((a != b).any(axis=1).sum())} of {n} rays differ"
    assert (a[:, 3] != 0xFFFFFFFF).mean() > 0.5
