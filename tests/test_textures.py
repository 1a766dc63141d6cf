"""Material texture sampling (light.wgsl:748-794, include/hk_texture.h): the oracle's sampler
against an independent numpy restatement, and a textured scene through the whole oracle frame."""
import numpy as np
import pytest

from parity import canon_plane


def _np_decode(byte, srgb):
    c = byte.astype(np.float32) / np.float32(255.0)
    if not srgb:
        return c
    lin = c / np.float32(12.92)
    hi = ((c.astype(np.float64) + 0.055) / 1.055) ** 2.4
    return np.where(c <= np.float32(0.04045), lin, hi.astype(np.float32))


def _np_address(i, n, mode):
    if mode == 1:
        return np.mod(i, n)
    if mode == 2:
        r = np.mod(i, 2 * n)
        return np.where(r < n, r, 2 * n - 1 - r)
    return np.clip(i, 0, n - 1)


def _np_sample(tex, uv):
    """float64 restatement of textureSampleLevel(.., 0) (tolerance check, not bit-exact)."""
    a = tex.rgba8
    h, w = a.shape[:2]
    dec = np.stack([_np_decode(a[..., k], tex.srgb and k < 3) for k in range(4)], axis=-1).astype(np.float64)
    u, v = uv[:, 0].astype(np.float64), uv[:, 1].astype(np.float64)
    if tex.filter == 0:
        i = _np_address(np.floor(u * w).astype(np.int64), w, tex.address_u)
        j = _np_address(np.floor(v * h).astype(np.int64), h, tex.address_v)
        return dec[j, i]
    x, y = u * w - 0.5, v * h - 0.5
    x0, y0 = np.floor(x), np.floor(y)
    fa, fb = (x - x0)[:, None], (y - y0)[:, None]
    i0, j0 = x0.astype(np.int64), y0.astype(np.int64)
    ia, ib = _np_address(i0, w, tex.address_u), _np_address(i0 + 1, w, tex.address_u)
    ja, jb = _np_address(j0, h, tex.address_v), _np_address(j0 + 1, h, tex.address_v)
    return (dec[ja, ia] * (1 - fa) + dec[ja, ib] * fa) * (1 - fb) + (dec[jb, ia] * (1 - fa) + dec[jb, ib] * fa) * fb


def test_oracle_sampler_matches_numpy_restatement():
    from hikari_amd import examples, load_noise
    from oracle import Oracle
    scene, cam, lights = examples.cornell_textured()
    desc = scene.build()
    o = Oracle(desc, load_noise(), 8, 8, 1.0, textures=scene.textures)
    rng = np.random.default_rng(3)
    uv = rng.uniform(-2.5, 3.5, (20000, 2)).astype(np.float32)
    uv[:50] = np.array([[0, 0], [1, 1], [0.5, 0.5], [-0.0, 1.0], [0.999999, 0.0000001]] * 10, np.float32)
    for tid, tex in enumerate(scene.textures):
        got = o.sample_texture(tid, uv)
        want = _np_sample(tex, uv)
        err = np.abs(got - want)
        assert err.max() < 2e-5, (tid, float(err.max()))


def test_texture_decode_lut_edges():
    from hikari_amd import Scene, Texture, examples, load_noise
    from oracle import Oracle
    scene, _, _ = examples.cornell()
    desc = scene.build()
    ramp = np.zeros((1, 256, 4), np.uint8)
    ramp[0, :, 0] = ramp[0, :, 1] = ramp[0, :, 2] = ramp[0, :, 3] = np.arange(256)
    o = Oracle(desc, load_noise(), 8, 8, 1.0, textures=[Texture(ramp, srgb=True, filter=0),
                                                         Texture(ramp, srgb=False, filter=0)])
    uv = np.stack([(np.arange(256) + 0.5) / 256, np.full(256, 0.5)], axis=1).astype(np.float32)
    s = o.sample_texture(0, uv)
    l_ = o.sample_texture(1, uv)
    assert s[0, 0] == 0.0 and s[255, 0] == 1.0 and l_[255, 0] == 1.0
    assert np.all(np.diff(s[:, 0]) > 0) and np.array_equal(s[:, 3], l_[:, 3])  # alpha linear in sRGB images
    assert np.abs(s[:, 0] - _np_decode(np.arange(256), True)).max() < 2e-7


def test_textured_frames_differ_from_untextured_and_are_deterministic():
    """The textured pipeline changes the image (it is really sampled) and is deterministic."""
    from hikari_amd import HikariSettings, Upscale, examples, frame_inputs, load_noise
    from oracle import Oracle
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0).to_c()
    outs = []
    for fn in ("cornell_textured", "cornell_textured", "cornell"):
        scene, cam, lights = examples.SCENES[fn]()
        desc = scene.build()
        o = Oracle(desc, load_noise(), 32, 24, 1.0, textures=scene.textures)
        for f in range(2):
            fi = frame_inputs(f, cam, lights, 32, 24)
            o.render_gbuffer(fi)
            o.render_frame(st, fi)
            o.denoise(st, fi)
            o.tone_sum(st)
        outs.append(canon_plane(10, o.output(10)).copy())
    assert np.array_equal(outs[0], outs[1])
    assert not np.array_equal(outs[0], outs[2])


def test_oracle_post_process_smaa_current_samples_and_sizes():
    """SMAA TU4x writes each input texel unchanged at its jittered output position
    (smaa.wgsl:123-126, 197) and the upscaled / TAA planes have the reference's sizes
    (post_process.rs:663-731: ceil(S * 2 / ratio))."""
    import math
    from hikari_amd import HikariSettings, Upscale, _abi, examples, frame_inputs, load_noise
    from oracle import Oracle
    W, H = 33, 21
    st = HikariSettings(upscale=Upscale.SMAA_TU_2_0)
    scene, cam, lights = examples.cornell()
    o = Oracle(scene.build(), load_noise(), W, H, st.upscale.ratio())
    s = st.to_c()
    for f in range(3):
        fi = frame_inputs(f, cam, lights, W, H)
        o.render_gbuffer(fi)
        o.render_frame(s, fi)
        o.denoise(s, fi)
        o.tone_sum(s)
        o.post_process(s, fi)
        tone = o.output(_abi.OUT_TONE_MAPPED).view(np.uint16).reshape(math.ceil(H / 2), math.ceil(W / 2), 4)
        up = o.output(_abi.OUT_UPSCALED).view(np.uint16)
        taa = o.output(_abi.OUT_TAA).view(np.uint16)
        assert up.shape[:2] == (H, W) and taa.shape[:2] == (H, W)
        up = up.reshape(H, W, 4)
        j = 0 if f % 2 == 0 else 1
        sub = up[j::2, j::2]
        hh, ww = sub.shape[:2]
        assert np.array_equal(sub[..., :3], tone[:hh, :ww, :3])
        assert np.all(sub[..., 3] == 0x3C00)  # alpha 1.0
        assert np.isfinite(taa.view(np.float16)).all()
