"""indirect_lit_ambient, spatial_reuse and the denoiser (incl. its firefly filter) pinned by
independent restatements (CPU).

The GPU kernels are checked bit for bit against the oracle (tests/test_gpu_*.py); the oracle and the
kernels were written by the same hands from the same reading of the WGSL, so a misreading made once would
pass both.  tests/indirect_python.py restates `indirect_lit_ambient` (one bounce and MULTIPLE_BOUNCES)
and `spatial_reuse` (indirect and EMISSIVE_LIT) from light.wgsl, tests/denoise_python.py restates
denoise.wgsl in float32 (demodulation, the four à-trous levels, FIREFLY_FILTERING), both without the
oracle's code.  Here the oracle renders frames 0..5 of the cornell, scene.rs and city.rs layouts; for
each frame the restatements run on the oracle's G-buffer and the reservoir buffers as they were before
the frame (history carried by the oracle, so every frame is an independent check) and every stored word
must equal the oracle's: the channels' render and variance planes, all reservoir buffers the passes
write, and the three denoised outputs.  Tolerance: none (bit-exact); the transcendentals sin / cos /
exp2 / log2 are the oracle library's pinned primitives.

Variant "default" is HikariSettings::default() at ratio 1 (one bounce, indirect spatial reuse, denoise).
Variant "multi" adds MULTIPLE_BOUNCES (indirect_bounces = 3), emissive spatial reuse (EMISSIVE_LIT; the
direct and emissive temporal passes then run in tests/direct_python.py first, because the emissive
spatial pass reads the pair they share), and max_reservoir_lifetime = 3 so spatial reuse takes both
sides of its lifetime test.
"""
import numpy as np
import pytest

import denoise_python as dnp
import direct_python as dp
import indirect_python as ip

W, H = 24, 20


def _gbuffer(o, w, h):
    pos = o.output(11).view(np.float32).reshape(h, w, 4)
    nrm_u = o.output(12).view(np.uint32).reshape(h, w)
    nrm = np.stack([np.maximum(((nrm_u >> (8 * k)) & 0xFF).astype(np.uint8).view(np.int8).astype(np.float32) /
                               np.float32(127.0), np.float32(-1.0)) for k in range(3)], -1).astype(np.float32)
    im = o.output(14).view(np.float32).reshape(h, w, 2)
    vel = o.output(15).view(np.float32).reshape(h, w, 4)
    grad = o.output(13).view(np.float32).reshape(h, w, 2)
    return {"position": pos, "normal": nrm, "instance_material": im, "velocity_uv": vel, "depth_gradient": grad}


def _frame_dict(f, s, fi, L):
    return {"number": f, "size": (W, H), "ratio": np.float32(1.0),
            "direct_validate_interval": s.direct_validate_interval,
            "emissive_validate_interval": s.emissive_validate_interval,
            "max_temporal_reuse_count": s.max_temporal_reuse_count,
            "max_spatial_reuse_count": s.max_spatial_reuse_count,
            "max_reservoir_lifetime": np.float32(s.max_reservoir_lifetime),
            "indirect_bounces": s.indirect_bounces,
            "max_indirect_luminance": np.float32(s.max_indirect_luminance),
            "temporal_reuse": s.temporal_reuse,
            "direction_to_light": tuple(np.float32(v) for v in fi.lights.direction_to_light),
            "directional": tuple(np.float32(v) for v in fi.lights.directional_color[:3]),
            "ambient": tuple(np.float32(v) for v in fi.lights.ambient_color[:3]),
            "cos_solar": np.float32(L.hko_cos(float(np.float32(s.solar_angle)))),
            "view_position": tuple(np.float32(v) for v in fi.view.world_position)}


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _check_channel(o, ch, bufs, spatial_pair_ids, tag):
    got_r = o.output(4 + ch).view(np.uint16).reshape(H, W, 4)
    want_r = bufs["render"].astype(np.float16).view(np.uint16)
    bad = np.argwhere((got_r != want_r).any(-1))
    assert len(bad) == 0, (tag, "render", bad[:5].tolist())
    got_v = _bits(o.output(1 + ch).view(np.float32).reshape(H, W))
    bad = np.argwhere(got_v != _bits(bufs["variance"]))
    assert len(bad) == 0, (tag, "variance", bad[:5].tolist())
    for name, k in spatial_pair_ids:
        got = o.reservoirs(k).view(np.uint32).reshape(-1, 16)[: W * H]
        bad = np.argwhere((got != bufs[name]).any(1)).ravel()
        assert len(bad) == 0, (tag, name, k, bad[:5].tolist(), got[bad[0]].tolist(), bufs[name][bad[0]].tolist())


@pytest.mark.parametrize("variant", ["default", "multi"])
@pytest.mark.parametrize("scene_fn", ["cornell", "scene", "city"])
def test_indirect_spatial_denoise_match_python_restatement(scene_fn, variant):
    import oracle as orc
    from hikari_amd import HikariSettings, Taa, Upscale, examples, frame_inputs, load_noise
    from oracle import Oracle
    scene, cam, lights = examples.SCENES[scene_fn]()
    desc = scene.build()
    sc = dp.Scene(scene.arrays(), orc.lib())
    noise = load_noise().reshape(16, 64, 64, 4)
    multi = variant == "multi"
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, taa=Taa.None_, indirect_spatial_reuse=True, denoise=True,
                        indirect_bounces=3 if multi else 1, emissive_spatial_reuse=multi,
                        max_reservoir_lifetime=3.0 if multi else 100.0)
    s = st.to_c()
    o = Oracle(desc, load_noise(), W, H, 1.0, threads=1)
    L = orc.lib()
    counts = {"top": 0, "emitter": 0}
    reused = lifetime_kept = 0
    stats = {}
    for f in range(6):
        before = [o.reservoirs(k).view(np.uint32).reshape(-1, 16)[: W * H].copy() for k in range(10)]
        fi = frame_inputs(f, cam, lights, W, H)
        o.render_gbuffer(fi)
        o.render_frame(s, fi)
        o.denoise(s, fi)
        gb = _gbuffer(o, W, H)
        fr = _frame_dict(f, s, fi, L)
        fm = ip.Frame(fr, gb, noise)
        current, previous = f % 2, 1 - f % 2
        pixels = [(x, y) for y in range(H) for x in range(W)]

        if multi:  # direct + emissive temporal (proven in test_direct_independent), then EMISSIVE_LIT spatial
            pair = {"prev_spatial": before[current + 4].copy(), "spatial": before[previous + 4].copy()}
            for ch, emissive_lit in ((0, False), (1, True)):
                bufs = dict(pair, prev=before[current + 2 * ch], cur=before[previous + 2 * ch].copy(),
                            variance=np.zeros((H, W), np.float32), render=np.zeros((H, W, 4), np.float32))
                for x, y in pixels:
                    dp.direct_lit(sc, fr, gb, noise, bufs, x, y, emissive_lit, counts)
            for x, y in pixels:
                ip.spatial_reuse(sc, fm, bufs, x, y, True)
            _check_channel(o, 1, bufs, (("cur", previous + 2), ("prev_spatial", current + 4),
                                        ("spatial", previous + 4)), (scene_fn, f, "emissive"))

        bufs = {"prev": before[current + 6], "cur": before[previous + 6].copy(),
                "prev_spatial": before[current + 8].copy(), "spatial": before[previous + 8].copy(),
                "variance": np.zeros((H, W), np.float32), "render": np.zeros((H, W, 4), np.float32)}
        for x, y in pixels:
            ip.indirect_lit_ambient(sc, fm, bufs, x, y, counts)
        lifetimes = [dp.unpack_reservoir(bufs["cur"][x + W * y])["lifetime"] for x, y in pixels]
        lifetime_kept += sum(lt > np.float32(3.0) for lt in lifetimes)
        spatial_before = bufs["spatial"].copy()
        for x, y in pixels:
            ip.spatial_reuse(sc, fm, bufs, x, y, False)
        reused += int((bufs["spatial"] != spatial_before).any(1).sum())
        _check_channel(o, 2, bufs, (("cur", previous + 6), ("prev_spatial", current + 8), ("spatial", previous + 8)),
                       (scene_fn, f, "indirect"))

        # denoiser on the (now verified) planes: all three channels, firefly on emissive / indirect
        albedo = o.output(0).view(np.float16).reshape(H, W, 4).astype(np.float32)
        pl = dnp.Planes(gb, albedo)
        for ch in range(3):
            render = o.output(4 + ch).view(np.float16).reshape(H, W, 4).astype(np.float32)
            variance = o.output(1 + ch).view(np.float32).reshape(H, W)
            out, _ = dnp.denoise_channel(L, pl, render, variance, ch >= 1, f, stats=stats)
            got = o.output(7 + ch).view(np.uint16).reshape(H, W, 4)
            bad = np.argwhere((got != out.astype(np.float16).view(np.uint16)).any(-1))
            assert len(bad) == 0, (scene_fn, f, "denoised", ch, bad[:5].tolist())
    assert counts["top"] > 0 and reused > 0
    if multi:
        assert lifetime_kept > 0  # spatial reuse kept the temporal record (lifetime > max_reservoir_lifetime)
    assert stats.get("firefly", 0) > 0  # the firefly branch scaled at least one pixel
