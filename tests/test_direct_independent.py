"""direct_lit + select_light_candidate pinned by an independent restatement (CPU).

The GPU kernels are checked bit for bit against the oracle (tests/test_gpu_*.py); the oracle and
the kernels were written by the same hands from the same reading of light.wgsl, so a misreading
made once would pass both.  tests/direct_python.py restates `direct_lit` (RENDER_EMISSIVE and
EMISSIVE_LIT), `select_light_candidate` (light-BVH pick, alias table, triangle sampling, emitter
BLAS walk), the TLAS/BLAS walks on the reference-format arrays, the reservoir packing and the Bevy
shading in pure Python from the WGSL; here it runs the direct and emissive passes of 16x16 Cornell
frames 0..5 — and of the scene.rs and city.rs layouts (directional light, emissive sphere, City
proxy) — (validation frames of both passes included, reservoir history carried) on the oracle's
G-buffer and previous reservoirs, and every stored word must equal the oracle's: render and variance
planes, the temporal reservoirs and the shared spatial pair.  Tolerance: none (bit-exact); the
transcendentals sin / cos / exp2 come from the oracle's pinned implementations.
"""
import numpy as np
import pytest

import direct_python as dp


def _gbuffer(o, w, h):
    pos = o.output(11).view(np.float32).reshape(h, w, 4)
    nrm_u = o.output(12).view(np.uint32).reshape(h, w)
    nrm = np.stack([np.maximum(((nrm_u >> (8 * k)) & 0xFF).astype(np.uint8).view(np.int8).astype(np.float32) /
                               np.float32(127.0), np.float32(-1.0)) for k in range(3)], -1).astype(np.float32)
    im = o.output(14).view(np.float32).reshape(h, w, 2)
    vel = o.output(15).view(np.float32).reshape(h, w, 4)
    return {"position": pos, "normal": nrm, "instance_material": im, "velocity_uv": vel}


@pytest.mark.parametrize("scene_fn", ["cornell", "scene", "city"])
def test_direct_passes_match_python_restatement(scene_fn):
    import oracle as orc
    from hikari_amd import HikariSettings, Taa, Upscale, examples, frame_inputs, load_noise
    from oracle import Oracle
    w = h = 16
    scene, cam, lights = examples.SCENES[scene_fn]()
    desc = scene.build()
    sc = dp.Scene(scene.arrays(), orc.lib())
    noise = load_noise().reshape(16, 64, 64, 4)
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, taa=Taa.None_, indirect_spatial_reuse=False, denoise=False)
    s = st.to_c()
    o = Oracle(desc, load_noise(), w, h, 1.0, threads=1)
    L = orc.lib()
    emitted = 0
    for f in range(6):
        before = [o.reservoirs(k).view(np.uint32).reshape(-1, 16)[: w * h].copy() for k in range(10)]
        fi = frame_inputs(f, cam, lights, w, h)
        o.render_gbuffer(fi)
        o.render_frame(s, fi)
        gb = _gbuffer(o, w, h)
        fr = {"number": f, "size": (w, h), "ratio": np.float32(1.0),
              "direct_validate_interval": s.direct_validate_interval,
              "emissive_validate_interval": s.emissive_validate_interval,
              "max_temporal_reuse_count": s.max_temporal_reuse_count, "temporal_reuse": s.temporal_reuse,
              "direction_to_light": tuple(np.float32(v) for v in fi.lights.direction_to_light),
              "directional": tuple(np.float32(v) for v in fi.lights.directional_color[:3]),
              "ambient": tuple(np.float32(v) for v in fi.lights.ambient_color[:3]),
              "cos_solar": np.float32(L.hko_cos(float(np.float32(s.solar_angle)))),
              "view_position": tuple(np.float32(v) for v in fi.view.world_position)}
        current, previous = f % 2, 1 - f % 2
        spatial_pair = {"prev_spatial": before[current + 4].copy(), "spatial": before[previous + 4].copy()}
        counts = {"top": 0, "emitter": 0}
        for ch, emissive_lit in ((0, False), (1, True)):
            base = 2 * ch
            bufs = dict(spatial_pair, prev=before[current + base], cur=before[previous + base].copy(),
                        variance=np.zeros((h, w), np.float32), render=np.zeros((h, w, 4), np.float32))
            for y in range(h):
                for x in range(w):
                    dp.direct_lit(sc, fr, gb, noise, bufs, x, y, emissive_lit, counts)
            got_r = o.output(4 + ch).view(np.float16).reshape(h, w, 4)
            assert np.array_equal(got_r.view(np.uint16), bufs["render"].astype(np.float16).view(np.uint16)), \
                (f, ch, "render")
            got_v = o.output(1 + ch).view(np.float32).reshape(h, w)
            assert np.array_equal(got_v.view(np.uint32), bufs["variance"].view(np.uint32)), (f, ch, "variance")
            got_c = o.reservoirs(previous + base).view(np.uint32).reshape(-1, 16)[: w * h]
            bad = np.argwhere((got_c != bufs["cur"]).any(1))
            assert len(bad) == 0, (f, ch, "reservoir", bad[:5].ravel().tolist(), got_c[bad[0][0]], bufs["cur"][bad[0][0]])
        for name, k in (("prev_spatial", current + 4), ("spatial", previous + 4)):
            got = o.reservoirs(k).view(np.uint32).reshape(-1, 16)[: w * h]
            assert np.array_equal(got, spatial_pair[name]), (f, name)
        emitted += counts["emitter"]
    assert emitted > 0  # the emitter BLAS walk and the alias-table pick ran
