"""GPU parity of the wavefront indirect pass (hk_set_wavefront: BASELINE configs[4]'s material-sorted
shading; hk_kernels.hip k_wf_*): live pixels compacted with wave64 ballots, the bounce walk writing SoA
hit records, the queue grouped by the hit's material, the shading / NEE / shadow / temporal tail in
that order.  Every plane, reservoir buffer and ray counter must equal the CPU oracle's (which runs
light.wgsl's one-thread-per-pixel order), frame after frame."""
import numpy as np
import pytest

from parity import canon_plane, canon_reservoirs, mismatch_report

pytestmark = pytest.mark.gpu


def _pair(scene_fn, w, h, settings):
    from hikari_amd import HikariRenderer, examples, load_noise
    from oracle import Oracle
    scene, cam, lights = examples.SCENES[scene_fn]()
    desc = scene.build()
    r = HikariRenderer(0)
    r.set_noise()
    r.upload_scene(scene)
    r.resize(w, h, settings.upscale.ratio())
    r.set_wavefront(True)
    o = Oracle(desc, load_noise(), w, h, settings.upscale.ratio(), textures=scene.textures)
    return scene, cam, lights, r, o


def _frames(scene_fn, w, h, settings, frames):
    from hikari_amd import frame_inputs
    scene, cam, lights, r, o = _pair(scene_fn, w, h, settings)
    s = settings.to_c()
    errors = []
    for f in range(frames):
        fi = frame_inputs(f, cam, lights, w, h)
        for x in (r, o):
            x.render_gbuffer(fi)
            x.render_frame(s, fi)
            x.denoise(s, fi)
            x.tone_sum(s)
        for oid in range(0, 17):
            m = mismatch_report(canon_plane(oid, r.output(oid)), canon_plane(oid, o.output(oid)), f"frame {f} output {oid}")
            if m:
                errors.append(m)
        for rid in range(10):
            g = r.reservoirs(rid)
            m = mismatch_report(canon_reservoirs(g), canon_reservoirs(o.reservoirs(rid)[: len(g)]),
                                f"frame {f} reservoir {rid}")
            if m:
                errors.append(m)
        if errors:
            break
    assert not errors, "\n".join(errors[:20])
    assert r.counters() == o.counters()
    return r, o


@pytest.mark.parametrize("lds", ["0", "1"])
@pytest.mark.parametrize("size", [(64, 64), (96, 72)])
def test_wavefront_cornell_bit_exact(hk_options, lds, size):
    from hikari_amd import HikariSettings, Upscale
    hk_options["lds_scene"] = int(lds)
    _frames("cornell", size[0], size[1], HikariSettings(upscale=Upscale.SMAA_TU_1_0), 7)


@pytest.mark.parametrize("scene_fn,size", [("city", (64, 40)), ("scene", (64, 40)), ("cornell_textured", (64, 48))])
def test_wavefront_scenes_bit_exact(scene_fn, size):
    """City proxy (79 material bins, directional light, emissive sphere), scene.rs, textured cornell
    (material textures fetched in material order), upscale ratio 1."""
    from hikari_amd import HikariSettings, Upscale
    _frames(scene_fn, size[0], size[1], HikariSettings(upscale=Upscale.SMAA_TU_1_0), 4)


def test_wavefront_ratio_two_bit_exact():
    """Upscale ratio 2 (integrator at half resolution, jittered deferred lookups)."""
    from hikari_amd import HikariSettings, Upscale
    _frames("cornell", 64, 48, HikariSettings(upscale=Upscale.SMAA_TU_2_0), 5)


def test_city_4k_16spp_bit_exact():
    """BASELINE configs[4] at full size: city.rs 3840x2160, 16 integrator sub-frames per displayed
    frame (each one reference frame: G-buffer, light passes with the wavefront indirect pass, spatial
    reuse, denoise, tone-sum), accumulated and resolved on the GPU, over 2 displayed frames.
    * whole frame: the wavefront context (G-buffer reuse on: 30 of the 32 sub-frames keep the planes they
      find) equals a megakernel context tracing every sub-frame (whose full-size parity with the oracle
      test_full_size_bench_workloads_bit_exact establishes) on OUT_ACCUMULATED of both displayed frames,
      every plane and reservoir buffer of the last sub-frame and the ray counters;
    * against the oracle: rows 1040..1119 (through the sphere and the houses) rendered by the oracle
      as a band with a 40-row halo (exact for the band's own rows, test_gpu_row_bands_match_whole_frame),
      its 32 tone-mapped sub-frames accumulated in numpy (f32 running sum, / 16, rounded to f16),
      bit for bit against the GPU's OUT_ACCUMULATED rows."""
    from hikari_amd import HikariRenderer, HikariSettings, Taa, Upscale, _abi, examples, frame_inputs, load_noise
    from oracle import Oracle
    import bench
    cfg = bench.CONFIGS["city-4k-16spp"]
    w, h, spp = cfg["width"], cfg["height"], cfg["spp"]
    y0, rows = 1040, 80
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, taa=Taa.None_, indirect_spatial_reuse=cfg["spatial"],
                        denoise=cfg["denoise"])
    scene, cam, lights = examples.SCENES[cfg["scene"]]()
    desc = scene.build()
    ctx = []
    for wavefront in (True, False):
        # the wavefront context reuses the G-buffer of the static sub-frames (the default), the megakernel
        # context traces every sub-frame (gbuffer_reuse = 0): their equality pins the reuse at full size
        r = HikariRenderer(0, options={"gbuffer_reuse": 1 if wavefront else 0})
        r.set_noise()
        r.upload_scene(scene)
        r.resize(w, h, 1.0)
        r.set_wavefront(wavefront)
        ctx.append(r)
    o = Oracle(desc, load_noise(), w, h, 1.0)
    o.set_band(y0, rows, 40)
    s = st.to_c()
    errors = []
    for shown in range(2):
        acc = np.zeros((rows, w, 4), np.float32)
        for k in range(spp):
            fi = frame_inputs(shown * spp + k, cam, lights, w, h)
            for r in ctx:
                r.render_gbuffer(fi)
                r.render_frame(s, fi)
                r.denoise(s, fi)
                r.tone_sum(s)
                r.accumulate(reset=(k == 0))
            o.render_gbuffer(fi)
            o.render_frame(s, fi)
            o.denoise(s, fi)
            o.tone_sum(s)
            t = o.output(_abi.OUT_TONE_MAPPED)[y0:y0 + rows].view(np.float16).reshape(rows, w, 4).astype(np.float32)
            acc = (acc + t).astype(np.float32)
        for r in ctx:
            r.resolve_accumulation()
        a, b = (canon_plane(10, r.output(_abi.OUT_ACCUMULATED)) for r in ctx)
        m = mismatch_report(a, b, f"displayed frame {shown}: wavefront vs megakernel accumulated")
        if m:
            errors.append(m)
        want = canon_plane(10, (acc / np.float32(spp)).astype(np.float16).view(np.uint8).reshape(rows, w, 8))
        m = mismatch_report(a[y0:y0 + rows], want, f"displayed frame {shown}: rows {y0}..{y0 + rows - 1} vs oracle")
        if m:
            errors.append(m)
        assert float(np.abs(want.view(np.float16).astype(np.float32)).mean()) > 0.01  # a lit band
    for oid in range(0, 17):
        m = mismatch_report(*(canon_plane(oid, r.output(oid)) for r in ctx), f"last sub-frame output {oid}")
        if m:
            errors.append(m)
    for rid in range(10):
        m = mismatch_report(*(canon_reservoirs(r.reservoirs(rid)) for r in ctx), f"reservoir {rid}")
        if m:
            errors.append(m)
    assert not errors, "\n".join(errors[:20])
    assert ctx[0].counters() == ctx[1].counters()
    assert ctx[0].primary_reused() == (2 * spp - 2) * w * h and ctx[1].primary_reused() == 0
