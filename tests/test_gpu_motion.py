"""GPU parity with motion: moving camera, moving instances, TAA jitter and host-supplied G-buffer
planes (prepass.wgsl:30-54,84-100; view.rs:31-73 PreviousViewUniform; transform.rs:32-44
GlobalTransformQueue).

Reprojection reads the previous reservoirs at previous_uv (light.wgsl:181-190) and scatters
rejected history into the previous *spatial* reservoir buffer at the reprojected pixel
(light.wgsl:1092-1095, 1199-1202, 1330-1333).  Several pixels can scatter to one target in one
dispatch: the reference's result there depends on the GPU's write order, so the
oracle runs single-threaded (raster order) and the four spatial-pair buffers (4, 5, 8, 9) are
compared with a stated tolerance: at least 97 % of their records bit-exact.  Everything the
scatter does not reach — the G-buffer (incl. velocity), render / variance / albedo planes and
the temporal reservoirs — is compared bit-exact, and with spatial reuse off nothing reads the
spatial pair, so the frames stay bit-exact frame after frame.
"""
import copy

import numpy as np
import pytest

from parity import canon_plane, canon_reservoirs, mismatch_report

pytestmark = pytest.mark.gpu

RACY = (4, 5, 8, 9)  # previous-spatial scatter targets (light.wgsl:1092-1095)
RACY_MIN_EXACT = 0.97


def _pair(scene_fn, w, h, settings, threads=1):
    from hikari_amd import HikariRenderer, examples, load_noise
    from oracle import Oracle
    scene, cam, lights = examples.SCENES[scene_fn]()
    desc = scene.build()
    r = HikariRenderer(0)
    r.set_noise()
    r.upload_scene(scene)
    r.resize(w, h, settings.upscale.ratio())
    o = Oracle(desc, load_noise(), w, h, settings.upscale.ratio(), threads=threads, textures=scene.textures)
    return scene, cam, lights, r, o


def _compare(r, o, frame, errors, outputs=range(0, 17), stats=None, racy=RACY, rids=range(10)):
    for oid in outputs:
        m = mismatch_report(canon_plane(oid, r.output(oid)), canon_plane(oid, o.output(oid)), f"frame {frame} output {oid}")
        if m:
            errors.append(m)
    for rid in rids:
        g = canon_reservoirs(r.reservoirs(rid))
        c = canon_reservoirs(o.reservoirs(rid)[: len(g)])
        if rid in racy:
            exact = float((g == c).all(axis=1).mean())
            if stats is not None:
                stats.append((frame, rid, exact))
            if exact < RACY_MIN_EXACT:
                errors.append(f"frame {frame} reservoir {rid}: only {exact:.4f} of records exact")
        else:
            m = mismatch_report(g, c, f"frame {frame} reservoir {rid}")
            if m:
                errors.append(m)


def _orbit(cam, f, radius_step=0.05, angle_step=0.04):
    """The camera moved along an orbit around the Cornell box's centre: frame f's camera."""
    from hikari_amd import Camera, Transform
    t = cam.transform.translation
    a = angle_step * f
    c, s = np.cos(a), np.sin(a)
    eye = (float(c * t[0] + s * t[2]), float(t[1] + 0.02 * f), float(-s * t[0] + c * t[2]) + radius_step * f)
    return Camera(Transform.from_xyz(*eye).looking_at((0.0, 1.0, 0.0)))


@pytest.mark.parametrize("size", [(64, 64), (96, 72)])
def test_moving_camera_bit_exact(size):
    """A camera orbiting the Cornell box: every frame's G-buffer (velocity from the previous view),
    light and denoise planes bit-exact; motion vectors present; spatial-pair scatter within the
    stated tolerance."""
    from hikari_amd import HikariSettings, Upscale, frame_inputs
    w, h = size
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=False, denoise=True)
    scene, cam, lights, r, o = _pair("cornell", w, h, st)
    s = st.to_c()
    errors, stats = [], []
    prev = None
    moved = 0
    for f in range(7):
        c = _orbit(cam, f)
        fi = frame_inputs(f, c, lights, w, h, previous_camera=prev)
        prev = copy.deepcopy(c)
        for x in (r, o):
            x.render_gbuffer(fi)
            x.render_frame(s, fi)
            x.denoise(s, fi)
            x.tone_sum(s)
        _compare(r, o, f, errors, stats=stats)
        vel = r.output(15).view(np.float32).reshape(h, w, 4)[..., :2]
        moved += int((vel != 0).any(axis=-1).sum())
        if errors:
            break
    assert not errors, "\n".join(errors[:20])
    assert moved > w * h  # the camera moved: most covered pixels carry a motion vector
    assert r.counters() == o.counters()


def test_moving_camera_1080p_bit_exact():
    """The bench's moving-camera workload at full size (bench.py cornell-1080p-nee-orbit: cornell
    1920x1080, traversal + NEE, the examples' orbit camera at 0.5 deg/frame, examples.orbit): 3 frames,
    every plane bit-exact, the spatial-pair scatter targets within the stated tolerance.  With motion
    the fused direct/emissive launch is off and the direct pair's background stores are kept, while the
    passes' own background targets and the indirect pair still elide (the direct pair bit off, the indirect
    pair bit kept): this covers the separate launches and motion-time elision at bench size."""
    from hikari_amd import HikariSettings, Taa, Upscale, examples, frame_inputs
    w, h = 1920, 1080
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, taa=Taa.None_, indirect_spatial_reuse=False, denoise=False)
    scene, cam, lights, r, o = _pair("cornell", w, h, st)
    s = st.to_c()
    target = examples.ORBIT_TARGETS["cornell"]
    errors, stats = [], []
    moved = 0
    for f in range(3):
        fi = frame_inputs(f, examples.orbit(cam, target, f), lights, w, h,
                          previous_camera=examples.orbit(cam, target, f - 1) if f else None)
        for x in (r, o):
            x.render_gbuffer(fi)
            x.render_frame(s, fi)
            x.tone_sum(s)
        _compare(r, o, f, errors, outputs=(0, 1, 2, 3, 4, 5, 6, 10, 11, 12, 13, 14, 15), stats=stats)
        vel = r.output(15).view(np.float32).reshape(h, w, 4)[..., :2]
        moved += int((vel != 0).any(axis=-1).sum())
        if errors:
            break
    assert not errors, "\n".join(errors[:20])
    assert moved > w * h // 4
    assert r.counters() == o.counters()


def test_moving_camera_spatial_reuse_within_tolerance():
    """Moving camera with indirect spatial reuse and the denoiser: spatial reuse reads the racy
    scatter target (load_previous_spatial_reservoir at previous_uv, light.wgsl:1581-1583), so its
    render plane and everything downstream is compared within a stated tolerance: >= 95 % of
    pixels bit-exact and a mean relative difference of the tone-mapped frame <= 2 %; the
    G-buffer, albedo and the temporal passes' planes stay bit-exact."""
    from hikari_amd import HikariSettings, Upscale, frame_inputs
    w, h = 64, 64
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=True, denoise=True)
    scene, cam, lights, r, o = _pair("cornell", w, h, st)
    s = st.to_c()
    errors = []
    prev = None
    for f in range(6):
        c = _orbit(cam, f)
        fi = frame_inputs(f, c, lights, w, h, previous_camera=prev)
        prev = copy.deepcopy(c)
        for x in (r, o):
            x.render_gbuffer(fi)
            x.render_frame(s, fi)
            x.denoise(s, fi)
            x.tone_sum(s)
        # exact: albedo, direct/emissive variance + render, G-buffer planes
        _compare(r, o, f, errors, outputs=(0, 1, 2, 4, 5, 11, 12, 13, 14, 15), stats=[])
        for oid in (6, 9, 10):  # indirect render (spatial output), denoised indirect, tone-mapped
            a = canon_plane(oid, r.output(oid)).reshape(h, w, 4)
            b = canon_plane(oid, o.output(oid)).reshape(h, w, 4)
            exact = float((a == b).all(axis=-1).mean())
            fa = a.view(np.float16).astype(np.float32)[..., :3]
            fb = b.view(np.float16).astype(np.float32)[..., :3]
            rel = float(np.abs(fa - fb).sum() / max(np.abs(fb).sum(), 1e-6))
            if exact < 0.95 or rel > 0.02:
                errors.append(f"frame {f} output {oid}: {exact:.4f} of pixels exact, mean relative difference {rel:.4f}")
        if errors:
            break
    assert not errors, "\n".join(errors[:20])


def _rotate_instance(scene, k, m0, angle):
    """sphere_rotate_system (city.rs:290-294): rotate_local_z — model = model0 * Rz(angle)."""
    c, s = np.cos(angle), np.sin(angle)
    rz = np.array([[c, -s, 0, 0], [s, c, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]])
    mesh, mat, _ = scene.instances[k]
    scene.instances[k] = (mesh, mat, m0 @ rz)


@pytest.mark.parametrize("scene_fn", ["city", "cornell"])
def test_moving_instances_bit_exact(scene_fn):
    """Instances moving between frames (hk_update_instances on the GPU, a host rebuild for the
    oracle): the G-buffer's per-instance previous models (GlobalTransformQueue) give motion vectors
    on the moving instance only; frames bit-exact.  city: the emissive sphere rotating about its
    local z axis as in city.rs:290-294 (larger steps, seen from close by); cornell: the tall box."""
    from hikari_amd import Camera, HikariSettings, Transform, Upscale, frame_inputs
    w, h = 64, 48
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=False, denoise=True)
    scene, cam, lights, r, o = _pair(scene_fn, w, h, st)
    if scene_fn == "city":
        k = [i for i, (m, _, _) in enumerate(scene.instances) if len(scene.meshes[m].positions) == 37 * 19][-1]
        cam = Camera(Transform.from_xyz(0.6, 1.4, 2.2).looking_at((0.0, 1.0, 0.0)))
        step = 0.35
    else:
        k = 1
        step = 0.12
    m0 = np.asarray(scene.instances[k][2], np.float64)
    s = st.to_c()
    errors = []
    moving_pixels = 0
    for f in range(5):
        if f > 0:
            _rotate_instance(scene, k, m0, step * f)
            desc = scene.build()
            r.update_instances(scene.instance_models(), scene.instance_local_aabbs())
            o.set_scene(desc)
        fi = frame_inputs(f, cam, lights, w, h)
        for x in (r, o):
            x.render_gbuffer(fi)
            x.render_frame(s, fi)
            x.denoise(s, fi)
            x.tone_sum(s)
        _compare(r, o, f, errors)
        vel = r.output(15).view(np.float32).reshape(h, w, 4)[..., :2]
        ids = r.output(14).view(np.float32).reshape(h, w, 2)[..., 0]
        moving = (vel != 0).any(axis=-1)
        moving_pixels += int(moving.sum())
        # only the moving instance's pixels carry motion
        assert not (moving & (ids.astype(np.int64) != k)).any(), f"frame {f}: motion outside instance {k}"
        if errors:
            break
    assert not errors, "\n".join(errors[:20])
    assert moving_pixels > 0


@pytest.mark.parametrize("jitter", [1, 2], ids=["taa", "taa_smaa"])
def test_taa_jitter_bit_exact(jitter):
    """Halton-jittered primary rays (TEMPORAL_ANTI_ALIASING, with and without SMAA_TU4X's halved
    index; prepass.wgsl:30-38,52-54) over 6 frames, every plane bit-exact.  The jitter changes the
    G-buffer but not the velocity (computed from the unjittered view_proj, prepass.wgsl:96)."""
    from hikari_amd import HikariSettings, Upscale, frame_inputs
    w, h = 64, 48
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=True, denoise=True)
    scene, cam, lights, r, o = _pair("cornell", w, h, st, threads=0)
    s = st.to_c()
    errors = []
    positions = []
    for f in range(6):
        fi = frame_inputs(f, cam, lights, w, h, jitter=jitter)
        for x in (r, o):
            x.render_gbuffer(fi)
            x.render_frame(s, fi)
            x.denoise(s, fi)
            x.tone_sum(s)
        _compare(r, o, f, errors, racy=())
        vel = r.output(15).view(np.float32).reshape(h, w, 4)[..., :2]
        assert (vel == 0).all()
        positions.append(r.output(11).tobytes())
        if errors:
            break
    assert not errors, "\n".join(errors[:20])
    assert len(set(positions)) > 1  # the jitter moved the primary rays


def test_host_gbuffer_planes_bit_exact():
    """The route that keeps the reference's raster prepass: G-buffer planes handed
    over with hk_set_gbuffer_plane (here: another context's k_gbuffer output of a moving camera),
    full_screen_albedo as its own pass (k_albedo), separate direct / emissive launches; every
    plane bit-exact against the oracle."""
    from hikari_amd import HikariRenderer, HikariSettings, Upscale, frame_inputs
    w, h = 64, 48
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=False, denoise=True)
    scene, cam, lights, src, o = _pair("cornell", w, h, st)
    r = HikariRenderer(0)
    r.set_noise()
    r.upload_scene(scene)
    r.resize(w, h, 1.0)
    s = st.to_c()
    errors = []
    prev = None
    for f in range(5):
        c = _orbit(cam, f)
        fi = frame_inputs(f, c, lights, w, h, previous_camera=prev)
        prev = copy.deepcopy(c)
        src.render_gbuffer(fi)
        o.render_gbuffer(fi)
        for plane, oid in enumerate((11, 12, 13, 14, 15)):
            r.set_gbuffer_plane(plane, src.output(oid))
        for x in (r, o):
            x.render_frame(s, fi)
            x.denoise(s, fi)
            x.tone_sum(s)
        _compare(r, o, f, errors)
        if errors:
            break
    assert not errors, "\n".join(errors[:20])


@pytest.mark.parametrize("lds", ["0", "1"])
def test_forced_kernel_variants_bit_exact(hk_options, lds):
    """Kernel variants the size thresholds normally pick only at large sizes, forced on a small
    frame: k_direct_lit_w4 (4 waves per SIMD; direct_w4_min_px=0 with fuse=0), the fused
    direct+emissive launch next to the indirect side stream (fuse_min_px=0, merge=0: its emitter walks per
    pixel; with compact_emitter=1 compacted per workgroup, k_direct_fused_cw<VD, false>; with compact_shadow=1
    its shadow walks and the indirect pass's compacted too, k_direct_fused_cw<VD, true>) and the
    merged direct+indirect launch (k_light_merged, merge=1: the default only for small frames without
    spatial reuse; here with spatial reuse after it) and the persistent-wave indirect pass
    (k_indirect_persist, persistent_indirect=1, an opt-in), each with and without LDS scene staging."""
    from hikari_amd import HikariSettings, Upscale, frame_inputs
    hk_options["lds_scene"] = int(lds)
    w, h = 64, 48
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0)
    s = st.to_c()
    for env in ({"direct_w4_min_px": 0, "fuse": 0}, {"fuse_min_px": 0, "merge": 0},
                {"fuse_min_px": 0, "merge": 0, "compact_emitter": 1},
                {"fuse_min_px": 0, "merge": 0, "compact_shadow": 1},
                {"merge": 1}, {"persistent_indirect": 1, "merge": 0}):
        hk_options.clear()
        hk_options.update(lds_scene=int(lds), **env)
        scene, cam, lights, r, o = _pair("cornell", w, h, st, threads=0)
        errors = []
        for f in range(6):
            fi = frame_inputs(f, cam, lights, w, h)
            for x in (r, o):
                x.render_gbuffer(fi)
                x.render_frame(s, fi)
                x.denoise(s, fi)
                x.tone_sum(s)
            _compare(r, o, f, errors, racy=())
            if errors:
                break
        assert not errors, f"{env}: " + "\n".join(errors[:20])
        assert r.counters() == o.counters()


@pytest.mark.parametrize("launch", ["fused", "separate"])
def test_background_elision_bit_exact(hk_options, launch):
    """Background store elision (ChannelArgs::bg, hk_kernels.hip bg_elide): the direct / emissive
    launches (fused, or separate sharing one mask) and the indirect pass skip a background pixel's constant zero stores once
    every target buffer holds them.  A sequence that exercises every way the mask can go stale:
    static frames (elision active from the third frame), camera motion (separate launches: each pass's
    own background targets keep eliding, the direct pair's bit is cleared and its stores resume, the
    indirect pair's bit stays), static again (the pair bit rebuilt), and a reservoir upload over the spatial pairs,
    after which the next frame must store the background records again.  Every plane and all 10
    reservoir buffers bit-exact against the oracle (which never elides) on every frame."""
    from hikari_amd import HikariSettings, Upscale, frame_inputs
    if launch == "fused":
        hk_options["fuse_min_px"] = 0
    else:  # direct_lit and the emissive pass as two launches sharing the mask (k_direct_lit_w4 too)
        hk_options["fuse"] = 0
        hk_options["direct_w4_min_px"] = 0
    w, h = 64, 48
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=False, denoise=True)
    scene, cam, lights, r, o = _pair("cornell", w, h, st)
    s = st.to_c()
    errors = []
    prev = None
    for f in range(12):
        c = _orbit(cam, min(max(f - 3, 0), 2))  # frames 4, 5 move; 0-3 and 6-11 are static
        fi = frame_inputs(f, c, lights, w, h, previous_camera=prev)
        prev = copy.deepcopy(c)
        if f == 11:
            # garbage over both spatial pairs' buffers: the elision masks must be dropped
            from hikari_amd.plugin import RESERVOIR_DTYPE
            rng = np.random.default_rng(5)
            counters = r.counters()
            assert counters == o.counters()
            for rid in RACY:
                r.load_reservoirs(rid, np.frombuffer(rng.bytes(w * h * RESERVOIR_DTYPE.itemsize), RESERVOIR_DTYPE))
        for x in (r, o):
            x.render_gbuffer(fi)
            x.render_frame(s, fi)
            x.denoise(s, fi)
            x.tone_sum(s)
        if f < 11:
            # frames 4-5 move: their spatial-pair scatter is racy (light.wgsl:1092-1095), and
            # with spatial reuse off nothing reads those records afterwards
            _compare(r, o, f, errors, racy=RACY if f >= 4 else ())
        else:
            _compare(r, o, f, errors, racy=(), rids=[k for k in range(10) if k not in RACY])
            depth = r.output(11).view(np.float32).reshape(h * w, 4)[:, 3]
            bg = depth < np.finfo(np.float32).eps
            assert bg.sum() > 0
            for rid in RACY:  # every background record rewritten with the zero reservoir
                g = canon_reservoirs(r.reservoirs(rid))[bg]
                c0 = canon_reservoirs(o.reservoirs(rid)[: w * h])[bg]
                m = mismatch_report(g, c0, f"frame {f} reservoir {rid} background records")
                if m:
                    errors.append(m)
        if errors:
            break
    assert not errors, "\n".join(errors[:20])


@pytest.mark.parametrize("jitter", [0, 1], ids=["static", "taa_jitter"])
def test_background_elision_spatial_pairs_bit_exact(hk_options, jitter):
    """Background store elision with both spatial reuse passes on (emissive_spatial_reuse and
    indirect_spatial_reuse): the fused launch's background pixels then skip their own targets but
    still store the spatial pair (the spatial passes rewrite it with a repacked record), and with TAA
    jitter the silhouettes move every frame while the velocity stays zero, so elision stays on over a
    changing coverage.  Static camera (no scatter race): every plane and all 10 reservoir buffers
    bit-exact on every frame, including after garbage is uploaded over the spatial pairs."""
    from hikari_amd import HikariSettings, Upscale, frame_inputs
    from hikari_amd.plugin import RESERVOIR_DTYPE
    hk_options["fuse_min_px"] = 0
    w, h = 64, 48
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, emissive_spatial_reuse=True, indirect_spatial_reuse=True,
                        denoise=True)
    scene, cam, lights, r, o = _pair("cornell", w, h, st, threads=0)
    s = st.to_c()
    errors = []
    rng = np.random.default_rng(9)
    for f in range(9):
        if f == 7:  # garbage over both spatial pairs, on both sides: the elision masks must be dropped
            for rid in RACY:
                garbage = np.frombuffer(rng.bytes(w * h * RESERVOIR_DTYPE.itemsize), RESERVOIR_DTYPE)
                r.load_reservoirs(rid, garbage)
                o.load_reservoirs(rid, garbage)
        fi = frame_inputs(f, cam, lights, w, h, jitter=jitter)
        for x in (r, o):
            x.render_gbuffer(fi)
            x.render_frame(s, fi)
            x.denoise(s, fi)
            x.tone_sum(s)
        _compare(r, o, f, errors, racy=())
        if errors:
            break
    assert not errors, "\n".join(errors[:20])
