"""GPU tests of the runtime's scheduling features (hk_runtime.hip), each against the CPU oracle or against
the same frames with the feature switched off through hk_set_option:
* G-buffer reuse (option gbuffer_reuse): static sub-frames keep the planes of the slot they reuse;
* foreign-stream output copies (hk_copy_output_rows on a communication stream, as bench.py's all-gather
  path issues them): each copy sees its frame's finished plane while the frames stay pipelined, and the
  plane's next write waits for the copy;
* a row band fed host G-buffer planes with motion runs every pass on its whole band;
* foreign-stream copies of the denoiser's internal variance, and the option value checks.
"""
import copy
import ctypes

import numpy as np
import pytest

from parity import canon_plane, canon_reservoirs, mismatch_report

pytestmark = pytest.mark.gpu


def _pair(scene_fn, w, h, settings, options=None):
    from hikari_amd import HikariRenderer, examples, load_noise
    from oracle import Oracle
    scene, cam, lights = examples.SCENES[scene_fn]()
    desc = scene.build()
    r = HikariRenderer(0, options=options)
    r.set_noise()
    r.upload_scene(scene)
    r.resize(w, h, settings.upscale.ratio())
    o = Oracle(desc, load_noise(), w, h, settings.upscale.ratio(), textures=scene.textures)
    return scene, cam, lights, r, o


RACY = (4, 5, 8, 9)  # previous-spatial scatter targets under motion (light.wgsl:1092-1095; test_gpu_motion.py)


def _compare(r, o, frame, errors, racy=()):
    for oid in range(0, 17):
        m = mismatch_report(canon_plane(oid, r.output(oid)), canon_plane(oid, o.output(oid)), f"frame {frame} output {oid}")
        if m:
            errors.append(m)
    for rid in range(10):
        g = canon_reservoirs(r.reservoirs(rid))
        c = canon_reservoirs(o.reservoirs(rid)[: len(g)])
        if rid in racy:  # written by the reference's racy scatter: the motion tests' tolerance
            exact = float((g == c).all(axis=1).mean())
            if exact < 0.97:
                errors.append(f"frame {frame} reservoir {rid}: only {exact:.4f} of records exact")
            continue
        m = mismatch_report(g, c, f"frame {frame} reservoir {rid}")
        if m:
            errors.append(m)


def _hip():
    maps = [ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln]
    path = next((m for m in maps if m.startswith("/opt/rocm")), maps[0] if maps else "libamdhip64.so")
    hip = ctypes.CDLL(path)
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    return hip


def test_gbuffer_reuse_bit_exact():
    """Static frames with frame pipelining forced on (pipeline_min_px = 0): from the third frame on the
    G-buffer slot already holds the frame's planes and k_gbuffer is skipped.  Then the camera moves (no
    reuse: new planes, motion vectors), stands still again (reuse resumes once both slots hold the new
    view and no motion vectors), and TAA jitter changes the primary rays every frame (no reuse).  Every plane, every reservoir
    buffer and the counters equal the oracle's (which traces every frame) on every frame — from the camera
    move on, the spatial-pair buffers that the reference's temporal passes scatter into under motion within
    the motion tests' tolerance (spatial reuse is off, so nothing reads them); the primary-ray count includes
    the reused frames, and primary_reused is exactly their pixels."""
    from hikari_amd import HikariSettings, Upscale, frame_inputs
    w, h = 96, 72
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=False, denoise=True)
    scene, cam, lights, r, o = _pair("cornell", w, h, st, options={"pipeline_min_px": 0})
    s = st.to_c()
    moved = copy.deepcopy(cam)
    moved.transform.translation = np.array([0.05, 1.02, 4.0])
    # (camera, previous camera, jitter) per frame
    plan = [(cam, None, 0)] * 5 + [(moved, cam, 0)] + [(moved, None, 0)] * 4 + [(moved, None, 1)] * 3
    # frame 5 has motion vectors, so its slot is not reusable either: frame 7 traces again
    expect_reused = [False, False, True, True, True, False, False, False, True, True, False, False, False]
    errors = []
    reused = 0
    for f, (c, prev, jitter) in enumerate(plan):
        fi = frame_inputs(f, c, lights, w, h, previous_camera=prev, jitter=jitter)
        for x in (r, o):
            x.render_gbuffer(fi)
            x.render_frame(s, fi)
            x.denoise(s, fi)
            x.tone_sum(s)
        now = r.primary_reused()
        assert (now > reused) == expect_reused[f], f"frame {f}: reused {now - reused} rays"
        if expect_reused[f]:
            assert now - reused == w * h
        reused = now
        _compare(r, o, f, errors, racy=RACY if f >= 5 else ())
        if errors:
            break
    assert not errors, "\n".join(errors[:20])
    assert r.counters() == o.counters()
    # off: the same frames traced every time
    scene, cam, lights, r2, o2 = _pair("cornell", w, h, st, options={"pipeline_min_px": 0, "gbuffer_reuse": 0})
    for f, (c, prev, jitter) in enumerate(plan):
        fi = frame_inputs(f, c, lights, w, h, previous_camera=prev, jitter=jitter)
        r2.render_gbuffer(fi)
        r2.render_frame(s, fi)
        r2.denoise(s, fi)
        r2.tone_sum(s)
    assert r2.primary_reused() == 0
    for oid in range(0, 17):
        m = mismatch_report(canon_plane(oid, r.output(oid)), canon_plane(oid, r2.output(oid)), f"reuse on/off output {oid}")
        assert not m, m


@pytest.mark.parametrize("denoise", [True, False], ids=["denoise", "tone_only"])
def test_foreign_stream_copies_keep_frames_exact(denoise):
    """bench.py's all-gather path: each frame's tone-mapped rows copied with hk_copy_output_rows on a
    stream of the caller's own (not the frame stream), into two alternating device buffers, while the next
    frames are queued without any readback (pipelined: pipeline_min_px = 0).  Every copy holds its own
    frame's plane bit for bit (oracle), so the copy waited for the frame's tail and the tone-sum two frames
    later waited for the copy; the frames themselves stay exact."""
    from hikari_amd import HikariSettings, Upscale, _abi, frame_inputs
    hip = _hip()
    w, h = 96, 72
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=denoise, denoise=denoise)
    scene, cam, lights, r, o = _pair("cornell", w, h, st, options={"pipeline_min_px": 0})
    s = st.to_c()
    stream = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(stream)) == 0
    y0, rows = 8, 48
    nbytes = rows * w * 8
    bufs = [ctypes.c_void_p(), ctypes.c_void_p()]
    for b in bufs:
        assert hip.hipMalloc(ctypes.byref(b), nbytes) == 0
    want = {}
    got = {}
    frames = 8
    for f in range(frames):
        fi = frame_inputs(f, cam, lights, w, h)
        r.render_gbuffer(fi)
        r.render_frame(s, fi)
        r.denoise(s, fi)
        r.tone_sum(s)
        r.copy_output_rows(_abi.OUT_TONE_MAPPED, y0, rows, bufs[f & 1].value, False, stream.value)
        o.render_gbuffer(fi)
        o.render_frame(s, fi)
        o.denoise(s, fi)
        o.tone_sum(s)
        want[f] = canon_plane(10, o.output(10)[y0:y0 + rows])
        if f >= 1 and f % 3 == 0:  # read the previous frame's copy back (its buffer is rewritten next frame)
            assert hip.hipStreamSynchronize(stream) == 0
            out = np.empty((rows, w, 8), np.uint8)
            assert hip.hipMemcpy(out.ctypes.data, bufs[(f - 1) & 1], nbytes, 2) == 0
            got[f - 1] = canon_plane(10, out)
    assert hip.hipStreamSynchronize(stream) == 0
    out = np.empty((rows, w, 8), np.uint8)
    assert hip.hipMemcpy(out.ctypes.data, bufs[(frames - 1) & 1], nbytes, 2) == 0
    got[frames - 1] = canon_plane(10, out)
    for f, g in got.items():
        m = mismatch_report(g, want[f], f"frame {f} copied rows")
        assert not m, m
    errors = []
    _compare(r, o, frames - 1, errors)
    assert not errors, "\n".join(errors[:20])
    for b in bufs:
        hip.hipFree(b)
    hip.hipStreamDestroy(stream)


def test_foreign_copies_of_the_internal_variance():
    """hk_copy_output_rows of HK_OUT_DENOISE_INTERNAL_VARIANCE on a foreign stream registers a read of
    that plane, so the next hk_denoise (which rewrites it) waits for the copy.  Each frame's copy must hold that
    frame's plane (the oracle's), with frames queued pipelined behind the copies."""
    from hikari_amd import HikariSettings, Upscale, _abi, frame_inputs
    hip = _hip()
    w, h = 96, 72
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=True, denoise=True)
    scene, cam, lights, r, o = _pair("cornell", w, h, st, options={"pipeline_min_px": 0})
    s = st.to_c()
    stream = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(stream)) == 0
    nbytes = h * w * 4
    bufs = [ctypes.c_void_p() for _ in range(4)]
    for b in bufs:
        assert hip.hipMalloc(ctypes.byref(b), nbytes) == 0
    want = []
    for f in range(4):
        fi = frame_inputs(f, cam, lights, w, h)
        r.render_gbuffer(fi)
        r.render_frame(s, fi)
        r.denoise(s, fi)
        r.tone_sum(s)
        r.copy_output_rows(_abi.OUT_DENOISE_INTERNAL_VARIANCE, 0, h, bufs[f].value, False, stream.value)
        o.render_gbuffer(fi)
        o.render_frame(s, fi)
        o.denoise(s, fi)
        want.append(canon_plane(16, o.output(16)))
    assert hip.hipStreamSynchronize(stream) == 0
    for f in range(4):
        out = np.empty((h, w, 4), np.uint8)
        assert hip.hipMemcpy(out.ctypes.data, bufs[f], nbytes, 2) == 0
        m = mismatch_report(canon_plane(16, out), want[f], f"frame {f} internal variance copy")
        assert not m, m
    for b in bufs:
        hip.hipFree(b)
    hip.hipStreamDestroy(stream)


def test_option_values():
    """hk_set_option: on/off switches and modes take integers only (0.5 used to count as on), the
    pixel-count thresholds any value in range; unknown keys and out-of-range values are refused."""
    from hikari_amd import HikariRenderer
    from hikari_amd._abi import HikariError
    r = HikariRenderer(0)
    for key, bad in (("gbuffer_reuse", 0.5), ("lds_scene", 1.5), ("merge", 0.3), ("lds_scene", 3), ("nope", 1)):
        with pytest.raises(HikariError):
            r.set_option(key, bad)
    r.set_option("fuse_min_px", 1234.5)
    r.set_option("lds_scene", 2)
    r.set_option("merge", -1)
    assert (r.get_option("fuse_min_px"), r.get_option("lds_scene"), r.get_option("merge")) == (1234.5, 2.0, -1.0)


def test_band_with_host_planes_under_motion_runs_whole_band():
    """A row band fed G-buffer planes through hk_set_gbuffer_plane (the raster-prepass route) with a moving
    camera: the planes carry non-zero velocity, so temporal reprojection reads other rows and every pass
    must run on the whole band.  The band's outputs with the default per-pass row windows equal those with
    band_full_windows = 1 (spatial reuse off: nothing reads the racy scatter targets)."""
    from hikari_amd import HikariRenderer, HikariSettings, Upscale, examples, frame_inputs
    w, h = 64, 192
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=False, denoise=True)
    scene, cam, lights = examples.SCENES["cornell"]()
    s = st.to_c()
    src = HikariRenderer(0)
    src.set_noise()
    src.upload_scene(scene)
    src.resize(w, h, 1.0)
    bands = []
    for full in (0, 1):
        b = HikariRenderer(0, options={"band_full_windows": full})
        b.set_noise()
        b.upload_scene(scene)
        b.set_band_halo(40)
        b.resize(w, h, 1.0, 64, 64)
        bands.append(b)
    row0, rows, core0, core_rows = bands[0].band_info()
    assert rows < h and core_rows == 64
    prev = None
    for f in range(5):
        c = copy.deepcopy(cam)
        c.transform.translation = np.array([0.03 * f, 1.0 + 0.01 * f, 4.0])
        fi = frame_inputs(f, c, lights, w, h, previous_camera=prev)
        prev = copy.deepcopy(c)
        src.render_gbuffer(fi)
        planes = [src.output(oid)[row0:row0 + rows] for oid in (11, 12, 13, 14, 15)]
        assert f == 0 or np.abs(planes[4].view(np.float32)[..., :2]).max() > 0  # motion vectors present
        for b in bands:
            for plane, data in enumerate(planes):
                b.set_gbuffer_plane(plane, data)
            b.render_frame(s, fi)
            b.denoise(s, fi)
            b.tone_sum(s)
        for oid in (1, 2, 3, 4, 5, 6, 7, 8, 9, 10):
            a, z = (canon_plane(oid, b.output(oid)[core0:core0 + core_rows]) for b in bands)
            m = mismatch_report(a, z, f"frame {f} output {oid}: row windows vs whole band")
            assert not m, m


@pytest.mark.parametrize("scene_fn", ["cornell", "city"])
def test_gbuffer_stack_bound_after_instance_updates(scene_fn):
    """The shallow G-buffer walk takes exactly the scene's stack bound (TLAS + BLAS inner levels) of LDS
    levels, a bound the runtime recomputes from the device TLAS after every hk_update_instances (ADVICE r03:
    an undercount would push past the workgroup's LDS).  After several GPU rebuilds with seeded transforms,
    the G-buffer planes of the default walk equal those of the same walk with all 16 LDS levels
    (gbuffer_stack_full), of the deep variant with its scratch stack (gbuffer_deep), of both without the
    small-frame scene staging (gbuffer_lds_max_px = 0: node loads from global memory), and the oracle's."""
    from hikari_amd import HikariRenderer, examples, frame_inputs, load_noise
    from oracle import Oracle
    from test_gpu_parity import _moved
    w, h = 128, 72
    scene, cam, lights = examples.SCENES[scene_fn]()
    ctx = []
    for opts in ({}, {"gbuffer_stack_full": 1}, {"gbuffer_deep": 1}, {"gbuffer_lds_max_px": 0},
                 {"gbuffer_lds_max_px": 0, "gbuffer_deep": 1}):
        r = HikariRenderer(0, options=opts)
        r.set_noise()
        r.upload_scene(scene)
        r.resize(w, h, 1.0)
        ctx.append(r)
    for f, seed in enumerate((3, 11, 19)):
        moved, _, _ = _moved(scene_fn, seed)
        for r in ctx:
            r.update_instances(moved.instance_models(), moved.instance_local_aabbs())
            r.render_gbuffer(frame_inputs(f, cam, lights, w, h))
        o = Oracle(moved.build(), load_noise(), w, h, 1.0)
        o.render_gbuffer(frame_inputs(f, cam, lights, w, h))
        for oid in (0, 11, 12, 13, 14):  # albedo, position, normal, depth gradient, ids (velocity: see motion tests)
            planes = [canon_plane(oid, r.output(oid)) for r in ctx]
            for k in range(1, len(ctx)):
                m = mismatch_report(planes[0], planes[k], f"update {f} output {oid}: default vs variant {k}")
                assert not m, m
            if oid != 0:  # (the oracle computes full_screen_albedo in its frame pass, not with the G-buffer)
                m = mismatch_report(planes[0], canon_plane(oid, o.output(oid)), f"update {f} output {oid} vs oracle")
                assert not m, m
