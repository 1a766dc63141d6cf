"""`HikariPlugin` host mirror: one `HikariRenderer` per camera, driving libhikari_amd.so.

The reference's per-frame render-graph work for a `hikari` camera is
    PrepassNode::run (raster G-buffer)                 -> render_gbuffer()  (primary rays, f1)
    LightNode::run (light.rs:590-702)                  -> render_frame()
    PostProcessNode::run denoise block (post_process.rs:1190-1224) -> denoise()
    tone_mapping dispatch (post_process.rs:1226-1234)  -> tone_sum()
`HikariPlugin.frame()` runs them in that order, like the `hikari` sub-graph (lib.rs:238-367).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _abi
from .scene import Scene, load_noise, texture_array
from .settings import HikariSettings, HikariUniversalSettings

RESERVOIR_DTYPE = np.dtype([("radiance", "<u4", 2), ("random", "<u4", 2), ("visible_position", "<f4", 4),
                            ("sample_position", "<f4", 4), ("visible_normal", "<u4"), ("sample_normal", "<u4"),
                            ("reservoir", "<u4", 2)])
assert RESERVOIR_DTYPE.itemsize == 64


def _stream(stream):
    """A hipStream_t handle for the C ABI: None (the context's own stream), an integer address (e.g.
    torch.cuda.Stream.cuda_stream) or a ctypes.c_void_p; anything else is refused here, before it
    reaches HIP."""
    if stream is None or isinstance(stream, (int, C.c_void_p)):
        return stream
    raise TypeError(f"stream must be None or an integer hipStream_t handle, not {type(stream).__name__}")


def _check(ctx, rc: int, what: str) -> None:
    if rc != 0:
        msg = _abi.lib().hk_last_error(ctx).decode() if ctx else ""
        raise _abi.HikariError(f"{what} failed ({rc}): {msg}")


class HikariRenderer:
    """A camera's integrator context (hk_ctx)."""

    # options (hk_set_option) applied to every context this class creates; tests use it to force kernel
    # variants and schedules for all the contexts of a test (tests/conftest.py `hk_options`)
    defaults: dict = {}

    def __init__(self, device: int = 0, options: Optional[dict] = None):
        L = _abi.lib()
        h = C.c_void_p()
        rc = L.hk_create(device, C.byref(h))
        if rc != 0:
            raise _abi.HikariError(f"hk_create({device}) failed ({rc}): no usable gfx950 device")
        self._L = L
        self.ctx = h.value
        self.width = self.height = 0
        for k, v in {**self.defaults, **(options or {})}.items():
            self.set_option(k, v)

    def close(self):
        if getattr(self, "ctx", None):
            self._L.hk_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        self.close()

    # ---- runtime options (hk_set_option): schedule / kernel-variant choices, results unchanged
    def set_option(self, key: str, value: float) -> None:
        _check(self.ctx, self._L.hk_set_option(self.ctx, key.encode(), float(value)), f"hk_set_option({key})")

    def get_option(self, key: str) -> float:
        v = C.c_double()
        _check(self.ctx, self._L.hk_get_option(self.ctx, key.encode(), C.byref(v)), f"hk_get_option({key})")
        return v.value

    def options(self) -> dict:
        """{key: value} of every option of this context."""
        out, i = {}, 0
        while True:
            k = self._L.hk_option_name(i)
            if k is None:
                return out
            out[k.decode()] = self.get_option(k.decode())
            i += 1

    def set_options(self, opts: dict) -> dict:
        """Set several options; returns their previous values (for restoring)."""
        old = {k: self.get_option(k) for k in opts}
        for k, v in opts.items():
            self.set_option(k, v)
        return old

    # ---- resources
    def upload_scene(self, scene: Scene) -> None:
        desc = scene.desc if scene.desc is not None else scene.build()
        _check(self.ctx, self._L.hk_scene_upload(self.ctx, C.byref(desc)), "hk_scene_upload")
        tex = texture_array(scene.textures)
        _check(self.ctx, self._L.hk_texture_upload(self.ctx, tex, len(scene.textures)), "hk_texture_upload")

    def set_noise(self, noise: Optional[np.ndarray] = None) -> None:
        n = np.ascontiguousarray(load_noise() if noise is None else noise, np.uint8)
        _check(self.ctx, self._L.hk_set_noise(self.ctx, n.ctypes.data, 16, 64), "hk_set_noise")

    def resize(self, width: int, height: int, ratio: float = 1.0, band_y0: int = 0, band_rows: int = 0) -> None:
        _check(self.ctx, self._L.hk_resize(self.ctx, width, height, ratio, band_y0, band_rows), "hk_resize")
        self.width, self.height = width, height

    def resize_striped(self, width: int, height: int, rank: int, world: int) -> None:
        """Interleaved 8-row stripes rank, rank + world, ... of the frame (bands.stripes_of)."""
        _check(self.ctx, self._L.hk_resize_striped(self.ctx, width, height, rank, world), "hk_resize_striped")
        self.width, self.height = width, height

    def resize_tile(self, width: int, height: int, x0: int, cols: int, y0: int, rows: int) -> None:
        """A 2-D tile of the frame: columns [x0, x0 + cols) of rows [y0, y0 + rows) plus halo (hk_resize_tile)."""
        _check(self.ctx, self._L.hk_resize_tile(self.ctx, width, height, x0, cols, y0, rows), "hk_resize_tile")
        self.width, self.height = width, height

    def tile_info(self):
        v = [C.c_int32(), C.c_int32()]
        _check(self.ctx, self._L.hk_tile_info(self.ctx, C.byref(v[0]), C.byref(v[1])), "hk_tile_info")
        return v[0].value, v[1].value

    def copy_output_rect(self, output_id: int, row0: int, rows: int, col0: int, cols: int, dst_ptr: int,
                         dst_pitch: int = 0, to_host: bool = False, stream=None) -> None:
        _check(self.ctx, self._L.hk_copy_output_rect(self.ctx, output_id, row0, rows, col0, cols, dst_ptr, dst_pitch,
                                                     int(to_host), _stream(stream)), "hk_copy_output_rect")

    def set_band_halo(self, rows: int) -> None:
        _check(self.ctx, self._L.hk_set_band_halo(self.ctx, rows), "hk_set_band_halo")

    def copy_output_rows(self, output_id: int, row0: int, rows: int, dst_ptr: int, to_host: bool = False,
                         stream=None) -> None:
        _check(self.ctx, self._L.hk_copy_output_rows(self.ctx, output_id, row0, rows, dst_ptr, int(to_host), _stream(stream)),
               "hk_copy_output_rows")

    def band_info(self):
        v = [C.c_int32() for _ in range(4)]
        _check(self.ctx, self._L.hk_band_info(self.ctx, *[C.byref(x) for x in v]), "hk_band_info")
        return tuple(x.value for x in v)

    def band_window_grow(self, settings: _abi.hk_settings, commit: bool = False) -> np.ndarray:
        """(10, 4) int32: per reservoir buffer the (frame row, rows) above and below the band's core whose records
        the next hk_render_frame with `settings` needs from their owner bands (hk_band_window_grow); commit widens
        the band's windows without zero-filling (after the rows were loaded)."""
        ranges = np.zeros((_abi.RESERVOIR_BUFFERS, 4), np.int32)
        rc = self._L.hk_band_window_grow(self.ctx, C.byref(settings), ranges.ctypes.data, int(commit))
        _check(self.ctx, min(rc, 0), "hk_band_window_grow")
        return ranges

    def reservoir_rows_bytes(self, rows: int) -> int:
        return 4 * rows * self.width * 16

    def reservoir_rows(self, buffer_id: int, frame_row0: int, rows: int, data=None, store: bool = False,
                       stream=None):
        """Records of frame rows [frame_row0, frame_row0 + rows) of a reservoir buffer in the row-exchange layout
        (hk_reservoir_rows): store False copies them out (into `data`: a uint8 array, or a device address; a new
        array when None, returned), store True copies `data` in."""
        if data is None:
            data = np.empty(self.reservoir_rows_bytes(rows), np.uint8)
        if isinstance(data, np.ndarray):
            if not data.flags.c_contiguous or data.nbytes != self.reservoir_rows_bytes(rows):
                raise ValueError("reservoir row data must be a contiguous array of reservoir_rows_bytes(rows) bytes")
            ptr = data.ctypes.data
        else:
            ptr = int(data)
        _check(self.ctx, self._L.hk_reservoir_rows(self.ctx, buffer_id, frame_row0, rows, ptr, int(store),
                                                   _stream(stream)), "hk_reservoir_rows")
        return data

    # ---- per frame
    def render_gbuffer(self, inputs: _abi.hk_frame_inputs, stream=None) -> None:
        _check(self.ctx, self._L.hk_render_gbuffer(self.ctx, C.byref(inputs), _stream(stream)), "hk_render_gbuffer")

    def render_frame(self, settings: _abi.hk_settings, inputs: _abi.hk_frame_inputs, stream=None) -> None:
        _check(self.ctx, self._L.hk_render_frame(self.ctx, C.byref(settings), C.byref(inputs), _stream(stream)),
               "hk_render_frame")

    def denoise(self, settings: _abi.hk_settings, inputs: _abi.hk_frame_inputs, stream=None) -> None:
        _check(self.ctx, self._L.hk_denoise(self.ctx, C.byref(settings), C.byref(inputs), _stream(stream)), "hk_denoise")

    def tone_sum(self, settings: _abi.hk_settings, stream=None) -> None:
        _check(self.ctx, self._L.hk_tone_sum(self.ctx, C.byref(settings), _stream(stream)), "hk_tone_sum")

    def update_instances(self, models: np.ndarray, local_aabbs: np.ndarray, stream=None) -> None:
        """New transforms of every instance (hk_update_instances): (n, 16) column-major models and
        (n, 6) local AABBs (center, half extents); the GPU rebuilds instances, TLAS, emissives and
        the light BVH."""
        m = np.ascontiguousarray(models, np.float32).reshape(-1, 16)
        a = np.ascontiguousarray(local_aabbs, np.float32).reshape(-1, 6)
        if len(m) != len(a):
            raise ValueError("models and local_aabbs differ in length")
        _check(self.ctx, self._L.hk_update_instances(self.ctx, m.ctypes.data, a.ctypes.data, len(m), _stream(stream)),
               "hk_update_instances")

    def scene_array(self, array: int, dtype, count: int) -> np.ndarray:
        """Device copy of group-2 scene array `array` (hk_scene_desc order) as `count` records."""
        out = np.empty(count, dtype)
        _check(self.ctx, self._L.hk_read_scene_array(self.ctx, array, out.ctypes.data, out.nbytes),
               "hk_read_scene_array")
        return out

    def post_process(self, settings: _abi.hk_settings, inputs: _abi.hk_frame_inputs, stream=None) -> None:
        """SMAA TU4x + TAA Jasmine after tone mapping (hk_post_process)."""
        _check(self.ctx, self._L.hk_post_process(self.ctx, C.byref(settings), C.byref(inputs), _stream(stream)),
               "hk_post_process")

    def accumulate(self, reset: bool = False, stream=None) -> None:
        """Add the tone-mapped output to the sub-frame accumulator (hk_accumulate)."""
        _check(self.ctx, self._L.hk_accumulate(self.ctx, int(reset), _stream(stream)), "hk_accumulate")

    def resolve_accumulation(self, stream=None) -> None:
        """Accumulator / sub-frame count -> OUT_ACCUMULATED (RGBA16F)."""
        _check(self.ctx, self._L.hk_resolve_accumulation(self.ctx, _stream(stream)), "hk_resolve_accumulation")

    # ---- readback
    def output_info(self, output_id: int):
        w, h, b = C.c_uint32(), C.c_uint32(), C.c_uint32()
        _check(self.ctx, self._L.hk_output_info(self.ctx, output_id, C.byref(w), C.byref(h), C.byref(b)),
               "hk_output_info")
        return w.value, h.value, b.value

    def output(self, output_id: int) -> np.ndarray:
        """Raw bytes of an output plane as (rows, width, bytes_per_pixel) uint8."""
        w, h, b = self.output_info(output_id)
        out = np.empty((h, w, b), np.uint8)
        _check(self.ctx, self._L.hk_get_output(self.ctx, output_id, out.ctypes.data, out.nbytes, 1, None),
               "hk_get_output")
        return out

    def output_device_ptr(self, output_id: int) -> int:
        """Device address of the plane for this frame (call sync(stream) before reading it there)."""
        return self._L.hk_output_device_ptr(self.ctx, output_id)

    def set_wavefront(self, enable: bool = True) -> None:
        """Indirect pass as a wavefront with material-sorted shading (hk_set_wavefront)."""
        _check(self.ctx, self._L.hk_set_wavefront(self.ctx, int(enable)), "hk_set_wavefront")

    def sync(self, stream=None) -> None:
        """`stream` waits for the context's own streams (hk_sync)."""
        _check(self.ctx, self._L.hk_sync(self.ctx, _stream(stream)), "hk_sync")

    def set_gbuffer_plane(self, plane: int, data: np.ndarray, stream=None) -> None:
        """A host G-buffer plane (hk_set_gbuffer_plane; 0..4 = position, normal, depth gradient,
        instance/material, velocity/uv), the route that keeps the reference's raster prepass."""
        d = np.ascontiguousarray(data)
        _check(self.ctx, self._L.hk_set_gbuffer_plane(self.ctx, plane, d.ctypes.data, d.nbytes, 0, _stream(stream)),
               "hk_set_gbuffer_plane")

    def reservoirs(self, buffer_id: int) -> np.ndarray:
        w, h, _ = self.output_info(_abi.OUT_VARIANCE[0])
        out = np.empty(w * h, RESERVOIR_DTYPE)
        _check(self.ctx, self._L.hk_dump_reservoirs(self.ctx, buffer_id, out.ctypes.data, w * h, None),
               "hk_dump_reservoirs")
        return out

    def load_reservoirs(self, buffer_id: int, data: np.ndarray) -> None:
        data = np.ascontiguousarray(data, RESERVOIR_DTYPE)
        _check(self.ctx, self._L.hk_load_reservoirs(self.ctx, buffer_id, data.ctypes.data, len(data), None),
               "hk_load_reservoirs")

    def reset_counters(self) -> None:
        _check(self.ctx, self._L.hk_reset_counters(self.ctx, None), "hk_reset_counters")

    def counters(self) -> dict:
        c = _abi.hk_counters()
        _check(self.ctx, self._L.hk_read_counters(self.ctx, C.byref(c), None), "hk_read_counters")
        return {"traverse_top": c.traverse_top, "traverse_emitter": c.traverse_emitter, "primary": c.primary}

    def primary_reused(self) -> int:
        """Primary rays (included in counters()["primary"]) of frames whose G-buffer planes were reused
        rather than traced (option gbuffer_reuse)."""
        c = _abi.hk_counters()
        _check(self.ctx, self._L.hk_read_counters(self.ctx, C.byref(c), None), "hk_read_counters")
        return c.primary_reused

    def enable_kernel_timing(self, enable: bool = True) -> None:
        _check(self.ctx, self._L.hk_enable_kernel_timing(self.ctx, int(enable)), "hk_enable_kernel_timing")

    def set_kernel_timing_interval(self, every: int) -> None:
        """Time only frames whose frame_number % every == 0 (hk_set_kernel_timing_interval)."""
        _check(self.ctx, self._L.hk_set_kernel_timing_interval(self.ctx, int(every)), "hk_set_kernel_timing_interval")

    def lane_stats(self) -> dict:
        """{kernel: (active lanes, walk iterations)} of traverse_top (instrumented builds only)."""
        names = (C.c_char_p * 64)()
        act = (C.c_uint64 * 64)()
        its = (C.c_uint64 * 64)()
        n = self._L.hk_lane_stats(self.ctx, names, act, its, 64)
        return {names[i].decode(): (int(act[i]), int(its[i])) for i in range(min(n, 64))}

    def kernel_timing(self) -> dict:
        names = (C.c_char_p * 64)()
        ms = (C.c_float * 64)()
        n = self._L.hk_kernel_timing(self.ctx, names, ms, 64)
        return {names[i].decode(): float(ms[i]) for i in range(min(n, 64))}

    def trace(self, rays: np.ndarray, max_distance=None, early_distance=None, exclude=None) -> np.ndarray:
        """Stand-alone traverse_top over n rays (n, 6) -> (n, 5) uint32 {u, v, t bits, instance, primitive}."""
        rays = np.ascontiguousarray(rays, np.float32)
        n = len(rays)
        hits = np.empty((n, 5), np.uint32)
        keep = [None if a is None else np.ascontiguousarray(a, dt)
                for a, dt in ((max_distance, np.float32), (early_distance, np.float32), (exclude, np.uint32))]
        ptr = [None if a is None else a.ctypes.data for a in keep]
        _check(self.ctx, self._L.hk_trace(self.ctx, rays.ctypes.data, ptr[0], ptr[1], ptr[2], n, hits.ctypes.data, 0,
                                          None), "hk_trace")
        return hits

    def selftest_rcp(self, lo: int, hi: int) -> int:
        """f32 bit patterns in [lo, hi) (both signs) where the kernels' rcp_exact(x) != 1 / x."""
        n = C.c_uint64()
        _check(self.ctx, self._L.hk_selftest_rcp(self.ctx, lo, hi, C.byref(n)), "hk_selftest_rcp")
        return n.value

    def selftest_div(self, divisor: float, lo: int, hi: int) -> int:
        """Mismatches of the kernels' division by a frame dimension against IEEE x / divisor."""
        n = C.c_uint64()
        _check(self.ctx, self._L.hk_selftest_div(self.ctx, divisor, lo, hi, C.byref(n)), "hk_selftest_div")
        return n.value

    def selftest_f16(self, values: np.ndarray) -> np.ndarray:
        """The kernels' own f32 -> f16 conversion applied to `values` (uint16 bit patterns)."""
        v = np.ascontiguousarray(values, np.float32)
        out = np.empty(len(v), np.uint16)
        _check(self.ctx, self._L.hk_selftest_f16(self.ctx, v.ctypes.data, len(v), out.ctypes.data), "hk_selftest_f16")
        return out


class HikariPlugin:
    """`app.add_plugin(HikariPlugin)` for one camera: owns the renderer and the frame counter
    (`FrameCounter`, view.rs:75-103; frame numbers 0, 1, 2, ...)."""

    def __init__(self, scene: Scene, settings: HikariSettings = None, device: int = 0,
                 universal: HikariUniversalSettings = None):
        self.settings = settings or HikariSettings()
        self.universal = universal or HikariUniversalSettings()
        self.renderer = HikariRenderer(device)
        self.renderer.set_noise()
        if self.universal.build_mesh_acceleration_structure and self.universal.build_instance_acceleration_structure:
            self.renderer.upload_scene(scene)
        self.frame_number = 0
        self._previous_camera = None

    def resize(self, width: int, height: int, band_y0: int = 0, band_rows: int = 0):
        self.renderer.resize(width, height, self.settings.upscale.ratio(), band_y0, band_rows)

    def frame(self, camera, lights, gbuffer: bool = True, stream=None) -> None:
        """One frame.  The previous frame's camera is the PreviousViewUniform of the motion vectors
        (view.rs:47-73; the first frame has none: static) and the prepass jitters the primary rays
        when TAA is on (prepass.rs:194-199)."""
        import copy

        from .scene import frame_inputs, jitter_mode
        r = self.renderer
        s = self.settings.to_c()
        fi = frame_inputs(self.frame_number, camera, lights, r.width, r.height,
                          previous_camera=self._previous_camera, jitter=jitter_mode(self.settings))
        self._previous_camera = copy.deepcopy(camera)
        if gbuffer:
            r.render_gbuffer(fi, stream)
        r.render_frame(s, fi, stream)
        if self.settings.denoise:
            r.denoise(s, fi, stream)
        r.tone_sum(s, stream)
        self.frame_number += 1
