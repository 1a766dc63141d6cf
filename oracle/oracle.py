"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (oracle/_build/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
The product (bevy-hikari_amd/hikari_amd) never does.  Parity status: see hk_oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "_build" / "liboracle.so"

_L = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib() -> C.CDLL:
    global _L
    if _L is not None:
        return _L
    if not LIB.exists():
        build()
    L = C.CDLL(str(LIB))
    vp, u32, f = C.c_void_p, C.c_uint32, C.c_float
    sigs = {
        "hko_create": (vp, [vp, vp, u32, u32, f, C.c_int]),
        "hko_destroy": (None, [vp]),
        "hko_set_band": (None, [vp, C.c_int32, C.c_int32, C.c_int32]),
        "hko_set_tile": (None, [vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
        "hko_set_stripes": (None, [vp, C.c_int32, C.c_int32]),
        "hko_render_gbuffer": (None, [vp, vp]),
        "hko_set_scene": (None, [vp, vp]),
        "hko_render_frame": (None, [vp, vp, vp]),
        "hko_denoise": (None, [vp, vp, vp]),
        "hko_tone_sum": (None, [vp, vp]),
        "hko_output": (vp, [vp, C.c_int, C.POINTER(u32), C.POINTER(u32), C.POINTER(u32)]),
        "hko_reservoirs": (vp, [vp, C.c_int, C.POINTER(u32)]),
        "hko_counters": (None, [vp, vp]),
        "hko_reset_counters": (None, [vp]),
        "hko_set_light_walk": (None, [vp, C.c_int]),
        "hko_light_walk_stats": (None, [vp, vp]),
        "hko_trace": (None, [vp, vp, vp, vp, vp, u32, vp]),
        "hko_trace_ordered": (None, [vp, vp, u32, vp]),
        "hko_primary_hits": (None, [vp, vp, vp]),
        "hko_intersects_aabb": (f, [vp, vp, vp, vp]),
        "hko_intersects_triangle": (None, [vp, vp, vp, vp, vp, vp]),
        "hko_pack_reservoir_roundtrip": (None, [vp, vp, vp]),
        "hko_pow": (f, [f, f]),
        "hko_pow_int": (f, [f, C.c_int]),
        "hko_exp2": (f, [f]),
        "hko_math_form_mismatches": (None, [u32, vp]),
        "hko_exp_weight_mismatches": (C.c_uint64, [u32]),
        "hko_log2": (f, [f]),
        "hko_sin": (f, [f]),
        "hko_cos": (f, [f]),
        "hko_f32_to_f16": (u32, [f]),
        "hko_f32_to_f16_array": (None, [C.c_void_p, C.c_size_t, C.c_void_p]),
        "hko_set_textures": (C.c_int, [vp, vp, u32]),
        "hko_post_process": (None, [vp, vp, vp]),
        "hko_sample_texture": (None, [vp, u32, vp, u32, vp]),
        "hko_hash": (u32, [u32]),
        "hko_unpack_fast_mismatches": (u32, []),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _L = L
    return L


def default_threads() -> int:
    """OpenMP threads: OMP_NUM_THREADS if set (the GPU box sets it to the job's core share), else
    the cores this process may run on (os.cpu_count() counts the whole machine there)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except AttributeError:
        return os.cpu_count() or 1


class Oracle:
    """CPU restatement of one camera's integrator state (same API shape as HikariRenderer)."""

    WALK_REFERENCE, WALK_ORDERED, WALK_CHECK = 0, 1, 2

    def __init__(self, scene_desc, noise: np.ndarray, width: int, height: int, ratio: float = 1.0, threads: int = 0,
                 textures=None, light_walk: int = 0):
        """light_walk (analysis, tests/test_light_walks.py): the closest-hit light walks in light.wgsl's order (0, the
        restatement), the bounce walk with the ordered rule (1), or light.wgsl's order with every bounce ray also
        walked with the ordered rule and render_frame raising if any ray's two results differ (2, WALK_CHECK)."""
        L = lib()
        self._L = L
        self._noise = np.ascontiguousarray(noise, np.uint8)
        self.ctx = L.hko_create(C.byref(scene_desc), self._noise.ctypes.data, width, height, ratio,
                                threads or default_threads())
        self.width, self.height = width, height
        if textures:
            self.set_textures(textures)
        self.light_walk = int(light_walk)
        L.hko_set_light_walk(self.ctx, self.light_walk)

    def set_textures(self, textures):
        """Material textures (a list of hikari_amd.Texture), as hk_texture_upload."""
        from hikari_amd.scene import texture_array
        self._textures = list(textures)
        arr = texture_array(self._textures)
        self._L.hko_set_textures(self.ctx, arr, len(self._textures))

    def sample_texture(self, texture_id: int, uv: np.ndarray) -> np.ndarray:
        uv = np.ascontiguousarray(uv, np.float32).reshape(-1, 2)
        out = np.empty((len(uv), 4), np.float32)
        self._L.hko_sample_texture(self.ctx, texture_id, uv.ctypes.data, len(uv), out.ctypes.data)
        return out

    def close(self):
        if getattr(self, "ctx", None):
            self._L.hko_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        self.close()

    def set_band(self, y0: int, rows: int, halo: int = 40):
        self._L.hko_set_band(self.ctx, y0, rows, halo)

    def set_tile(self, x0: int, cols: int, y0: int, rows: int, halo: int = 40):
        """Compute only a 2-D tile plus its halo on every side (hk_resize_tile's pixels)."""
        self._L.hko_set_tile(self.ctx, x0, cols, y0, rows, halo)

    def set_stripes(self, rank: int, world: int):
        """Compute only this rank's 8-row stripes (hk_resize_striped's rows)."""
        self._L.hko_set_stripes(self.ctx, rank, world)

    def post_process(self, settings, inputs):
        self._L.hko_post_process(self.ctx, C.byref(settings), C.byref(inputs))

    def set_scene(self, scene_desc):
        """Replace the scene arrays (moved instances); the motion vectors' previous models stay."""
        self._L.hko_set_scene(self.ctx, C.byref(scene_desc))

    def render_gbuffer(self, inputs):
        self._L.hko_render_gbuffer(self.ctx, C.byref(inputs))

    def render_frame(self, settings, inputs):
        self._L.hko_render_frame(self.ctx, C.byref(settings), C.byref(inputs))
        if self.light_walk == self.WALK_CHECK:
            st = self.light_walk_stats()
            if st["bounce_differ"]:
                raise AssertionError(f"the ordered bounce walk differs from light.wgsl's order: {st}")

    def denoise(self, settings, inputs):
        self._L.hko_denoise(self.ctx, C.byref(settings), C.byref(inputs))

    def tone_sum(self, settings):
        self._L.hko_tone_sum(self.ctx, C.byref(settings))

    def output(self, output_id: int) -> np.ndarray:
        w, h, b = C.c_uint32(), C.c_uint32(), C.c_uint32()
        p = self._L.hko_output(self.ctx, output_id, C.byref(w), C.byref(h), C.byref(b))
        if not p:
            raise KeyError(output_id)
        n = w.value * h.value * b.value
        return np.frombuffer(C.string_at(p, n), np.uint8).reshape(h.value, w.value, b.value).copy()

    def reservoirs(self, buffer_id: int) -> np.ndarray:
        from hikari_amd.plugin import RESERVOIR_DTYPE
        cnt = C.c_uint32()
        p = self._L.hko_reservoirs(self.ctx, buffer_id, C.byref(cnt))
        return np.frombuffer(C.string_at(p, cnt.value * 64), RESERVOIR_DTYPE).copy()

    def load_reservoirs(self, buffer_id: int, records: np.ndarray):
        """Overwrite reservoir buffer `buffer_id` (the first len(records) records), as hk_load_reservoirs."""
        cnt = C.c_uint32()
        p = self._L.hko_reservoirs(self.ctx, buffer_id, C.byref(cnt))
        data = np.ascontiguousarray(records).view(np.uint8)
        if data.nbytes > cnt.value * 64:
            raise ValueError("more records than the buffer holds")
        C.memmove(p, data.ctypes.data, data.nbytes)

    def counters(self) -> dict:
        v = (C.c_uint64 * 4)()  # hk_counters (include/hikari_amd.h): the oracle traces every frame, [3] = 0
        self._L.hko_counters(self.ctx, v)
        return {"traverse_top": v[0], "traverse_emitter": v[1], "primary": v[2]}

    def reset_counters(self):
        self._L.hko_reset_counters(self.ctx)

    def set_light_walk(self, mode: int):
        """The closest-hit light walks: light.wgsl's order (0), the bounce walk with the ordered rule (1), or light.wgsl's
        order with every bounce and emitter walk also walked with the ordered rule and the differing rays counted (2)."""
        self.light_walk = int(mode)
        self._L.hko_set_light_walk(self.ctx, self.light_walk)

    def light_walk_stats(self) -> dict:
        v = (C.c_uint64 * 4)()
        self._L.hko_light_walk_stats(self.ctx, v)
        return {"bounce_checked": v[0], "bounce_differ": v[1], "emitter_checked": v[2], "emitter_differ": v[3]}

    def primary_hits(self, frame_inputs) -> np.ndarray:
        """(h, w, 2, 3) words: [ordered walk, reference-order walk] x (instance, primitive, distance bits)."""
        out = np.empty((self.height, self.width, 2, 3), np.uint32)
        self._L.hko_primary_hits(self.ctx, C.byref(frame_inputs), out.ctypes.data)
        return out

    def trace_ordered(self, rays) -> np.ndarray:
        """Closest-hit rays with the ordered rule; hits as trace()."""
        rays = np.ascontiguousarray(rays, np.float32)
        hits = np.empty((len(rays), 5), np.uint32)
        self._L.hko_trace_ordered(self.ctx, rays.ctypes.data, len(rays), hits.ctypes.data)
        return hits

    def trace(self, rays, max_distance=None, early_distance=None, exclude=None) -> np.ndarray:
        rays = np.ascontiguousarray(rays, np.float32)
        hits = np.empty((len(rays), 5), np.uint32)
        keep = [None if a is None else np.ascontiguousarray(a, dt)
                for a, dt in ((max_distance, np.float32), (early_distance, np.float32), (exclude, np.uint32))]
        self._L.hko_trace(self.ctx, rays.ctypes.data, *[None if a is None else a.ctypes.data for a in keep],
                          len(rays), hits.ctypes.data)
        return hits
