"""ctypes mirror of include/hikari_amd.h and include/hikari_scene.h.

The product path is libhikari_amd.so (HIP kernels for gfx950).  Loading fails loudly if the
library is missing: there is no CPU fallback anywhere in this package.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ["HK_LIB"]) if os.environ.get("HK_LIB") else HERE / "libhikari_amd.so"  # HK_LIB: experiment builds

HK_OK = 0
HK_ERR_INVALID = -1
HK_ERR_HIP = -2
HK_ERR_STATE = -3
HK_ERR_NO_DEVICE = -4

RESERVOIR_BUFFERS = 10  # HK_RESERVOIR_BUFFERS

# hk_output_id
OUT_ALBEDO = 0
OUT_VARIANCE = (1, 2, 3)
OUT_RENDER = (4, 5, 6)
OUT_DENOISED = (7, 8, 9)
OUT_TONE_MAPPED = 10
OUT_GBUF_POSITION = 11
OUT_GBUF_NORMAL = 12
OUT_GBUF_DEPTH_GRADIENT = 13
OUT_GBUF_INSTANCE_MATERIAL = 14
OUT_GBUF_VELOCITY_UV = 15
OUT_ACCUMULATED = 17
OUT_UPSCALED = 18
OUT_TAA = 19
OUT_TONE_MAPPED_PREVIOUS = 20
OUT_DENOISE_INTERNAL_VARIANCE = 16
RESERVOIR_BUFFERS = 10


class hk_array(C.Structure):
    _fields_ = [("data", C.c_void_p), ("count", C.c_uint32)]


class hk_scene_desc(C.Structure):
    _fields_ = [(n, hk_array) for n in ("vertices", "primitives", "asset_nodes", "alias_table", "instances",
                                       "instance_nodes", "materials", "emissive_nodes", "emissives")]


class hk_texture(C.Structure):
    """include/hikari_amd.h hk_texture (one GpuImage level 0 + its sampler)."""
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("format", C.c_uint32), ("address_u", C.c_uint32),
                ("address_v", C.c_uint32), ("filter", C.c_uint32), ("rgba8", C.c_void_p)]


TEXTURE_RGBA8_SRGB, TEXTURE_RGBA8_UNORM = 0, 1
ADDRESS_CLAMP_TO_EDGE, ADDRESS_REPEAT, ADDRESS_MIRROR_REPEAT = 0, 1, 2
FILTER_NEAREST, FILTER_LINEAR = 0, 1


class hk_settings(C.Structure):
    _fields_ = [
        ("direct_validate_interval", C.c_uint32),
        ("emissive_validate_interval", C.c_uint32),
        ("max_temporal_reuse_count", C.c_uint32),
        ("max_spatial_reuse_count", C.c_uint32),
        ("max_reservoir_lifetime", C.c_float),
        ("solar_angle", C.c_float),
        ("indirect_bounces", C.c_uint32),
        ("max_indirect_luminance", C.c_float),
        ("clear_color", C.c_float * 4),
        ("temporal_reuse", C.c_uint32),
        ("emissive_spatial_reuse", C.c_uint32),
        ("indirect_spatial_reuse", C.c_uint32),
        ("denoise", C.c_uint32),
        ("taa", C.c_uint32),
        ("upscale_ratio", C.c_float),
        ("upscale", C.c_uint32),
    ]


class hk_view(C.Structure):
    _fields_ = [
        ("world_position", C.c_float * 3),
        ("_pad0", C.c_float),
        ("view_proj", C.c_float * 16),
        ("inverse_view_proj", C.c_float * 16),
        ("projection", C.c_float * 16),
    ]


class hk_lights(C.Structure):
    _fields_ = [
        ("directional_color", C.c_float * 4),
        ("direction_to_light", C.c_float * 3),
        ("_pad0", C.c_float),
        ("ambient_color", C.c_float * 4),
    ]


JITTER_NONE, JITTER_TAA, JITTER_TAA_SMAA = 0, 1, 2


class hk_frame_inputs(C.Structure):
    _fields_ = [("frame_number", C.c_uint32), ("jitter", C.c_uint32), ("has_previous_view", C.c_uint32),
                ("_pad", C.c_uint32), ("view", hk_view), ("lights", hk_lights),
                ("previous_view_proj", C.c_float * 16)]


class hk_counters(C.Structure):
    _fields_ = [("traverse_top", C.c_uint64), ("traverse_emitter", C.c_uint64), ("primary", C.c_uint64),
                ("primary_reused", C.c_uint64)]


# std430 record sizes (include/hk_types.h)
SIZEOF = {"vertex": 32, "primitive": 48, "node": 32, "alias": 8, "instance": 176, "material": 80, "emissive": 64,
          "reservoir": 64}


class HikariError(RuntimeError):
    pass


_lib = None


def lib() -> C.CDLL:
    """Load libhikari_amd.so (built by `make -C bevy-hikari_amd`). Raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise HikariError(f"{LIB_PATH} is missing: build it with `make -C bevy-hikari_amd` "
                          "(no CPU fallback exists for the integrator)")
    L = C.CDLL(str(LIB_PATH))
    vp, i32, u32 = C.c_void_p, C.c_int, C.c_uint32
    sig = {
        "hk_abi_version": (i32, []),
        "hk_create": (i32, [i32, C.POINTER(vp)]),
        "hk_destroy": (None, [vp]),
        "hk_last_error": (C.c_char_p, [vp]),
        "hk_settings_default": (None, [C.POINTER(hk_settings)]),
        "hk_set_option": (i32, [vp, C.c_char_p, C.c_double]),
        "hk_get_option": (i32, [vp, C.c_char_p, C.POINTER(C.c_double)]),
        "hk_option_name": (C.c_char_p, [i32]),
        "hk_scene_upload": (i32, [vp, C.POINTER(hk_scene_desc)]),
        "hk_set_noise": (i32, [vp, vp, u32, u32]),
        "hk_texture_upload": (i32, [vp, vp, u32]),
        "hk_resize": (i32, [vp, u32, u32, C.c_float, u32, u32]),
        "hk_set_band_halo": (i32, [vp, u32]),
        "hk_resize_striped": (i32, [vp, u32, u32, u32, u32]),
        "hk_band_info": (i32, [vp] + [C.POINTER(C.c_int32)] * 4),
        "hk_band_window_grow": (i32, [vp, C.POINTER(hk_settings), vp, i32]),
        "hk_resize_tile": (i32, [vp, u32, u32, u32, u32, u32, u32]),
        "hk_tile_info": (i32, [vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
        "hk_copy_output_rect": (i32, [vp, i32, u32, u32, u32, u32, vp, C.c_size_t, i32, vp]),
        "hk_reservoir_rows": (i32, [vp, i32, C.c_int32, C.c_int32, vp, i32, vp]),
        "hk_copy_output_rows": (i32, [vp, i32, u32, u32, vp, i32, vp]),
        "hk_render_gbuffer": (i32, [vp, C.POINTER(hk_frame_inputs), vp]),
        "hk_set_gbuffer_plane": (i32, [vp, i32, vp, C.c_size_t, i32, vp]),
        "hk_render_frame": (i32, [vp, C.POINTER(hk_settings), C.POINTER(hk_frame_inputs), vp]),
        "hk_denoise": (i32, [vp, C.POINTER(hk_settings), C.POINTER(hk_frame_inputs), vp]),
        "hk_tone_sum": (i32, [vp, C.POINTER(hk_settings), vp]),
        "hk_accumulate": (i32, [vp, i32, vp]),
        "hk_post_process": (i32, [vp, C.POINTER(hk_settings), C.POINTER(hk_frame_inputs), vp]),
        "hk_update_instances": (i32, [vp, vp, vp, u32, vp]),
        "hk_read_scene_array": (i32, [vp, i32, vp, C.c_size_t]),
        "hk_resolve_accumulation": (i32, [vp, vp]),
        "hk_output_info": (i32, [vp, i32, C.POINTER(u32), C.POINTER(u32), C.POINTER(u32)]),
        "hk_get_output": (i32, [vp, i32, vp, C.c_size_t, i32, vp]),
        "hk_output_device_ptr": (vp, [vp, i32]),
        "hk_sync": (i32, [vp, vp]),
        "hk_set_wavefront": (i32, [vp, i32]),
        "hk_lane_stats": (i32, [vp, C.POINTER(C.c_char_p), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), i32]),
        "hk_dump_reservoirs": (i32, [vp, i32, vp, C.c_size_t, vp]),
        "hk_load_reservoirs": (i32, [vp, i32, vp, C.c_size_t, vp]),
        "hk_reset_counters": (i32, [vp, vp]),
        "hk_read_counters": (i32, [vp, C.POINTER(hk_counters), vp]),
        "hk_enable_kernel_timing": (i32, [vp, i32]),
        "hk_kernel_timing": (i32, [vp, C.POINTER(C.c_char_p), C.POINTER(C.c_float), i32]),
        "hk_set_kernel_timing_interval": (i32, [vp, u32]),
        "hk_trace": (i32, [vp, vp, vp, vp, vp, u32, vp, i32, vp]),
        "hk_selftest_f16": (i32, [vp, vp, u32, vp]),
        "hk_selftest_div": (i32, [vp, C.c_float, u32, u32, C.POINTER(C.c_uint64)]),
        "hk_selftest_rcp": (i32, [vp, u32, u32, C.POINTER(C.c_uint64)]),
        "hks_create": (vp, []),
        "hks_destroy": (None, [vp]),
        "hks_last_error": (C.c_char_p, [vp]),
        "hks_add_mesh": (i32, [vp, vp, vp, vp, u32, vp, u32, i32]),
        "hks_add_material": (i32, [vp, vp]),
        "hks_add_instance": (i32, [vp, u32, u32, vp]),
        "hks_build": (i32, [vp, i32]),
        "hks_get_desc": (i32, [vp, C.POINTER(hk_scene_desc)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


# symbols include/*.h declare (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = [
    "hk_abi_version", "hk_create", "hk_destroy", "hk_last_error", "hk_settings_default", "hk_set_option",
    "hk_get_option", "hk_option_name", "hk_scene_upload",
    "hk_set_noise", "hk_texture_upload", "hk_resize", "hk_resize_striped", "hk_set_band_halo", "hk_band_info", "hk_band_window_grow", "hk_reservoir_rows", "hk_resize_tile", "hk_tile_info", "hk_copy_output_rect", "hk_copy_output_rows", "hk_render_gbuffer", "hk_set_gbuffer_plane", "hk_render_frame",
    "hk_denoise", "hk_tone_sum", "hk_update_instances", "hk_read_scene_array", "hk_post_process", "hk_accumulate", "hk_resolve_accumulation", "hk_output_info", "hk_get_output", "hk_output_device_ptr", "hk_sync", "hk_set_wavefront", "hk_lane_stats", "hk_dump_reservoirs",
    "hk_load_reservoirs", "hk_reset_counters", "hk_read_counters", "hk_enable_kernel_timing", "hk_kernel_timing", "hk_set_kernel_timing_interval",
    "hk_trace", "hk_selftest_f16", "hk_selftest_div", "hk_selftest_rcp", "hks_create", "hks_destroy", "hks_last_error", "hks_add_mesh", "hks_add_material",
    "hks_add_instance", "hks_build", "hks_get_desc",
]


def gpu_visible() -> bool:
    """True when a HIP device may be present (never initialises the GPU itself)."""
    return bool(os.environ.get("HIP_VISIBLE_DEVICES", "x")) and Path("/dev/kfd").exists()
