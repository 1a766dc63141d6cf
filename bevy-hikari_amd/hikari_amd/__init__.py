"""hikari_amd — MI355X-native drop-in for bevy-hikari's per-pixel integrator + SVGF denoiser.

Python host mirror of the reference's plugin API over the C ABI of libhikari_amd.so
(include/hikari_amd.h).  See DESIGN.md for the path, boundary and kernel layout.
"""
from . import _abi
from ._abi import HikariError
from .plugin import HikariPlugin, HikariRenderer, RESERVOIR_DTYPE
from .scene import (AmbientLight, Camera, DirectionalLight, Mesh, Scene, StandardMaterial, Texture, Transform,
                    frame_inputs, jitter_mode, load_glb, load_noise, make_lights, plane_mesh, texture_array, uv_sphere_mesh)
from .settings import HikariSettings, HikariUniversalSettings, Taa, Upscale

__all__ = [
    "HikariError", "HikariPlugin", "HikariRenderer", "RESERVOIR_DTYPE", "AmbientLight", "Camera", "DirectionalLight",
    "Mesh", "Scene", "StandardMaterial", "Texture", "texture_array", "Transform", "frame_inputs", "jitter_mode", "load_glb", "load_noise", "make_lights",
    "plane_mesh", "uv_sphere_mesh", "HikariSettings", "HikariUniversalSettings", "Taa", "Upscale", "_abi",
]
