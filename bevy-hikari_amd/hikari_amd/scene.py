"""Scene side of the host mirror: meshes, StandardMaterial, instances, camera and lights.

What the reference gets from Bevy (glTF loader, `shape::*` meshes, `Transform`,
`PerspectiveProjection`, `DirectionalLight`, `AmbientLight`) is restated here in the
small subset the benchmark scenes need; the `mesh_material` upload path itself
(mesh -> primitives, BLAS/TLAS/light-BVH builds, alias tables) runs in the C++ builder
of libhikari_amd.so (`hks_*`, include/hikari_scene.h).
"""
from __future__ import annotations

import ctypes as C
import json
import math
import struct
from dataclasses import dataclass, field
from pathlib import Path
from typing import List, Optional, Sequence

import numpy as np

from . import _abi
from .settings import srgb_to_linear

ASSETS = Path(__file__).resolve().parent / "assets"
U32_MAX = 0xFFFFFFFF


# ---------------------------------------------------------------- math (glam conventions, column-major)
def quat_from_axis_angle(axis, angle) -> np.ndarray:
    axis = np.asarray(axis, dtype=np.float64)
    axis = axis / np.linalg.norm(axis)
    s = math.sin(0.5 * angle)
    return np.array([axis[0] * s, axis[1] * s, axis[2] * s, math.cos(0.5 * angle)])


def quat_mul(a, b) -> np.ndarray:
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw, aw * bw - ax * bx - ay * by - az * bz])


def quat_from_euler_xyz(a, b, c) -> np.ndarray:
    """glam `Quat::from_euler(EulerRot::XYZ, a, b, c)` = Rx(a) * Ry(b) * Rz(c)."""
    return quat_mul(quat_mul(quat_from_axis_angle([1, 0, 0], a), quat_from_axis_angle([0, 1, 0], b)),
                    quat_from_axis_angle([0, 0, 1], c))


def quat_to_mat3(q) -> np.ndarray:
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def mat3_to_quat(m) -> np.ndarray:
    t = m[0, 0] + m[1, 1] + m[2, 2]
    if t > 0:
        s = math.sqrt(t + 1.0) * 2
        return np.array([(m[2, 1] - m[1, 2]) / s, (m[0, 2] - m[2, 0]) / s, (m[1, 0] - m[0, 1]) / s, 0.25 * s])
    i = int(np.argmax([m[0, 0], m[1, 1], m[2, 2]]))
    j, k = (i + 1) % 3, (i + 2) % 3
    s = math.sqrt(1.0 + m[i, i] - m[j, j] - m[k, k]) * 2
    q = np.zeros(4)
    q[i] = 0.25 * s
    q[j] = (m[j, i] + m[i, j]) / s
    q[k] = (m[k, i] + m[i, k]) / s
    q[3] = (m[k, j] - m[j, k]) / s
    return q


@dataclass
class Transform:
    translation: np.ndarray = field(default_factory=lambda: np.zeros(3))
    rotation: np.ndarray = field(default_factory=lambda: np.array([0.0, 0.0, 0.0, 1.0]))
    scale: np.ndarray = field(default_factory=lambda: np.ones(3))

    @staticmethod
    def from_xyz(x, y, z) -> "Transform":
        return Transform(translation=np.array([x, y, z], dtype=np.float64))

    def looking_at(self, target, up=(0.0, 1.0, 0.0)) -> "Transform":
        """Bevy `Transform::looking_at`: forward (-Z) points at `target`."""
        back = np.asarray(self.translation, np.float64) - np.asarray(target, np.float64)
        back /= np.linalg.norm(back)
        right = np.cross(np.asarray(up, np.float64), back)
        right /= np.linalg.norm(right)
        up2 = np.cross(back, right)
        self.rotation = mat3_to_quat(np.stack([right, up2, back], axis=1))
        return self

    def matrix(self) -> np.ndarray:
        """4x4 (row-major numpy) = T * R * S (glam `from_scale_rotation_translation`)."""
        m = np.eye(4)
        m[:3, :3] = quat_to_mat3(self.rotation) * np.asarray(self.scale)[None, :]
        m[:3, 3] = self.translation
        return m

    def back(self) -> np.ndarray:
        return quat_to_mat3(self.rotation) @ np.array([0.0, 0.0, 1.0])


def col_major(m: np.ndarray) -> np.ndarray:
    """numpy 4x4 -> 16 float32 in glam's column-major order."""
    return np.ascontiguousarray(np.asarray(m, np.float64).T.reshape(16).astype(np.float32))


def perspective_infinite_reverse_rh(fov_y: float, aspect: float, near: float) -> np.ndarray:
    f = 1.0 / math.tan(0.5 * fov_y)
    m = np.zeros((4, 4))
    m[0, 0] = f / aspect
    m[1, 1] = f
    m[3, 2] = -1.0
    m[2, 3] = near
    return m


@dataclass
class Camera:
    """Camera3dBundle with Bevy's default PerspectiveProjection (fov pi/4, near 0.1)."""

    transform: Transform
    fov_y: float = math.pi / 4.0
    near: float = 0.1

    def view(self, width: int, height: int) -> _abi.hk_view:
        # the view of an unchanged camera is computed once (the per-frame host work of a static camera is then
        # a struct copy: ~80 -> ~10 us per frame_inputs)
        key = (width, height, self.fov_y, self.near, tuple(np.asarray(self.transform.translation, np.float64)),
               tuple(np.asarray(self.transform.rotation, np.float64)), tuple(np.asarray(self.transform.scale, np.float64)))
        cache = self.__dict__.setdefault("_view_cache", {})
        hit = cache.get(key)
        if hit is None:
            if len(cache) > 64:
                cache.clear()
            hit = cache[key] = self._view(width, height)
        return _abi.hk_view.from_buffer_copy(hit)

    def _view(self, width: int, height: int) -> _abi.hk_view:
        proj = perspective_infinite_reverse_rh(self.fov_y, width / height, self.near)
        world = self.transform.matrix()
        view_proj = proj @ np.linalg.inv(world)
        v = _abi.hk_view()
        for i in range(3):
            v.world_position[i] = float(np.float32(self.transform.translation[i]))
        for arr, m in ((v.view_proj, view_proj), (v.inverse_view_proj, np.linalg.inv(view_proj)), (v.projection, proj)):
            cm = col_major(m)
            for i in range(16):
                arr[i] = float(cm[i])
        return v


@dataclass
class DirectionalLight:
    """`DirectionalLightBundle`; GPU colour = linear rgba * illuminance * exposure, where Bevy 0.9's
    default exposure (f/4, 1/250 s, ISO 100: EV100 = log2(4000)) gives 1/4800."""

    illuminance: float = 100000.0
    color: tuple = (1.0, 1.0, 1.0, 1.0)  # sRGB
    transform: Transform = field(default_factory=Transform)


@dataclass
class AmbientLight:
    color: tuple = (1.0, 1.0, 1.0, 1.0)  # sRGB
    brightness: float = 0.05


def make_lights(directional: Optional[DirectionalLight], ambient: AmbientLight = AmbientLight()) -> _abi.hk_lights:
    L = _abi.hk_lights()
    if directional is not None:
        lin = [srgb_to_linear(c) for c in directional.color[:3]] + [directional.color[3]]
        intensity = directional.illuminance / (2.0 ** math.log2(4000.0) * 1.2)
        for i in range(4):
            L.directional_color[i] = float(np.float32(lin[i] * intensity))
        d = directional.transform.back()
        d = d / np.linalg.norm(d)
        for i in range(3):
            L.direction_to_light[i] = float(np.float32(d[i]))
    lin = [srgb_to_linear(c) for c in ambient.color[:3]] + [ambient.color[3]]
    for i in range(4):
        L.ambient_color[i] = float(np.float32(lin[i] * ambient.brightness))
    return L


def jitter_mode(settings) -> int:
    """The prepass shader defs of HikariSettings (prepass.rs:194-199): TEMPORAL_ANTI_ALIASING when
    taa is Jasmine, plus SMAA_TU4X when the upscaler is SMAA TU4x."""
    if settings.taa.value != 0:
        return _abi.JITTER_NONE
    return _abi.JITTER_TAA_SMAA if settings.upscale.kind == "SmaaTu4x" else _abi.JITTER_TAA


def frame_inputs(number: int, camera: Camera, lights: _abi.hk_lights, width: int, height: int,
                 previous_camera: Optional[Camera] = None, jitter: int = 0) -> _abi.hk_frame_inputs:
    """hk_frame_inputs of frame `number`.  previous_camera: the camera of the previous frame
    (PreviousViewUniform, view.rs:47-73; None = a static camera); jitter: hk_frame_inputs.jitter."""
    f = _abi.hk_frame_inputs()
    f.frame_number = int(number)
    f.jitter = int(jitter)
    f.view = camera.view(width, height)
    f.lights = lights
    if previous_camera is not None:
        f.has_previous_view = 1
        pv = previous_camera.view(width, height)
        for i in range(16):
            f.previous_view_proj[i] = pv.view_proj[i]
    return f


# ---------------------------------------------------------------- assets
@dataclass
class Mesh:
    positions: np.ndarray  # (n, 3) f32
    normals: np.ndarray    # (n, 3) f32
    uvs: np.ndarray        # (n, 2) f32
    indices: Optional[np.ndarray] = None  # u32
    topology: int = 0      # 0 = TriangleList, 1 = TriangleStrip


@dataclass
class StandardMaterial:
    """Bevy 0.9 `StandardMaterial` defaults; colours given as linear RGBA.  Texture fields hold
    indices into `Scene.textures` (the ids `MaterialTextures::id` assigns, material.rs:78-86)."""

    base_color: tuple = (1.0, 1.0, 1.0, 1.0)
    emissive: tuple = (0.0, 0.0, 0.0, 1.0)
    perceptual_roughness: float = 0.089
    metallic: float = 0.01
    reflectance: float = 0.5
    base_color_texture: Optional[int] = None
    emissive_texture: Optional[int] = None
    metallic_roughness_texture: Optional[int] = None
    normal_map_texture: Optional[int] = None
    occlusion_texture: Optional[int] = None

    def record(self) -> bytes:
        """GpuStandardMaterial std430 bytes (material.rs:162-199)."""
        def tid(t):
            return U32_MAX if t is None else int(t)
        return struct.pack("<4fI3I4fIffIfIII", *self.base_color, tid(self.base_color_texture), 0, 0, 0,
                           *self.emissive, tid(self.emissive_texture), self.perceptual_roughness, self.metallic,
                           tid(self.metallic_roughness_texture), self.reflectance, tid(self.normal_map_texture),
                           tid(self.occlusion_texture), 0)


@dataclass
class Texture:
    """One Bevy `Image` as the renderer sees it: level-0 RGBA8 texels (rows, cols, 4) + sampler.
    sRGB for base colour / emissive images, linear for metallic-roughness / occlusion."""

    rgba8: np.ndarray
    srgb: bool = True
    address_u: int = _abi.ADDRESS_REPEAT
    address_v: int = _abi.ADDRESS_REPEAT
    filter: int = _abi.FILTER_LINEAR

    def c_struct(self) -> "_abi.hk_texture":
        a = np.ascontiguousarray(self.rgba8, np.uint8)
        if a.ndim != 3 or a.shape[2] != 4:
            raise ValueError("texture texels must be (rows, cols, 4) uint8")
        self._keep = a
        return _abi.hk_texture(a.shape[1], a.shape[0],
                               _abi.TEXTURE_RGBA8_SRGB if self.srgb else _abi.TEXTURE_RGBA8_UNORM,
                               self.address_u, self.address_v, self.filter, a.ctypes.data)


def texture_array(textures) -> "C.Array":
    """ctypes array of hk_texture for hk_texture_upload / hko_set_textures (keeps texels alive
    through the Texture objects)."""
    arr = (_abi.hk_texture * max(1, len(textures)))()
    for i, t in enumerate(textures):
        arr[i] = t.c_struct()
    return arr


def plane_mesh(size: float = 1.0) -> Mesh:
    """bevy `shape::Plane` (0.9)."""
    e = size / 2.0
    pos = np.array([[e, 0, -e], [e, 0, e], [-e, 0, e], [-e, 0, -e]], np.float32)
    nrm = np.tile(np.array([[0, 1, 0]], np.float32), (4, 1))
    uv = np.array([[1, 1], [1, 0], [0, 0], [0, 1]], np.float32)
    return Mesh(pos, nrm, uv, np.array([0, 2, 1, 0, 3, 2], np.uint32))


def uv_sphere_mesh(radius: float = 0.5, sectors: int = 36, stacks: int = 18) -> Mesh:
    """bevy `shape::UVSphere` (0.9)."""
    pos, nrm, uv, idx = [], [], [], []
    sector_step = 2.0 * math.pi / sectors
    stack_step = math.pi / stacks
    for i in range(stacks + 1):
        stack_angle = math.pi / 2.0 - i * stack_step
        xy = radius * math.cos(stack_angle)
        z = radius * math.sin(stack_angle)
        for j in range(sectors + 1):
            a = j * sector_step
            x, y = xy * math.cos(a), xy * math.sin(a)
            pos.append([x, y, z])
            nrm.append([x / radius, y / radius, z / radius])
            uv.append([j / sectors, i / stacks])
    for i in range(stacks):
        k1 = i * (sectors + 1)
        k2 = k1 + sectors + 1
        for _ in range(sectors):
            if i != 0:
                idx += [k1, k2, k1 + 1]
            if i != stacks - 1:
                idx += [k1 + 1, k2, k2 + 1]
            k1 += 1
            k2 += 1
    return Mesh(np.array(pos, np.float32), np.array(nrm, np.float32), np.array(uv, np.float32),
                np.array(idx, np.uint32))


class Scene:
    """Meshes + materials + visible instances -> std430 buffers via the C++ builder."""

    def __init__(self):
        self.meshes: List[Mesh] = []
        self.materials: List[StandardMaterial] = []
        self.instances: List[tuple] = []  # (mesh, material, 4x4 numpy)
        self.textures: List[Texture] = []
        self._h = None
        self.desc: Optional[_abi.hk_scene_desc] = None

    def add_mesh(self, mesh: Mesh) -> int:
        self.meshes.append(mesh)
        return len(self.meshes) - 1

    def add_material(self, material: StandardMaterial) -> int:
        self.materials.append(material)
        return len(self.materials) - 1

    def add_texture(self, texture: "Texture") -> int:
        self.textures.append(texture)
        return len(self.textures) - 1

    def add_instance(self, mesh: int, material: int, matrix: np.ndarray) -> int:
        self.instances.append((mesh, material, np.asarray(matrix, np.float64)))
        return len(self.instances) - 1

    def build(self, buckets: int = 6) -> _abi.hk_scene_desc:
        L = _abi.lib()
        if self._h is not None:
            L.hks_destroy(self._h)
        h = L.hks_create()
        self._h = h
        keep = []
        for m in self.meshes:
            p = np.ascontiguousarray(m.positions, np.float32)
            n = np.ascontiguousarray(m.normals, np.float32)
            u = np.ascontiguousarray(m.uvs, np.float32)
            ix = None if m.indices is None else np.ascontiguousarray(m.indices, np.uint32)
            keep += [p, n, u, ix]
            rc = L.hks_add_mesh(h, p.ctypes.data, n.ctypes.data, u.ctypes.data, len(p),
                                None if ix is None else ix.ctypes.data, 0 if ix is None else len(ix), m.topology)
            if rc < 0:
                raise _abi.HikariError(f"hks_add_mesh: {L.hks_last_error(h).decode()}")
        for mat in self.materials:
            rec = C.create_string_buffer(mat.record(), 80)
            if L.hks_add_material(h, rec) < 0:
                raise _abi.HikariError("hks_add_material failed")
        for mesh, mat, m in self.instances:
            cm = col_major(m)
            if L.hks_add_instance(h, mesh, mat, cm.ctypes.data) < 0:
                raise _abi.HikariError(f"hks_add_instance: {L.hks_last_error(h).decode()}")
        if L.hks_build(h, buckets) != 0:
            raise _abi.HikariError(f"hks_build: {L.hks_last_error(h).decode()}")
        d = _abi.hk_scene_desc()
        L.hks_get_desc(h, C.byref(d))
        self.desc = d
        return d

    def instance_models(self) -> np.ndarray:
        """(n, 16) float32 column-major model matrices of the instances, in upload order."""
        return np.stack([col_major(m) for _, _, m in self.instances]).astype(np.float32)

    def instance_local_aabbs(self) -> np.ndarray:
        """(n, 6) float32 Bevy `Aabb` of each instance's mesh (center xyz, half extents xyz),
        from the mesh's vertex bounds with the builder's float operations."""
        out = np.empty((len(self.instances), 6), np.float32)
        cache = {}
        for i, (mesh, _, _) in enumerate(self.instances):
            if mesh not in cache:
                p = np.asarray(self.meshes[mesh].positions, np.float32)
                mn, mx = p.min(axis=0), p.max(axis=0)
                cache[mesh] = np.concatenate([(mn + mx) * np.float32(0.5), (mx - mn) * np.float32(0.5)])
            out[i] = cache[mesh]
        return out

    def arrays(self) -> dict:
        """numpy views (copies) of the built std430 buffers."""
        assert self.desc is not None
        out = {}
        for name, size in (("vertices", 32), ("primitives", 48), ("asset_nodes", 32), ("alias_table", 8),
                           ("instances", 176), ("instance_nodes", 32), ("materials", 80), ("emissive_nodes", 32),
                           ("emissives", 64)):
            a = getattr(self.desc, name)
            n = a.count * size
            out[name] = np.frombuffer(C.string_at(a.data, n), np.uint8).copy() if n else np.zeros(0, np.uint8)
        return out

    def __del__(self):
        if getattr(self, "_h", None) is not None and _abi._lib is not None:
            _abi._lib.hks_destroy(self._h)
            self._h = None


# ---------------------------------------------------------------- glTF / GLB (the subset Bevy's loader uses here)
_COMP = {5126: np.float32, 5125: np.uint32, 5123: np.uint16, 5121: np.uint8}
_NCOMP = {"SCALAR": 1, "VEC2": 2, "VEC3": 3, "VEC4": 4}


def _node_matrix(n: dict) -> np.ndarray:
    if "matrix" in n:
        return np.asarray(n["matrix"], np.float64).reshape(4, 4).T
    t = Transform(np.asarray(n.get("translation", [0, 0, 0]), np.float64),
                  np.asarray(n.get("rotation", [0, 0, 0, 1]), np.float64),
                  np.asarray(n.get("scale", [1, 1, 1]), np.float64))
    return t.matrix()


def load_glb(scene: Scene, path: Path, root: np.ndarray = np.eye(4)) -> None:
    """Spawn a glTF scene (SceneBundle): one Mesh asset per primitive, one StandardMaterial per glTF
    material (Bevy 0.9 loader: linear factors, reflectance 0.5), instances in node DFS order."""
    data = Path(path).read_bytes()
    magic, _, _ = struct.unpack_from("<III", data, 0)
    assert magic == 0x46546C67, "not a GLB file"
    jlen, _ = struct.unpack_from("<II", data, 12)
    g = json.loads(data[20:20 + jlen])
    off = 20 + jlen
    blen, _ = struct.unpack_from("<II", data, off)
    binary = data[off + 8: off + 8 + blen]

    def accessor(i):
        a = g["accessors"][i]
        bv = g["bufferViews"][a["bufferView"]]
        dt = np.dtype(_COMP[a["componentType"]])
        nc = _NCOMP[a["type"]]
        start = bv.get("byteOffset", 0) + a.get("byteOffset", 0)
        stride = bv.get("byteStride", dt.itemsize * nc)
        raw = np.frombuffer(binary, np.uint8, count=stride * (a["count"] - 1) + dt.itemsize * nc, offset=start)
        if stride == dt.itemsize * nc:
            return np.frombuffer(raw.tobytes(), dt).reshape(a["count"], nc)
        out = np.empty((a["count"], nc), dt)
        for k in range(a["count"]):
            out[k] = np.frombuffer(raw[k * stride: k * stride + dt.itemsize * nc].tobytes(), dt)
        return out

    mat_ids = []
    for m in g.get("materials", []):
        pbr = m.get("pbrMetallicRoughness", {})
        e = m.get("emissiveFactor", [0.0, 0.0, 0.0])
        mat_ids.append(scene.add_material(StandardMaterial(
            base_color=tuple(pbr.get("baseColorFactor", [1.0, 1.0, 1.0, 1.0])),
            emissive=(e[0], e[1], e[2], 1.0),
            perceptual_roughness=pbr.get("roughnessFactor", 1.0),
            metallic=pbr.get("metallicFactor", 1.0))))
    default_mat = None
    mesh_ids = []
    for m in g["meshes"]:
        prims = []
        for p in m["primitives"]:
            at = p["attributes"]
            pos = accessor(at["POSITION"]).astype(np.float32)
            nrm = accessor(at["NORMAL"]).astype(np.float32)
            uv = accessor(at["TEXCOORD_0"]).astype(np.float32)
            idx = accessor(p["indices"]).reshape(-1).astype(np.uint32) if "indices" in p else None
            mid = scene.add_mesh(Mesh(pos, nrm, uv, idx, 1 if p.get("mode", 4) == 5 else 0))
            if "material" in p:
                mat = mat_ids[p["material"]]
            else:
                if default_mat is None:
                    default_mat = scene.add_material(StandardMaterial())
                mat = default_mat
            prims.append((mid, mat))
        mesh_ids.append(prims)

    def visit(ni, parent):
        n = g["nodes"][ni]
        world = parent @ _node_matrix(n)
        if "mesh" in n:
            for mid, mat in mesh_ids[n["mesh"]]:
                scene.add_instance(mid, mat, world)
        for c in n.get("children", []):
            visit(c, world)

    for r in g["scenes"][g.get("scene", 0)]["nodes"]:
        visit(r, np.asarray(root, np.float64))


def load_noise() -> np.ndarray:
    return np.fromfile(ASSETS / "blue_noise_16x64x64_rgba8.bin", np.uint8)
