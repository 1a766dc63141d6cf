"""Benchmark scene definitions (BASELINE.json configs), restating the reference examples.

* cornell()  — examples/cornell.rs: cornell.glb, camera (0,1,4) -> (0,1,0), no directional light.
* scene()    — examples/scene.rs layout; `models/scene.gltf` is missing from the checkout, so its
               geometry is the deterministic City proxy (see city_proxy_meshes).
* city()     — examples/city.rs layout; the Low-Poly houses are missing, so the City proxy is placed
               at the 12 house slots (city.rs:154-195).
"""
from __future__ import annotations

import json
import math
from typing import List, Tuple

import numpy as np

from .scene import (ASSETS, AmbientLight, Camera, DirectionalLight, Mesh, Scene, StandardMaterial, Transform,
                    load_glb, make_lights, plane_mesh, quat_from_axis_angle, quat_from_euler_xyz, uv_sphere_mesh,
                    _node_matrix)
from .settings import srgb_to_linear

PROXY_SEED = 0x48494B41


def cornell():
    scene = Scene()
    load_glb(scene, ASSETS / "cornell.glb")
    camera = Camera(Transform.from_xyz(0.0, 1.0, 4.0).looking_at((0.0, 1.0, 0.0)))
    lights = make_lights(None)  # cornell.rs spawns no DirectionalLight
    return scene, camera, lights


def cornell_textured():
    """cornell.rs with procedural material textures on every texture slot the integrator samples
    (light.wgsl:748-794): sRGB checker base colours (repeat / linear and mirror-repeat / nearest),
    a linear metallic-roughness gradient (clamp-to-edge), an occlusion ramp and an sRGB emissive
    pattern on the light.  The reference scene has no textures; this exercises the textured
    pipeline on the same geometry."""
    from . import _abi
    from .scene import Texture
    scene, camera, lights = cornell()
    rng = np.random.default_rng(0x48494B41)
    y, x = np.mgrid[0:64, 0:64]
    checker = (((x // 8) + (y // 8)) % 2).astype(np.uint8)
    base = np.stack([np.where(checker, 230, 60), np.where(checker, 200, 90), np.where(checker, 170, 200),
                     np.full_like(checker, 255)], axis=-1).astype(np.uint8)
    noise = rng.integers(0, 256, (16, 16, 4), dtype=np.uint8)
    noise[..., 3] = 255
    grad = np.stack([np.tile(np.linspace(0, 255, 32, dtype=np.uint8), (32, 1))] * 3
                    + [np.full((32, 32), 255, np.uint8)], axis=-1)
    ramp = np.stack([np.repeat(np.linspace(80, 255, 8, dtype=np.uint8)[:, None], 8, axis=1)] * 4, axis=-1)
    t_base = scene.add_texture(Texture(base, srgb=True, address_u=_abi.ADDRESS_REPEAT, address_v=_abi.ADDRESS_REPEAT,
                                       filter=_abi.FILTER_LINEAR))
    t_noise = scene.add_texture(Texture(noise, srgb=True, address_u=_abi.ADDRESS_MIRROR_REPEAT,
                                        address_v=_abi.ADDRESS_REPEAT, filter=_abi.FILTER_NEAREST))
    t_mr = scene.add_texture(Texture(grad, srgb=False, address_u=_abi.ADDRESS_CLAMP_TO_EDGE,
                                     address_v=_abi.ADDRESS_CLAMP_TO_EDGE, filter=_abi.FILTER_LINEAR))
    t_occ = scene.add_texture(Texture(ramp, srgb=False, address_u=_abi.ADDRESS_REPEAT,
                                      address_v=_abi.ADDRESS_MIRROR_REPEAT, filter=_abi.FILTER_LINEAR))
    for i, m in enumerate(scene.materials):
        if max(m.emissive[:3]) > 0:
            m.emissive_texture = t_noise
            continue
        m.base_color_texture = t_base if i % 2 == 0 else t_noise
        if i % 3 == 0:
            m.metallic = 0.8
            m.metallic_roughness_texture = t_mr
        if i % 3 == 1:
            m.occlusion_texture = t_occ
    return scene, camera, lights


def _srgb(c):
    return tuple([srgb_to_linear(x) for x in c[:3]] + [c[3] if len(c) > 3 else 1.0])


def box_grid_mesh(mn, mx, triangles: int, rng: np.random.Generator) -> Mesh:
    """Deterministic stand-in for a missing mesh: `triangles` triangles tessellating the surface of
    the AABB [mn, mx] (faces split into grids, small seeded jitter inwards so faces are not coplanar
    duplicates)."""
    mn = np.asarray(mn, np.float64)
    mx = np.asarray(mx, np.float64)
    ext = np.maximum(mx - mn, 1e-3)
    quads = max(1, triangles // 2)
    per_face = max(1, quads // 6)
    g = max(1, int(math.sqrt(per_face)))
    pos, nrm, uv, idx = [], [], [], []
    faces = [(0, 1, 2, -1), (0, 1, 2, +1), (1, 2, 0, -1), (1, 2, 0, +1), (2, 0, 1, -1), (2, 0, 1, +1)]
    tri_count = 0
    for f, (a, b, c, side) in enumerate(faces):
        base = len(pos)
        for i in range(g + 1):
            for j in range(g + 1):
                p = np.empty(3)
                p[a] = mn[a] + ext[a] * i / g
                p[b] = mn[b] + ext[b] * j / g
                p[c] = mx[c] if side > 0 else mn[c]
                p[c] -= side * ext[c] * 0.02 * rng.random()
                n = np.zeros(3)
                n[c] = side
                pos.append(p)
                nrm.append(n)
                uv.append([i / g, j / g])
        for i in range(g):
            for j in range(g):
                k = base + i * (g + 1) + j
                if tri_count + 2 <= triangles:
                    idx += [k, k + g + 1, k + 1, k + 1, k + g + 1, k + g + 2]
                    tri_count += 2
    # pad with thin triangles until the exact triangle count is reached
    while tri_count < triangles:
        k = len(pos)
        p = mn + ext * rng.random(3)
        pos += [p, p + ext * 0.01 * np.array([1, 0, 0]), p + ext * 0.01 * np.array([0, 1, 0])]
        nrm += [[0, 0, 1]] * 3
        uv += [[0, 0], [1, 0], [0, 1]]
        idx += [k, k + 1, k + 2]
        tri_count += 1
    return Mesh(np.array(pos, np.float32), np.array(nrm, np.float32), np.array(uv, np.float32),
                np.array(idx[: 3 * triangles], np.uint32))


def city_proxy_assets(scene: Scene):
    """Mesh + material assets of the City glTF proxy (exact per-mesh triangle counts, AABBs and
    emissive factors from assets/models/City/scene.gltf); returns a handle for city_proxy_spawn."""
    layout = json.loads((ASSETS / "city_layout.json").read_text())
    rng = np.random.default_rng(PROXY_SEED)
    mats = []
    for m in layout["materials"]:
        e = m["emissive"]
        mats.append(scene.add_material(StandardMaterial(base_color=tuple(m["base_color"]), emissive=(e[0], e[1], e[2], 1.0),
                                                        perceptual_roughness=m["roughness"], metallic=m["metallic"])))
    mesh_ids = []
    for prims in layout["meshes"]:
        ids = []
        for p in prims:
            if not (p["has_normal"] and p["has_uv"]):  # GpuMesh::try_from rejects it (mod.rs:391-397)
                ids.append(None)
                continue
            t = p["index_count"] // 3
            ids.append((scene.add_mesh(box_grid_mesh(p["min"], p["max"], t, rng)), mats[p["material"]], t))
        mesh_ids.append(ids)
    return layout, mesh_ids


def city_proxy_spawn(scene: Scene, assets, root: np.ndarray, scale: float = 1.0) -> int:
    """Spawn one SceneBundle of the proxy (instances in node DFS order). Returns traced triangles."""
    layout, mesh_ids = assets
    S = np.diag([scale, scale, scale, 1.0])
    tris = 0

    def visit(ni, parent):
        nonlocal tris
        n = layout["nodes"][ni]
        world = parent @ _node_matrix(n)
        if "mesh" in n:
            for entry in mesh_ids[n["mesh"]]:
                if entry is not None:
                    scene.add_instance(entry[0], entry[1], world)
                    tris += entry[2]
        for c in n.get("children", []):
            visit(c, world)

    for r in layout["scene_roots"]:
        visit(r, np.asarray(root, np.float64) @ S)
    return tris


def city_proxy(scene: Scene, root: np.ndarray, scale: float = 1.0) -> int:
    return city_proxy_spawn(scene, city_proxy_assets(scene), root, scale)


def _emissive_sphere(scene: Scene, translation) -> None:
    mesh = scene.add_mesh(uv_sphere_mesh(0.5))
    mat = scene.add_material(StandardMaterial(base_color=(1.0, 1.0, 1.0, 1.0), emissive=(1.0, 1.0, 1.0, 0.5)))
    t = Transform(np.asarray(translation, np.float64), quat_from_axis_angle([1, 0, 0], -math.pi / 2.0))
    scene.add_instance(mesh, mat, t.matrix())


def scene_rs():
    """examples/scene.rs with the City proxy standing in for models/scene.gltf (0.01 scale: cm -> m)."""
    scene = Scene()
    plane = scene.add_mesh(plane_mesh(1.0))
    pm = scene.add_material(StandardMaterial(base_color=_srgb((0.8, 0.7, 0.6)), perceptual_roughness=0.9))
    scene.add_instance(plane, pm, Transform(np.array([0.0, -3.0, 0.0]), scale=np.array([10000.0, 1.0, 10000.0])).matrix())
    city_proxy(scene, np.eye(4), scale=0.01)
    _emissive_sphere(scene, (2.0, 2.0, 0.0))
    sun = DirectionalLight(illuminance=100000.0,
                           transform=Transform(np.array([0.0, 5.0, 0.0]), quat_from_euler_xyz(-math.pi / 4, math.pi / 4, 0)))
    camera = Camera(Transform.from_xyz(-20.0, 10.0, 20.0).looking_at((0.0, 0.0, 0.0)))
    return scene, camera, make_lights(sun)


def city():
    """examples/city.rs with the City proxy at the 12 Low-Poly house slots (city.rs:154-195)."""
    scene = Scene()
    plane = scene.add_mesh(plane_mesh(1.0))
    pm = scene.add_material(StandardMaterial(base_color=_srgb((0.8, 0.7, 0.6)), perceptual_roughness=0.9))
    scene.add_instance(plane, pm, Transform(np.zeros(3), scale=np.array([100.0, 1.0, 100.0])).matrix())
    _emissive_sphere(scene, (0.0, 1.0, 0.0))
    slots = [(4.0 * l, 0.0, 0.0) for l in (-3, -1, 1, 3)]
    slots += [(4.0 * l, 0.0, 8.0 * (1.0 if i % 2 == 0 else -1.0)) for i, l in enumerate((-3, -1, 1, 3))]
    slots += [(4.0 * l, 0.0, 8.0 * (-1.0 if i % 2 == 0 else 1.0)) for i, l in enumerate((-3, -1, 1, 3))]
    assets = city_proxy_assets(scene)  # one asset set, 12 spawns (like one glb handle)
    for s in slots:
        city_proxy_spawn(scene, assets, Transform(np.asarray(s, np.float64)).matrix(), scale=0.0005)
    sun = DirectionalLight(illuminance=10000.0,
                           transform=Transform(np.array([0.0, 5.0, 0.0]), quat_from_euler_xyz(-math.pi / 4, math.pi / 4, 0)))
    camera = Camera(Transform.from_xyz(-20.0, 10.0, 20.0).looking_at((0.0, 0.0, 0.0)))
    return scene, camera, make_lights(sun)


SCENES = {"cornell": cornell, "cornell_textured": cornell_textured, "scene": scene_rs, "city": city}

# OrbitCameraBundle targets of the examples (cornell.rs:56-60, scene.rs:123-142, city.rs:134-138); the
# eyes are the scenes' camera translations
ORBIT_TARGETS = {"cornell": (0.0, 1.0, 0.0), "cornell_textured": (0.0, 1.0, 0.0), "scene": (0.0, 0.0, 0.0),
                 "city": (0.0, 0.0, 0.0)}
ORBIT_YAW_PER_FRAME = math.radians(0.5)  # a steady mouse orbit: 30 deg/s at 60 frames/s


def orbit(camera: Camera, target, frame: int, yaw_per_frame: float = ORBIT_YAW_PER_FRAME) -> Camera:
    """The examples' orbit camera (OrbitCameraController, user-driven in the reference) as a deterministic
    benchmark motion: the eye yawed about the vertical axis through `target` by frame * yaw_per_frame,
    looking at the target."""
    t = np.asarray(camera.transform.translation, np.float64) - np.asarray(target, np.float64)
    a = yaw_per_frame * frame
    c, s = math.cos(a), math.sin(a)
    eye = np.array([c * t[0] + s * t[2], t[1], -s * t[0] + c * t[2]]) + np.asarray(target, np.float64)
    return Camera(Transform.from_xyz(*eye).looking_at(tuple(target)))
