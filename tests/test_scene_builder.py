"""Host scene builder (mesh_material upload path restated in C++): buffer layouts, skip-pointer
BVH invariants of bvh 0.7.1's flatten_custom, alias tables, emissive list (instance.rs:377-428)."""
import numpy as np
import pytest

NODE = np.dtype([("min", "<f4", 3), ("entry", "<u4"), ("max", "<f4", 3), ("exit", "<u4")])
LEAF = 0x80000000


def nodes_of(arrs, name):
    return np.frombuffer(arrs[name].tobytes(), NODE)


def check_skip_bvh(nodes, shape_count, leaf_bounds=None):
    """DFS skip-pointer invariants: 3n-2 nodes; entry = next for inner; exit > index; walking
    with every AABB test true visits every node once and every shape once."""
    n = len(nodes)
    if shape_count == 0:
        assert n == 0
        return
    assert n == 3 * shape_count - 2
    seen = []
    i = 0
    steps = 0
    while i < n:
        e, x = int(nodes[i]["entry"]), int(nodes[i]["exit"])
        assert x > i and x <= n
        if e >= LEAF:
            seen.append(e - LEAF)
            assert x == i + 1
            i = x
        else:
            assert e == i + 1
            i = e
        steps += 1
    assert steps == n
    assert sorted(seen) == list(range(shape_count))
    # exit of an entry node skips exactly its subtree: the leaves reachable between i+1 and exit
    # all lie inside the entry node's AABB
    if leaf_bounds is not None:
        for i in range(n):
            e, x = int(nodes[i]["entry"]), int(nodes[i]["exit"])
            if e < LEAF:
                mn, mx = nodes[i]["min"], nodes[i]["max"]
                for j in range(i + 1, x):
                    ej = int(nodes[j]["entry"])
                    if ej >= LEAF:
                        lb = leaf_bounds[ej - LEAF]
                        assert np.all(lb[0] >= mn - 1e-6) and np.all(lb[1] <= mx + 1e-6)


def test_cornell_buffers():
    from hikari_amd import examples
    scene, cam, lights = examples.cornell()
    d = scene.build()
    counts = {n: getattr(d, n).count for n in ("vertices", "primitives", "asset_nodes", "alias_table", "instances",
                                                "instance_nodes", "materials", "emissive_nodes", "emissives")}
    # 78 vtx, 32 prims, 8 inst, 8 mats, 1 emissive (2 alias entries), 80 BLAS + 22 TLAS + 1 light nodes
    assert counts == {"vertices": 78, "primitives": 32, "asset_nodes": 80, "alias_table": 2, "instances": 8,
                      "instance_nodes": 22, "materials": 8, "emissive_nodes": 1, "emissives": 1}
    arrs = scene.arrays()
    inst = np.frombuffer(arrs["instances"].tobytes(), np.uint8).reshape(-1, 176)
    # TLAS over instance AABBs
    ib = []
    for row in inst:
        f = row.view(np.float32)
        ib.append((f[0:3], f[4:7]))
    check_skip_bvh(nodes_of(arrs, "instance_nodes"), 8, ib)
    # each mesh's BLAS
    prims = np.frombuffer(arrs["primitives"].tobytes(), np.float32).reshape(-1, 12)
    blas = nodes_of(arrs, "asset_nodes")
    for row in inst:
        u = row.view(np.uint32)
        voff, poff, noff, nlen = u[40], u[41], u[42], u[43]
        sub = blas[noff:noff + nlen]
        nprim = (nlen + 2) // 3
        pb = []
        for k in range(nprim):
            t = prims[poff + k].reshape(3, 4)[:, :3]
            pb.append((t.min(0), t.max(0)))
        check_skip_bvh(sub, nprim, pb)
    # the light: emissive 1,1,1 -> intensity 255*sqrt(3); radius = half diagonal + sqrt(intensity)
    em = np.frombuffer(arrs["emissives"].tobytes(), np.uint8)
    f = em.view(np.float32)
    u = em.view(np.uint32)
    assert list(f[0:4]) == [1.0, 1.0, 1.0, 1.0]
    light = inst[u[8]].view(np.float32)
    half_diag = 0.5 * np.linalg.norm(light[4:7] - light[0:3])
    assert f[7] == pytest.approx(half_diag + np.sqrt(255.0 * np.sqrt(3.0)), rel=1e-5)
    assert u[10] == 0 and u[11] == 2  # alias table (offset, length)


def test_alias_table_reproduces_area_distribution():
    """GpuMesh::build_alias_table (mod.rs:330-376): P(pick i) = (1 - prob_i + sum_{j: alias_j = i} prob_j)/n."""
    from hikari_amd import Scene, StandardMaterial
    from hikari_amd.scene import Mesh
    rng = np.random.default_rng(1)
    pos, idx = [], []
    areas = []
    for t in range(9):
        s = 0.2 + rng.random() * 2.0
        base = np.array([t * 3.0, 0, 0])
        pos += [base, base + [s, 0, 0], base + [0, s * (1 + t % 3), 0]]
        idx += [3 * t, 3 * t + 1, 3 * t + 2]
        areas.append(0.5 * s * s * (1 + t % 3))
    pos = np.array(pos, np.float32)
    mesh = Mesh(pos, np.tile([[0, 0, 1]], (len(pos), 1)).astype(np.float32), np.zeros((len(pos), 2), np.float32),
                np.array(idx, np.uint32))
    sc = Scene()
    m = sc.add_mesh(mesh)
    mat = sc.add_material(StandardMaterial(emissive=(1.0, 0.5, 0.2, 1.0)))
    sc.add_instance(m, mat, np.eye(4))
    sc.build()
    arrs = sc.arrays()
    alias = np.frombuffer(arrs["alias_table"].tobytes(), [("prob", "<f4"), ("index", "<u4")])
    n = len(alias)
    assert n == 9
    p = np.zeros(n)
    for i, e in enumerate(alias):
        p[i] += (1.0 - e["prob"]) / n
        p[e["index"]] += e["prob"] / n
    want = np.array(areas) / np.sum(areas)
    assert np.allclose(p, want, atol=1e-5)
    em = np.frombuffer(arrs["emissives"].tobytes(), np.float32)
    assert em[12] == pytest.approx(np.sum(areas), rel=1e-5)  # surface_area


def test_mesh_errors_match_prepare_mesh_error():
    import ctypes as C

    import hikari_amd
    L = hikari_amd._abi.lib()
    h = L.hks_create()
    p = np.zeros((3, 3), np.float32)
    uv = np.zeros((3, 2), np.float32)
    assert L.hks_add_mesh(h, p.ctypes.data, None, uv.ctypes.data, 3, None, 0, 0) == -11  # MissingAttributeNormal
    assert L.hks_add_mesh(h, p.ctypes.data, p.ctypes.data, None, 3, None, 0, 0) == -12   # MissingAttributeUV
    ix = np.array([0, 1], np.uint32)
    assert L.hks_add_mesh(h, p.ctypes.data, p.ctypes.data, uv.ctypes.data, 3, ix.ctypes.data, 2, 0) == -13
    assert L.hks_add_mesh(h, p.ctypes.data, p.ctypes.data, uv.ctypes.data, 3, None, 0, 5) == -13
    assert L.hks_add_mesh(h, p.ctypes.data, p.ctypes.data, uv.ctypes.data, 3, None, 0, 0) == 0
    # triangle strip: winding alternates (mod.rs:431-445)
    p4 = np.zeros((4, 3), np.float32)
    uv4 = np.zeros((4, 2), np.float32)
    assert L.hks_add_mesh(h, p4.ctypes.data, p4.ctypes.data, uv4.ctypes.data, 4, None, 0, 1) == 1
    L.hks_destroy(h)


def test_city_proxy_triangle_count():
    """The City proxy keeps the glTF JSON's per-mesh triangle counts (139,865 traced)."""
    from hikari_amd import Scene, examples
    sc = Scene()
    tris = examples.city_proxy(sc, np.eye(4))
    assert tris == 139865
    assert sum(len(m.indices) // 3 for m in sc.meshes) == 139865


def test_large_bvh_invariants():
    from hikari_amd import Scene, StandardMaterial
    from hikari_amd.scene import Mesh
    rng = np.random.default_rng(3)
    n = 3000
    c = rng.random((n, 3)).astype(np.float32) * 10
    pos = np.concatenate([c, c + [0.1, 0, 0], c + [0, 0.1, 0]], axis=1).reshape(-1, 3).astype(np.float32)
    mesh = Mesh(pos, np.tile([[0, 0, 1]], (len(pos), 1)).astype(np.float32), np.zeros((len(pos), 2), np.float32))
    sc = Scene()
    m = sc.add_mesh(mesh)
    mat = sc.add_material(StandardMaterial())
    sc.add_instance(m, mat, np.eye(4))
    sc.build()
    arrs = sc.arrays()
    prims = np.frombuffer(arrs["primitives"].tobytes(), np.float32).reshape(-1, 12)
    pb = [(p.reshape(3, 4)[:, :3].min(0), p.reshape(3, 4)[:, :3].max(0)) for p in prims]
    check_skip_bvh(nodes_of(arrs, "asset_nodes"), n, pb)
