"""Independent pure-Python restatement of light.wgsl's `direct_lit` entry point (both variants:
RENDER_EMISSIVE and EMISSIVE_LIT) with `select_light_candidate`, the TLAS/BLAS walks, hit_info and
the Bevy PBR shading it calls (light.wgsl:77-223, 306-533, 537-708, 714-952, 1007-1017, 1044-1261;
utils.wgsl; SURVEY Appendix B for the Bevy 0.9.1 functions).

TEST INFRASTRUCTURE.  Written from the WGSL, not from oracle/hk_oracle.c or csrc/hk_device.h:
scalar float32 arithmetic (numpy float32 scalars; NEP 50 keeps Python literals weak), every WGSL
expression evaluated left to right, the build's conventions where WGSL leaves the result
implementation-defined: dot = ((x x' + y y') + z z'), normalize(v) = v * (1 / sqrt(dot)),
mix(a, b, t) = a (1 - t) + b t, min / max / clamp = IEEE minNum / maxNum, pow(x, 2 | 5) by
multiplication, f32 -> f16 round-to-nearest-even.  The transcendental primitives sin / cos / exp2
are taken from the oracle library (hko_sin / hko_cos / hko_exp2 — the build's pinned implementations,
checked separately against libm by test_transcendentals_accuracy), so any difference in a result
is a difference in the algorithm.
Scene data are the reference-format std430 arrays (leaf boxes recomputed from the triangle as
light.wgsl:411-412 does, no build-side node copies).
"""
from __future__ import annotations

import math

import numpy as np

from test_oracle_kat import np_slab, np_triangle

F = np.float32
F32_MAX = F(3.402823466e38)
F32_EPSILON = F(1.1920929e-7)
U32_MAX = 0xFFFFFFFF
LEAF = 0x80000000
RAY_BIAS = F(0.02)
DISTANCE_MAX = F(65535.0)
GOLDEN_RATIO = F(1.618033989)
TAU = F(6.283185307)
INV_TAU = F(0.159154943)
PI = F(3.141592653589793)
DONT_SAMPLE_EMISSIVE = 0x80000000
MAX_VARIANCE = F(10.0)
NODE = np.dtype([("min", "<f4", 3), ("entry", "<u4"), ("max", "<f4", 3), ("exit", "<u4")])


# ------------------------------------------------------------------ vectors (tuples of float32)
def v3(a, b, c):
    return (F(a), F(b), F(c))


def add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def mul(a, b):
    return (a[0] * b[0], a[1] * b[1], a[2] * b[2])


def scale(a, s):
    return (a[0] * s, a[1] * s, a[2] * s)


def dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def normalize(a):
    return scale(a, F(1.0) / np.sqrt(dot(a, a)))


def fmin(a, b):
    return F(np.fmin(a, b))


def fmax(a, b):
    return F(np.fmax(a, b))


def clamp(x, lo, hi):
    return fmin(fmax(x, F(lo)), F(hi))


def fract(x):
    return x - F(math.floor(x))


def lum(c):
    return dot(c, v3(0.2126, 0.7152, 0.0722))


def f2u(x):
    """u32(f32): truncation, saturating (NaN -> 0)."""
    if not (x > 0):
        return 0
    return 0xFFFFFFFF if x >= F(4294967296.0) else int(x)


def f2i(x):
    if x != x:
        return 0
    return max(-2 ** 31, min(2 ** 31 - 1, int(x)))


def f16(x):
    return F(np.float16(x))


def mat_vec(m16, v4):
    """column-major mat4 * vec4"""
    return tuple(((m16[r] * v4[0] + m16[4 + r] * v4[1]) + m16[8 + r] * v4[2]) + m16[12 + r] * v4[3] for r in range(4))


# ------------------------------------------------------------------ scene
class Scene:
    def __init__(self, arrays: dict, lib):
        self.lib = lib
        a = arrays
        self.vert = np.frombuffer(a["vertices"].tobytes(), F).reshape(-1, 8)
        self.prim = np.frombuffer(a["primitives"].tobytes(), F).reshape(-1, 3, 4)
        self.prim_u = np.frombuffer(a["primitives"].tobytes(), np.uint32).reshape(-1, 3, 4)
        self.blas = np.frombuffer(a["asset_nodes"].tobytes(), NODE)
        self.alias = np.frombuffer(a["alias_table"].tobytes(), np.uint32).reshape(-1, 2)
        self.inst_f = np.frombuffer(a["instances"].tobytes(), F).reshape(-1, 44)
        self.inst_u = self.inst_f.view(np.uint32)
        self.tlas = np.frombuffer(a["instance_nodes"].tobytes(), NODE)
        self.mat_f = np.frombuffer(a["materials"].tobytes(), F).reshape(-1, 20)
        self.lbvh = np.frombuffer(a["emissive_nodes"].tobytes(), NODE)
        self.emis_f = np.frombuffer(a["emissives"].tobytes(), F).reshape(-1, 16)
        self.emis_u = self.emis_f.view(np.uint32)

    def sin(self, x):
        return F(self.lib.hko_sin(float(x)))

    def cos(self, x):
        return F(self.lib.hko_cos(float(x)))

    def exp2(self, x):
        return F(self.lib.hko_exp2(float(x)))

    # instance fields (mod.rs:147-156 layout)
    def model(self, i):
        return self.inst_f[i, 8:24]

    def itm(self, i):
        return self.inst_f[i, 24:40]

    def mesh(self, i):
        u = self.inst_u[i]
        return int(u[40]), int(u[41]), int(u[42]), int(u[43])  # vertex, primitive, node offset, node count

    def world_to_local_point(self, i, p):
        m = self.itm(i)  # inverse model = transpose(itm): row r of it is column r of itm
        v = (p[0], p[1], p[2], F(1.0))
        r = [((m[4 * k] * v[0] + m[4 * k + 1] * v[1]) + m[4 * k + 2] * v[2]) + m[4 * k + 3] * v[3] for k in range(4)]
        return (r[0] / r[3], r[1] / r[3], r[2] / r[3])

    def world_to_local_dir(self, i, d):
        m = self.itm(i)
        v = (d[0], d[1], d[2], F(0.0))
        return tuple(((m[4 * k] * v[0] + m[4 * k + 1] * v[1]) + m[4 * k + 2] * v[2]) + m[4 * k + 3] * v[3] for k in range(3))

    def local_to_world_point(self, i, p):
        r = mat_vec(self.model(i), (p[0], p[1], p[2], F(1.0)))
        return (r[0] / r[3], r[1] / r[3], r[2] / r[3])

    def local_to_world_normal(self, i, n):
        m = self.itm(i)
        r = tuple((m[k] * n[0] + m[4 + k] * n[1]) + m[8 + k] * n[2] for k in range(3))
        return normalize(r)


# ------------------------------------------------------------------ walks (light.wgsl:400-486)
def _inv(d):
    with np.errstate(divide="ignore"):
        return np.array([F(1.0) / d[0], F(1.0) / d[1], F(1.0) / d[2]], F)


def traverse_bottom(sc, hit, origin, direction, mesh, early):
    _, poff, noff, ncount = mesh
    o = np.array(origin, F)
    d = np.array(direction, F)
    inv = _inv(direction)
    intersected = False
    j = 0
    with np.errstate(all="ignore"):
        while j < ncount:
            m = sc.blas[noff + j]
            if m["entry"] >= LEAF:
                pi = poff + int(m["entry"]) - LEAF
                t3 = sc.prim[pi][:, :3]
                mn = np.fmin(t3[0], np.fmin(t3[1], t3[2]))
                mx = np.fmax(t3[0], np.fmax(t3[1], t3[2]))
                if np_slab(o, inv, mn, mx) < hit["t"]:
                    u, v, t = np_triangle(o, d, t3[0], t3[1], t3[2])
                    if t < hit["t"]:
                        hit.update(uv=(F(u), F(v)), t=F(t), prim=pi)
                        intersected = True
                        if t < early:
                            return True
                j = int(m["exit"])
            else:
                j = int(m["entry"]) if np_slab(o, inv, m["min"], m["max"]) < hit["t"] else int(m["exit"])
    return intersected


def traverse_top(sc, origin, direction, max_distance, early, exclude):
    hit = {"uv": (F(0), F(0)), "t": F(max_distance), "inst": U32_MAX, "prim": U32_MAX}
    o = np.array(origin, F)
    inv = _inv(direction)
    i = 0
    with np.errstate(all="ignore"):
        while i < len(sc.tlas):
            n = sc.tlas[i]
            if n["entry"] >= LEAF:
                ii = int(n["entry"]) - LEAF
                if ii != exclude and np_slab(o, inv, sc.inst_f[ii, 0:3], sc.inst_f[ii, 4:7]) < hit["t"]:
                    lo = sc.world_to_local_point(ii, origin)
                    ld = sc.world_to_local_dir(ii, direction)
                    if traverse_bottom(sc, hit, lo, ld, sc.mesh(ii), early):
                        hit["inst"] = ii
                        if hit["t"] < early:
                            return hit
                i = int(n["exit"])
            else:
                i = int(n["entry"]) if np_slab(o, inv, n["min"], n["max"]) < hit["t"] else int(n["exit"])
    return hit


def empty_hit_info(position, direction):
    p = add(position, scale(direction, DISTANCE_MAX))
    return {"position": (p[0], p[1], p[2], F(0.0)), "normal": v3(0, 0, 0), "uv": (F(0), F(0)),
            "inst": U32_MAX, "mat": U32_MAX}


def hit_info(sc, origin, direction, hit):
    if hit["inst"] == U32_MAX:
        p = add(origin, scale(direction, DISTANCE_MAX))
        return {"position": (p[0], p[1], p[2], F(0.0)), "normal": v3(0, 0, 0), "uv": (F(0), F(0)),
                "inst": U32_MAX, "mat": U32_MAX}
    ii = hit["inst"]
    vbase = sc.mesh(ii)[0]
    idx = [int(sc.prim_u[hit["prim"], k, 3]) for k in range(3)]
    vs = [sc.vert[vbase + k] for k in idx]
    u, v = hit["uv"]
    uv = tuple((vs[0][c] + u * (vs[1][c] - vs[0][c])) + v * (vs[2][c] - vs[0][c]) for c in (3, 7))
    n0, n1, n2 = (tuple(vv[4:7]) for vv in vs)
    n = add(add(n0, scale(sub(n1, n0), u)), scale(sub(n2, n0), v))
    p = add(origin, scale(direction, hit["t"]))
    return {"position": (p[0], p[1], p[2], F(1.0)), "normal": sc.local_to_world_normal(ii, n), "uv": uv,
            "inst": ii, "mat": int(sc.inst_u[ii, 3])}


def occlude_hit_info(origin, direction, hit, info):
    if hit["inst"] != U32_MAX:
        p = add(origin, scale(direction, hit["t"]))
        info.update(inst=hit["inst"], mat=U32_MAX, position=(p[0], p[1], p[2], F(1.0)), normal=v3(0, 0, 0))


# ------------------------------------------------------------------ sampling (light.wgsl:537-708)
def normal_basis(n):
    s = fmin(F(np.sign(n[2])) * F(2.0) + F(1.0), F(1.0))
    u = F(-1.0) / (s + n[2])
    v = (n[0] * n[1]) * u
    t = (F(1.0) + ((s * n[0]) * n[0]) * u, s * v, -s * n[0])
    b = (v, s + (n[1] * n[1]) * u, -n[1])
    return t, b, n


def basis_mul(tbn, d):
    t, b, n = tbn
    return add(add(scale(t, d[0]), scale(b, d[1])), scale(n, d[2]))


def sample_uniform_cone(sc, rand, cos_angle):
    z = F(1.0) - (F(1.0) - cos_angle) * rand[0]
    theta = TAU * rand[1]
    r = np.sqrt(F(1.0) - z * z)
    return (r * sc.cos(theta), r * sc.sin(theta), z)


def inside_aabb(p, mn, mx):
    return (p[0] > mn[0] and p[1] > mn[1] and p[2] > mn[2]) and (p[0] < mx[0] and p[1] < mx[1] and p[2] < mx[2])


def select_light_candidate(sc, fr, rand, position, normal, instance):
    cand = {"max": F32_MAX, "min": DISTANCE_MAX, "emissive": DONT_SAMPLE_EMISSIVE, "p": F(1.0), "emitter_rays": 0}
    cone = fr["direction_to_light"]
    rand_direction = basis_mul(normal_basis(cone), sample_uniform_cone(sc, (rand[2], rand[3]), fr["cos_solar"]))
    cand["direction"] = rand_direction
    info = empty_hit_info(position, rand_direction)
    if instance == DONT_SAMPLE_EMISSIVE:
        return cand, info
    count = F(0.0)
    index = 0
    rand_1d = rand[0]
    picked = None
    while index < len(sc.lbvh):
        node = sc.lbvh[index]
        if node["entry"] >= LEAF:
            ei = int(node["entry"]) - LEAF
            e = sc.emis_f[ei]
            pos, rad = tuple(e[4:7]), e[7]
            mn = (pos[0] - rad, pos[1] - rad, pos[2] - rad)
            mx = (pos[0] + rad, pos[1] + rad, pos[2] + rad)
            if instance != int(sc.emis_u[ei, 8]) and inside_aabb(position, mn, mx):
                rand_1d = fract(rand_1d + GOLDEN_RATIO)
                count = count + F(1.0)
                if rand_1d < F(1.0) / count:
                    cand["emissive"] = int(sc.emis_u[ei, 8])
                    picked = ei
            index = int(node["exit"])
        else:
            index = int(node["entry"]) if inside_aabb(position, tuple(node["min"]), tuple(node["max"])) else int(node["exit"])
    if cand["emissive"] != DONT_SAMPLE_EMISSIVE:
        eu, ef = sc.emis_u[picked], sc.emis_f[picked]
        a_off, a_len = int(eu[10]), int(eu[11])
        alias_index = min(f2u(rand[0] * F(a_len)), a_len - 1)
        prob = sc.alias[a_off + alias_index].view(F)[0]
        primitive_index = int(sc.alias[a_off + alias_index][1]) if rand[1] < prob else alias_index
        ein = cand["emissive"]
        _, poff, _, _ = sc.mesh(ein)
        vp = [tuple(sc.prim[poff + primitive_index][k][:3]) for k in range(3)]
        srx = np.sqrt(rand[2])
        b = (F(1.0) - srx, rand[3] * srx)
        lp = add(add(scale(vp[0], b[0]), scale(vp[1], b[1])), scale(vp[2], (F(1.0) - b[0]) - b[1]))
        p = sc.local_to_world_point(ein, lp)
        origin = add(position, scale(normal, RAY_BIAS))
        direction = normalize(sub(p, position))
        hit = {"uv": (F(0), F(0)), "t": F32_MAX, "inst": U32_MAX, "prim": U32_MAX}
        cand["direction"] = direction
        traced = False
        if dot(direction, normal) > 0:
            cand["emitter_rays"] = 1
            lo = sc.world_to_local_point(ein, origin)
            ld = sc.world_to_local_dir(ein, direction)
            traced = traverse_bottom(sc, hit, lo, ld, sc.mesh(ein), F(0.0))
        if traced:
            hit["inst"] = int(eu[8])
            info = hit_info(sc, origin, direction, hit)
            cand["max"] = hit["t"]
            cand["min"] = hit["t"] - F(0.1)
            delta = sub(info["position"][:3], position)
            cand["p"] = dot(delta, delta) / abs(dot(direction, info["normal"]) * ef[12])
            cand["p"] = cand["p"] / count
        else:
            info = empty_hit_info(origin, direction)
            cand["emissive"] = DONT_SAMPLE_EMISSIVE
            cand["direction"] = rand_direction
            cand["p"] = F(1.0)
    return cand, info


# ------------------------------------------------------------------ shading (light.wgsl:714-908, Bevy 0.9.1)
def retreive_surface(sc, m):
    f = sc.mat_f[m]
    pr = clamp(f[13], 0.089, 1.0)
    return {"base": tuple(f[0:3]), "emissive": tuple(f[8:12]), "metallic": f[14], "occlusion": F(1.0),
            "roughness": pr * pr, "reflectance": f[16]}


def F_Schlick(f0, f90, voh):
    x = F(1.0) - voh
    x2 = x * x
    return f0 + (f90 - f0) * ((x2 * x2) * x)


def env_brdf_approx(sc, f0, r, nov):
    c0 = (F(-1.0), F(-0.0275), F(-0.572), F(0.022))
    c1 = (F(1.0), F(0.0425), F(1.04), F(-0.04))
    r4 = tuple(r * c0[k] + c1[k] for k in range(4))
    a004 = fmin(r4[0] * r4[0], sc.exp2(F(-9.28) * nov)) * r4[0] + r4[1]
    ab = (F(-1.04) * a004 + r4[2], F(1.04) * a004 + r4[3])
    return (f0[0] * ab[0] + ab[1], f0[1] * ab[0] + ab[1], f0[2] * ab[0] + ab[1])


def shading(sc, fr, V, N, L, surface, radiance4):
    base = surface["base"]
    refl, rough, metal, occl = surface["reflectance"], surface["roughness"], surface["metallic"], surface["occlusion"]
    f0s = ((F(0.16) * refl) * refl) * (F(1.0) - metal)
    F0 = (f0s + base[0] * metal, f0s + base[1] * metal, f0s + base[2] * metal)
    diffuse_color = scale(base, F(1.0) - metal)
    # lit (light.wgsl:796-818)
    H = normalize(add(L, V))
    NoL = clamp(dot(N, L), 0.0, 1.0)
    NoH = clamp(dot(N, H), 0.0, 1.0)
    LoH = clamp(dot(L, H), 0.0, 1.0)
    NdotV = fmax(dot(N, V), F(0.0001))
    f90 = F(0.5) + ((F(2.0) * rough) * LoH) * LoH
    fd = (F_Schlick(F(1.0), f90, NoL) * F_Schlick(F(1.0), f90, NdotV)) * (F(1.0) / PI)
    diffuse = scale(diffuse_color, fd)
    a = NoH * rough
    k = rough / ((F(1.0) - NoH * NoH) + a * a)
    D = (k * k) * (F(1.0) / PI)
    a2 = rough * rough
    lambdaV = NoL * np.sqrt((NdotV - a2 * NdotV) * NdotV + a2)
    lambdaL = NdotV * np.sqrt((NoL - a2 * NoL) * NoL + a2)
    Vis = F(0.5) / (lambdaV + lambdaL)
    fr90 = clamp(dot(F0, v3(16.5, 16.5, 16.5)), 0.0, 1.0)
    Fr = tuple(F_Schlick(F0[c], fr90, LoH) for c in range(3))
    specular = scale(Fr, (F(1.0) * D) * Vis)
    lit = scale(mul(add(specular, diffuse), radiance4[:3]), NoL)
    # ambient (light.wgsl:820-833)
    da = env_brdf_approx(sc, diffuse_color, F(1.0), NdotV)
    sa = env_brdf_approx(sc, F0, rough, NdotV)
    amb = mul(scale(add(da, sa), occl), fr["ambient"])
    t = F(1.0) - radiance4[3]
    it = F(1.0) - t
    return (lit[0] * it + amb[0] * t, lit[1] * it + amb[1] * t, lit[2] * it + amb[2] * t)


def input_radiance(sc, fr, direction, info, sample_directional, sample_emissive, sample_ambient):
    radiance, ambient = v3(0, 0, 0), F(0.0)
    if info["inst"] == U32_MAX:
        hit_directional = dot(direction, fr["direction_to_light"]) >= fr["cos_solar"]
        if sample_directional and hit_directional:
            radiance, ambient = fr["directional"], F(0.0)
        else:
            radiance = fr["ambient"] if sample_ambient else v3(0, 0, 0)
            ambient = F(1.0)
    elif sample_emissive == info["inst"]:
        e = sc.mat_f[info["mat"]][8:12]
        radiance = scale(tuple(e[:3]), F(255.0) * e[3])
    return (radiance[0], radiance[1], radiance[2], F(1.0) - ambient)


# ------------------------------------------------------------------ reservoirs (light.wgsl:77-223, 913-952)
def zero_reservoir():
    return {"radiance": (F(0),) * 4, "random": (F(0),) * 4, "visible_position": (F(0),) * 4, "visible_normal": v3(0, 0, 0),
            "visible_instance": 0, "sample_position": (F(0),) * 4, "sample_normal": v3(0, 0, 0),
            "count": F(0), "lifetime": F(0), "w": F(0), "w_sum": F(0), "w2_sum": F(0)}


SAMPLE_KEYS = ("radiance", "random", "visible_position", "visible_normal", "visible_instance", "sample_position",
               "sample_normal")


def unpack_reservoir(rec):
    """rec: 16 u32 words of a PackedReservoir (light.wgsl:35-43)."""
    w = [int(x) for x in rec]
    h = lambda u: (F(np.uint16(u & 0xFFFF).view(np.float16)), F(np.uint16(u >> 16).view(np.float16)))  # noqa: E731
    unorm = lambda u: (F(u & 0xFFFF) / F(65535.0), F(u >> 16) / F(65535.0))  # noqa: E731

    def snorm(u):
        return tuple(fmax(F(np.int8(np.uint8((u >> (8 * k)) & 0xFF))) / F(127.0), F(-1.0)) for k in range(4))

    f = np.array(w, np.uint32).view(F)
    r = zero_reservoir()
    r["count"], r["w"] = h(w[14])
    r["w_sum"], r["w2_sum"] = h(w[15])
    r["radiance"] = h(w[0]) + h(w[1])
    r["random"] = unorm(w[2]) + unorm(w[3])
    vn = snorm(w[12])
    r["visible_position"] = tuple(f[4:8])
    r["visible_normal"] = normalize(vn[:3])
    r["lifetime"] = F(127.0) * (F(1.0) + vn[3])
    sn = snorm(w[13])
    r["sample_position"] = (f[8], f[9], f[10], sn[3])
    r["sample_normal"] = normalize(sn[:3])
    r["visible_instance"] = f2u(f[11])
    return r


def pack_reservoir(r):
    def ph(a, b):
        return int(np.float16(a).view(np.uint16)) | (int(np.float16(b).view(np.uint16)) << 16)

    def pu(a, b):
        q = lambda e: int(math.floor(F(0.5) + F(65535.0) * fmin(F(1.0), fmax(F(0.0), e))))  # noqa: E731
        return q(a) | (q(b) << 16)

    def ps(v):
        out = 0
        for k, e in enumerate(v):
            q = int(math.floor(F(0.5) + F(127.0) * fmin(F(1.0), fmax(F(-1.0), F(e)))))
            out |= (q & 0xFF) << (8 * k)
        return out

    w = [0] * 16
    w[14] = ph(r["count"], r["w"])
    w[15] = ph(r["w_sum"], r["w2_sum"])
    w[0], w[1] = ph(*r["radiance"][:2]), ph(*r["radiance"][2:])
    w[2], w[3] = pu(*r["random"][:2]), pu(*r["random"][2:])
    vp = np.array(r["visible_position"], F).view(np.uint32)
    sp = np.array(list(r["sample_position"][:3]) + [F(r["visible_instance"])], F).view(np.uint32)
    w[4:8] = [int(x) for x in vp]
    w[8:12] = [int(x) for x in sp]
    w[12] = ps(tuple(r["visible_normal"]) + (r["lifetime"] / F(127.0) - F(1.0),))
    w[13] = ps(tuple(r["sample_normal"]) + (r["sample_position"][3],))
    return np.array(w, np.uint32)


def update_reservoir(r, s, w_new):
    r["w_sum"] = r["w_sum"] + w_new
    r["w2_sum"] = r["w2_sum"] + w_new * w_new
    r["count"] = r["count"] + F(1.0)
    rnd = fract(((s["random"][0] + s["random"][1]) + s["random"][2]) + s["random"][3])
    if rnd < w_new / r["w_sum"]:
        for k in SAMPLE_KEYS:
            r[k] = s[k]


def set_reservoir(r, s, w_new):
    r["count"], r["lifetime"], r["w_sum"], r["w2_sum"] = F(1.0), F(0.0), w_new, w_new * w_new
    for k in SAMPLE_KEYS:
        r[k] = s[k]


def check_previous_reservoir(r, s):
    with np.errstate(all="ignore"):
        depth_ratio = r["visible_position"][3] / s["visible_position"][3]
        depth_ratio = F(1.0) / depth_ratio if depth_ratio < 1.0 else depth_ratio
    depth_miss = depth_ratio > F(1.05) * (F(1.0) + F(0.5) * s["random"][0])
    instance_miss = r["visible_instance"] != s["visible_instance"]
    normal_miss = dot(s["visible_normal"], r["visible_normal"]) < 0.9
    if depth_miss or normal_miss or instance_miss:
        r.update(zero_reservoir())
        return False
    return True


# ------------------------------------------------------------------ direct_lit (light.wgsl:1044-1261)
def direct_lit(sc, fr, gb, noise, bufs, x, y, emissive_lit, counts):
    """One pixel of one direct pass; writes into bufs {'prev', 'cur', 'prev_spatial', 'spatial':
    (N, 16) u32 arrays; 'variance': (H, W) f32; 'render': (H, W, 4) f32 (rounded to f16)}."""
    W, H = fr["size"]
    idx = x + W * y
    n = fr["number"]
    uv = ((F(x) + F(0.5)) / F(W), (F(y) + F(0.5)) / F(H))
    j = F(-0.25) if n & 1 == 0 else F(0.25)
    duv = tuple(uv[k] + (j * (F(1.0) / F(fr["size"][k]))) * (fr["ratio"] - F(1.0)) for k in range(2))
    dx, dy = f2i(duv[0] * F(W)), f2i(duv[1] * F(H))
    pd = gb["position"][dy, dx]
    position = (pd[0], pd[1], pd[2], F(1.0))
    depth = pd[3]
    s = zero_reservoir()
    if depth < F32_EPSILON:
        r = zero_reservoir()
        set_reservoir(r, s, F(0.0))
        for b in ("cur", "spatial", "prev_spatial"):
            bufs[b][idx] = pack_reservoir(r)
        bufs["variance"][y, x] = F(0.0)
        bufs["render"][y, x] = 0.0
        return
    normal = gb["normal"][dy, dx]
    im = gb["instance_material"][dy, dx]
    im_x, im_y = f2u(im[0]), f2u(im[1])
    velocity_uv = gb["velocity_uv"][dy, dx]
    # blue noise: nearest + repeat (lib.rs:189-219)
    nu = (F(x) + F(n) + F(0.5)) / F(64.0)
    nv = (F(y) + F(n) + F(0.5)) / F(64.0)
    tx, ty = int(math.floor(fract(nu) * F(64.0))), int(math.floor(fract(nv) * F(64.0)))
    texel = noise[n % 16, ty, tx]
    fn = F(n) * GOLDEN_RATIO
    s["random"] = tuple(fract(F(t) / F(255.0) + fn) for t in texel)
    s["visible_position"] = (position[0], position[1], position[2], depth)
    s["visible_normal"] = tuple(normal)
    s["visible_instance"] = im_x
    previous_uv = (duv[0] - velocity_uv[0], duv[1] - velocity_uv[1])
    r = zero_reservoir()
    if abs(previous_uv[0] - F(0.5)) < 0.5 and abs(previous_uv[1] - F(0.5)) < 0.5:
        pc = (f2i(previous_uv[0] * F(W)), f2i(previous_uv[1] * F(H)))
        r = unpack_reservoir(bufs["prev"][pc[0] + W * pc[1]])
    inside = abs(previous_uv[0] - F(0.5)) <= 0.5 and abs(previous_uv[1] - F(0.5)) <= 0.5
    if not check_previous_reservoir(r, s) and inside:
        pc = (f2i(previous_uv[0] * F(W)), f2i(previous_uv[1] * F(H)))
        bufs["prev_spatial"][pc[0] + W * pc[1]] = pack_reservoir(r)
    interval = fr["emissive_validate_interval"] if emissive_lit else fr["direct_validate_interval"]
    select_instance = im_x if emissive_lit else DONT_SAMPLE_EMISSIVE
    vis_pos3 = s["visible_position"][:3]
    info = None
    if (n % interval if interval else 0) != 0 or r["count"] < F(4.0):
        cand, info = select_light_candidate(sc, fr, s["random"], vis_pos3, s["visible_normal"], select_instance)
        counts["emitter"] += cand["emitter_rays"]
        origin = add(position[:3], scale(normal, RAY_BIAS))
        direction = cand["direction"]
        trace = dot(direction, normal) > 0 and cand["p"] > 0
        if emissive_lit:
            trace = trace and cand["emissive"] != DONT_SAMPLE_EMISSIVE
        if trace:
            counts["top"] += 1
            hit = traverse_top(sc, origin, direction, cand["max"], cand["min"], cand["emissive"])
            occlude_hit_info(origin, direction, hit, info)
            if emissive_lit:
                s["radiance"] = input_radiance(sc, fr, direction, info, False, cand["emissive"], False)
            else:
                s["radiance"] = input_radiance(sc, fr, direction, info, True, DONT_SAMPLE_EMISSIVE, False)
        s["sample_position"] = info["position"]
        s["sample_normal"] = info["normal"]
        w_new = lum(s["radiance"][:3]) / cand["p"] if cand["p"] > 0 else F(0.0)
        update_reservoir(r, s, w_new)
        m = F(fr["max_temporal_reuse_count"])
        if r["count"] > m:
            r["w_sum"] = r["w_sum"] * (m / r["count"])
            r["w2_sum"] = r["w2_sum"] * (m / r["count"])
            r["count"] = m
    if (n % interval if interval else 0) == 0:
        cand, info = select_light_candidate(sc, fr, r["random"], r["visible_position"][:3], r["visible_normal"],
                                            select_instance)
        counts["emitter"] += cand["emitter_rays"]
        origin = add(vis_pos3, scale(s["visible_normal"], RAY_BIAS))
        direction = normalize(sub(r["sample_position"][:3], vis_pos3))
        validate_radiance = (F(0),) * 4
        trace = dot(cand["direction"], r["visible_normal"]) > 0 and cand["p"] > 0
        if emissive_lit:
            trace = trace and cand["emissive"] != DONT_SAMPLE_EMISSIVE
        if trace:
            counts["top"] += 1
            hit = traverse_top(sc, origin, direction, cand["max"], cand["min"], cand["emissive"])
            occlude_hit_info(origin, direction, hit, info)
            if emissive_lit:
                validate_radiance = input_radiance(sc, fr, direction, info, False, cand["emissive"], False)
            else:
                validate_radiance = input_radiance(sc, fr, direction, info, True, DONT_SAMPLE_EMISSIVE, False)
        if r["count"] >= F(4.0):
            s["random"] = r["random"]
            s["sample_position"] = info["position"]
            s["sample_normal"] = info["normal"]
            s["radiance"] = validate_radiance
        ratio = lum(validate_radiance[:3]) / fmax(lum(r["radiance"][:3]), F(0.0001))
        if ratio > F(1.25) or ratio < F(0.8):
            if inside:
                pc = (f2i(previous_uv[0] * F(W)), f2i(previous_uv[1] * F(H)))
                bufs["prev_spatial"][pc[0] + W * pc[1]] = pack_reservoir(r)
            w_new = lum(s["radiance"][:3]) / cand["p"] if cand["p"] > 0 else F(0.0)
            set_reservoir(r, s, w_new)
    total_lum = r["count"] * lum(r["radiance"][:3])
    r["w"] = r["w_sum"] / total_lum if total_lum > 0 else F(0.0)
    r["visible_position"] = s["visible_position"]
    r["visible_normal"] = s["visible_normal"]
    r["lifetime"] = r["lifetime"] + F(1.0)
    with np.errstate(all="ignore"):
        q = r["w_sum"] / r["count"]
        variance = r["w2_sum"] / r["count"] - q * q
        variance = variance if r["count"] < 1.0 else variance / r["count"]
    bufs["variance"][y, x] = fmin(variance, MAX_VARIANCE)
    if fr["temporal_reuse"]:
        bufs["cur"][idx] = pack_reservoir(r)
    surface = retreive_surface(sc, im_y)
    wp = position[:3]
    V = normalize(sub(fr["view_position"], wp))
    L = normalize(sub(r["sample_position"][:3], r["visible_position"][:3]))
    with np.errstate(all="ignore"):
        out = scale(shading(sc, fr, V, r["visible_normal"], L, surface, r["radiance"]), r["w"])
    if not emissive_lit:
        e = surface["emissive"]
        out = add(out, scale(tuple(e[:3]), F(255.0) * e[3]))
    bufs["render"][y, x] = [f16(out[0]), f16(out[1]), f16(out[2]), F(1.0)]
