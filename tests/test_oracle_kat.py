"""Pins the CPU oracle with independent known-answer restatements (numpy / pure Python).

The reference ships no tests or golden vectors and cannot run here, so
these KATs restate the WGSL building blocks a second time, independently of oracle/hk_oracle.c:
utils.wgsl hash/random_float, the WGSL pack*/unpack* built-ins (pack_reservoir/unpack_reservoir,
light.wgsl:77-136), the slab test (light.wgsl:344-362), Möller–Trumbore (light.wgsl:364-398),
the stackless TLAS/BLAS walk (light.wgsl:400-486) and the à-trous denoiser (denoise.wgsl).
"""
import ctypes as C
import math

import numpy as np
import pytest

f32 = np.float32


# ------------------------------------------------------------------ utils.wgsl
def py_hash(v):
    m = 0xFFFFFFFF
    s = v & m
    s ^= 2747636419
    s = (s * 2654435769) & m
    s ^= s >> 16
    s = (s * 2654435769) & m
    s ^= s >> 16
    s = (s * 2654435769) & m
    return s


def test_hash_known_answers(oracle_lib):
    rng = np.random.default_rng(0)
    for v in [0, 1, 2, 3, 15, 16, 255, 2 ** 31, 2 ** 32 - 1] + list(rng.integers(0, 2 ** 32, 200)):
        assert oracle_lib.hko_hash(int(v)) == py_hash(int(v))
    assert py_hash(0) == oracle_lib.hko_hash(0)


# ------------------------------------------------------------------ packing
def test_f32_to_f16_matches_ieee_rne(oracle_lib):
    rng = np.random.default_rng(1)
    vals = np.concatenate([
        rng.standard_normal(20000).astype(f32) * f32(100),
        rng.uniform(-1, 1, 5000).astype(f32) * f32(6e-5),           # f16 subnormal range
        np.array([0.0, -0.0, 65504.0, 65519.9, 65520.0, 1e9, -1e9, np.inf, -np.inf, 5.9604645e-08,
                  2.9802322e-08, 2.98023259e-08, 1.0009765625, 1.00048828125, 1.00146484375], f32)])
    # exact halfway cases between consecutive f16 values
    h = np.arange(0x0001, 0x7BFF, 97, dtype=np.uint16)
    lo = h.view(np.float16).astype(f32)
    hi = (h + 1).view(np.float16).astype(f32)
    vals = np.concatenate([vals, ((lo.astype(np.float64) + hi.astype(np.float64)) / 2).astype(f32)])
    want = vals.astype(np.float16).view(np.uint16)
    got = np.array([oracle_lib.hko_f32_to_f16(float(v)) for v in vals], np.uint16)
    assert np.array_equal(got, want), f"{int((got != want).sum())} mismatches"


def np_pack_reservoir(fl):
    """Independent restatement of pack_reservoir (light.wgsl:111-136) with numpy's IEEE f16."""
    def pk16f(a, b):
        return int(np.array([a], f32).astype(np.float16).view(np.uint16)[0]) | \
            (int(np.array([b], f32).astype(np.float16).view(np.uint16)[0]) << 16)

    def unorm16(e):
        return int(np.rint(np.clip(f32(e), f32(0), f32(1)) * f32(65535.0)))

    def snorm8(e):
        return int(np.rint(np.clip(f32(e), f32(-1), f32(1)) * f32(127.0))) & 0xFF

    count, w, w_sum, w2_sum, lifetime = fl[0:5]
    rad, rnd, vp, vn, vi, sp, sn = fl[5:9], fl[9:13], fl[13:17], fl[17:20], fl[20], fl[21:25], fl[25:28]
    words = [pk16f(rad[0], rad[1]), pk16f(rad[2], rad[3]),
             unorm16(rnd[0]) | (unorm16(rnd[1]) << 16), unorm16(rnd[2]) | (unorm16(rnd[3]) << 16)]
    words += list(np.array(vp, f32).view(np.uint32))
    words += list(np.array([sp[0], sp[1], sp[2], f32(int(vi))], f32).view(np.uint32))
    lw = f32(f32(lifetime) / f32(127.0)) - f32(1.0)
    words.append(snorm8(vn[0]) | snorm8(vn[1]) << 8 | snorm8(vn[2]) << 16 | snorm8(lw) << 24)
    words.append(snorm8(sn[0]) | snorm8(sn[1]) << 8 | snorm8(sn[2]) << 16 | snorm8(sp[3]) << 24)
    words += [pk16f(count, w), pk16f(w_sum, w2_sum)]
    return np.array(words, np.uint32)


def test_pack_reservoir_roundtrip(oracle_lib):
    rng = np.random.default_rng(2)
    for trial in range(300):
        n1 = rng.standard_normal(3)
        n1 /= np.linalg.norm(n1)
        n2 = rng.standard_normal(3)
        n2 /= np.linalg.norm(n2)
        fl = np.array([rng.integers(0, 60), rng.random() * 3, rng.random() * 100, rng.random() * 1000,
                       rng.integers(0, 200), *(rng.random(4) * 300), *rng.random(4), *(rng.standard_normal(4) * 9),
                       *n1, rng.integers(0, 90), *(rng.standard_normal(3) * 9), rng.choice([0.0, 1.0]), *n2], f32)
        packed = (C.c_uint32 * 16)()
        out = (C.c_float * 28)()
        oracle_lib.hko_pack_reservoir_roundtrip(fl.ctypes.data, packed, out)
        got = np.frombuffer(bytes(packed), np.uint32)
        want = np_pack_reservoir(fl)
        assert np.array_equal(got, want), (trial, got, want)
        u = np.frombuffer(bytes(out), f32)
        # unpack (light.wgsl:77-109): f16 fields, unorm16 / 65535, lifetime = 127 (1 + snorm), id via f32
        assert u[0] == np.float16(fl[0]) and u[20] == int(fl[20])
        assert np.allclose(u[9:13], np.rint(fl[9:13] * 65535) / 65535, atol=1e-7)
        life = 127.0 * (1.0 + max(np.rint(np.clip(fl[4] / 127.0 - 1.0, -1, 1) * 127) / 127, -1.0))
        assert abs(u[4] - life) < 1e-4
        assert abs(np.linalg.norm(u[17:20]) - 1.0) < 1e-5 and abs(np.linalg.norm(u[25:28]) - 1.0) < 1e-5


# ------------------------------------------------------------------ intersection
def np_slab(o, inv, mn, mx):
    t1 = (mn - o) * inv
    t2 = (mx - o) * inv
    tmin = np.fmin(t1[0], t2[0])
    tmax = np.fmax(t1[0], t2[0])
    tmin = np.fmax(tmin, np.fmin(t1[1], t2[1]))
    tmax = np.fmin(tmax, np.fmax(t1[1], t2[1]))
    tmin = np.fmax(tmin, np.fmin(t1[2], t2[2]))
    tmax = np.fmin(tmax, np.fmax(t1[2], t2[2]))
    return tmin if (tmax >= tmin and tmax >= 0) else f32(3.402823466e38)


def test_intersects_aabb_known_answers(oracle_lib):
    rng = np.random.default_rng(3)
    with np.errstate(all="ignore"):
        for k in range(3000):
            o = rng.uniform(-2, 2, 3).astype(f32)
            d = rng.standard_normal(3).astype(f32)
            if k % 7 == 0:
                d[k % 3] = 0.0  # axis-parallel: inv = +-inf, 0 * inf = NaN ignored by minNum
            inv = (f32(1.0) / d).astype(f32)
            mn = rng.uniform(-1, 0, 3).astype(f32)
            mx = (mn + rng.uniform(0, 1.5, 3)).astype(f32)
            if k % 11 == 0:
                o[k % 3] = mn[k % 3]  # origin on the slab plane
            want = np_slab(o, inv, mn, mx)
            got = oracle_lib.hko_intersects_aabb(o.ctypes.data, inv.ctypes.data, mn.ctypes.data, mx.ctypes.data)
            assert np.float32(got).view(np.uint32) == np.float32(want).view(np.uint32), (k, got, want)
    # ray inside a box: t_min < 0 still counts as a hit
    o = np.zeros(3, f32)
    inv = np.array([1, 1, 1], f32)
    assert oracle_lib.hko_intersects_aabb(o.ctypes.data, inv.ctypes.data, np.array([-1, -1, -1], f32).ctypes.data,
                                          np.array([1, 1, 1], f32).ctypes.data) == -1.0


def np_triangle(o, d, a, b, c):
    F32_EPS = f32(1.1920929e-7)
    miss = f32(3.402823466e38)
    ab, ac = b - a, c - a
    def dot(x, y): return f32(f32(x[0] * y[0] + x[1] * y[1]) + x[2] * y[2])
    def cross(x, y): return np.array([x[1] * y[2] - x[2] * y[1], x[2] * y[0] - x[0] * y[2], x[0] * y[1] - x[1] * y[0]], f32)
    u_vec = cross(d, ac)
    det = dot(ab, u_vec)
    if abs(det) < F32_EPS:
        return (f32(0), f32(0), miss)
    inv_det = f32(f32(1.0) / det)
    ao = o - a
    u = f32(dot(ao, u_vec) * inv_det)
    if u < 0 or u > 1:
        return (u, f32(0), miss)
    v_vec = cross(ao, ab)
    v = f32(dot(d, v_vec) * inv_det)
    if v < 0 or f32(u + v) > 1:
        return (u, v, miss)
    t = f32(dot(ac, v_vec) * inv_det)
    return (u, v, t if t > F32_EPS else miss)


def test_intersects_triangle_known_answers(oracle_lib):
    rng = np.random.default_rng(4)
    out = np.zeros(3, f32)
    # exact cases
    a, b, c = np.array([0, 0, 0], f32), np.array([1, 0, 0], f32), np.array([0, 1, 0], f32)
    o, d = np.array([0.25, 0.25, 1], f32), np.array([0, 0, -1], f32)
    oracle_lib.hko_intersects_triangle(o.ctypes.data, d.ctypes.data, a.ctypes.data, b.ctypes.data, c.ctypes.data,
                                       out.ctypes.data)
    assert list(out) == [0.25, 0.25, 1.0]
    # parallel ray: det == 0 -> miss
    d2 = np.array([1, 0, 0], f32)
    oracle_lib.hko_intersects_triangle(o.ctypes.data, d2.ctypes.data, a.ctypes.data, b.ctypes.data, c.ctypes.data,
                                       out.ctypes.data)
    assert out[2] == np.float32(3.402823466e38)
    # two-sided: hit from below too
    o3, d3 = np.array([0.2, 0.3, -2], f32), np.array([0, 0, 1], f32)
    oracle_lib.hko_intersects_triangle(o3.ctypes.data, d3.ctypes.data, a.ctypes.data, b.ctypes.data, c.ctypes.data,
                                       out.ctypes.data)
    assert out[2] == 2.0
    with np.errstate(all="ignore"):
        for k in range(3000):
            tri = rng.uniform(-1, 1, (3, 3)).astype(f32)
            o = rng.uniform(-2, 2, 3).astype(f32)
            tgt = (tri[0] + rng.uniform(-0.2, 1, 1)[0] * (tri[1] - tri[0]) + rng.uniform(-0.2, 1, 1)[0] *
                   (tri[2] - tri[0])).astype(f32)
            d = (tgt - o).astype(f32)
            oracle_lib.hko_intersects_triangle(o.ctypes.data, d.ctypes.data, tri[0].ctypes.data, tri[1].ctypes.data,
                                               tri[2].ctypes.data, out.ctypes.data)
            want = np.array(np_triangle(o, d, tri[0], tri[1], tri[2]), f32)
            assert np.array_equal(out.view(np.uint32), want.view(np.uint32)), (k, out, want)


# ------------------------------------------------------------------ pinned transcendentals
@pytest.mark.parametrize("name,fn,lo,hi", [
    ("sin", math.sin, -7.0, 7.0), ("cos", math.cos, -7.0, 7.0), ("exp2", lambda x: 2.0 ** x, -20.0, 20.0),
    ("log2", math.log2, 1e-6, 1e6)])
def test_transcendentals_accuracy(oracle_lib, name, fn, lo, hi):
    rng = np.random.default_rng(5)
    xs = rng.uniform(lo, hi, 20000).astype(f32) if name != "log2" else np.exp(rng.uniform(np.log(lo), np.log(hi),
                                                                                          20000)).astype(f32)
    f = getattr(oracle_lib, f"hko_{name}")
    worst = 0.0
    for x in xs:
        got = f(float(x))
        ref = fn(float(x))
        ulp = float(np.spacing(np.float32(abs(ref)) if ref != 0 else np.float32(1e-30)))
        err = abs(got - ref) / max(ulp, float(np.spacing(np.float32(1e-7))) if name in ("sin", "cos") else ulp)
        worst = max(worst, err)
    assert worst <= 4.0, f"{name}: {worst} ulp"


def test_branch_free_exp2_log2_equal_the_branchy_forms(oracle_lib):
    """hk_math.h's hk_exp2 / hk_log2 / hk_sincos are written branch-free since round 5 (each case computed, the
    result selected); they must give the bits of the round-4 branchy forms (kept in the oracle as the reference) on
    every input.  Every 7th of the 2^32 bit patterns here (all of them: 0 / 0 / 0 when run with stride 1)."""
    import ctypes as C
    v = (C.c_uint64 * 3)()
    oracle_lib.hko_math_form_mismatches(7, v)
    assert list(v) == [0, 0, 0], list(v)
    # the selected special cases
    assert math.isnan(oracle_lib.hko_exp2(float("nan"))) and math.isnan(oracle_lib.hko_log2(-1.0))
    assert oracle_lib.hko_exp2(128.0) == float("inf") and oracle_lib.hko_exp2(-151.5) == 0.0
    assert oracle_lib.hko_exp2(-149.0) == 2.0 ** -149 and oracle_lib.hko_log2(0.0) == -float("inf")
    assert oracle_lib.hko_log2(float("inf")) == float("inf") and oracle_lib.hko_log2(2.0 ** -140) == -140.0


def test_exp_weight_equals_exp(oracle_lib):
    """hk_exp_weight (the denoise levels' weights, arguments <= 0) gives hk_exp's bits wherever that is a normal
    float, 0 where hk_exp is subnormal (flushed) and for NaN: every 5th input here (all of them: 0 when run with
    stride 1)."""
    assert oracle_lib.hko_exp_weight_mismatches(5) == 0


def test_pow_special_cases(oracle_lib):
    assert oracle_lib.hko_pow(0.0, 5.0) == 0.0
    assert oracle_lib.hko_pow(0.0, 0.25) == 0.0
    assert oracle_lib.hko_pow(1.0, 16.0) == 1.0
    assert math.isnan(oracle_lib.hko_pow(-1.0, 2.0))
    assert abs(oracle_lib.hko_pow(0.5, 16.0) - 0.5 ** 16) <= 4 * np.spacing(np.float32(0.5 ** 16))
    assert abs(oracle_lib.hko_pow(3.0, 2.0) - 9.0) <= 4 * np.spacing(np.float32(9.0))


# ------------------------------------------------------------------ traversal (pure Python restatement)
NODE = np.dtype([("min", "<f4", 3), ("entry", "<u4"), ("max", "<f4", 3), ("exit", "<u4")])


def py_traverse_top(arrs, o, d, max_distance, early, exclude):
    inst = arrs["instances"].reshape(-1, 176)
    tlas = np.frombuffer(arrs["instance_nodes"].tobytes(), NODE)
    blas = np.frombuffer(arrs["asset_nodes"].tobytes(), NODE)
    prims = np.frombuffer(arrs["primitives"].tobytes(), f32).reshape(-1, 3, 4)
    FMAX = f32(3.402823466e38)
    hit = {"uv": (f32(0), f32(0)), "t": f32(max_distance), "inst": 0xFFFFFFFF, "prim": 0xFFFFFFFF}
    with np.errstate(all="ignore"):
        inv = (f32(1) / d).astype(f32)
        i = 0
        while i < len(tlas):
            n = tlas[i]
            if n["entry"] >= 0x80000000:
                ii = int(n["entry"]) - 0x80000000
                row = inst[ii]
                fv = row.view(f32)
                uv = row.view(np.uint32)
                if ii != exclude and np_slab(o, inv, fv[0:3], fv[4:7]) < hit["t"]:
                    itm = fv[24:40]
                    def tm(p, w):
                        return np.array([f32(f32(f32(itm[4 * r] * p[0] + itm[4 * r + 1] * p[1]) + itm[4 * r + 2] * p[2])
                                             + itm[4 * r + 3] * f32(w)) for r in range(4)], f32)
                    po = tm(o, 1.0)
                    lo = (po[:3] / po[3]).astype(f32)
                    ld = tm(d, 0.0)[:3]
                    linv = (f32(1) / ld).astype(f32)
                    noff, nlen, poff = int(uv[42]), int(uv[43]), int(uv[41])
                    j = 0
                    got = False
                    done = False
                    while j < nlen:
                        m = blas[noff + j]
                        if m["entry"] >= 0x80000000:
                            pi = poff + int(m["entry"]) - 0x80000000
                            t3 = prims[pi][:, :3]
                            mn = np.fmin(t3[0], np.fmin(t3[1], t3[2]))
                            mx = np.fmax(t3[0], np.fmax(t3[1], t3[2]))
                            if np_slab(lo, linv, mn, mx) < hit["t"]:
                                u, v, t = np_triangle(lo, ld, t3[0], t3[1], t3[2])
                                if t < hit["t"]:
                                    hit.update(uv=(u, v), t=t, prim=pi)
                                    got = True
                                    if t < early:
                                        done = True
                                        break
                            j = int(m["exit"])
                        else:
                            j = int(m["entry"]) if np_slab(lo, linv, m["min"], m["max"]) < hit["t"] else int(m["exit"])
                    if got:
                        hit["inst"] = ii
                        if hit["t"] < early:
                            return hit
                i = int(n["exit"])
            else:
                i = int(n["entry"]) if np_slab(o, inv, n["min"], n["max"]) < hit["t"] else int(n["exit"])
    return hit


def test_traversal_matches_python_restatement(oracle_lib):
    from oracle import Oracle

    from hikari_amd import examples, load_noise
    scene, cam, lights = examples.cornell()
    desc = scene.build()
    arrs = scene.arrays()
    o = Oracle(desc, load_noise(), 8, 8, 1.0, threads=1)
    rng = np.random.default_rng(6)
    n = 160
    org = rng.uniform([-0.9, 0.1, -0.9], [0.9, 1.9, 0.9], (n, 3)).astype(f32)
    d = rng.standard_normal((n, 3)).astype(f32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(f32)
    early = np.where(np.arange(n) % 2 == 0, 0.0, 65535.0).astype(f32)
    excl = (np.arange(n) % 9).astype(np.uint32)
    rays = np.concatenate([org, d], axis=1).astype(f32)
    got = o.trace(rays, None, early, excl)
    for k in range(n):
        h = py_traverse_top(arrs, org[k], d[k], f32(3.402823466e38), early[k], int(excl[k]))
        want = [np.float32(h["uv"][0]).view(np.uint32), np.float32(h["uv"][1]).view(np.uint32),
                np.float32(h["t"]).view(np.uint32), h["inst"], h["prim"]]
        assert list(got[k]) == want, (k, list(got[k]), want)
    assert (got[:, 3] != 0xFFFFFFFF).sum() > n // 2


# The denoiser's independent check is the float32 restatement of all three channels, incl. the firefly
# filter, in tests/denoise_python.py (bit-exact, tests/test_indirect_independent.py).


def test_f16_conversion_matches_numpy_ieee_sweep():
    """hk_f32_to_f16 (software RNE, shared by the oracle) equals IEEE-754 binaryfloat16 conversion
    (numpy's astype) on a 2^24-pattern stride sweep of all f32 bit patterns (NaNs: quiet NaN)."""
    import oracle as orc
    L = orc.lib()
    bits = np.arange(0, 1 << 32, 256, dtype=np.uint64).astype(np.uint32) + np.uint32(0x1000 - 3)
    vals = bits.view(np.float32)
    got = np.empty(len(vals), np.uint16)
    L.hko_f32_to_f16_array(vals.ctypes.data, len(vals), got.ctypes.data)
    with np.errstate(over="ignore"):
        want = vals.astype(np.float16).view(np.uint16)
    nan = np.isnan(vals)
    assert np.array_equal(got[~nan], want[~nan])
    assert ((got[nan] & 0x7C00) == 0x7C00).all() and ((got[nan] & 0x3FF) != 0).all()


def test_integer_pow_accuracy_and_domain():
    """hk_pow2/5/16 (literal-exponent pow): within a few ulp of the float64 power on [0, 4],
    and the same special values as hk_pow (x < 0 / NaN -> NaN, +-0 -> +0, inf -> inf)."""
    import math
    import oracle as orc
    L = orc.lib()
    rng = np.random.default_rng(5)
    xs = np.concatenate([rng.uniform(0, 1, 3000), rng.uniform(1, 4, 1000), [0.5, 1.0, 2.0]]).astype(np.float32)
    for n, tol in ((2, 1), (5, 3), (16, 16)):
        for x in xs:
            got = np.float32(L.hko_pow_int(float(x), n))
            want = float(x) ** n
            if want == 0 or not math.isfinite(want) or want > 3.4e38:
                continue
            ulp = np.spacing(np.float32(want))
            assert abs(float(got) - want) <= tol * ulp, (n, x, got, want)
        assert math.isnan(L.hko_pow_int(-1.0, n)) and math.isnan(L.hko_pow_int(float("nan"), n))
        assert math.copysign(1.0, L.hko_pow_int(-0.0, n)) == 1.0 and L.hko_pow_int(0.0, n) == 0.0
        assert L.hko_pow_int(float("inf"), n) == float("inf")


def test_divide_free_unorm16_snorm8_decodes_are_exact(oracle_lib):
    """hk_unpack_unorm16_fast / hk_unpack_snorm8_fast / hk_unorm8_fast (device kernels: x * RN(1/d) plus
    one residual correction) equal unpack2x16unorm / unpack4x8snorm / the RGBA8 texel's divisions for every
    code: compiled (host C,
    hko_unpack_fast_mismatches) and as a formula in exact rational arithmetic."""
    from fractions import Fraction as Fr
    assert oracle_lib.hko_unpack_fast_mismatches() == 0

    def rn(x):  # exact rational -> nearest f32, ties to even
        a = np.float32(float(x))
        c = [np.nextafter(a, np.float32(-np.inf)), a, np.nextafter(a, np.float32(np.inf))]
        return min(c, key=lambda v: (abs(Fr(float(v)) - x), int(np.float32(v).view(np.uint32)) & 1))

    for d, codes in ((65535, range(0, 65536, 7)), (127, range(-128, 128)), (255, range(256))):
        r = rn(Fr(1, d))
        for v in codes:
            q0 = rn(Fr(v) * Fr(float(r)))
            e = rn(Fr(float(-q0)) * d + v)
            q1 = rn(Fr(float(e)) * Fr(float(r)) + Fr(float(q0)))
            assert q1 == rn(Fr(v, d)), (d, v)
