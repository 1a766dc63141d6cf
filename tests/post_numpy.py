"""Independent numpy restatement of SMAA TU4x and TAA "Jasmine" (smaa.wgsl:47-271, taa.wgsl:20-170).

TEST INFRASTRUCTURE.  Written from the WGSL and the WGSL/wgpu texture rules, NOT from
include/hk_post.h (the per-pixel code the oracle and the GPU share), so that tests can pin that
header against a second reading of the shaders.  Vectorised over all pixels in float32; vector
expressions evaluated left to right per component, `dot` as ((x + y) + z) (+ w).
Texture access (post_process.rs:697-708 samplers: default address mode = clamp-to-edge, LOD 0):
  nearest  texel (floor(u W), floor(v H)), clamped;
  linear   ideal bilinear filter of the 2x2 footprint at (u W - 0.5, v H - 0.5), clamped texels;
  gather   component c of that footprint in WGSL order (u_min, v_max), (u_max, v_max), (u_max,
           v_min), (u_min, v_min);
  load     out-of-bounds textureLoad -> 0.
min / max / clamp follow IEEE minNum / maxNum (a NaN operand yields the other one), the build's
convention for WGSL's implementation-defined NaN behaviour; textureStore rounds to f16.
"""
from __future__ import annotations

import numpy as np

F = np.float32
TAU = F(6.283185307)


def f32(x):
    return np.asarray(x, dtype=np.float32)


def clampf(x, lo, hi):
    return np.fmin(np.fmax(x, lo), hi)


def coords_to_uv(x, y, w, h):
    return (f32(x) + F(0.5)) / F(w), (f32(y) + F(0.5)) / F(h)


def _index(t, u, v):
    h, w = t.shape[:2]
    fx, fy = np.floor(f32(u) * F(w)), np.floor(f32(v) * F(h))
    ix = np.clip(np.nan_to_num(fx, nan=0.0, posinf=w, neginf=-1), -1, w).astype(np.int64)
    iy = np.clip(np.nan_to_num(fy, nan=0.0, posinf=h, neginf=-1), -1, h).astype(np.int64)
    return np.clip(ix, 0, w - 1), np.clip(iy, 0, h - 1)


def nearest(t, u, v):
    ix, iy = _index(t, u, v)
    return t[iy, ix]


def _footprint(t, u, v):
    h, w = t.shape[:2]
    x, y = f32(u) * F(w) - F(0.5), f32(v) * F(h) - F(0.5)
    x0, y0 = np.floor(x), np.floor(y)
    a, b = x - x0, y - y0
    i0 = np.clip(np.nan_to_num(x0, nan=0.0, posinf=w, neginf=-1), -1, w).astype(np.int64)
    j0 = np.clip(np.nan_to_num(y0, nan=0.0, posinf=h, neginf=-1), -1, h).astype(np.int64)
    c = lambda i, n: np.clip(i, 0, n - 1)  # noqa: E731
    return c(i0, w), c(i0 + 1, w), c(j0, h), c(j0 + 1, h), a, b


def linear(t, u, v):
    i0, i1, j0, j1, a, b = _footprint(t, u, v)
    a, b = a[..., None], b[..., None]
    ia, ib = F(1.0) - a, F(1.0) - b
    return (t[j0, i0] * ia + t[j0, i1] * a) * ib + (t[j1, i0] * ia + t[j1, i1] * a) * b


def gather(t, comp, u, v):
    i0, i1, j0, j1, _, _ = _footprint(t, u, v)
    return np.stack([t[j1, i0, comp], t[j1, i1, comp], t[j0, i1, comp], t[j0, i0, comp]], axis=-1)


def rgb_to_ycocg(c):
    r, g, b = c[..., 0], c[..., 1], c[..., 2]
    y = ((r / F(4.0)) + (g / F(2.0))) + (b / F(4.0))
    co = (r / F(2.0)) - (b / F(2.0))
    cg = ((-r / F(4.0)) + (g / F(2.0))) - (b / F(4.0))
    return np.stack([y, co, cg], axis=-1)


def ycocg_to_rgb(c):
    x, y, z = c[..., 0], c[..., 1], c[..., 2]
    return clampf(np.stack([(x + y) - z, x + z, (x - y) - z], axis=-1), F(0.0), F(1.0))


def clip_towards_aabb_center(prev, mn, mx):
    p = F(0.5) * (mx + mn)
    e = F(0.5) * (mx - mn)
    v = prev - p
    with np.errstate(divide="ignore", invalid="ignore"):
        a = np.abs(v / e)
    ma = np.fmax(a[..., 0], np.fmax(a[..., 1], a[..., 2]))
    with np.errstate(divide="ignore", invalid="ignore"):
        clipped = p + v / ma[..., None]
    return np.where((ma > F(1.0))[..., None], clipped, prev)


def nearest_velocity(position, velocity_uv, u, v, sized):
    """smaa.wgsl:52-71 / taa.wgsl:54-73; texel size = 1 / dims of `sized` (position for SMAA,
    render for TAA)."""
    h, w = sized.shape[:2]
    tx, ty = F(1.0) / F(w), F(1.0) / F(h)
    d = np.stack([nearest(position, u + tx, v + ty)[..., 3], nearest(position, u + -tx, v + ty)[..., 3],
                  nearest(position, u + tx, v + -ty)[..., 3], nearest(position, u + -tx, v + -ty)[..., 3]], -1)
    max_depth = np.fmax(np.fmax(d[..., 0], d[..., 1]), np.fmax(d[..., 2], d[..., 3]))
    depth = nearest(position, u, v)[..., 3]
    hit = d == max_depth[..., None]
    sx = np.where(hit, f32([1.0, -1.0, 1.0, -1.0]), F(0.0))
    sy = np.where(hit, f32([1.0, 1.0, -1.0, -1.0]), F(0.0))
    ox = ((tx * sx[..., 0] + tx * sx[..., 1]) + tx * sx[..., 2]) + tx * sx[..., 3]
    oy = ((ty * sy[..., 0] + ty * sy[..., 1]) + ty * sy[..., 2]) + ty * sy[..., 3]
    use = depth < max_depth
    ox, oy = np.where(use, ox, F(0.0)), np.where(use, oy, F(0.0))
    vel = nearest(velocity_uv, u + ox, v + oy)
    return vel[..., 0], vel[..., 1]


def _distance2(ax, ay, bx, by):
    dx, dy = ax - bx, ay - by
    return np.sqrt(dx * dx + dy * dy)


def smaa_tu4x(number, render, previous_render, position, previous_position, velocity_uv, previous_velocity_uv,
              instance_material, output):
    """smaa.wgsl:81-199 over every input pixel; writes into `output` (H, W, 4) float32 in place."""
    ih, iw = render.shape[:2]
    oh, ow = output.shape[:2]
    y, x = np.mgrid[0:ih, 0:iw]
    u, v = coords_to_uv(x, y, iw, ih)
    tsx, tsy = F(1.0) / F(ow), F(1.0) / F(oh)
    biases = [(F(0.0), F(0.0)), (F(2.5) * tsx, F(2.5) * tsy), (F(-2.5) * tsx, F(2.5) * tsy),
              (F(2.5) * tsx, F(-2.5) * tsy), (F(-2.5) * tsx, F(-2.5) * tsy)]
    cj = 0 if number & 1 == 0 else 1
    pj = 1 if number & 1 == 0 else 0
    current = nearest(render, u, v)[..., :3]
    px, py = 2 * x + pj, 2 * y + pj
    pu, pv = coords_to_uv(px, py, ow, oh)
    vx, vy = nearest_velocity(position, velocity_uv, pu, pv, position)
    ru, rv = pu - vx, pv - vy
    prev = nearest(previous_render, ru, rv)[..., :3]
    boundary_miss = (np.abs(ru - F(0.5)) > F(0.5)) | (np.abs(rv - F(0.5)) > F(0.5))
    current_instance = nearest(instance_material, pu, pv)[..., 0]
    current_depth = nearest(position, pu, pv)[..., 3]
    depth_miss = current_depth == F(0.0)
    instance_miss = np.zeros_like(depth_miss)
    with np.errstate(divide="ignore", invalid="ignore"):
        for bx, by in biases:
            pd = gather(previous_position, 3, ru + bx, rv + by)
            ratio = np.where(pd == F(0.0), F(1.0), current_depth[..., None] / pd)
            low = (ratio < F(0.95)).any(-1)
            depth_miss = depth_miss | low
            pi = nearest(instance_material, ru + bx, rv + by)[..., 0]
            instance_miss = instance_miss | (low & (np.abs(pi - current_instance) > F(1.0)))
    pvel = nearest(previous_velocity_uv, ru, rv)
    velocity_miss = _distance2(vx, vy, pvel[..., 0], pvel[..., 1]) > F(0.0001)
    clip = boundary_miss | ((depth_miss | instance_miss) & velocity_miss)
    # 2x2 YCoCg variance clipping around the nearest-depth footprint
    ubx, uby = np.zeros_like(u), np.zeros_like(v)
    min_ds = np.full_like(u, F(10.0))
    for bx, by in biases:
        ds = gather(position, 3, pu + bx, pv + by)
        e = current_depth[..., None] - ds
        dds = np.sqrt(((e[..., 0] * e[..., 0] + e[..., 1] * e[..., 1]) + e[..., 2] * e[..., 2]) + e[..., 3] * e[..., 3])
        take = dds < min_ds
        ubx, uby = np.where(take, bx, ubx), np.where(take, by, uby)
        min_ds = np.fmin(min_ds, dds)
    cr, cg, cb = (gather(render, k, pu + ubx, pv + uby) for k in range(3))
    s = [rgb_to_ycocg(np.stack([cr[..., q], cg[..., q], cb[..., q]], -1)) for q in range(4)]
    m1 = ((s[0] + s[1]) + s[2]) + s[3]
    m2 = ((s[0] * s[0] + s[1] * s[1]) + s[2] * s[2]) + s[3] * s[3]
    mean = m1 / F(4.0)
    with np.errstate(invalid="ignore"):
        var = np.sqrt((m2 / F(4.0)) - (mean * mean))
        clipped = ycocg_to_rgb(clip_towards_aabb_center(rgb_to_ycocg(prev), mean - var, mean + var))
    prev = np.where(clip[..., None], clipped, prev)
    spx = vx / (F(2.0) * tsx)
    spy = vy / (F(2.0) * tsy)
    blend = np.fmax(spx - np.floor(spx), spy - np.floor(spy))
    blend = clampf(-np.cos(blend * TAU).astype(np.float32), F(0.0), F(1.0))
    remix = linear(render, pu, pv)[..., :3]
    b = blend[..., None]
    prev = prev * (F(1.0) - b) + remix * b
    one = np.ones_like(u)[..., None]
    cx, cy = 2 * x + cj, 2 * y + cj
    _store(output, cx, cy, np.concatenate([current, one], -1))
    _store(output, px, py, np.concatenate([prev, one], -1))


def _store(out, x, y, c):
    """textureStore into an rgba16float storage texture: values rounded to f16 (out-of-bounds
    stores are dropped)."""
    oh, ow = out.shape[:2]
    ok = (x >= 0) & (y >= 0) & (x < ow) & (y < oh)
    out[y[ok], x[ok]] = c[ok].astype(np.float16).astype(np.float32)


def _load(out, x, y):
    oh, ow = out.shape[:2]
    ok = (x >= 0) & (y >= 0) & (x < ow) & (y < oh)
    r = np.zeros(x.shape + (4,), np.float32)
    r[ok] = out[y[ok], x[ok]]
    return r


def _lum(c):
    return (c[..., 0] * F(0.2126) + c[..., 1] * F(0.7152)) + c[..., 2] * F(0.0722)


def smaa_extrapolate(output, ih, iw):
    """smaa.wgsl:239-271 over every input pixel (the output's other two quad texels)."""
    y, x = np.mgrid[0:ih, 0:iw]
    t = _load(output, 2 * x, 2 * y)
    b = _load(output, 2 * x + 1, 2 * y + 1)
    n = _load(output, 2 * x + 1, 2 * y - 1)
    e = _load(output, 2 * x + 2, 2 * y)
    s = _load(output, 2 * x, 2 * y + 2)
    w = _load(output, 2 * x - 1, 2 * y + 1)
    dh0, dh1 = _lum(np.abs(w[..., :3] - b[..., :3])), _lum(np.abs(t[..., :3] - e[..., :3]))
    dv0, dv1 = _lum(np.abs(t[..., :3] - s[..., :3])), _lum(np.abs(n[..., :3] - b[..., :3]))
    fx = np.fmax(dv0, F(0.001)) * np.fmax(dv1, F(0.001))
    fy = np.fmax(dh0, F(0.001)) * np.fmax(dh1, F(0.001))
    fz = F(1.0) / (fx + fy)

    def blend(tt, bb, ll, rr):
        c = F(0.0) + (ll + rr) * fx[..., None]
        c = c + (tt + bb) * fy[..., None]
        return (F(0.5) * fz)[..., None] * c

    xc = blend(t, s, w, b)
    yc = blend(n, b, t, e)
    _store(output, 2 * x, 2 * y + 1, xc)
    _store(output, 2 * x + 1, 2 * y, yc)


def taa(upscale_ratio, clear_color, render, previous_render, position, previous_position, velocity_uv,
        previous_velocity_uv, oh, ow):
    """taa.wgsl:75-170 over every output pixel; returns (oh, ow, 4) float32."""
    y, x = np.mgrid[0:oh, 0:ow]
    tsx, tsy = F(1.0) / F(ow), F(1.0) / F(oh)
    u, v = coords_to_uv(x, y, ow, oh)
    original = nearest(render, u, v)
    current = original[..., :3]
    vx, vy = nearest_velocity(position, velocity_uv, u, v, render)
    qu, qv = u - vx, v - vy
    boundary_miss = (np.abs(qu - F(0.5)) > F(0.5)) | (np.abs(qv - F(0.5)) > F(0.5))
    biases = [(F(0.0), F(0.0)), (F(1.5) * tsx, F(1.5) * tsy), (F(-1.5) * tsx, F(1.5) * tsy),
              (F(1.5) * tsx, F(-1.5) * tsy), (F(-1.5) * tsx, F(-1.5) * tsy)]
    cpd = nearest(position, u, v)
    has_content = cpd[..., 3] > F(0.0)
    depth_miss = cpd[..., 3] == F(0.0)
    position_miss = cpd[..., 3] == F(0.0)
    with np.errstate(divide="ignore", invalid="ignore"):
        for bx, by in biases:
            pd = gather(previous_position, 3, qu + bx, qv + by)
            ratio = np.where(pd == F(0.0), F(1.0), cpd[..., 3:4] / pd)
            has_content = has_content | (pd > F(0.0)).any(-1)
            depth_miss = depth_miss | (ratio < F(0.95)).any(-1)
            pp = nearest(previous_position, qu + bx, qv + by)
            d = cpd[..., :3] - pp[..., :3]
            position_miss = position_miss | (np.sqrt((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]) > F(0.5))
    pvel = nearest(previous_velocity_uv, qu, qv)
    velocity_miss = _distance2(vx, vy, pvel[..., 0], pvel[..., 1]) > F(0.00005)
    # 5-tap Catmull-Rom
    out_w = []
    for k, (uu, vel, size, ts) in enumerate(((u, vx, ow, tsx), (v, vy, oh, tsy))):
        sp = (uu - vel) * F(size)
        t1 = np.floor(sp - F(0.5)) + F(0.5)
        f = sp - t1
        w0 = f * (F(-0.5) + f * (F(1.0) - F(0.5) * f))
        w1 = F(1.0) + (f * f) * (F(-2.5) + F(1.5) * f)
        w2 = f * (F(0.5) + f * (F(2.0) - F(1.5) * f))
        w3 = (f * f) * (F(-0.5) + F(0.5) * f)
        with np.errstate(divide="ignore", invalid="ignore"):
            o12 = w2 / (w1 + w2)
        out_w.append((w0, w1 + w2, w3, (t1 - F(1.0)) * ts, (t1 + o12) * ts, (t1 + F(2.0)) * ts))
    (w0x, w12x, w3x, t0x, t12x, t3x), (w0y, w12y, w3y, t0y, t12y, t3y) = out_w

    def prev_tap(tu, tv):
        return clampf(linear(previous_render, tu, tv)[..., :3], F(0.0), F(1.0))

    prev = np.zeros_like(current)
    for tu, tv, wa, wb in ((t12x, t0y, w12x, w0y), (t0x, t12y, w0x, w12y), (t12x, t12y, w12x, w12y),
                           (t3x, t12y, w3x, w12y), (t12x, t3y, w12x, w3y)):
        prev = prev + (prev_tap(tu, tv) * wa[..., None]) * wb[..., None]

    def sample(du, dv):
        return rgb_to_ycocg(clampf(nearest(render, u + du, v + dv)[..., :3], F(0.0), F(1.0)))

    taps = [sample(-tsx, tsy), sample(F(0.0), tsy), sample(tsx, tsy), sample(-tsx, -F(0.0)), rgb_to_ycocg(current),
            sample(tsx, F(0.0)), sample(-tsx, -tsy), sample(-F(0.0), -tsy), sample(tsx, -tsy)]
    m1, m2 = taps[0], taps[0] * taps[0]
    for s in taps[1:]:
        m1 = m1 + s
        m2 = m2 + s * s
    mean = m1 / F(9.0)
    with np.errstate(invalid="ignore", divide="ignore"):
        var = np.sqrt((m2 / F(9.0)) - (mean * mean))
        clipped = ycocg_to_rgb(clip_towards_aabb_center(rgb_to_ycocg(prev), mean - var, mean + var))
    clip = boundary_miss | (position_miss & velocity_miss & depth_miss)
    prev = np.where(clip[..., None], clipped, prev)
    t = F(0.1) / F(upscale_ratio)
    out = np.concatenate([prev * (F(1.0) - t) + current * t, original[..., 3:4]], -1)
    return np.where(has_content[..., None], out, f32(clear_color))
