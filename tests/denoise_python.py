"""Independent float32 restatement of denoise.wgsl: `demodulation` with `accumulate_variance`
(denoise.wgsl:116-162) and the four à-trous levels of `denoise` with `accumulate_irradiance`, the
edge-stopping weights and the FIREFLY_FILTERING branch (denoise.wgsl:43-65, 71-114, 164-319), dispatched
per channel as post_process.rs:1190-1224 does (direct without, emissive and indirect with the firefly
filter; the indirect channel dropped when indirect_bounces == 0, post_process.rs:949-954).

TEST INFRASTRUCTURE.  Written from the WGSL, not from oracle/hk_oracle.c or csrc/: scalar float32
arithmetic evaluated left to right with the conventions of DESIGN.md §3 (dot = (x x' + y y') + z z',
normalize(v) = v * (1 / sqrt(dot)), IEEE minNum / maxNum, pow(x, 16) by repeated squaring with WGSL pow's
domain).  The transcendentals are the build's pinned primitives from the oracle library: exp(x) =
exp2(x * log2(e)) and pow(x, 0.25) = exp2(0.25 * log2(x)) (WGSL's own definition of pow) over hko_exp2 /
hko_log2, so a difference in a result is a difference in the algorithm.  Sampled texels
(textureSampleLevel with the nearest sampler) are the texel floor(uv * size), clamped to the edge.
"""
from __future__ import annotations

import math

import numpy as np

F = np.float32
F32_EPSILON = F(1.1920929e-7)
F32_MAX = F(3.402823466e38)
LOG2E = F(1.4426950408889634)
KERNEL = ((F(0.0625), F(0.125), F(0.0625)), (F(0.125), F(0.25), F(0.125)), (F(0.0625), F(0.125), F(0.0625)))
TAPS = ((-1, -1), (0, -1), (1, -1), (-1, 0), (1, 0), (-1, 1), (0, 1), (1, 1))  # denoise.wgsl:252-259
VARIANCE_TAPS = ((-1, -1), (-1, 0), (-1, 1), (0, -1), (0, 0), (0, 1), (1, -1), (1, 0), (1, 1))  # 152-160


def f16(x):
    with np.errstate(over="ignore"):
        return F(np.float16(x))


def is_nan(v):
    return not (v < 0 or 0 < v or v == 0)


class Math:
    def __init__(self, lib):
        self.lib = lib

    def exp(self, x):
        return F(self.lib.hko_exp2(float(F(x) * LOG2E)))

    def pow_quarter(self, x):
        return F(self.lib.hko_exp2(float(F(0.25) * F(self.lib.hko_log2(float(x))))))


def pow16(x):
    if not (x >= 0):
        return F(np.nan)
    x = x + F(0.0)
    x2 = x * x
    x4 = x2 * x2
    x8 = x4 * x4
    return x8 * x8


def dot3(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def normalize3(a):
    with np.errstate(all="ignore"):
        k = F(1.0) / np.sqrt(dot3(a, a))
        return (a[0] * k, a[1] * k, a[2] * k)


def luminance(c):
    return (c[0] * F(0.2126) + c[1] * F(0.7152)) + c[2] * F(0.0722)


class Planes:
    """The textures the denoiser binds (deferred_bindings.wgsl + light/post-process textures), as float32
    arrays: position (H, W, 4), normal (H, W, 3, snorm-decoded), depth_gradient (H, W, 2),
    instance_material (H, W, 2), albedo (H, W, 4), per channel render (H, W, 4) and variance (H, W)."""

    def __init__(self, gb: dict, albedo: np.ndarray):
        self.gb, self.albedo = gb, albedo
        self.H, self.W = albedo.shape[:2]

    @staticmethod
    def nearest(a, uv):
        h, w = a.shape[:2]
        x = min(max(int(math.floor(uv[0] * F(w))), 0), w - 1)
        y = min(max(int(math.floor(uv[1] * F(h))), 0), h - 1)
        return a[y, x]


def coords_to_uv(x, y, w, h):
    return ((F(x) + F(0.5)) / F(w), (F(y) + F(0.5)) / F(h))


def jittered_deferred_uv(uv, number, ratio, dsize):
    j = F(-0.5) if (number & 1) == 0 else F(0.5)
    r = F(ratio) - F(1.0)
    return tuple(uv[k] + (j * (F(1.0) / F(dsize[k]))) * r for k in range(2))


def demodulation(pl: Planes, render, variance, number, ratio):
    """-> internal_0 (H, W, 4) f16-rounded, internal_variance (H, W) f32."""
    H, W = render.shape[:2]
    dsize = (pl.gb["position"].shape[1], pl.gb["position"].shape[0])
    out = np.zeros((H, W, 4), F)
    ivar = np.zeros((H, W), F)
    for y in range(H):
        for x in range(W):
            uv = coords_to_uv(x, y, W, H)
            duv = jittered_deferred_uv(uv, number, ratio, dsize)
            albedo = Planes.nearest(pl.albedo, duv)[:3]
            irr = Planes.nearest(render, uv)[:3]
            with np.errstate(all="ignore"):
                irr = tuple(F(0.0) if albedo[k] < F(0.01) else irr[k] / albedo[k] for k in range(3))
            out[y, x] = [f16(irr[0]), f16(irr[1]), f16(irr[2]), F(1.0)]
            sv = F(0.0)
            for ox, oy in VARIANCE_TAPS:
                suv = (uv[0] + F(ox) / F(W), uv[1] + F(oy) / F(H))
                if suv[0] < F(0.0) or suv[1] < F(0.0) or suv[0] > F(1.0) or suv[1] > F(1.0):
                    continue
                v = Planes.nearest(variance, suv)
                if v > F32_MAX:
                    continue
                sv = sv + KERNEL[oy + 1][ox + 1] * F(np.fmax(v, F(0.0)))
            ivar[y, x] = sv
    return out, ivar


def denoise_level(m: Math, pl: Planes, inp, ivar, level, firefly, number, ratio, stats=None):
    """One à-trous level: internal_L -> internal_{L+1} (L3: x albedo -> output), f16-rounded.
    stats["firefly"] counts the pixels the firefly filter scaled."""
    H, W = inp.shape[:2]
    step = 8 >> level
    dsize = (pl.gb["position"].shape[1], pl.gb["position"].shape[0])
    out = np.zeros((H, W, 4), F)
    g = pl.gb
    for y in range(H):
        for x in range(W):
            uv = coords_to_uv(x, y, W, H)
            duv = jittered_deferred_uv(uv, number, ratio, dsize)
            depth = Planes.nearest(g["position"], duv)[3]
            grad = Planes.nearest(g["depth_gradient"], duv)
            normal = normalize3(Planes.nearest(g["normal"], duv))
            instance = Planes.nearest(g["instance_material"], duv)[0]
            if depth < F32_EPSILON:
                continue  # store_output(0)
            variance = ivar[y, x]
            irr = tuple(inp[y, x, :3])
            k11 = KERNEL[1][1]
            s_irr = [irr[0] * k11, irr[1] * k11, irr[2] * k11]
            s_w = k11
            if any(is_nan(c) for c in irr) or any(c > F32_MAX for c in irr):
                irr = (F(0.0),) * 3
                s_irr = [F(0.0)] * 3
                s_w = F(0.0)
            lum = luminance(irr)
            m1 = m2 = cnt = F(0.0)
            for ox, oy in TAPS:
                sx, sy = x + ox * step, y + oy * step
                suv = coords_to_uv(sx, sy, W, H)
                sduv = jittered_deferred_uv(suv, number, ratio, dsize)
                if suv[0] < F(0.0) or suv[1] < F(0.0) or suv[0] > F(1.0) or suv[1] > F(1.0):
                    continue
                t = inp[sy, sx, :3] if (0 <= sx < W and 0 <= sy < H) else np.zeros(3, F)
                if any(is_nan(c) for c in t) or any(c > F32_MAX for c in t):
                    continue
                sn = normalize3(Planes.nearest(g["normal"], sduv))
                sdepth = Planes.nearest(g["position"], sduv)[3]
                sinst = Planes.nearest(g["instance_material"], sduv)[0]
                slum = luminance(t)
                with np.errstate(all="ignore"):
                    w_normal = pow16(F(np.fmax(F(0.0), dot3(normal, sn))))
                    w_depth = m.exp((-abs(depth - sdepth)) / (abs(grad[0] * F(ox) + grad[1] * F(oy)) + F(0.01)))
                    w_instance = F(np.fmax(F(0.0), F(1.0) - abs(instance - sinst)))
                    w_lum = m.exp((-abs(lum - slum)) / (F(4.0) * m.pow_quarter(variance) + F(0.001)))
                    w = F(np.fmin(F(np.fmax(((w_normal * w_depth) * w_instance) * w_lum, F(0.0))), F(1.0))) * \
                        KERNEL[oy + 1][ox + 1]
                s_irr = [s_irr[k] + t[k] * w for k in range(3)]
                s_w = s_w + w
                if firefly:
                    m1 = m1 + slum
                    m2 = m2 + slum * slum
                    cnt = cnt + F(1.0)
            with np.errstate(all="ignore"):
                res = [F(0.0)] * 3 if s_w < F(0.0001) else [s_irr[k] / s_w for k in range(3)]
                if firefly:
                    mean = m1 / cnt
                    var = m2 / cnt - mean * mean
                    if lum > mean + F(3.0) * np.sqrt(var):
                        res = [(mean / lum) * c for c in res]
                        if stats is not None:
                            stats["firefly"] = stats.get("firefly", 0) + 1
            color = [res[0], res[1], res[2], F(1.0)]
            if level == 3:
                a = Planes.nearest(pl.albedo, duv)
                with np.errstate(all="ignore"):
                    color = [color[k] * a[k] for k in range(4)]
            out[y, x] = [f16(c) for c in color]
    return out


def denoise_channel(lib, pl: Planes, render, variance, firefly, number, ratio=1.0, stats=None):
    """demodulation + L0..L3 of one channel -> (denoised output (H, W, 4), internal variance)."""
    m = Math(lib)
    buf, ivar = demodulation(pl, render, variance, number, ratio)
    for level in range(4):
        buf = denoise_level(m, pl, buf, ivar, level, firefly, number, ratio, stats)
    return buf, ivar
