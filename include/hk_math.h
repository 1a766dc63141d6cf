/*
 * hk_math.h — the pinned scalar math library used on BOTH sides of the parity check
 * (the gcc-built CPU oracle and the hipcc-built gfx950 kernels).
 *
 * WGSL leaves sin/cos/exp/exp2/pow/log2 implementation-defined (a few ulp), so there is
 * no single "reference" bit pattern for them.  To make CPU-vs-GPU parity bit-exact we
 * fix ONE implementation of each built-in here, written only with IEEE-754 single
 * operations that both targets round identically: +, -, *, correctly-rounded / and
 * sqrt, rint/floor, integer bit manipulation.  Both sides compile with
 * -ffp-contract=off, so no mul+add is ever fused.  Accuracy vs libm is checked by
 * tests/test_math.py (<= 4 ulp on the ranges the integrator uses).
 *
 * Plain C99 + HIP: HK_HD marks functions callable from host and device.
 */
#ifndef HK_MATH_H
#define HK_MATH_H

#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define HK_HD __host__ __device__ static inline
#else
#define HK_HD static inline
#endif

#define HK_PI 3.141592653589793f
#define HK_TAU 6.283185307f      /* light.wgsl:226 */
#define HK_INV_TAU 0.159154943f  /* light.wgsl:227 */
#define HK_F32_EPSILON 1.1920929E-7f
#define HK_F32_MAX 3.402823466E+38f
#define HK_GOLDEN_RATIO 1.618033989f

typedef union { float f; uint32_t u; int32_t i; } hk_fbits;

/* Horner step of the exp2 / log2 polynomials: one fused multiply-add (correctly rounded on the CPU's fmaf and the
 * GPU's v_fma_f32 alike, so both sides keep the same bits).  WGSL leaves exp2 / log2 implementation-defined; the
 * build fixes them here.  Round 5: fused instead of a rounded product and sum (city 4K a-trous level 0.339 -> 0.325
 * ms, profiles/r05/c6); the accuracy bound of test_transcendentals_accuracy (<= 4 ulp) still holds. */
#define HK_MAD(a, b, c) fmaf((a), (b), (c))

HK_HD uint32_t hk_f2u(float f) { hk_fbits b; b.f = f; return b.u; }
HK_HD float hk_u2f(uint32_t u) { hk_fbits b; b.u = u; return b.f; }

HK_HD float hk_minf(float a, float b) { return fminf(a, b); } /* IEEE minNum */
HK_HD float hk_maxf(float a, float b) { return fmaxf(a, b); } /* IEEE maxNum */
HK_HD float hk_clampf(float x, float lo, float hi) { return hk_minf(hk_maxf(x, lo), hi); }
HK_HD float hk_saturate(float x) { return hk_clampf(x, 0.0f, 1.0f); }
HK_HD float hk_fract(float x) { return x - floorf(x); }
HK_HD float hk_absf(float x) { return hk_u2f(hk_f2u(x) & 0x7FFFFFFFu); }
HK_HD float hk_signf(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
HK_HD float hk_mixf(float a, float b, float t) { return a * (1.0f - t) + b * t; }

/* 2^x.  Range-reduce to n + f, |f| <= 0.5; degree-7 Taylor of e^(f ln2) in Horner form.
 * Written without branches: every case's value is computed and the result selected at the end
 * (x NaN -> x; x >= 128 -> +inf; x < -151 -> 0; n >= -126 -> p * 2^n; else the subnormal result in
 * two exact-exponent steps, the last one rounding once).  The same bits as the branchy form for all
 * 2^32 inputs (oracle hko_math_form_mismatches, tests/test_oracle_kat.py); on the GPU a wave then runs
 * one straight sequence instead of three exec-mask regions per call (35 calls per a-trous pixel). */
HK_HD float hk_exp2(float x)
{
    float n = rintf(x);
    float f = x - n;
    float p = 1.5252733804059840e-05f;        /* ln2^7/7! */
    p = HK_MAD(p, f, 1.5403530393381608e-04f);      /* ln2^6/6! */
    p = HK_MAD(p, f, 1.3333558146428443e-03f);      /* ln2^5/5! */
    p = HK_MAD(p, f, 9.6181291076284772e-03f);      /* ln2^4/4! */
    p = HK_MAD(p, f, 5.5504108664821580e-02f);      /* ln2^3/3! */
    p = HK_MAD(p, f, 2.4022650695910071e-01f);      /* ln2^2/2! */
    p = HK_MAD(p, f, 6.9314718055994531e-01f);      /* ln2 */
    p = HK_MAD(p, f, 1.0f);
    /* n clamped before the conversion (only the selected cases use it: -151 <= n <= 128) */
    const int32_t ni = (int32_t)hk_minf(hk_maxf(n, -160.0f), 160.0f);
    const int normal = ni >= -126;
    const float s1 = hk_u2f((uint32_t)(normal ? ni + 127 : ni + 64 + 127) << 23);
    const float s2 = normal ? 1.0f : hk_u2f((uint32_t)(-64 + 127) << 23);
    float r = (p * s1) * s2; /* x 1.0 is exact */
    r = x < -151.0f ? 0.0f : r;
    r = x >= 128.0f ? hk_u2f(0x7F800000u) : r;
    return x != x ? x : r;
}

HK_HD float hk_exp(float x) { return hk_exp2(x * 1.4426950408889634f); }

/* hk_exp(x) for the denoiser's edge-stopping weights (denoise.wgsl:44-69: exp of -|a| / b, b > 0, so x <= 0 or NaN),
 * which are then clamped to [0, 1]: y clamped below at -160 (so a huge |x| or a NaN gives 0, which the clamp makes of
 * a NaN weight anyway) and a one-step scale that flushes a weight below 2^-126 to 0 (WGSL leaves subnormal results
 * to the implementation), without hk_exp's selects.  The same bits as hk_exp wherever that is a normal float;
 * checked on every input x <= 0 (hko_exp_weight_mismatches). */
HK_HD float hk_exp_weight(float x)
{
    const float y = hk_maxf(x * 1.4426950408889634f, -160.0f);
    float n = rintf(y);
    float f = y - n;
    float p = 1.5252733804059840e-05f;
    p = HK_MAD(p, f, 1.5403530393381608e-04f);
    p = HK_MAD(p, f, 1.3333558146428443e-03f);
    p = HK_MAD(p, f, 9.6181291076284772e-03f);
    p = HK_MAD(p, f, 5.5504108664821580e-02f);
    p = HK_MAD(p, f, 2.4022650695910071e-01f);
    p = HK_MAD(p, f, 6.9314718055994531e-01f);
    p = HK_MAD(p, f, 1.0f);
    /* 2^n as an exponent field: 0 for n <= -127; for n >= -126 hk_exp's operations */
    const int32_t ni = (int32_t)hk_maxf(n, -127.0f);
    return p * hk_u2f((uint32_t)(ni + 127) << 23);
}

/* log2(x): x = m * 2^e with m in [sqrt(1/2), sqrt(2)); log2(m) via atanh series of s=(m-1)/(m+1).
 * Branch-free like hk_exp2 (x NaN -> x; x < 0 -> NaN; x == 0 -> -inf; x == +inf -> +inf; subnormal
 * x normalised first); the same bits as the branchy form for all 2^32 inputs. */
HK_HD float hk_log2(float x)
{
    const int sub = x < 1.17549435e-38f; /* normalize subnormals (x <= 0 and NaN are selected away below) */
    const float xn = sub ? x * 8388608.0f : x;
    const uint32_t u = hk_f2u(xn);
    int32_t e = (sub ? -23 : 0) + (int32_t)((u >> 23) & 0xFF) - 127;
    float m = hk_u2f((u & 0x007FFFFFu) | 0x3F800000u); /* [1,2) */
    const int big = m > 1.41421356f;
    m = big ? m * 0.5f : m;
    e += big ? 1 : 0;
    float s = (m - 1.0f) / (m + 1.0f);
    float s2 = s * s;
    float p = 0.11111111111111111f;          /* 1/9 */
    p = HK_MAD(p, s2, 0.14285714285714285f);       /* 1/7 */
    p = HK_MAD(p, s2, 0.2f);                       /* 1/5 */
    p = HK_MAD(p, s2, 0.33333333333333333f);       /* 1/3 */
    p = HK_MAD(p, s2, 1.0f);
    float lm = (p * s) * 2.8853900817779268f; /* 2/ln2 */
    float r = (float)e + lm;
    r = x == hk_u2f(0x7F800000u) ? x : r;
    r = x == 0.0f ? hk_u2f(0xFF800000u) : r;
    r = x < 0.0f ? hk_u2f(0x7FC00000u) : r;
    return x != x ? x : r;
}

/* WGSL pow(x, y) = exp2(y * log2(x)) for x >= 0 (NaN for x < 0). */
HK_HD float hk_pow(float x, float y) { return hk_exp2(y * hk_log2(x)); }

/* pow(x, n) for the literal integer exponents of the shaders — 5.0 in F_Schlick (Bevy
 * pbr lighting), 2.0 in the reservoir variance (light.wgsl:976), 16.0 in the denoiser's normal
 * weight (denoise.wgsl:48).  WGSL pins pow only to the accuracy of exp2(y * log2(x)), so the
 * build evaluates these by repeated multiplication (<= 3 ulp for n = 5, well inside that bound)
 * with hk_pow's domain: x < 0 or NaN -> NaN, +-0 -> +0, +inf -> +inf. */
HK_HD float hk_pow2(float x)
{
    if (!(x >= 0.0f)) return hk_u2f(0x7FC00000u);
    x = x + 0.0f; /* -0 -> +0 */
    return x * x;
}
HK_HD float hk_pow5(float x)
{
    if (!(x >= 0.0f)) return hk_u2f(0x7FC00000u);
    x = x + 0.0f;
    float x2 = x * x;
    return (x2 * x2) * x;
}
HK_HD float hk_pow16(float x)
{
    if (!(x >= 0.0f)) return hk_u2f(0x7FC00000u);
    x = x + 0.0f;
    float x2 = x * x;
    float x4 = x2 * x2;
    float x8 = x4 * x4;
    return x8 * x8;
}

/* sin/cos with Cody-Waite reduction by pi/2 and Taylor kernels on [-pi/4, pi/4]. */
HK_HD float hk_sin_kernel(float r)
{
    float r2 = r * r;
    float p = 2.7557319223985893e-06f;      /* 1/9! */
    p = p * r2 - 1.9841269841269841e-04f;   /* 1/7! */
    p = p * r2 + 8.3333333333333333e-03f;   /* 1/5! */
    p = p * r2 - 1.6666666666666667e-01f;   /* 1/3! */
    return r + (r * r2) * p;
}

HK_HD float hk_cos_kernel(float r)
{
    float r2 = r * r;
    float p = 2.4801587301587302e-05f;      /* 1/8! */
    p = p * r2 - 1.3888888888888889e-03f;   /* 1/6! */
    p = p * r2 + 4.1666666666666667e-02f;   /* 1/4! */
    p = p * r2 - 0.5f;
    return 1.0f + r2 * p;
}

/* Branch-free (round 5): both kernels computed, the quadrant's pair and the NaN / inf case selected — the same bits
 * as the branchy form on every input (oracle hko_math_form_mismatches); 16 calls per spatial-reuse pixel. */
HK_HD void hk_sincos(float x, float* s, float* c)
{
    const int special = x != x || hk_absf(x) == hk_u2f(0x7F800000u);
    float k = rintf(x * 0.63661977236758134f); /* 2/pi */
    /* pi/2 split into three parts; the first two have short mantissas */
    float r = x - k * 1.5703125f;
    r = r - k * 4.837512969970703125e-4f;
    r = r - k * 7.54978995489188216e-8f;
    /* k clamped before the conversion: |x| < 2^31 * pi/2 keeps it exact, larger |x| only select the quadrant */
    const int32_t q = ((int32_t)hk_minf(hk_maxf(k, -2147483520.0f), 2147483520.0f)) & 3;
    const float sk = hk_sin_kernel(r);
    const float ck = hk_cos_kernel(r);
    const int swap = q & 1;                  /* q = 1, 3: (s, c) = (+-ck, -+sk) */
    const float a = swap ? ck : sk, b = swap ? sk : ck;
    const float sa = (q == 2 || q == 3) ? -a : a;
    const float sb = (q == 1 || q == 2) ? -b : b;
    *s = special ? hk_u2f(0x7FC00000u) : sa;
    *c = special ? hk_u2f(0x7FC00000u) : sb;
}

HK_HD float hk_sin(float x) { float s, c; hk_sincos(x, &s, &c); return s; }
HK_HD float hk_cos(float x) { float s, c; hk_sincos(x, &s, &c); return c; }

/* ---- texel packing (WGSL pack / unpack built-ins) ---- */

/* f32 -> f16 bits, round-to-nearest-even, overflow -> inf, NaN -> quiet NaN. */
HK_HD uint32_t hk_f32_to_f16(float f)
{
    uint32_t x = hk_f2u(f);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t ex = (x >> 23) & 0xFFu;
    uint32_t man = x & 0x7FFFFFu;
    if (ex == 0xFFu) return sign | 0x7C00u | (man ? 0x200u : 0u);
    int32_t e = (int32_t)ex - 127 + 15;
    if (e >= 31) return sign | 0x7C00u;
    if (e <= 0) {
        if (e < -10) return sign;
        uint32_t m = man | 0x800000u;
        uint32_t shift = (uint32_t)(14 - e);
        uint32_t h = m >> shift;
        uint32_t rem = m & ((1u << shift) - 1u);
        uint32_t half = 1u << (shift - 1u);
        if (rem > half || (rem == half && (h & 1u))) h++;
        return sign | h;
    }
    uint32_t h = sign | ((uint32_t)e << 10) | (man >> 13);
    uint32_t rem = man & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return h;
}

HK_HD float hk_f16_to_f32(uint32_t h)
{
    uint32_t sign = (h & 0x8000u) << 16;
    uint32_t ex = (h >> 10) & 0x1Fu;
    uint32_t man = h & 0x3FFu;
    if (ex == 0) {
        if (man == 0) return hk_u2f(sign);
        /* subnormal: man * 2^-24, exact in f32 */
        float v = (float)man * 5.9604644775390625e-08f;
        return sign ? -v : v;
    }
    if (ex == 31) return hk_u2f(sign | 0x7F800000u | (man << 13));
    return hk_u2f(sign | ((ex + 112u) << 23) | (man << 13));
}

HK_HD uint32_t hk_pack2x16float(float a, float b) { return hk_f32_to_f16(a) | (hk_f32_to_f16(b) << 16); }
HK_HD float hk_unpack_lo16float(uint32_t v) { return hk_f16_to_f32(v & 0xFFFFu); }
HK_HD float hk_unpack_hi16float(uint32_t v) { return hk_f16_to_f32(v >> 16); }

/* pack2x16unorm: u16(round(clamp(e, 0, 1) * 65535)), round = nearest-even */
HK_HD uint32_t hk_unorm16(float e) { return (uint32_t)rintf(hk_clampf(e, 0.0f, 1.0f) * 65535.0f); }
HK_HD uint32_t hk_pack2x16unorm(float a, float b) { return hk_unorm16(a) | (hk_unorm16(b) << 16); }
HK_HD float hk_unpack_unorm16(uint32_t v) { return (float)(v & 0xFFFFu) / 65535.0f; }

/* pack4x8snorm: i8(round(clamp(e, -1, 1) * 127)) */
HK_HD uint32_t hk_snorm8(float e) { return ((uint32_t)(int32_t)rintf(hk_clampf(e, -1.0f, 1.0f) * 127.0f)) & 0xFFu; }
HK_HD uint32_t hk_pack4x8snorm(float x, float y, float z, float w)
{
    return hk_snorm8(x) | (hk_snorm8(y) << 8) | (hk_snorm8(z) << 16) | (hk_snorm8(w) << 24);
}
/* unpack4x8snorm component: max(f32(i8) / 127, -1) */
HK_HD float hk_unpack_snorm8(uint32_t v, int c)
{
    int32_t i = (int32_t)(int8_t)((v >> (8 * c)) & 0xFFu);
    return hk_maxf((float)i / 127.0f, -1.0f);
}

/* The same two decodes without the divide, for the device kernels (the oracle keeps the divisions
 * above as its restatement): q0 = v * RN(1/d) and one residual correction give RN(v / d) for every
 * input of these integer domains — all 65,536 unorm16 and all 256 snorm8 / unorm8 codes, checked exhaustively
 * by hko_unpack_fast_mismatches (tests/test_oracle_kat.py) and, for the formula itself, in exact
 * rational arithmetic.  3 instructions instead of the IEEE divide sequence. */
#define HK_INV_65535 0x1.00010p-16f /* RN(1 / 65535) */
#define HK_INV_127 0x1.020408p-7f   /* RN(1 / 127) */
#define HK_INV_255 0x1.010102p-8f   /* RN(1 / 255) */
HK_HD float hk_unpack_unorm16_fast(uint32_t v)
{
    const float x = (float)(v & 0xFFFFu);
    const float q = x * HK_INV_65535;
    return fmaf(fmaf(-q, 65535.0f, x), HK_INV_65535, q);
}
/* f32(byte) / 255 (an RGBA8 unorm texel, e.g. the blue noise) the same way: exact for all 256 codes */
HK_HD float hk_unorm8_fast(uint32_t byte)
{
    const float x = (float)(byte & 0xFFu);
    const float q = x * HK_INV_255;
    return fmaf(fmaf(-q, 255.0f, x), HK_INV_255, q);
}
HK_HD float hk_unpack_snorm8_fast(uint32_t v, int c)
{
    const float x = (float)(int32_t)(int8_t)((v >> (8 * c)) & 0xFFu);
    const float q = x * HK_INV_127;
    return hk_maxf(fmaf(fmaf(-q, 127.0f, x), HK_INV_127, q), -1.0f);
}

/* utils.wgsl:15-29 */
HK_HD uint32_t hk_hash(uint32_t value)
{
    uint32_t state = value;
    state = state ^ 2747636419u;
    state = state * 2654435769u;
    state = state ^ (state >> 16);
    state = state * 2654435769u;
    state = state ^ (state >> 16);
    state = state * 2654435769u;
    return state;
}

HK_HD float hk_random_float(uint32_t value) { return (float)hk_hash(value) / 4294967295.0f; }

/* utils.wgsl:62-64 (Rec. 709) */
HK_HD float hk_luminance(float r, float g, float b)
{
    return (r * 0.2126f + g * 0.7152f) + b * 0.0722f;
}

#endif /* HK_MATH_H */
