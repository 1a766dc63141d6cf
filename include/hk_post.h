/*
 * hk_post.h — SMAA TU4x and TAA "Jasmine" (post_process.rs:1236-1276, smaa.wgsl, taa.wgsl),
 * written once for both sides of the parity check: the CPU oracle calls these per pixel, the
 * gfx950 kernels (csrc/hk_post.hip) call the same functions from one thread per pixel.
 *
 * Textures are planes: RGBA16F render targets (4 x u16 per texel) or f32 G-buffer planes.
 * Samplers restate the reference's `nearest_sampler` / `linear_sampler` (post_process.rs:697-708,
 * default address mode = clamp-to-edge) at LOD 0:
 *   nearest  : texel (floor(u W), floor(v H)) clamped;
 *   linear   : x = u W - 0.5, i0 = floor(x), a = x - i0 (y alike), clamped texels,
 *              (t00 (1-a) + t10 a)(1-b) + (t01 (1-a) + t11 a) b   (one fixed f32 evaluation; GPU
 *              filtering precision is implementation-defined);
 *   gather   : component c of the linear footprint in WGSL order (i0,j1), (i1,j1), (i1,j0), (i0,j0);
 *   load     : textureLoad, out of bounds -> 0;  store: out of bounds ignored, f32 -> f16 RNE.
 * WGSL vector expressions are evaluated left to right per component (-ffp-contract=off).
 */
#ifndef HK_POST_H
#define HK_POST_H

#include <stdint.h>

#include "hk_math.h"

typedef struct hk_pp_tex {
    const void* data;
    uint32_t w, h;
    uint32_t f16;   /* 1: RGBA16F (u16 x 4), 0: f32 x comps */
    uint32_t comps; /* f32 planes: 4 (position, velocity_uv) or 2 (instance_material) */
} hk_pp_tex;

typedef struct hk_pp_out {
    uint16_t* data; /* RGBA16F */
    uint32_t w, h;
} hk_pp_out;

typedef struct hk_pp_frame {
    uint32_t number;
    float clear_color[4];
    float upscale_ratio;
} hk_pp_frame;

HK_HD int32_t hk_pp_f2i(float x)
{
    if (x != x) return 0;
    if (x >= 2147483520.0f) return 2147483647;
    if (x <= -2147483648.0f) return (int32_t)0x80000000u;
    return (int32_t)x;
}
HK_HD int32_t hk_pp_clampi(int32_t i, int32_t n) { return i < 0 ? 0 : (i >= n ? n - 1 : i); }
HK_HD void hk_pp_texel(const hk_pp_tex* t, int32_t x, int32_t y, float* o)
{
    const size_t i = (size_t)y * t->w + (size_t)x;
    if (t->f16) {
        const uint16_t* p = (const uint16_t*)t->data + 4 * i;
        for (int k = 0; k < 4; ++k) o[k] = hk_f16_to_f32(p[k]);
    } else {
        const float* p = (const float*)t->data + (size_t)t->comps * i;
        for (int k = 0; k < 4; ++k) o[k] = k < (int)t->comps ? p[k] : (k == 3 ? 1.0f : 0.0f);
    }
}
HK_HD void hk_pp_nearest(const hk_pp_tex* t, float u, float v, float* o)
{
    const int32_t x = hk_pp_clampi(hk_pp_f2i(floorf(u * (float)t->w)), (int32_t)t->w);
    const int32_t y = hk_pp_clampi(hk_pp_f2i(floorf(v * (float)t->h)), (int32_t)t->h);
    hk_pp_texel(t, x, y, o);
}
HK_HD void hk_pp_footprint(const hk_pp_tex* t, float u, float v, int32_t* i, int32_t* j, float* a, float* b)
{
    const float x = u * (float)t->w - 0.5f, y = v * (float)t->h - 0.5f;
    const float x0 = floorf(x), y0 = floorf(y);
    *a = x - x0;
    *b = y - y0;
    const int32_t ix = hk_pp_f2i(x0), iy = hk_pp_f2i(y0);
    i[0] = hk_pp_clampi(ix, (int32_t)t->w);
    i[1] = hk_pp_clampi(ix == 2147483647 ? ix : ix + 1, (int32_t)t->w);
    j[0] = hk_pp_clampi(iy, (int32_t)t->h);
    j[1] = hk_pp_clampi(iy == 2147483647 ? iy : iy + 1, (int32_t)t->h);
}
HK_HD void hk_pp_linear(const hk_pp_tex* t, float u, float v, float* o)
{
    int32_t i[2], j[2];
    float a, b;
    hk_pp_footprint(t, u, v, i, j, &a, &b);
    float t00[4], t10[4], t01[4], t11[4];
    hk_pp_texel(t, i[0], j[0], t00);
    hk_pp_texel(t, i[1], j[0], t10);
    hk_pp_texel(t, i[0], j[1], t01);
    hk_pp_texel(t, i[1], j[1], t11);
    const float ia = 1.0f - a, ib = 1.0f - b;
    for (int k = 0; k < 4; ++k) o[k] = (t00[k] * ia + t10[k] * a) * ib + (t01[k] * ia + t11[k] * a) * b;
}
HK_HD void hk_pp_gather(const hk_pp_tex* t, int comp, float u, float v, float* o)
{
    int32_t i[2], j[2];
    float a, b, c[4];
    hk_pp_footprint(t, u, v, i, j, &a, &b);
    hk_pp_texel(t, i[0], j[1], c);
    o[0] = c[comp];
    hk_pp_texel(t, i[1], j[1], c);
    o[1] = c[comp];
    hk_pp_texel(t, i[1], j[0], c);
    o[2] = c[comp];
    hk_pp_texel(t, i[0], j[0], c);
    o[3] = c[comp];
}
HK_HD void hk_pp_load(const hk_pp_out* t, int32_t x, int32_t y, float* o)
{
    if (x < 0 || y < 0 || (uint32_t)x >= t->w || (uint32_t)y >= t->h) {
        o[0] = o[1] = o[2] = o[3] = 0.0f;
        return;
    }
    const uint16_t* p = t->data + 4 * ((size_t)y * t->w + (size_t)x);
    for (int k = 0; k < 4; ++k) o[k] = hk_f16_to_f32(p[k]);
}
HK_HD void hk_pp_store(const hk_pp_out* t, int32_t x, int32_t y, const float* c)
{
    if (x < 0 || y < 0 || (uint32_t)x >= t->w || (uint32_t)y >= t->h) return;
    uint16_t* p = t->data + 4 * ((size_t)y * t->w + (size_t)x);
    for (int k = 0; k < 4; ++k) p[k] = (uint16_t)hk_f32_to_f16(c[k]);
}
HK_HD void hk_pp_uv(int32_t x, int32_t y, uint32_t w, uint32_t h, float* uv)
{
    uv[0] = ((float)x + 0.5f) / (float)w;
    uv[1] = ((float)y + 0.5f) / (float)h;
}

/* Playdead YCoCg helpers (taa.wgsl:20-42, smaa.wgsl:23-45) */
HK_HD void hk_pp_rgb_to_ycocg(const float* c, float* o)
{
    const float y = ((c[0] / 4.0f) + (c[1] / 2.0f)) + (c[2] / 4.0f);
    const float co = (c[0] / 2.0f) - (c[2] / 2.0f);
    const float cg = ((-c[0] / 4.0f) + (c[1] / 2.0f)) - (c[2] / 4.0f);
    o[0] = y, o[1] = co, o[2] = cg;
}
HK_HD void hk_pp_ycocg_to_rgb(const float* c, float* o)
{
    const float r = (c[0] + c[1]) - c[2];
    const float g = c[0] + c[2];
    const float b = (c[0] - c[1]) - c[2];
    o[0] = hk_clampf(r, 0.0f, 1.0f), o[1] = hk_clampf(g, 0.0f, 1.0f), o[2] = hk_clampf(b, 0.0f, 1.0f);
}
HK_HD void hk_pp_clip_towards_aabb_center(float* prev, const float* mn, const float* mx)
{
    float p[3], v[3], a[3];
    for (int k = 0; k < 3; ++k) {
        p[k] = 0.5f * (mx[k] + mn[k]);
        const float e = 0.5f * (mx[k] - mn[k]);
        v[k] = prev[k] - p[k];
        a[k] = hk_absf(v[k] / e);
    }
    const float ma = hk_maxf(a[0], hk_maxf(a[1], a[2]));
    if (ma > 1.0f)
        for (int k = 0; k < 3; ++k) prev[k] = p[k] + v[k] / ma;
}
HK_HD float hk_pp_dot4(const float* a, const float* b) { return ((a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]) + a[3] * b[3]; }

/* nearest_velocity (taa.wgsl:54-73, smaa.wgsl:52-71); texel = 1 / dims of `sized` */
HK_HD void hk_pp_nearest_velocity(const hk_pp_tex* position, const hk_pp_tex* velocity_uv, uint32_t sw, uint32_t sh,
                                  const float* uv, float* out)
{
    const float tx = 1.0f / (float)sw, ty = 1.0f / (float)sh;
    float d[4], c[4];
    hk_pp_nearest(position, uv[0] + tx, uv[1] + ty, c);
    d[0] = c[3];
    hk_pp_nearest(position, uv[0] + -tx, uv[1] + ty, c);
    d[1] = c[3];
    hk_pp_nearest(position, uv[0] + tx, uv[1] + -ty, c);
    d[2] = c[3];
    hk_pp_nearest(position, uv[0] + -tx, uv[1] + -ty, c);
    d[3] = c[3];
    const float max_depth = hk_maxf(hk_maxf(d[0], d[1]), hk_maxf(d[2], d[3]));
    hk_pp_nearest(position, uv[0], uv[1], c);
    const float depth = c[3];
    float ox = 0.0f, oy = 0.0f;
    if (depth < max_depth) {
        const float txv[4] = {tx, tx, tx, tx}, tyv[4] = {ty, ty, ty, ty};
        float sx[4], sy[4];
        const float px[4] = {1.0f, -1.0f, 1.0f, -1.0f}, py[4] = {1.0f, 1.0f, -1.0f, -1.0f};
        for (int k = 0; k < 4; ++k) {
            sx[k] = d[k] == max_depth ? px[k] : 0.0f;
            sy[k] = d[k] == max_depth ? py[k] : 0.0f;
        }
        ox = hk_pp_dot4(txv, sx);
        oy = hk_pp_dot4(tyv, sy);
    }
    hk_pp_nearest(velocity_uv, uv[0] + ox, uv[1] + oy, c);
    out[0] = c[0], out[1] = c[1];
}

typedef struct hk_pp_inputs {
    hk_pp_tex render, previous_render;           /* smaa: tone[current] / tone[previous]; taa: input / taa[previous] */
    hk_pp_tex position, previous_position, velocity_uv, previous_velocity_uv, instance_material;
    hk_pp_out output;
} hk_pp_inputs;

/* smaa.wgsl:81-199 — one thread per input pixel, writes 2 output pixels */
HK_HD void hk_pp_smaa_tu4x(const hk_pp_frame* F, const hk_pp_inputs* I, int32_t x, int32_t y)
{
    const uint32_t ow = I->output.w, oh = I->output.h;
    float uv[2];
    hk_pp_uv(x, y, I->render.w, I->render.h, uv);
    const float tsx = 1.0f / (float)ow, tsy = 1.0f / (float)oh;
    const float bias[5][2] = {{0.0f, 0.0f}, {2.5f * tsx, 2.5f * tsy}, {-2.5f * tsx, 2.5f * tsy},
                              {2.5f * tsx, -2.5f * tsy}, {-2.5f * tsx, -2.5f * tsy}};
    const int32_t cj = (F->number & 1u) == 0u ? 0 : 1, pj = (F->number & 1u) == 0u ? 1 : 0;
    const int32_t cx = 2 * x + cj, cy = 2 * y + cj;
    float c4[4];
    hk_pp_nearest(&I->render, uv[0], uv[1], c4);
    const float current[3] = {c4[0], c4[1], c4[2]};
    const int32_t px = 2 * x + pj, py = 2 * y + pj;
    float puv[2];
    hk_pp_uv(px, py, ow, oh, puv);
    float vel[2];
    hk_pp_nearest_velocity(&I->position, &I->velocity_uv, I->position.w, I->position.h, puv, vel);
    const float ru[2] = {puv[0] - vel[0], puv[1] - vel[1]};
    hk_pp_nearest(&I->previous_render, ru[0], ru[1], c4);
    float prev[3] = {c4[0], c4[1], c4[2]};
    const int boundary_miss = hk_absf(ru[0] - 0.5f) > 0.5f || hk_absf(ru[1] - 0.5f) > 0.5f;
    hk_pp_nearest(&I->instance_material, puv[0], puv[1], c4);
    const float current_instance = c4[0];
    int instance_miss = 0;
    hk_pp_nearest(&I->position, puv[0], puv[1], c4);
    const float current_depth = c4[3];
    int depth_miss = current_depth == 0.0f;
    for (int i = 0; i < 5; ++i) {
        float pd[4];
        hk_pp_gather(&I->previous_position, 3, ru[0] + bias[i][0], ru[1] + bias[i][1], pd);
        int any_low = 0;
        for (int k = 0; k < 4; ++k) {
            const float ratio = pd[k] == 0.0f ? 1.0f : current_depth / pd[k];
            any_low = any_low || ratio < 0.95f;
        }
        depth_miss = depth_miss || any_low;
        hk_pp_nearest(&I->instance_material, ru[0] + bias[i][0], ru[1] + bias[i][1], c4);
        instance_miss = instance_miss || (any_low && hk_absf(c4[0] - current_instance) > 1.0f);
    }
    hk_pp_nearest(&I->previous_velocity_uv, ru[0], ru[1], c4);
    const float dvx = vel[0] - c4[0], dvy = vel[1] - c4[1];
    const int velocity_miss = sqrtf(dvx * dvx + dvy * dvy) > 0.0001f;
    if (boundary_miss || ((depth_miss || instance_miss) && velocity_miss)) {
        float ub[2] = {0.0f, 0.0f};
        float min_ds = 10.0f;
        for (int i = 0; i < 5; ++i) {
            float ds[4];
            hk_pp_gather(&I->position, 3, puv[0] + bias[i][0], puv[1] + bias[i][1], ds);
            float e[4];
            for (int k = 0; k < 4; ++k) e[k] = current_depth - ds[k];
            const float dds = sqrtf(hk_pp_dot4(e, e));
            if (dds < min_ds) ub[0] = bias[i][0], ub[1] = bias[i][1];
            min_ds = hk_minf(min_ds, dds);
        }
        float cr[4], cg[4], cb[4];
        hk_pp_gather(&I->render, 0, puv[0] + ub[0], puv[1] + ub[1], cr);
        hk_pp_gather(&I->render, 1, puv[0] + ub[0], puv[1] + ub[1], cg);
        hk_pp_gather(&I->render, 2, puv[0] + ub[0], puv[1] + ub[1], cb);
        float s[4][3], m1[3], m2[3], mean[3], var[3], lo[3], hi[3];
        for (int q = 0; q < 4; ++q) {
            const float rgb[3] = {cr[q], cg[q], cb[q]};
            hk_pp_rgb_to_ycocg(rgb, s[q]);
        }
        for (int k = 0; k < 3; ++k) {
            m1[k] = ((s[0][k] + s[1][k]) + s[2][k]) + s[3][k];
            m2[k] = ((s[0][k] * s[0][k] + s[1][k] * s[1][k]) + s[2][k] * s[2][k]) + s[3][k] * s[3][k];
            mean[k] = m1[k] / 4.0f;
            var[k] = sqrtf((m2[k] / 4.0f) - (mean[k] * mean[k]));
            lo[k] = mean[k] - var[k];
            hi[k] = mean[k] + var[k];
        }
        float py_[3];
        hk_pp_rgb_to_ycocg(prev, py_);
        hk_pp_clip_towards_aabb_center(py_, lo, hi);
        hk_pp_ycocg_to_rgb(py_, prev);
    }
    const float spx = vel[0] / (2.0f * tsx), spy = vel[1] / (2.0f * tsy);
    float blend = hk_maxf(hk_fract(spx), hk_fract(spy));
    blend = hk_clampf(-hk_cos(blend * 6.283185307f), 0.0f, 1.0f);
    hk_pp_linear(&I->render, puv[0], puv[1], c4);
    for (int k = 0; k < 3; ++k) prev[k] = prev[k] * (1.0f - blend) + c4[k] * blend;
    const float co[4] = {current[0], current[1], current[2], 1.0f};
    const float po[4] = {prev[0], prev[1], prev[2], 1.0f};
    hk_pp_store(&I->output, cx, cy, co);
    hk_pp_store(&I->output, px, py, po);
}

/* smaa.wgsl:201-271 */
HK_HD void hk_pp_smaa_extrapolate(const hk_pp_out* O, int32_t x, int32_t y)
{
    float t[4], b[4], n[4], e[4], s[4], w[4];
    hk_pp_load(O, 2 * x, 2 * y, t);
    hk_pp_load(O, 2 * x + 1, 2 * y + 1, b);
    hk_pp_load(O, 2 * x + 1, 2 * y - 1, n);
    hk_pp_load(O, 2 * x + 2, 2 * y, e);
    hk_pp_load(O, 2 * x, 2 * y + 2, s);
    hk_pp_load(O, 2 * x - 1, 2 * y + 1, w);
    float d[3];
    for (int k = 0; k < 3; ++k) d[k] = hk_absf(w[k] - b[k]);
    const float dh0 = hk_luminance(d[0], d[1], d[2]);
    for (int k = 0; k < 3; ++k) d[k] = hk_absf(t[k] - e[k]);
    const float dh1 = hk_luminance(d[0], d[1], d[2]);
    for (int k = 0; k < 3; ++k) d[k] = hk_absf(t[k] - s[k]);
    const float dv0 = hk_luminance(d[0], d[1], d[2]);
    for (int k = 0; k < 3; ++k) d[k] = hk_absf(n[k] - b[k]);
    const float dv1 = hk_luminance(d[0], d[1], d[2]);
    const float fx = hk_maxf(dv0, 0.001f) * hk_maxf(dv1, 0.001f);
    const float fy = hk_maxf(dh0, 0.001f) * hk_maxf(dh1, 0.001f);
    const float fz = 1.0f / (fx + fy);
    float xc[4], yc[4];
    for (int k = 0; k < 4; ++k) {
        /* differential_blend(t, b, l, r): 0 + (l + r) fx + (t + b) fy, times 0.5 fz */
        float cx_ = 0.0f + (w[k] + b[k]) * fx;
        cx_ = cx_ + (t[k] + s[k]) * fy;
        xc[k] = (0.5f * fz) * cx_;
        float cy_ = 0.0f + (t[k] + e[k]) * fx;
        cy_ = cy_ + (n[k] + b[k]) * fy;
        yc[k] = (0.5f * fz) * cy_;
    }
    hk_pp_store(O, 2 * x, 2 * y + 1, xc);
    hk_pp_store(O, 2 * x + 1, 2 * y, yc);
}

/* taa.wgsl:75-170 */
HK_HD void hk_pp_taa(const hk_pp_frame* F, const hk_pp_inputs* I, int32_t x, int32_t y)
{
    const uint32_t ow = I->output.w, oh = I->output.h;
    const float tsx = 1.0f / (float)ow, tsy = 1.0f / (float)oh;
    float uv[2];
    hk_pp_uv(x, y, ow, oh, uv);
    float orig[4];
    hk_pp_nearest(&I->render, uv[0], uv[1], orig);
    const float current[3] = {orig[0], orig[1], orig[2]};
    float vel[2];
    hk_pp_nearest_velocity(&I->position, &I->velocity_uv, I->render.w, I->render.h, uv, vel);
    const float pu[2] = {uv[0] - vel[0], uv[1] - vel[1]};
    const int boundary_miss = hk_absf(pu[0] - 0.5f) > 0.5f || hk_absf(pu[1] - 0.5f) > 0.5f;
    const float bias[5][2] = {{0.0f, 0.0f}, {1.5f * tsx, 1.5f * tsy}, {-1.5f * tsx, 1.5f * tsy},
                              {1.5f * tsx, -1.5f * tsy}, {-1.5f * tsx, -1.5f * tsy}};
    float cpd[4];
    hk_pp_nearest(&I->position, uv[0], uv[1], cpd);
    int has_content = cpd[3] > 0.0f;
    int depth_miss = cpd[3] == 0.0f;
    int position_miss = cpd[3] == 0.0f;
    for (int i = 0; i < 5; ++i) {
        float pd[4], pp[4];
        hk_pp_gather(&I->previous_position, 3, pu[0] + bias[i][0], pu[1] + bias[i][1], pd);
        int any_pos = 0, any_low = 0;
        for (int k = 0; k < 4; ++k) {
            const float ratio = pd[k] == 0.0f ? 1.0f : cpd[3] / pd[k];
            any_pos = any_pos || pd[k] > 0.0f;
            any_low = any_low || ratio < 0.95f;
        }
        has_content = has_content || any_pos;
        depth_miss = depth_miss || any_low;
        hk_pp_nearest(&I->previous_position, pu[0] + bias[i][0], pu[1] + bias[i][1], pp);
        const float dx = cpd[0] - pp[0], dy = cpd[1] - pp[1], dz = cpd[2] - pp[2];
        position_miss = position_miss || sqrtf((dx * dx + dy * dy) + dz * dz) > 0.5f;
    }
    if (!has_content) {
        hk_pp_store(&I->output, x, y, F->clear_color);
        return;
    }
    float pv[4];
    hk_pp_nearest(&I->previous_velocity_uv, pu[0], pu[1], pv);
    const float dvx = vel[0] - pv[0], dvy = vel[1] - pv[1];
    const int velocity_miss = sqrtf(dvx * dvx + dvy * dvy) > 0.00005f;
    /* 5-tap Catmull-Rom */
    const float size[2] = {(float)ow, (float)oh}, ts[2] = {tsx, tsy};
    float w0[2], w3[2], w12[2], t0[2], t3[2], t12[2];
    for (int k = 0; k < 2; ++k) {
        const float sp = (uv[k] - vel[k]) * size[k];
        const float t1 = floorf(sp - 0.5f) + 0.5f;
        const float f = sp - t1;
        w0[k] = f * (-0.5f + f * (1.0f - 0.5f * f));
        const float w1 = 1.0f + (f * f) * (-2.5f + 1.5f * f);
        const float w2 = f * (0.5f + f * (2.0f - 1.5f * f));
        w3[k] = (f * f) * (-0.5f + 0.5f * f);
        w12[k] = w1 + w2;
        const float o12 = w2 / (w1 + w2);
        t0[k] = (t1 - 1.0f) * ts[k];
        t3[k] = (t1 + 2.0f) * ts[k];
        t12[k] = (t1 + o12) * ts[k];
    }
    float prev[3] = {0.0f, 0.0f, 0.0f}, c4[4];
    const float taps[5][4] = {{t12[0], t0[1], w12[0], w0[1]},
                              {t0[0], t12[1], w0[0], w12[1]},
                              {t12[0], t12[1], w12[0], w12[1]},
                              {t3[0], t12[1], w3[0], w12[1]},
                              {t12[0], t3[1], w12[0], w3[1]}};
    for (int i = 0; i < 5; ++i) {
        hk_pp_linear(&I->previous_render, taps[i][0], taps[i][1], c4);
        for (int k = 0; k < 3; ++k) prev[k] = prev[k] + (hk_clampf(c4[k], 0.0f, 1.0f) * taps[i][2]) * taps[i][3];
    }
    if (boundary_miss || (position_miss && velocity_miss && depth_miss)) {
        const float off[9][2] = {{-tsx, tsy}, {0.0f, tsy}, {tsx, tsy}, {-tsx, -0.0f}, {0.0f, 0.0f},
                                 {tsx, 0.0f}, {-tsx, -tsy}, {-0.0f, -tsy}, {tsx, -tsy}};
        float s[9][3];
        for (int q = 0; q < 9; ++q) {
            float rgb[3];
            if (q == 4) {
                for (int k = 0; k < 3; ++k) rgb[k] = current[k];
            } else {
                /* uv - vec2(t, 0) for the ml / bm / bl taps: uv + (-t) */
                hk_pp_nearest(&I->render, uv[0] + off[q][0], uv[1] + off[q][1], c4);
                for (int k = 0; k < 3; ++k) rgb[k] = hk_clampf(c4[k], 0.0f, 1.0f);
            }
            hk_pp_rgb_to_ycocg(rgb, s[q]);
        }
        float lo[3], hi[3];
        for (int k = 0; k < 3; ++k) {
            float m1 = s[0][k], m2 = s[0][k] * s[0][k];
            for (int q = 1; q < 9; ++q) {
                m1 = m1 + s[q][k];
                m2 = m2 + s[q][k] * s[q][k];
            }
            const float mean = m1 / 9.0f;
            const float var = sqrtf((m2 / 9.0f) - (mean * mean));
            lo[k] = mean - var;
            hi[k] = mean + var;
        }
        float py_[3];
        hk_pp_rgb_to_ycocg(prev, py_);
        hk_pp_clip_towards_aabb_center(py_, lo, hi);
        hk_pp_ycocg_to_rgb(py_, prev);
    }
    const float t = 0.1f / F->upscale_ratio;
    float o[4];
    for (int k = 0; k < 3; ++k) o[k] = prev[k] * (1.0f - t) + current[k] * t;
    o[3] = orig[3];
    hk_pp_store(&I->output, x, y, o);
}

#endif /* HK_POST_H */
