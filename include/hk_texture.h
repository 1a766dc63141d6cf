/*
 * hk_texture.h — material texture sampling shared by the CPU oracle and the gfx950 kernels.
 *
 * Restates the textured retreive_surface / retreive_emissive of light.wgsl:748-794:
 * `textureSampleLevel(textures[id], samplers[id], uv, 0.0)` on a Bevy `GpuImage` (RGBA8, sRGB
 * for base colour / emissive, linear for metallic-roughness / occlusion) with the image's
 * sampler (address mode per axis, magnification filter; explicit LOD 0 = the base level).
 * Hardware filtering precision is implementation-defined in WGSL/Vulkan (fixed-point weights on
 * most GPUs), so the build fixes ONE definition in IEEE f32, evaluated in the same order on both
 * sides (-ffp-contract=off):
 *   texel decode : LUT[byte] — sRGB: c <= 0.04045 ? c/12.92 : ((c+0.055)/1.055)^2.4 with
 *                  c = byte/255 (hk_pow), unorm: byte/255; 4 channels, alpha always unorm;
 *   nearest      : i = floor(u*W), j = floor(v*H);
 *   linear       : x = u*W - 0.5, i0 = floor(x), a = x - i0 (same for y), result =
 *                  (t00*(1-a) + t10*a)*(1-b) + (t01*(1-a) + t11*a)*b;
 *   addressing   : clamp-to-edge, repeat, mirror-repeat (WebGPU GPUAddressMode) on integer
 *                  texel coordinates; float->int conversion saturates, NaN -> 0.
 */
#ifndef HK_TEXTURE_H
#define HK_TEXTURE_H

#include <stdint.h>

#include "hk_math.h"

#define HK_TEXTURE_RGBA8_SRGB 0u
#define HK_TEXTURE_RGBA8_UNORM 1u
#define HK_ADDRESS_CLAMP_TO_EDGE 0u
#define HK_ADDRESS_REPEAT 1u
#define HK_ADDRESS_MIRROR_REPEAT 2u
#define HK_FILTER_NEAREST 0u
#define HK_FILTER_LINEAR 1u

/* device-side descriptor of one uploaded texture (32 bytes) */
typedef struct hk_texture_desc {
    uint32_t offset; /* first texel in the packed RGBA8 texel array */
    uint32_t width, height;
    uint32_t format, address_u, address_v, filter;
    uint32_t _pad;
} hk_texture_desc;

/* LUT[format * 256 + byte]: decoded channel value */
HK_HD float hk_texture_decode(uint32_t format, uint32_t byte)
{
    float c = (float)byte / 255.0f;
    if (format != HK_TEXTURE_RGBA8_SRGB) return c;
    if (c <= 0.04045f) return c / 12.92f;
    return hk_pow((c + 0.055f) / 1.055f, 2.4f);
}
HK_HD void hk_texture_build_lut(float* lut)
{
    for (uint32_t f = 0; f < 2; ++f)
        for (uint32_t b = 0; b < 256; ++b) lut[f * 256 + b] = hk_texture_decode(f, b);
}

HK_HD int32_t hk_tex_f2i(float x)
{
    if (x != x) return 0;
    if (x >= 2147483520.0f) return 2147483647;
    if (x <= -2147483648.0f) return (int32_t)0x80000000u;
    return (int32_t)x;
}
HK_HD int32_t hk_tex_address(int32_t i, int32_t n, uint32_t mode)
{
    if (mode == HK_ADDRESS_REPEAT) {
        int32_t r = i % n;
        return r < 0 ? r + n : r;
    }
    if (mode == HK_ADDRESS_MIRROR_REPEAT) {
        int64_t p = 2 * (int64_t)n;
        int64_t r = (int64_t)i % p;
        if (r < 0) r += p;
        return (int32_t)(r < n ? r : p - 1 - r);
    }
    return i < 0 ? 0 : (i >= n ? n - 1 : i);
}
HK_HD void hk_tex_fetch(const hk_texture_desc* t, const uint32_t* texels, const float* lut, int32_t x, int32_t y,
                        float* out)
{
    const uint32_t v = texels[t->offset + (uint32_t)y * t->width + (uint32_t)x];
    const float* l = lut + (t->format == HK_TEXTURE_RGBA8_SRGB ? 0 : 256);
    out[0] = l[v & 0xFFu];
    out[1] = l[(v >> 8) & 0xFFu];
    out[2] = l[(v >> 16) & 0xFFu];
    out[3] = lut[256 + (v >> 24)]; /* alpha is linear in sRGB formats */
}
/* textureSampleLevel(texture, sampler, uv, 0.0) -> out[4] */
HK_HD void hk_sample_texture(const hk_texture_desc* t, const uint32_t* texels, const float* lut, float u, float v,
                             float* out)
{
    const int32_t w = (int32_t)t->width, h = (int32_t)t->height;
    if (t->filter == HK_FILTER_NEAREST) {
        int32_t i = hk_tex_address(hk_tex_f2i(floorf(u * (float)w)), w, t->address_u);
        int32_t j = hk_tex_address(hk_tex_f2i(floorf(v * (float)h)), h, t->address_v);
        hk_tex_fetch(t, texels, lut, i, j, out);
        return;
    }
    const float x = u * (float)w - 0.5f, y = v * (float)h - 0.5f;
    const float x0 = floorf(x), y0 = floorf(y);
    const float a = x - x0, b = y - y0;
    const int32_t i0 = hk_tex_f2i(x0), j0 = hk_tex_f2i(y0);
    const int32_t ia = hk_tex_address(i0, w, t->address_u);
    const int32_t ib = hk_tex_address(i0 == 2147483647 ? i0 : i0 + 1, w, t->address_u);
    const int32_t ja = hk_tex_address(j0, h, t->address_v);
    const int32_t jb = hk_tex_address(j0 == 2147483647 ? j0 : j0 + 1, h, t->address_v);
    float t00[4], t10[4], t01[4], t11[4];
    hk_tex_fetch(t, texels, lut, ia, ja, t00);
    hk_tex_fetch(t, texels, lut, ib, ja, t10);
    hk_tex_fetch(t, texels, lut, ia, jb, t01);
    hk_tex_fetch(t, texels, lut, ib, jb, t11);
    const float ia_ = 1.0f - a, ib_ = 1.0f - b;
    for (int k = 0; k < 4; ++k) out[k] = (t00[k] * ia_ + t10[k] * a) * ib_ + (t01[k] * ia_ + t11[k] * a) * b;
}

#endif /* HK_TEXTURE_H */
