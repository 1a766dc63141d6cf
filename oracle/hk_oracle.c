/*
 * hk_oracle.c — TEST INFRASTRUCTURE ONLY (see hk_oracle.h for the parity status).
 *
 * Line-by-line C restatement of bevy-hikari's integrator and denoiser:
 *   src/shaders/light.wgsl      (entry points full_screen_albedo, direct_lit, indirect_lit_ambient,
 *                                spatial_reuse with the EMISSIVE_LIT / RENDER_EMISSIVE /
 *                                MULTIPLE_BOUNCES / NO_TEXTURE shader defs)
 *   src/shaders/denoise.wgsl    (demodulation, denoise levels 0-3, FIREFLY_FILTERING)
 *   src/shaders/tone_mapping.wgsl
 *   src/shaders/utils.wgsl, mesh_material_types.wgsl
 *   dispatch order of LightNode::run (light.rs:590-702) and the denoise block of
 *   PostProcessNode::run (post_process.rs:1190-1224), reservoir pairing light.rs:518-546
 *   Bevy 0.9.1 PBR functions (third-party, recalled)
 * The G-buffer comes from a primary-ray restatement of prepass.wgsl:84-100.
 *
 * Conventions that the WGSL leaves implementation-defined, fixed identically here and in
 * the HIP kernels: vector expressions evaluate left to right, dot = (x*x'+y*y')+z*z',
 * normalize(v) = v * (1/sqrt(dot(v,v))), mix(a,b,t) = a*(1-t)+b*t, min/max = IEEE
 * minNum/maxNum, transcendentals from include/hk_math.h, out-of-bounds textureLoad
 * returns 0, u32/i32 from f32 truncate and saturate (NaN -> 0), x % 0 == 0.
 */
#include "hk_oracle.h"
#include "../include/hk_math.h"
#include "../include/hk_texture.h"
#include "../include/hk_post.h"

#include <stdlib.h>
#include <stdio.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ vectors */
typedef struct { float x, y; } v2;
typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } v4;

static inline v2 V2(float x, float y) { v2 r = {x, y}; return r; }
static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v4 V4(float x, float y, float z, float w) { v4 r = {x, y, z, w}; return r; }
static inline v3 xyz(v4 a) { return V3(a.x, a.y, a.z); }
static inline v3 add3(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub3(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul3(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 scale3(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 div3s(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline v3 neg3(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline float dot3(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline float dot2(v2 a, v2 b) { return a.x * b.x + a.y * b.y; }
static inline v3 cross3(v3 a, v3 b)
{
    return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float length3(v3 a) { return sqrtf(dot3(a, a)); }
static inline v3 normalize3(v3 a) { return scale3(a, 1.0f / sqrtf(dot3(a, a))); }
static inline v3 min3(v3 a, v3 b) { return V3(hk_minf(a.x, b.x), hk_minf(a.y, b.y), hk_minf(a.z, b.z)); }
static inline v3 max3(v3 a, v3 b) { return V3(hk_maxf(a.x, b.x), hk_maxf(a.y, b.y), hk_maxf(a.z, b.z)); }
static inline v3 mix3(v3 a, v3 b, float t)
{
    float it = 1.0f - t;
    return V3(a.x * it + b.x * t, a.y * it + b.y * t, a.z * it + b.z * t);
}
static inline v3 fract3(v3 a) { return V3(hk_fract(a.x), hk_fract(a.y), hk_fract(a.z)); }
static inline v3 ld3(const float* p) { return V3(p[0], p[1], p[2]); }
static inline float sum4(v4 a) { return ((a.x + a.y) + a.z) + a.w; } /* dot(a, vec4(1.0)) */
static inline float lum3(v3 c) { return hk_luminance(c.x, c.y, c.z); }

/* WGSL u32(f32) / i32(f32): truncate toward zero, saturate, NaN -> 0 */
static inline uint32_t f2u32(float x)
{
    if (!(x > 0.0f)) return 0u;
    if (x >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)x;
}
static inline int32_t f2i32(float x)
{
    if (x != x) return 0;
    if (x >= 2147483648.0f) return 0x7FFFFFFF;
    if (x <= -2147483648.0f) return (int32_t)0x80000000u;
    return (int32_t)x;
}
static inline uint32_t umod(uint32_t a, uint32_t b) { return b ? a % b : 0u; }

/* column-major mat4 * vec4 = ((c0*x + c1*y) + c2*z) + c3*w */
static inline v4 mat4_mul(const float* m, v4 v)
{
    v4 r;
    r.x = ((m[0] * v.x + m[4] * v.y) + m[8] * v.z) + m[12] * v.w;
    r.y = ((m[1] * v.x + m[5] * v.y) + m[9] * v.z) + m[13] * v.w;
    r.z = ((m[2] * v.x + m[6] * v.y) + m[10] * v.z) + m[14] * v.w;
    r.w = ((m[3] * v.x + m[7] * v.y) + m[11] * v.z) + m[15] * v.w;
    return r;
}
/* transpose(m) * v: row i of m dotted with v in the same left-to-right order */
static inline v4 mat4_tmul(const float* m, v4 v)
{
    v4 r;
    r.x = ((m[0] * v.x + m[1] * v.y) + m[2] * v.z) + m[3] * v.w;
    r.y = ((m[4] * v.x + m[5] * v.y) + m[6] * v.z) + m[7] * v.w;
    r.z = ((m[8] * v.x + m[9] * v.y) + m[10] * v.z) + m[11] * v.w;
    r.w = ((m[12] * v.x + m[13] * v.y) + m[14] * v.z) + m[15] * v.w;
    return r;
}

/* ------------------------------------------------------------------ constants (light.wgsl:226-256) */
#define RAY_BIAS 0.02f
#define DISTANCE_MAX 65535.0f
#define NOISE_TEXTURE_COUNT 16u
#define MAX_VARIANCE 10.0f
#define DONT_EXCLUDE 0xFFFFFFFFu
#define DONT_SAMPLE_EMISSIVE 0x80000000u
#define SPATIAL_REUSE_TAPS 4u
#define DIRECT_VALIDATION_FRAME_SAMPLE_THRESHOLD 4u
#define SPATIAL_VARIANCE_SAMPLE_THRESHOLD 4u

/* ------------------------------------------------------------------ context */
struct hko_ctx {
    hk_vertex* vertices; uint32_t n_vertices;
    hk_primitive* primitives; uint32_t n_primitives;
    hk_node* asset_nodes; uint32_t n_asset_nodes;
    hk_alias_entry* alias_table; uint32_t n_alias;
    hk_instance* instances; uint32_t n_instances;
    hk_node* instance_nodes; uint32_t n_instance_nodes;
    hk_material* materials; uint32_t n_materials;
    hk_node* emissive_nodes; uint32_t n_emissive_nodes;
    hk_emissive* emissives; uint32_t n_emissives;
    /* GlobalTransformQueue[1] (transform.rs:32-44): every instance's model as of the previous
     * hko_render_gbuffer, read by the motion vectors (prepass.wgsl:50,96) */
    float* prev_models;
    /* material textures (hko_set_textures; none = the NO_TEXTURE pipeline) */
    hk_texture_desc* tex_desc; uint32_t* texels; uint32_t n_textures;
    float tex_lut[512];
    uint8_t noise[16 * 64 * 64 * 4];

    uint32_t S[2], s[2];
    float ratio;
    int threads;

    /* G-buffer (S) */
    float* g_position;        /* 4 */
    uint32_t* g_normal;       /* 1 */
    float* g_depth_gradient;  /* 2 */
    float* g_instance_material; /* 2 */
    float* g_velocity_uv;     /* 4 */
    float* g_prev_position;   /* previous frame's planes (prepass.rs:309-317 swap) */
    float* g_prev_velocity_uv;
    uint32_t head;            /* frame_number % 2 */
    /* light textures */
    uint16_t* albedo;         /* 4 x f16, S */
    float* variance[3];       /* s */
    uint16_t* render[3];      /* 4 x f16, s */
    hk_packed_reservoir* reservoirs[HK_RESERVOIR_BUFFERS]; /* S.x*S.y each */
    /* denoise */
    uint16_t* internal[4];
    float* internal_variance;
    uint16_t* denoised[3];
    uint16_t* tone;           /* = tone_buf[head] */
    uint16_t* tone_buf[2];
    uint16_t* upscale; uint32_t upscale_wh[2];
    uint16_t* taa_buf[2]; uint32_t taa_wh[2];
    hk_counters counters;
    int32_t band_y0, band_y1; /* rows computed by every pass (whole frame by default) */
    int32_t band_x0, band_x1; /* ... and columns (hko_set_tile; the whole width by default) */
    int32_t stripe_n, stripe_k; /* hko_set_stripes: only rows of 8-row stripes k, k + n, ... (n >= 2) */
    /* the closest-hit light walks (the indirect bounce, light.wgsl:1319,1401; the emitter BLAS walk of
     * select_light_candidate, light.wgsl:687): hko_set_light_walk */
    int light_walk;
    unsigned long long walk_checked[2], walk_differ[2]; /* [bounce, emitter], light_walk == HKO_WALK_CHECK */
};

typedef struct {
    uint64_t top, emitter, primary;
} Counts;

/* per-dispatch "bindings" */
typedef struct {
    const hko_ctx* c;
    const hk_settings* st;
    const hk_frame_inputs* in;
    uint32_t number;
    int emissive_lit, render_emissive, multiple_bounces;
    hk_packed_reservoir* previous_reservoir_buffer;
    hk_packed_reservoir* reservoir_buffer;
    hk_packed_reservoir* previous_spatial_reservoir_buffer;
    hk_packed_reservoir* spatial_reservoir_buffer;
    float* variance_texture;
    uint16_t* render_texture;
} Pass;

/* ------------------------------------------------------------------ texel helpers */
static inline void store_rgba16f(uint16_t* tex, uint32_t idx, v4 c)
{
    tex[4 * idx + 0] = (uint16_t)hk_f32_to_f16(c.x);
    tex[4 * idx + 1] = (uint16_t)hk_f32_to_f16(c.y);
    tex[4 * idx + 2] = (uint16_t)hk_f32_to_f16(c.z);
    tex[4 * idx + 3] = (uint16_t)hk_f32_to_f16(c.w);
}
static inline v4 load_rgba16f(const uint16_t* tex, uint32_t idx)
{
    return V4(hk_f16_to_f32(tex[4 * idx + 0]), hk_f16_to_f32(tex[4 * idx + 1]), hk_f16_to_f32(tex[4 * idx + 2]),
              hk_f16_to_f32(tex[4 * idx + 3]));
}
static inline int in_bounds(int32_t x, int32_t y, const uint32_t* size)
{
    return x >= 0 && y >= 0 && (uint32_t)x < size[0] && (uint32_t)y < size[1];
}
/* textureLoad on the deferred textures (size S); out of bounds -> 0 */
static inline v4 load_position(const hko_ctx* c, int32_t x, int32_t y)
{
    if (!in_bounds(x, y, c->S)) return V4(0, 0, 0, 0);
    const float* p = c->g_position + 4 * ((size_t)y * c->S[0] + x);
    return V4(p[0], p[1], p[2], p[3]);
}
static inline v3 load_normal(const hko_ctx* c, int32_t x, int32_t y)
{
    if (!in_bounds(x, y, c->S)) return V3(0, 0, 0);
    uint32_t n = c->g_normal[(size_t)y * c->S[0] + x];
    return V3(hk_unpack_snorm8(n, 0), hk_unpack_snorm8(n, 1), hk_unpack_snorm8(n, 2));
}
static inline v2 load_instance_material(const hko_ctx* c, int32_t x, int32_t y)
{
    if (!in_bounds(x, y, c->S)) return V2(0, 0);
    const float* p = c->g_instance_material + 2 * ((size_t)y * c->S[0] + x);
    return V2(p[0], p[1]);
}
static inline v4 load_velocity_uv(const hko_ctx* c, int32_t x, int32_t y)
{
    if (!in_bounds(x, y, c->S)) return V4(0, 0, 0, 0);
    const float* p = c->g_velocity_uv + 4 * ((size_t)y * c->S[0] + x);
    return V4(p[0], p[1], p[2], p[3]);
}
static inline v2 load_depth_gradient(const hko_ctx* c, int32_t x, int32_t y)
{
    if (!in_bounds(x, y, c->S)) return V2(0, 0);
    const float* p = c->g_depth_gradient + 2 * ((size_t)y * c->S[0] + x);
    return V2(p[0], p[1]);
}
/* nearest sampler, ClampToEdge: texel = clamp(floor(uv * size)) */
static inline void nearest_texel(v2 uv, const uint32_t* size, int32_t* x, int32_t* y)
{
    float fx = floorf(uv.x * (float)size[0]);
    float fy = floorf(uv.y * (float)size[1]);
    int32_t ix = f2i32(fx), iy = f2i32(fy);
    if (ix < 0) ix = 0;
    if (iy < 0) iy = 0;
    if (ix > (int32_t)size[0] - 1) ix = (int32_t)size[0] - 1;
    if (iy > (int32_t)size[1] - 1) iy = (int32_t)size[1] - 1;
    *x = ix;
    *y = iy;
}

/* utils.wgsl:41-44 */
static inline v2 coords_to_uv(int32_t x, int32_t y, const uint32_t* size)
{
    return V2(((float)x + 0.5f) / (float)size[0], ((float)y + 0.5f) / (float)size[1]);
}

/* light.wgsl:1007-1017 */
static inline v2 jittered_deferred_uv(const Pass* P, v2 uv)
{
    float tx = 1.0f / (float)P->c->S[0], ty = 1.0f / (float)P->c->S[1];
    float ratio = P->st->upscale_ratio - 1.0f;
    float j = (P->number & 1u) == 0u ? -0.25f : 0.25f;
    return V2(uv.x + (j * tx) * ratio, uv.y + (j * ty) * ratio);
}
static inline void jittered_deferred_coords(const Pass* P, v2 uv, int32_t* x, int32_t* y)
{
    v2 d = jittered_deferred_uv(P, uv);
    *x = f2i32(d.x * (float)P->c->S[0]);
    *y = f2i32(d.y * (float)P->c->S[1]);
}

/* ------------------------------------------------------------------ reservoirs (light.wgsl:45-223) */
typedef struct {
    v4 radiance;
    v4 random;
    v4 visible_position;
    v3 visible_normal;
    uint32_t visible_instance;
    v4 sample_position;
    v3 sample_normal;
} Sample;

typedef struct {
    Sample s;
    float count, lifetime, w, w_sum, w2_sum;
} Reservoir;

static Reservoir unpack_reservoir(const hk_packed_reservoir* p)
{
    Reservoir r;
    memset(&r, 0, sizeof(r));
    r.count = hk_unpack_lo16float(p->reservoir[0]);
    r.w = hk_unpack_hi16float(p->reservoir[0]);
    r.w_sum = hk_unpack_lo16float(p->reservoir[1]);
    r.w2_sum = hk_unpack_hi16float(p->reservoir[1]);
    r.s.radiance = V4(hk_unpack_lo16float(p->radiance[0]), hk_unpack_hi16float(p->radiance[0]),
                      hk_unpack_lo16float(p->radiance[1]), hk_unpack_hi16float(p->radiance[1]));
    r.s.random = V4(hk_unpack_unorm16(p->random[0]), hk_unpack_unorm16(p->random[0] >> 16),
                    hk_unpack_unorm16(p->random[1]), hk_unpack_unorm16(p->random[1] >> 16));
    uint32_t vn = p->visible_normal;
    r.s.visible_position = V4(p->visible_position[0], p->visible_position[1], p->visible_position[2],
                              p->visible_position[3]);
    r.s.visible_normal = normalize3(V3(hk_unpack_snorm8(vn, 0), hk_unpack_snorm8(vn, 1), hk_unpack_snorm8(vn, 2)));
    r.lifetime = 127.0f * (1.0f + hk_unpack_snorm8(vn, 3));
    uint32_t sn = p->sample_normal;
    r.s.sample_position = V4(p->sample_position[0], p->sample_position[1], p->sample_position[2], hk_unpack_snorm8(sn, 3));
    r.s.sample_normal = normalize3(V3(hk_unpack_snorm8(sn, 0), hk_unpack_snorm8(sn, 1), hk_unpack_snorm8(sn, 2)));
    r.s.visible_instance = f2u32(p->sample_position[3]);
    return r;
}

static void pack_reservoir(const Reservoir* r, hk_packed_reservoir* p)
{
    p->reservoir[0] = hk_pack2x16float(r->count, r->w);
    p->reservoir[1] = hk_pack2x16float(r->w_sum, r->w2_sum);
    p->radiance[0] = hk_pack2x16float(r->s.radiance.x, r->s.radiance.y);
    p->radiance[1] = hk_pack2x16float(r->s.radiance.z, r->s.radiance.w);
    p->random[0] = hk_pack2x16unorm(r->s.random.x, r->s.random.y);
    p->random[1] = hk_pack2x16unorm(r->s.random.z, r->s.random.w);
    p->visible_position[0] = r->s.visible_position.x;
    p->visible_position[1] = r->s.visible_position.y;
    p->visible_position[2] = r->s.visible_position.z;
    p->visible_position[3] = r->s.visible_position.w;
    p->sample_position[0] = r->s.sample_position.x;
    p->sample_position[1] = r->s.sample_position.y;
    p->sample_position[2] = r->s.sample_position.z;
    p->sample_position[3] = (float)r->s.visible_instance;
    p->visible_normal = hk_pack4x8snorm(r->s.visible_normal.x, r->s.visible_normal.y, r->s.visible_normal.z,
                                        r->lifetime / 127.0f - 1.0f);
    p->sample_normal = hk_pack4x8snorm(r->s.sample_normal.x, r->s.sample_normal.y, r->s.sample_normal.z,
                                       r->s.sample_position.w);
}

static void set_reservoir(Reservoir* r, const Sample* s, float w_new)
{
    r->count = 1.0f;
    r->lifetime = 0.0f;
    r->w_sum = w_new;
    r->w2_sum = w_new * w_new;
    r->s = *s;
}

static void update_reservoir(Reservoir* r, const Sample* s, float w_new)
{
    r->w_sum += w_new;
    r->w2_sum += w_new * w_new;
    r->count = r->count + 1.0f;
    float rand = hk_fract(sum4(s->random));
    if (rand < w_new / r->w_sum) r->s = *s;
}

static void merge_reservoir(Reservoir* r, const Reservoir* other, float p)
{
    float count = r->count;
    update_reservoir(r, &other->s, (p * other->w) * other->count);
    r->count = count + other->count;
}

static inline int uv_inside_open(v2 uv) /* all(abs(uv - 0.5) < vec2(0.5)) */
{
    return hk_absf(uv.x - 0.5f) < 0.5f && hk_absf(uv.y - 0.5f) < 0.5f;
}
static inline int uv_inside_closed(v2 uv) /* all(abs(uv - 0.5) <= vec2(0.5)) */
{
    return hk_absf(uv.x - 0.5f) <= 0.5f && hk_absf(uv.y - 0.5f) <= 0.5f;
}

static Reservoir load_previous_from(const hk_packed_reservoir* buf, v2 uv, const uint32_t* size)
{
    Reservoir r;
    memset(&r, 0, sizeof(r));
    if (uv_inside_open(uv)) {
        int32_t x = f2i32(uv.x * (float)size[0]);
        int32_t y = f2i32(uv.y * (float)size[1]);
        int32_t index = x + (int32_t)size[0] * y;
        r = unpack_reservoir(&buf[index]);
    }
    return r;
}

/* ------------------------------------------------------------------ tracing (light.wgsl:259-533) */
typedef struct { v3 origin, direction, inv_direction; } Ray;
typedef struct { v3 min, max; } Aabb;
typedef struct { v2 uv; float distance; } Intersection;
typedef struct { Intersection intersection; uint32_t instance_index, primitive_index; } Hit;
typedef struct { v4 base_color, emissive; float reflectance, metallic, roughness, occlusion; } Surface;
typedef struct { v4 position; v3 normal; v2 uv; uint32_t instance_index, material_index; } HitInfo;
typedef struct { v3 direction; float max_distance, min_distance; uint32_t emissive_instance; float p; } LightCandidate;

static inline v3 inv3(v3 d) { return V3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z); }

static inline const hk_instance* get_instance(const hko_ctx* c, uint32_t i)
{
    return &c->instances[i < c->n_instances ? i : c->n_instances - 1];
}
static inline const hk_material* get_material(const hko_ctx* c, uint32_t i)
{
    return &c->materials[i < c->n_materials ? i : c->n_materials - 1];
}

static v3 instance_position_world_to_local(const hk_instance* in, v3 p)
{
    v4 r = mat4_tmul(in->inverse_transpose_model, V4(p.x, p.y, p.z, 1.0f));
    return div3s(xyz(r), r.w);
}
static v3 instance_direction_world_to_local(const hk_instance* in, v3 p)
{
    return xyz(mat4_tmul(in->inverse_transpose_model, V4(p.x, p.y, p.z, 0.0f)));
}
static v3 instance_position_local_to_world(const hk_instance* in, v3 p)
{
    v4 r = mat4_mul(in->model, V4(p.x, p.y, p.z, 1.0f));
    return div3s(xyz(r), r.w);
}
static v3 instance_normal_local_to_world(const hk_instance* in, v3 n)
{
    const float* m = in->inverse_transpose_model;
    v3 r;
    r.x = (m[0] * n.x + m[4] * n.y) + m[8] * n.z;
    r.y = (m[1] * n.x + m[5] * n.y) + m[9] * n.z;
    r.z = (m[2] * n.x + m[6] * n.y) + m[10] * n.z;
    return normalize3(r);
}

static inline int inside_aabb(v3 p, Aabb a)
{
    return (p.x > a.min.x && p.y > a.min.y && p.z > a.min.z) && (p.x < a.max.x && p.y < a.max.y && p.z < a.max.z);
}

static float intersects_aabb(const Ray* ray, Aabb aabb)
{
    v3 t1 = mul3(sub3(aabb.min, ray->origin), ray->inv_direction);
    v3 t2 = mul3(sub3(aabb.max, ray->origin), ray->inv_direction);
    float t_min = hk_minf(t1.x, t2.x);
    float t_max = hk_maxf(t1.x, t2.x);
    t_min = hk_maxf(t_min, hk_minf(t1.y, t2.y));
    t_max = hk_minf(t_max, hk_maxf(t1.y, t2.y));
    t_min = hk_maxf(t_min, hk_minf(t1.z, t2.z));
    t_max = hk_minf(t_max, hk_maxf(t1.z, t2.z));
    float t = HK_F32_MAX;
    if (t_max >= t_min && t_max >= 0.0f) t = t_min;
    return t;
}

static Intersection intersects_triangle(const Ray* ray, const hk_primitive_vertex* tri)
{
    Intersection result;
    result.uv = V2(0, 0);
    result.distance = HK_F32_MAX;
    v3 p0 = ld3(tri[0].position), p1 = ld3(tri[1].position), p2 = ld3(tri[2].position);
    v3 ab = sub3(p1, p0);
    v3 ac = sub3(p2, p0);
    v3 u_vec = cross3(ray->direction, ac);
    float det = dot3(ab, u_vec);
    if (hk_absf(det) < HK_F32_EPSILON) return result;
    float inv_det = 1.0f / det;
    v3 ao = sub3(ray->origin, p0);
    float u = dot3(ao, u_vec) * inv_det;
    if (u < 0.0f || u > 1.0f) {
        result.uv = V2(u, 0.0f);
        return result;
    }
    v3 v_vec = cross3(ao, ab);
    float v = dot3(ray->direction, v_vec) * inv_det;
    result.uv = V2(u, v);
    if (v < 0.0f || u + v > 1.0f) return result;
    float distance = dot3(ac, v_vec) * inv_det;
    if (distance > HK_F32_EPSILON) result.distance = distance;
    return result;
}

#ifdef HKO_STATS
/* traversal statistics (analysis builds only): [class][calls, tlas nodes, instances entered,
 * blas nodes, triangle tests]; class 0 closest, 1 directional any-hit, 2 emissive any-hit,
 * 3 emitter BLAS walk of select_light_candidate */
unsigned long long hko_stats[4][5];
static __thread int hko_class = 3;
static __thread unsigned hko_ray_steps; /* node visits + leaf tests of the current traverse_top */
uint32_t* hko_steps_out;                 /* per-ray steps of hko_trace, if set */
unsigned long long hko_hit_infos;        /* hit_info calls (3 vertices + instance + material fetched) */
/* per-pixel walk steps of the light passes, if set: [pass 0 direct_lit, 1 emissive, 2 indirect][class][s pixel],
 * node visits + leaf tests of every walk of that class (the lane-efficiency model of tools/walk_lanes.py) */
uint32_t* hko_pixel_steps_out;
static __thread int32_t hko_pixel = -1, hko_pass = 0;
static __thread uint32_t hko_npix;
#define HKO_STAT(k) (__atomic_fetch_add(&hko_stats[hko_class][k], 1ull, __ATOMIC_RELAXED), hko_ray_steps++, \
                     (hko_pixel_steps_out && hko_pixel >= 0 ?                                                  \
                      (void)hko_pixel_steps_out[((size_t)hko_pass * 4u + (size_t)hko_class) * hko_npix + (size_t)hko_pixel]++ \
                      : (void)0))
#else
#define HKO_STAT(k) ((void)0)
#endif

static int traverse_bottom(const hko_ctx* c, Hit* hit, const Ray* ray, hk_mesh_index mesh, float early_distance)
{
    int intersected = 0;
    uint32_t index = 0u;
    while (index < mesh.node[1]) {
        HKO_STAT(3);
        uint32_t node_index = mesh.node[0] + index;
        const hk_node* node = &c->asset_nodes[node_index];
        Aabb aabb;
        if (node->entry_index >= HK_BVH_LEAF_FLAG) {
            uint32_t primitive_index = mesh.primitive + node->entry_index - HK_BVH_LEAF_FLAG;
            const hk_primitive_vertex* vertices = c->primitives[primitive_index].vertices;
            v3 a = ld3(vertices[0].position), b = ld3(vertices[1].position), d = ld3(vertices[2].position);
            aabb.min = min3(a, min3(b, d));
            aabb.max = max3(a, max3(b, d));
            if (intersects_aabb(ray, aabb) < hit->intersection.distance) {
                HKO_STAT(4);
                Intersection is = intersects_triangle(ray, vertices);
                if (is.distance < hit->intersection.distance) {
                    hit->intersection = is;
                    hit->primitive_index = primitive_index;
                    intersected = 1;
                    if (is.distance < early_distance) return intersected;
                }
            }
            index = node->exit_index;
        } else {
            aabb.min = ld3(node->min);
            aabb.max = ld3(node->max);
            index = intersects_aabb(ray, aabb) < hit->intersection.distance ? node->entry_index : node->exit_index;
        }
    }
    return intersected;
}

static Hit traverse_top(const hko_ctx* c, Counts* cnt, const Ray* ray, float max_distance, float early_distance,
                        uint32_t exclude_instance)
{
    cnt->top++;
#ifdef HKO_STATS
    hko_class = (max_distance == HK_F32_MAX && early_distance == 0.0f) ? 0 : (early_distance == 65535.0f ? 1 : 2);
    HKO_STAT(0);
#endif
    Hit hit;
    hit.intersection.uv = V2(0, 0);
    hit.intersection.distance = max_distance;
    hit.instance_index = HK_U32_MAX;
    hit.primitive_index = HK_U32_MAX;
    uint32_t index = 0u;
    while (index < c->n_instance_nodes) {
        HKO_STAT(1);
        const hk_node* node = &c->instance_nodes[index];
        Aabb aabb;
        if (node->entry_index >= HK_BVH_LEAF_FLAG) {
            uint32_t instance_index = node->entry_index - HK_BVH_LEAF_FLAG;
            const hk_instance* instance = &c->instances[instance_index];
            aabb.min = ld3(instance->min);
            aabb.max = ld3(instance->max);
            if (instance_index != exclude_instance && intersects_aabb(ray, aabb) < hit.intersection.distance) {
                Ray r;
                r.origin = instance_position_world_to_local(instance, ray->origin);
                r.direction = instance_direction_world_to_local(instance, ray->direction);
                r.inv_direction = inv3(r.direction);
                HKO_STAT(2);
                if (traverse_bottom(c, &hit, &r, instance->mesh, early_distance)) {
                    hit.instance_index = instance_index;
                    if (hit.intersection.distance < early_distance) return hit;
                }
            }
            index = node->exit_index;
        } else {
            aabb.min = ld3(node->min);
            aabb.max = ld3(node->max);
            index = intersects_aabb(ray, aabb) < hit.intersection.distance ? node->entry_index : node->exit_index;
        }
    }
    return hit;
}

/* The closest-hit light walks.  light.wgsl walks them with the stackless skip-pointer order of
 * traverse_top / traverse_bottom (light.wgsl:400-486): the bounce ray (`traverse_top(ray, F32_MAX, 0.0,
 * DONT_EXCLUDE)`, light.wgsl:1319,1401) and the emitter BLAS walk (`traverse_bottom(..., 0.0)`,
 * light.wgsl:687).  Neither has an early exit, so the hit they return is the closest one whatever the
 * visit order, except for exact-distance ties and box tests that round across the hit distance.  The
 * HIP kernels keep light.wgsl's order for both walks; the ordered rule (closest_hit_ordered: nearer child
 * first, the farther pushed and dropped on pop once it cannot win — the G-buffer's primary-visibility rule)
 * is the analysed alternative for the bounce walk, bit-identical on the bench scenes and measured slower in
 * the kernels.  hko_set_light_walk selects:
 *   HKO_WALK_REFERENCE  light.wgsl's order for both (what the HIP kernels run);
 *   HKO_WALK_ORDERED    the bounce walk with the ordered rule (the analysed alternative);
 *   HKO_WALK_CHECK      light.wgsl's order, and every bounce ray and emitter walk walked with the ordered rule
 *                       too; the rays whose two results differ in any bit (instance, primitive, distance, uv)
 *                       are counted (hko_light_walk_stats).  Zero bounce differences on a workload show that
 *                       the ordered bounce walk would return light.wgsl's results there (tests/test_light_walks.py);
 *                       the emitter count is analysis only: the kernels keep light.wgsl's order for the emitter
 *                       walk, which aims at sampled emitter points, shared triangle edges included, where the
 *                       ordered rule breaks ties differently. */
static Hit closest_hit_ordered(const hko_ctx* c, const Ray* ray);
static int emitter_walk_ordered(const hko_ctx* c, Hit* hit, const Ray* ray, const hk_mesh_index* mesh);
static int hit_differs(const Hit* a, const Hit* b)
{
    return a->instance_index != b->instance_index || a->primitive_index != b->primitive_index ||
           hk_f2u(a->intersection.distance) != hk_f2u(b->intersection.distance) ||
           hk_f2u(a->intersection.uv.x) != hk_f2u(b->intersection.uv.x) ||
           hk_f2u(a->intersection.uv.y) != hk_f2u(b->intersection.uv.y);
}
static void walk_tally(const hko_ctx* c, int k, int differ)
{
    hko_ctx* m = (hko_ctx*)c; /* counters only */
    __atomic_fetch_add(&m->walk_checked[k], 1ull, __ATOMIC_RELAXED);
    if (differ) __atomic_fetch_add(&m->walk_differ[k], 1ull, __ATOMIC_RELAXED);
}
/* the bounce ray: traverse_top(ray, F32_MAX, 0.0, DONT_EXCLUDE) */
static Hit bounce_walk(const hko_ctx* c, Counts* cnt, const Ray* ray)
{
    if (c->light_walk == HKO_WALK_ORDERED) {
        cnt->top++;
#ifdef HKO_STATS
        hko_class = 0;
        HKO_STAT(0);
#endif
        return closest_hit_ordered(c, ray);
    }
    Hit h = traverse_top(c, cnt, ray, HK_F32_MAX, 0.0f, DONT_EXCLUDE);
    if (c->light_walk == HKO_WALK_CHECK) {
        Hit o = closest_hit_ordered(c, ray);
        walk_tally(c, 0, hit_differs(&h, &o));
    }
    return h;
}
/* the emitter BLAS walk: traverse_bottom(hit, r, mesh, 0.0) from an empty hit */
static int emitter_walk(const hko_ctx* c, Hit* hit, const Ray* r, const hk_mesh_index* mesh)
{
    Hit start = *hit;
    int traced = traverse_bottom(c, hit, r, *mesh, 0.0f);
    if (c->light_walk == HKO_WALK_CHECK) {
        Hit o = start;
        int t2 = emitter_walk_ordered(c, &o, r, mesh);
        /* the instance field is the caller's (light.wgsl:689) */
        o.instance_index = hit->instance_index;
        walk_tally(c, 1, t2 != traced || hit_differs(hit, &o));
    }
    return traced;
}

static HitInfo empty_hit_info(v3 position, v3 direction)
{
    HitInfo info;
    memset(&info, 0, sizeof(info));
    info.instance_index = HK_U32_MAX;
    info.material_index = HK_U32_MAX;
    v3 p = add3(position, scale3(direction, DISTANCE_MAX));
    info.position = V4(p.x, p.y, p.z, 0.0f);
    return info;
}

static HitInfo hit_info(const hko_ctx* c, const Ray* ray, const Hit* hit)
{
    HitInfo info;
#ifdef HKO_STATS
    __atomic_fetch_add(&hko_hit_infos, 1ull, __ATOMIC_RELAXED);
#endif
    memset(&info, 0, sizeof(info));
    info.instance_index = hit->instance_index;
    info.material_index = HK_U32_MAX;
    if (hit->instance_index != HK_U32_MAX) {
        const hk_instance* instance = get_instance(c, hit->instance_index);
        const hk_primitive_vertex* vertices = c->primitives[hit->primitive_index].vertices;
        const hk_vertex* v0 = &c->vertices[instance->mesh.vertex + vertices[0].index];
        const hk_vertex* v1 = &c->vertices[instance->mesh.vertex + vertices[1].index];
        const hk_vertex* v2_ = &c->vertices[instance->mesh.vertex + vertices[2].index];
        v2 uv0 = V2(v0->u, v0->v), uv1 = V2(v1->u, v1->v), uv2 = V2(v2_->u, v2_->v);
        v2 uv = hit->intersection.uv;
        info.uv = V2((uv0.x + uv.x * (uv1.x - uv0.x)) + uv.y * (uv2.x - uv0.x),
                     (uv0.y + uv.x * (uv1.y - uv0.y)) + uv.y * (uv2.y - uv0.y));
        v3 n0 = ld3(v0->normal), n1 = ld3(v1->normal), n2 = ld3(v2_->normal);
        v3 n = add3(add3(n0, scale3(sub3(n1, n0), uv.x)), scale3(sub3(n2, n0), uv.y));
        info.normal = instance_normal_local_to_world(instance, n);
        v3 p = add3(ray->origin, scale3(ray->direction, hit->intersection.distance));
        info.position = V4(p.x, p.y, p.z, 1.0f);
        info.material_index = instance->material;
    } else {
        v3 p = add3(ray->origin, scale3(ray->direction, DISTANCE_MAX));
        info.position = V4(p.x, p.y, p.z, 0.0f);
    }
    return info;
}

static void occlude_hit_info(const Ray* ray, const Hit* hit, HitInfo* info)
{
    if (hit->instance_index != HK_U32_MAX) {
        info->instance_index = hit->instance_index;
        info->material_index = HK_U32_MAX;
        v3 p = add3(ray->origin, scale3(ray->direction, hit->intersection.distance));
        info->position = V4(p.x, p.y, p.z, 1.0f);
        info->normal = V3(0, 0, 0);
    }
}

/* ------------------------------------------------------------------ sampling (light.wgsl:537-708) */
static v2 sample_uniform_disk(v2 rand)
{
    float r = sqrtf(rand.x);
    float theta = (2.0f * HK_PI) * rand.y;
    float sn, cs;
    hk_sincos(theta, &sn, &cs);
    return V2(r * cs, r * sn);
}
static v4 sample_cosine_hemisphere(v2 rand)
{
    v2 t = sample_uniform_disk(rand);
    float z = sqrtf(1.0f - dot2(t, t));
    float pdf = (2.0f * HK_INV_TAU) * z;
    return V4(t.x, t.y, z, pdf);
}
static v4 sample_uniform_cone(v2 rand, float cos_angle)
{
    float z = 1.0f - (1.0f - cos_angle) * rand.x;
    float theta = HK_TAU * rand.y;
    float r = sqrtf(1.0f - z * z);
    float sn, cs;
    hk_sincos(theta, &sn, &cs);
    float pdf = HK_INV_TAU / (1.0f - cos_angle);
    return V4(r * cs, r * sn, z, pdf);
}
static v2 sample_uniform_triangle_barycentric(v2 rand)
{
    float srx = sqrtf(rand.x);
    return V2(1.0f - srx, rand.y * srx);
}
/* utils.wgsl:41-48: returns the columns (t, b, n) */
static void normal_basis(v3 n, v3* t, v3* b)
{
    float s = hk_minf(hk_signf(n.z) * 2.0f + 1.0f, 1.0f);
    float u = -1.0f / (s + n.z);
    float v = (n.x * n.y) * u;
    *t = V3(1.0f + ((s * n.x) * n.x) * u, s * v, -s * n.x);
    *b = V3(v, s + (n.y * n.y) * u, -n.y);
}
static inline v3 basis_mul(v3 t, v3 b, v3 n, v3 d) /* mat3x3(t, b, n) * d */
{
    return add3(add3(scale3(t, d.x), scale3(b, d.y)), scale3(n, d.z));
}
static inline v4 directional_cone(const Pass* P) /* light.wgsl:571-573 */
{
    const float* d = P->in->lights.direction_to_light;
    return V4(d[0], d[1], d[2], hk_cos(P->st->solar_angle));
}
static inline v3 compute_emissive_radiance(v4 e) { return scale3(xyz(e), 255.0f * e.w); }

static LightCandidate select_light_candidate(const Pass* P, Counts* cnt, v4 rand, v3 position, v3 normal,
                                             uint32_t instance, HitInfo* info)
{
    const hko_ctx* c = P->c;
    LightCandidate candidate;
    candidate.max_distance = HK_F32_MAX;
    candidate.min_distance = DISTANCE_MAX;
    candidate.emissive_instance = DONT_SAMPLE_EMISSIVE;

    v4 cone = directional_cone(P);
    v3 bt, bb;
    normal_basis(xyz(cone), &bt, &bb);
    v3 rand_direction = basis_mul(bt, bb, xyz(cone), xyz(sample_uniform_cone(V2(rand.z, rand.w), cone.w)));
    candidate.direction = rand_direction;
    candidate.p = 1.0f;
    *info = empty_hit_info(position, rand_direction);
    if (instance == DONT_SAMPLE_EMISSIVE) return candidate;

    const hk_emissive* emissive = NULL;
    float count = 0.0f;
    uint32_t index = 0u;
    float rand_1d = rand.x;
    while (index < c->n_emissive_nodes) {
        const hk_node* node = &c->emissive_nodes[index];
        Aabb aabb;
        if (node->entry_index >= HK_BVH_LEAF_FLAG) {
            uint32_t emissive_index = node->entry_index - HK_BVH_LEAF_FLAG;
            const hk_emissive* cur = &c->emissives[emissive_index];
            v3 ep = ld3(cur->position);
            aabb.min = V3(ep.x - cur->radius, ep.y - cur->radius, ep.z - cur->radius);
            aabb.max = V3(ep.x + cur->radius, ep.y + cur->radius, ep.z + cur->radius);
            if (instance != cur->instance && inside_aabb(position, aabb)) {
                rand_1d = hk_fract(rand_1d + HK_GOLDEN_RATIO);
                count += 1.0f;
                if (rand_1d < 1.0f / count) {
                    candidate.emissive_instance = cur->instance;
                    emissive = cur;
                }
            }
            index = node->exit_index;
        } else {
            aabb.min = ld3(node->min);
            aabb.max = ld3(node->max);
            index = inside_aabb(position, aabb) ? node->entry_index : node->exit_index;
        }
    }

    if (candidate.emissive_instance != DONT_SAMPLE_EMISSIVE) {
        uint32_t len = emissive->alias_table[1];
        uint32_t alias_index = f2u32(rand.x * (float)len);
        if (alias_index > len - 1u) alias_index = len - 1u;
        const hk_alias_entry* alias_entry = &c->alias_table[emissive->alias_table[0] + alias_index];
        uint32_t primitive_index = rand.y < alias_entry->prob ? alias_entry->index : alias_index;

        const hk_instance* emissive_instance = get_instance(c, candidate.emissive_instance);
        const hk_primitive_vertex* v = c->primitives[emissive_instance->mesh.primitive + primitive_index].vertices;
        v2 b = sample_uniform_triangle_barycentric(V2(rand.z, rand.w));
        v3 lp = add3(add3(scale3(ld3(v[0].position), b.x), scale3(ld3(v[1].position), b.y)),
                     scale3(ld3(v[2].position), (1.0f - b.x) - b.y));
        v3 p = instance_position_local_to_world(emissive_instance, lp);

        Hit hit;
        hit.intersection.uv = V2(0, 0);
        hit.intersection.distance = HK_F32_MAX;
        hit.instance_index = HK_U32_MAX;
        hit.primitive_index = HK_U32_MAX;

        Ray ray;
        ray.origin = add3(position, scale3(normal, RAY_BIAS));
        ray.direction = normalize3(sub3(p, position));
        ray.inv_direction = V3(0, 0, 0);
        Ray r;
        r.origin = instance_position_world_to_local(emissive_instance, ray.origin);
        r.direction = instance_direction_world_to_local(emissive_instance, ray.direction);
        r.inv_direction = inv3(r.direction);

        candidate.direction = ray.direction;
        int traced = 0;
        if (dot3(candidate.direction, normal) > 0.0f) {
            cnt->emitter++;
#ifdef HKO_STATS
            hko_class = 3;
            HKO_STAT(0);
#endif
            traced = emitter_walk(c, &hit, &r, &emissive_instance->mesh);
        }
        if (traced) {
            hit.instance_index = emissive->instance;
            *info = hit_info(c, &ray, &hit);
            candidate.max_distance = hit.intersection.distance;
            candidate.min_distance = hit.intersection.distance - 0.1f;
            v3 delta = sub3(xyz(info->position), position);
            candidate.p = dot3(delta, delta) / hk_absf(dot3(ray.direction, info->normal) * emissive->surface_area);
            candidate.p = candidate.p / count;
        } else {
            *info = empty_hit_info(ray.origin, ray.direction);
            candidate.emissive_instance = DONT_SAMPLE_EMISSIVE;
            candidate.direction = rand_direction;
            candidate.p = 1.0f;
        }
    }
    return candidate;
}

/* ------------------------------------------------------------------ shading (light.wgsl:714-908 + Bevy PBR) */
static v3 calculate_view(const Pass* P, v4 world_position, int is_orthographic)
{
    const hk_view* view = &P->in->view;
    if (is_orthographic)
        return normalize3(V3(view->view_proj[2], view->view_proj[6], view->view_proj[10]));
    return normalize3(sub3(ld3(view->world_position), xyz(world_position)));
}
static inline int is_orthographic(const Pass* P) { return P->in->view.projection[15] == 1.0f; }

/* light.wgsl:729-794: the NO_TEXTURE variant when the scene has no textures, otherwise every
 * texture id != U32_MAX modulates its factor by textureSampleLevel(.., uv, 0) (hk_texture.h) */
static int has_texture(const hko_ctx* c, uint32_t id) { return id != HK_U32_MAX && id < c->n_textures; }
static v4 sample_material_texture(const hko_ctx* c, uint32_t id, v2 uv)
{
    float t[4];
    hk_sample_texture(c->tex_desc + id, c->texels, c->tex_lut, uv.x, uv.y, t);
    return V4(t[0], t[1], t[2], t[3]);
}
static Surface retreive_surface(const Pass* P, uint32_t material_index, v2 uv)
{
    const hko_ctx* c = P->c;
    const hk_material* m = get_material(c, material_index);
    Surface s;
    s.base_color = V4(m->base_color[0], m->base_color[1], m->base_color[2], m->base_color[3]);
    s.emissive = V4(m->emissive[0], m->emissive[1], m->emissive[2], m->emissive[3]);
    s.metallic = m->metallic;
    s.occlusion = 1.0f;
    if (c->n_textures) {
        if (has_texture(c, m->base_color_texture)) {
            v4 t = sample_material_texture(c, m->base_color_texture, uv);
            s.base_color = V4(s.base_color.x * t.x, s.base_color.y * t.y, s.base_color.z * t.z, s.base_color.w * t.w);
        }
        if (has_texture(c, m->emissive_texture)) {
            v4 t = sample_material_texture(c, m->emissive_texture, uv);
            s.emissive = V4(s.emissive.x * t.x, s.emissive.y * t.y, s.emissive.z * t.z, s.emissive.w * t.w);
        }
        if (has_texture(c, m->metallic_roughness_texture))
            s.metallic = s.metallic * sample_material_texture(c, m->metallic_roughness_texture, uv).x;
        if (has_texture(c, m->occlusion_texture)) s.occlusion = sample_material_texture(c, m->occlusion_texture, uv).x;
    }
    float pr = hk_clampf(m->perceptual_roughness, 0.089f, 1.0f);
    s.roughness = pr * pr;
    s.reflectance = m->reflectance;
    return s;
}
static v4 retreive_emissive(const Pass* P, uint32_t material_index, v2 uv)
{
    const hko_ctx* c = P->c;
    const hk_material* m = get_material(c, material_index);
    v4 e = V4(m->emissive[0], m->emissive[1], m->emissive[2], m->emissive[3]);
    if (c->n_textures && has_texture(c, m->emissive_texture)) {
        v4 t = sample_material_texture(c, m->emissive_texture, uv);
        e = V4(e.x * t.x, e.y * t.y, e.z * t.z, e.w * t.w);
    }
    return e;
}

static float F_Schlick(float f0, float f90, float VoH)
{
    return f0 + (f90 - f0) * hk_pow5(1.0f - VoH);
}
static v3 F_Schlick_vec(v3 f0, float f90, float VoH)
{
    float k = hk_pow5(1.0f - VoH);
    return V3(f0.x + (f90 - f0.x) * k, f0.y + (f90 - f0.y) * k, f0.z + (f90 - f0.z) * k);
}
static v3 fresnel(v3 f0, float LoH)
{
    float f90 = hk_saturate(dot3(f0, V3(16.5f, 16.5f, 16.5f)));
    return F_Schlick_vec(f0, f90, LoH);
}
static float D_GGX(float roughness, float NoH)
{
    float one_minus = 1.0f - NoH * NoH;
    float a = NoH * roughness;
    float k = roughness / (one_minus + a * a);
    return (k * k) * (1.0f / HK_PI);
}
static float V_SmithGGXCorrelated(float roughness, float NoV, float NoL)
{
    float a2 = roughness * roughness;
    float lambdaV = NoL * sqrtf((NoV - a2 * NoV) * NoV + a2);
    float lambdaL = NoV * sqrtf((NoL - a2 * NoL) * NoL + a2);
    return 0.5f / (lambdaV + lambdaL);
}
static v3 specular(v3 f0, float roughness, float NoV, float NoL, float NoH, float LoH, float intensity)
{
    float D = D_GGX(roughness, NoH);
    float V = V_SmithGGXCorrelated(roughness, NoV, NoL);
    v3 F = fresnel(f0, LoH);
    return scale3(F, (intensity * D) * V);
}
static float Fd_Burley(float roughness, float NoV, float NoL, float LoH)
{
    float f90 = 0.5f + ((2.0f * roughness) * LoH) * LoH;
    float light_scatter = F_Schlick(1.0f, f90, NoL);
    float view_scatter = F_Schlick(1.0f, f90, NoV);
    return (light_scatter * view_scatter) * (1.0f / HK_PI);
}
static v3 EnvBRDFApprox(v3 f0, float perceptual_roughness, float NoV)
{
    float rx = perceptual_roughness * -1.0f + 1.0f;
    float ry = perceptual_roughness * -0.0275f + 0.0425f;
    float rz = perceptual_roughness * -0.572f + 1.04f;
    float rw = perceptual_roughness * 0.022f + -0.04f;
    float a004 = hk_minf(rx * rx, hk_exp2(-9.28f * NoV)) * rx + ry;
    float ABx = -1.04f * a004 + rz;
    float ABy = 1.04f * a004 + rw;
    return V3(f0.x * ABx + ABy, f0.y * ABx + ABy, f0.z * ABx + ABy);
}

static v3 lit(v3 radiance, v3 diffuse_color, float roughness, v3 F0, v3 L, v3 N, v3 V)
{
    v3 H = normalize3(add3(L, V));
    float NoL = hk_saturate(dot3(N, L));
    float NoH = hk_saturate(dot3(N, H));
    float LoH = hk_saturate(dot3(L, H));
    float NdotV = hk_maxf(dot3(N, V), 0.0001f);
    v3 diffuse = scale3(diffuse_color, Fd_Burley(roughness, NdotV, NoL, LoH));
    v3 specular_light = specular(F0, roughness, NdotV, NoL, NoH, LoH, 1.0f);
    return scale3(mul3(add3(specular_light, diffuse), radiance), NoL);
}

static v3 ambient(const Pass* P, v3 diffuse_color, float roughness, float occlusion, v3 F0, v3 N, v3 V)
{
    float NdotV = hk_maxf(dot3(N, V), 0.0001f);
    v3 diffuse_ambient = EnvBRDFApprox(diffuse_color, 1.0f, NdotV);
    v3 specular_ambient = EnvBRDFApprox(F0, roughness, NdotV);
    return mul3(scale3(add3(diffuse_ambient, specular_ambient), occlusion), ld3(P->in->lights.ambient_color));
}

static v4 input_radiance(const Pass* P, const Ray* ray, const HitInfo* info, int sample_directional,
                         uint32_t sample_emissive, int sample_ambient)
{
    v3 radiance = V3(0, 0, 0);
    float amb = 0.0f;
    if (info->instance_index == HK_U32_MAX) {
        v4 cone = directional_cone(P);
        int hit_directional = dot3(ray->direction, xyz(cone)) >= cone.w;
        if (sample_directional && hit_directional) {
            radiance = ld3(P->in->lights.directional_color);
            amb = 0.0f;
        } else {
            radiance = sample_ambient ? ld3(P->in->lights.ambient_color) : V3(0, 0, 0);
            amb = 1.0f;
        }
    } else {
        if (sample_emissive == info->instance_index) {
            v4 e = retreive_emissive(P, info->material_index, info->uv);
            radiance = compute_emissive_radiance(e);
        }
    }
    return V4(radiance.x, radiance.y, radiance.z, 1.0f - amb);
}

static v3 shading(const Pass* P, v3 V, v3 N, v3 L, const Surface* surface, v4 in_radiance)
{
    v3 base_color = xyz(surface->base_color);
    float reflectance = surface->reflectance;
    float roughness = surface->roughness;
    float metallic = surface->metallic;
    float occlusion = surface->occlusion;
    float f0s = ((0.16f * reflectance) * reflectance) * (1.0f - metallic);
    v3 F0 = V3(f0s + base_color.x * metallic, f0s + base_color.y * metallic, f0s + base_color.z * metallic);
    v3 diffuse_color = scale3(base_color, 1.0f - metallic);
    v3 lit_radiance = lit(xyz(in_radiance), diffuse_color, roughness, F0, L, N, V);
    v3 ambient_radiance = ambient(P, diffuse_color, roughness, occlusion, F0, N, V);
    return mix3(lit_radiance, ambient_radiance, 1.0f - in_radiance.w);
}

static v3 env_brdf(v3 V, v3 N, const Surface* surface)
{
    v3 base_color = xyz(surface->base_color);
    float reflectance = surface->reflectance;
    float roughness = surface->roughness;
    float metallic = surface->metallic;
    float occlusion = surface->occlusion;
    float NdotV = hk_maxf(dot3(N, V), 0.0001f);
    float f0s = ((0.16f * reflectance) * reflectance) * (1.0f - metallic);
    v3 F0 = V3(f0s + base_color.x * metallic, f0s + base_color.y * metallic, f0s + base_color.z * metallic);
    v3 diffuse_color = scale3(base_color, 1.0f - metallic);
    v3 diffuse_ambient = EnvBRDFApprox(diffuse_color, 1.0f, NdotV);
    v3 specular_ambient = EnvBRDFApprox(F0, roughness, NdotV);
    return scale3(add3(diffuse_ambient, specular_ambient), occlusion);
}

/* ------------------------------------------------------------------ ReSTIR (light.wgsl:913-1004) */
static float reservoir_lifetime(const Pass* P)
{
    return P->st->max_reservoir_lifetime <= 1.0f ? HK_F32_MAX : P->st->max_reservoir_lifetime;
}

static int check_previous_reservoir(Reservoir* r, const Sample* s)
{
    float depth_ratio = r->s.visible_position.w / s->visible_position.w;
    depth_ratio = depth_ratio < 1.0f ? 1.0f / depth_ratio : depth_ratio;
    int depth_miss = depth_ratio > 1.05f * (1.0f + 0.5f * s->random.x);
    int instance_miss = r->s.visible_instance != s->visible_instance;
    int normal_miss = dot3(s->visible_normal, r->s.visible_normal) < 0.9f;
    if (depth_miss || normal_miss || instance_miss) {
        memset(r, 0, sizeof(*r));
        return 0;
    }
    return 1;
}

static void temporal_restir(Reservoir* r, const Sample* s, float w_new, uint32_t max_sample_count)
{
    update_reservoir(r, s, w_new);
    float m = (float)max_sample_count;
    if (r->count > m) {
        r->w_sum *= m / r->count;
        r->w2_sum *= m / r->count;
        r->count = m;
    }
}

static float compute_jacobian(const Sample* q, const Sample* r)
{
    v3 normal = q->sample_normal;
    float cos_phi_1 = hk_absf(dot3(normalize3(sub3(xyz(r->visible_position), xyz(q->sample_position))), normal));
    float cos_phi_2 = hk_absf(dot3(normalize3(sub3(xyz(q->visible_position), xyz(q->sample_position))), normal));
    float term_1 = cos_phi_1 / hk_maxf(0.0001f, cos_phi_2);
    float num = length3(sub3(xyz(q->visible_position), xyz(q->sample_position)));
    num *= num;
    float denom = length3(sub3(xyz(r->visible_position), xyz(q->sample_position)));
    denom *= denom;
    float term_2 = num / hk_maxf(denom, 0.0001f);
    return hk_clampf(term_1 * term_2, 1.0f, 50.0f);
}

static float variance_of(const Reservoir* r)
{
    float variance = r->w2_sum / r->count - hk_pow2(r->w_sum / r->count);
    variance = r->count < 1.0f ? variance : variance / r->count;
    return hk_minf(variance, MAX_VARIANCE);
}

/* blue noise (light.wgsl:1075-1079): nearest + repeat => texel ((x + n) mod 64, (y + n) mod 64) */
static v4 noise_random(const Pass* P, int32_t x, int32_t y)
{
    uint32_t id = umod(P->number, NOISE_TEXTURE_COUNT);
    uint32_t tx = ((uint32_t)x + P->number) & 63u, ty = ((uint32_t)y + P->number) & 63u;
    const uint8_t* t = P->c->noise + (((size_t)id * 64 + ty) * 64 + tx) * 4;
    float fn = (float)P->number * HK_GOLDEN_RATIO;
    return V4(hk_fract((float)t[0] / 255.0f + fn), hk_fract((float)t[1] / 255.0f + fn),
              hk_fract((float)t[2] / 255.0f + fn), hk_fract((float)t[3] / 255.0f + fn));
}

/* ------------------------------------------------------------------ entry points */
static void full_screen_albedo(const Pass* P, int32_t x, int32_t y)
{
    const hko_ctx* c = P->c;
    uint32_t idx = (uint32_t)y * c->S[0] + (uint32_t)x;
    v4 position_depth = load_position(c, x, y);
    v4 position = V4(position_depth.x, position_depth.y, position_depth.z, 1.0f);
    float depth = position_depth.w;
    if (depth < HK_F32_EPSILON) {
        store_rgba16f(c->albedo, idx, V4(0, 0, 0, 0));
        return;
    }
    v3 normal = load_normal(c, x, y);
    v2 im = load_instance_material(c, x, y);
    uint32_t material = f2u32(im.y);
    v4 velocity_uv = load_velocity_uv(c, x, y);
    Surface surface = retreive_surface(P, material, V2(velocity_uv.z, velocity_uv.w));
    v3 view_direction = calculate_view(P, position, is_orthographic(P));
    v3 a = env_brdf(view_direction, normal, &surface);
    store_rgba16f(c->albedo, idx, V4(a.x, a.y, a.z, 1.0f));
}

static void direct_lit(const Pass* P, Counts* cnt, int32_t x, int32_t y)
{
    const hko_ctx* c = P->c;
    const uint32_t* render_size = c->s;
    int32_t idx = x + (int32_t)render_size[0] * y;
    v2 uv = coords_to_uv(x, y, render_size);
    Sample s;
    memset(&s, 0, sizeof(s));

    int32_t dx, dy;
    jittered_deferred_coords(P, uv, &dx, &dy);
    v4 position_depth = load_position(c, dx, dy);
    v4 position = V4(position_depth.x, position_depth.y, position_depth.z, 1.0f);
    float depth = position_depth.w;

    if (depth < HK_F32_EPSILON) {
        Reservoir r;
        memset(&r, 0, sizeof(r));
        set_reservoir(&r, &s, 0.0f);
        pack_reservoir(&r, &P->reservoir_buffer[idx]);
        pack_reservoir(&r, &P->spatial_reservoir_buffer[idx]);
        pack_reservoir(&r, &P->previous_spatial_reservoir_buffer[idx]);
        P->variance_texture[idx] = 0.0f;
        store_rgba16f(P->render_texture, (uint32_t)idx, V4(0, 0, 0, 0));
        return;
    }

    v3 normal = load_normal(c, dx, dy);
    v2 imf = load_instance_material(c, dx, dy);
    uint32_t im_x = f2u32(imf.x), im_y = f2u32(imf.y);
    v4 velocity_uv = load_velocity_uv(c, dx, dy);

    s.random = noise_random(P, x, y);
    s.visible_position = V4(position.x, position.y, position.z, depth);
    s.visible_normal = normal;
    s.visible_instance = im_x;

    Ray ray;
    memset(&ray, 0, sizeof(ray));
    Hit hit;
    HitInfo info;
    memset(&info, 0, sizeof(info));

    v2 juv = jittered_deferred_uv(P, uv);
    v2 previous_uv = V2(juv.x - velocity_uv.x, juv.y - velocity_uv.y);
    Reservoir r = load_previous_from(P->previous_reservoir_buffer, previous_uv, render_size);

    if (!check_previous_reservoir(&r, &s) && uv_inside_closed(previous_uv)) {
        int32_t px = f2i32(previous_uv.x * (float)render_size[0]);
        int32_t py = f2i32(previous_uv.y * (float)render_size[1]);
        pack_reservoir(&r, &P->previous_spatial_reservoir_buffer[px + (int32_t)render_size[0] * py]);
    }

    uint32_t validate_interval, select_light_instance;
    if (P->emissive_lit) {
        validate_interval = P->st->emissive_validate_interval;
        select_light_instance = im_x;
    } else {
        validate_interval = P->st->direct_validate_interval;
        select_light_instance = DONT_SAMPLE_EMISSIVE;
    }

    if (umod(P->number, validate_interval) != 0u || r.count < (float)DIRECT_VALIDATION_FRAME_SAMPLE_THRESHOLD) {
        LightCandidate candidate = select_light_candidate(P, cnt, s.random, xyz(s.visible_position), s.visible_normal,
                                                          select_light_instance, &info);
        ray.origin = add3(xyz(position), scale3(normal, RAY_BIAS));
        ray.direction = candidate.direction;
        ray.inv_direction = inv3(ray.direction);
        int trace_condition = dot3(candidate.direction, normal) > 0.0f;
        trace_condition = trace_condition && candidate.p > 0.0f;
        if (P->emissive_lit) trace_condition = trace_condition && candidate.emissive_instance != DONT_SAMPLE_EMISSIVE;
        if (trace_condition) {
            hit = traverse_top(c, cnt, &ray, candidate.max_distance, candidate.min_distance, candidate.emissive_instance);
            occlude_hit_info(&ray, &hit, &info);
            if (P->emissive_lit) s.radiance = input_radiance(P, &ray, &info, 0, candidate.emissive_instance, 0);
            else s.radiance = input_radiance(P, &ray, &info, 1, DONT_SAMPLE_EMISSIVE, 0);
        }
        s.sample_position = info.position;
        s.sample_normal = info.normal;
        float w_new = candidate.p > 0.0f ? lum3(xyz(s.radiance)) / candidate.p : 0.0f;
        temporal_restir(&r, &s, w_new, P->st->max_temporal_reuse_count);
    }

    if (umod(P->number, validate_interval) == 0u) {
        LightCandidate candidate = select_light_candidate(P, cnt, r.s.random, xyz(r.s.visible_position),
                                                          r.s.visible_normal, select_light_instance, &info);
        ray.origin = add3(xyz(s.visible_position), scale3(s.visible_normal, RAY_BIAS));
        ray.direction = normalize3(sub3(xyz(r.s.sample_position), xyz(s.visible_position)));
        ray.inv_direction = inv3(ray.direction);
        v4 validate_radiance = V4(0, 0, 0, 0);
        int trace_condition = dot3(candidate.direction, r.s.visible_normal) > 0.0f;
        trace_condition = trace_condition && candidate.p > 0.0f;
        if (P->emissive_lit) trace_condition = trace_condition && candidate.emissive_instance != DONT_SAMPLE_EMISSIVE;
        if (trace_condition) {
            hit = traverse_top(c, cnt, &ray, candidate.max_distance, candidate.min_distance, candidate.emissive_instance);
            occlude_hit_info(&ray, &hit, &info);
            if (P->emissive_lit) validate_radiance = input_radiance(P, &ray, &info, 0, candidate.emissive_instance, 0);
            else validate_radiance = input_radiance(P, &ray, &info, 1, DONT_SAMPLE_EMISSIVE, 0);
        }
        if (r.count >= (float)DIRECT_VALIDATION_FRAME_SAMPLE_THRESHOLD) {
            s.random = r.s.random;
            s.sample_position = info.position;
            s.sample_normal = info.normal;
            s.radiance = validate_radiance;
        }
        float luminance_ratio = lum3(xyz(validate_radiance)) / hk_maxf(lum3(xyz(r.s.radiance)), 0.0001f);
        if (luminance_ratio > 1.25f || luminance_ratio < 0.8f) {
            if (uv_inside_closed(previous_uv)) {
                int32_t px = f2i32(previous_uv.x * (float)render_size[0]);
                int32_t py = f2i32(previous_uv.y * (float)render_size[1]);
                pack_reservoir(&r, &P->previous_spatial_reservoir_buffer[px + (int32_t)render_size[0] * py]);
            }
            float w_new = candidate.p > 0.0f ? lum3(xyz(s.radiance)) / candidate.p : 0.0f;
            set_reservoir(&r, &s, w_new);
        }
    }

    float total_lum = r.count * lum3(xyz(r.s.radiance));
    r.w = total_lum > 0.0f ? r.w_sum / total_lum : 0.0f;
    r.s.visible_position = s.visible_position;
    r.s.visible_normal = s.visible_normal;
    r.lifetime += 1.0f;

    P->variance_texture[idx] = variance_of(&r);
    if (P->st->temporal_reuse > 0u) pack_reservoir(&r, &P->reservoir_buffer[idx]);

    Surface surface = retreive_surface(P, im_y, V2(velocity_uv.z, velocity_uv.w));
    v3 view_direction = calculate_view(P, position, is_orthographic(P));
    v3 out_radiance = shading(P, view_direction, r.s.visible_normal,
                              normalize3(sub3(xyz(r.s.sample_position), xyz(r.s.visible_position))), &surface,
                              r.s.radiance);
    out_radiance = scale3(out_radiance, r.w);
    v3 out_color = out_radiance;
    if (P->render_emissive) out_color = add3(out_radiance, compute_emissive_radiance(surface.emissive));
    store_rgba16f(P->render_texture, (uint32_t)idx, V4(out_color.x, out_color.y, out_color.z, 1.0f));
}

static void indirect_lit_ambient(const Pass* P, Counts* cnt, int32_t x, int32_t y)
{
    const hko_ctx* c = P->c;
    const uint32_t* render_size = c->s;
    int32_t idx = x + (int32_t)render_size[0] * y;
    v2 uv = coords_to_uv(x, y, render_size);
    int32_t dx, dy;
    jittered_deferred_coords(P, uv, &dx, &dy);
    v4 position_depth = load_position(c, dx, dy);
    v4 position = V4(position_depth.x, position_depth.y, position_depth.z, 1.0f);
    float depth = position_depth.w;

    Sample s;
    memset(&s, 0, sizeof(s));
    Reservoir r;
    memset(&r, 0, sizeof(r));

    if (P->st->indirect_bounces == 0u || depth < HK_F32_EPSILON) {
        pack_reservoir(&r, &P->reservoir_buffer[idx]);
        pack_reservoir(&r, &P->spatial_reservoir_buffer[idx]);
        pack_reservoir(&r, &P->previous_spatial_reservoir_buffer[idx]);
        P->variance_texture[idx] = 0.0f;
        store_rgba16f(P->render_texture, (uint32_t)idx, V4(0, 0, 0, 0));
        return;
    }

    v3 normal = normalize3(load_normal(c, dx, dy));
    v2 imf = load_instance_material(c, dx, dy);
    uint32_t im_x = f2u32(imf.x), im_y = f2u32(imf.y);
    v4 velocity_uv = load_velocity_uv(c, dx, dy);

    s.random = noise_random(P, x, y);
    s.visible_position = V4(position.x, position.y, position.z, depth);
    s.visible_normal = normal;
    s.visible_instance = im_x;

    Ray ray;
    memset(&ray, 0, sizeof(ray));
    Hit hit;
    HitInfo info;
    memset(&info, 0, sizeof(info));
    float pdf = 0.0f;
    Surface surface;
    memset(&surface, 0, sizeof(surface));

    if (P->multiple_bounces) {
        Sample bounce_sample = s;
        v3 color_transport = V3(1.0f, 1.0f, 1.0f);
        for (uint32_t n = 0u; n < P->st->indirect_bounces &&
                              (color_transport.x > 0.01f || color_transport.y > 0.01f || color_transport.z > 0.01f);
             n += 1u) {
            v4 rand_sample = sample_cosine_hemisphere(V2(bounce_sample.random.x, bounce_sample.random.y));
            ray.origin = add3(xyz(bounce_sample.visible_position), scale3(bounce_sample.visible_normal, RAY_BIAS));
            v3 bt, bb;
            normal_basis(bounce_sample.visible_normal, &bt, &bb);
            ray.direction = basis_mul(bt, bb, bounce_sample.visible_normal, xyz(rand_sample));
            ray.inv_direction = inv3(ray.direction);
            hit = bounce_walk(c, cnt, &ray);
            info = hit_info(c, &ray, &hit);
            if (n == 0u) {
                s.sample_position = info.position;
                s.sample_normal = info.normal;
                pdf = rand_sample.w;
            }
            bounce_sample.sample_position = info.position;
            bounce_sample.sample_normal = info.normal;
            if (hit.instance_index != HK_U32_MAX) {
                v3 out_radiance = V3(0, 0, 0);
                surface = retreive_surface(P, info.material_index, info.uv);
                surface.roughness = 1.0f;
                LightCandidate candidate = select_light_candidate(P, cnt, bounce_sample.random,
                                                                  xyz(bounce_sample.sample_position),
                                                                  bounce_sample.sample_normal, info.instance_index, &info);
                int sample_directional = candidate.emissive_instance == DONT_SAMPLE_EMISSIVE;
                v3 bounce_view_direction =
                    normalize3(sub3(xyz(bounce_sample.visible_position), xyz(bounce_sample.sample_position)));
                if (dot3(candidate.direction, bounce_sample.sample_normal) > 0.0f && candidate.p > 0.0f) {
                    ray.origin = add3(xyz(bounce_sample.sample_position), scale3(bounce_sample.sample_normal, RAY_BIAS));
                    ray.direction = candidate.direction;
                    ray.inv_direction = inv3(ray.direction);
                    hit = traverse_top(c, cnt, &ray, candidate.max_distance, candidate.min_distance,
                                       candidate.emissive_instance);
                    occlude_hit_info(&ray, &hit, &info);
                    v4 in_radiance = input_radiance(P, &ray, &info, sample_directional, candidate.emissive_instance, 0);
                    out_radiance = shading(P, bounce_view_direction, bounce_sample.sample_normal, ray.direction, &surface,
                                           in_radiance);
                    out_radiance = div3s(out_radiance, candidate.p);
                    if (n > 0u) {
                        out_radiance = rand_sample.w < 0.01f ? V3(0, 0, 0) : div3s(out_radiance, rand_sample.w);
                    }
                    float out_luminance = lum3(out_radiance);
                    if (out_luminance > P->st->max_indirect_luminance) {
                        out_radiance = div3s(scale3(out_radiance, P->st->max_indirect_luminance), out_luminance);
                    }
                    v3 add = mul3(color_transport, out_radiance);
                    s.radiance = V4(s.radiance.x + add.x, s.radiance.y + add.y, s.radiance.z + add.z, s.radiance.w + 1.0f);
                }
                color_transport = mul3(color_transport, env_brdf(bounce_view_direction, bounce_sample.sample_normal, &surface));
                float fn = (float)P->number * HK_GOLDEN_RATIO;
                bounce_sample.random = V4(hk_fract(bounce_sample.random.x + fn), hk_fract(bounce_sample.random.y + fn),
                                          hk_fract(bounce_sample.random.z + fn), hk_fract(bounce_sample.random.w + fn));
                bounce_sample.visible_position = bounce_sample.sample_position;
                bounce_sample.visible_normal = bounce_sample.sample_normal;
            } else {
                v3 out_radiance = xyz(input_radiance(P, &ray, &info, 0, DONT_SAMPLE_EMISSIVE, 1));
                v3 add = mul3(color_transport, out_radiance);
                s.radiance = V4(s.radiance.x + add.x, s.radiance.y + add.y, s.radiance.z + add.z, s.radiance.w + 0.0f);
                break;
            }
        }
    } else {
        v4 rand_sample = sample_cosine_hemisphere(V2(s.random.x, s.random.y));
        ray.origin = add3(xyz(s.visible_position), scale3(s.visible_normal, RAY_BIAS));
        v3 bt, bb;
        normal_basis(s.visible_normal, &bt, &bb);
        ray.direction = basis_mul(bt, bb, s.visible_normal, xyz(rand_sample));
        ray.inv_direction = inv3(ray.direction);
        hit = bounce_walk(c, cnt, &ray);
        info = hit_info(c, &ray, &hit);
        s.sample_position = info.position;
        s.sample_normal = info.normal;
        pdf = rand_sample.w;
        if (hit.instance_index != HK_U32_MAX) {
            v3 out_radiance = V3(0, 0, 0);
            surface = retreive_surface(P, info.material_index, info.uv);
            surface.roughness = 1.0f;
            LightCandidate candidate = select_light_candidate(P, cnt, s.random, xyz(s.sample_position), s.sample_normal,
                                                              info.instance_index, &info);
            int sample_directional = candidate.emissive_instance == DONT_SAMPLE_EMISSIVE;
            if (dot3(candidate.direction, s.sample_normal) > 0.0f && candidate.p > 0.0f) {
                ray.origin = add3(xyz(s.sample_position), scale3(s.sample_normal, RAY_BIAS));
                ray.direction = candidate.direction;
                ray.inv_direction = inv3(ray.direction);
                hit = traverse_top(c, cnt, &ray, candidate.max_distance, candidate.min_distance, candidate.emissive_instance);
                occlude_hit_info(&ray, &hit, &info);
                v4 in_radiance = input_radiance(P, &ray, &info, sample_directional, candidate.emissive_instance, 0);
                out_radiance = shading(P, normalize3(sub3(xyz(s.visible_position), xyz(s.sample_position))), s.sample_normal,
                                       ray.direction, &surface, in_radiance);
                out_radiance = div3s(out_radiance, candidate.p);
                s.radiance = V4(s.radiance.x + out_radiance.x, s.radiance.y + out_radiance.y,
                                s.radiance.z + out_radiance.z, s.radiance.w + 1.0f);
            }
        } else {
            v3 out_radiance = xyz(input_radiance(P, &ray, &info, 0, DONT_SAMPLE_EMISSIVE, 1));
            s.radiance = V4(s.radiance.x + out_radiance.x, s.radiance.y + out_radiance.y, s.radiance.z + out_radiance.z,
                            s.radiance.w + 0.0f);
        }
    }

    /* ReSTIR: temporal */
    v2 juv = jittered_deferred_uv(P, uv);
    v2 previous_uv = V2(juv.x - velocity_uv.x, juv.y - velocity_uv.y);
    r = load_previous_from(P->previous_reservoir_buffer, previous_uv, render_size);
    if (!check_previous_reservoir(&r, &s) && uv_inside_closed(previous_uv)) {
        int32_t px = f2i32(previous_uv.x * (float)render_size[0]);
        int32_t py = f2i32(previous_uv.y * (float)render_size[1]);
        pack_reservoir(&r, &P->previous_spatial_reservoir_buffer[px + (int32_t)render_size[0] * py]);
    }

    surface = retreive_surface(P, im_y, V2(velocity_uv.z, velocity_uv.w));
    v3 view_direction = calculate_view(P, position, is_orthographic(P));
    v3 sample_radiance = shading(P, view_direction, s.visible_normal,
                                 normalize3(sub3(xyz(s.sample_position), xyz(s.visible_position))), &surface, s.radiance);
    float w_new = pdf > 0.0f ? lum3(sample_radiance) / pdf : 0.0f;
    temporal_restir(&r, &s, w_new, P->st->max_temporal_reuse_count);

    v3 out_radiance = shading(P, view_direction, r.s.visible_normal,
                              normalize3(sub3(xyz(r.s.sample_position), xyz(r.s.visible_position))), &surface,
                              r.s.radiance);
    float total_lum = r.count * lum3(out_radiance);
    r.w = total_lum > 0.0f ? r.w_sum / total_lum : 0.0f;
    r.s.visible_position = s.visible_position;
    r.s.visible_normal = s.visible_normal;
    r.lifetime += 1.0f;

    P->variance_texture[idx] = variance_of(&r);
    if (P->st->temporal_reuse > 0u) pack_reservoir(&r, &P->reservoir_buffer[idx]);
    v3 o = scale3(out_radiance, r.w);
    store_rgba16f(P->render_texture, (uint32_t)idx, V4(o.x, o.y, o.z, 1.0f));
}

static void spatial_reuse(const Pass* P, int32_t x, int32_t y)
{
    const hko_ctx* c = P->c;
    const uint32_t* render_size = c->s;
    const uint32_t reuse_count = P->emissive_lit ? 8u : 16u;
    const float reuse_range = P->emissive_lit ? 10.0f : 20.0f;
    int32_t idx = x + (int32_t)render_size[0] * y;
    v2 uv = coords_to_uv(x, y, render_size);
    int32_t dx, dy;
    jittered_deferred_coords(P, uv, &dx, &dy);
    v4 position_depth = load_position(c, dx, dy);
    v4 position = V4(position_depth.x, position_depth.y, position_depth.z, 1.0f);
    float depth = position_depth.w;

    Reservoir r = unpack_reservoir(&P->reservoir_buffer[idx]);
    /* shared_reservoir / shared_depth (light.wgsl:1500-1524) hold exactly what the global
     * path reads for in-tile neighbours, so the restatement always takes the global path */
    if (depth < HK_F32_EPSILON) {
        pack_reservoir(&r, &P->spatial_reservoir_buffer[idx]);
        store_rgba16f(P->render_texture, (uint32_t)idx, V4(0, 0, 0, 0));
        return;
    }
    v2 imf = load_instance_material(c, dx, dy);
    uint32_t im_y = f2u32(imf.y);
    v4 velocity_uv = load_velocity_uv(c, dx, dy);
    Surface surface = retreive_surface(P, im_y, V2(velocity_uv.z, velocity_uv.w));
    int use_spatial_variance = r.count <= (float)SPATIAL_VARIANCE_SAMPLE_THRESHOLD;

    v2 juv = jittered_deferred_uv(P, uv);
    v2 previous_uv = V2(juv.x - velocity_uv.x, juv.y - velocity_uv.y);
    Reservoir q = r;
    Sample s = q.s;
    if (r.lifetime <= reservoir_lifetime(P))
        r = load_previous_from(P->previous_spatial_reservoir_buffer, previous_uv, render_size);

    v3 view_direction = calculate_view(P, position, is_orthographic(P));
    if (P->emissive_lit) {
        merge_reservoir(&r, &q, lum3(xyz(q.s.radiance)));
    } else {
        v3 out_radiance = shading(P, view_direction, s.visible_normal,
                                  normalize3(sub3(xyz(s.sample_position), xyz(s.visible_position))), &surface, s.radiance);
        merge_reservoir(&r, &q, lum3(out_radiance));
    }
    r.s.visible_position = s.visible_position;
    r.s.visible_normal = s.visible_normal;

    float rf = hk_random_float(P->number);
    float srand = sum4(s.random);
    for (uint32_t i = 1u; i <= reuse_count; i += 1u) {
        float px = HK_TAU * hk_fract(((float)i * HK_GOLDEN_RATIO + srand) + rf);
        float py = sqrtf((float)i / (float)reuse_count) * reuse_range;
        float sn, cs;
        hk_sincos(px, &sn, &cs);
        v2 offset = V2(py * cs, py * sn);
        int32_t scx = f2i32(offset.x + (float)x), scy = f2i32(offset.y + (float)y);
        v2 sample_uv = coords_to_uv(scx, scy, render_size);
        int32_t sdx, sdy;
        jittered_deferred_coords(P, sample_uv, &sdx, &sdy);
        if (sample_uv.x < 0.0f || sample_uv.y < 0.0f || sample_uv.x > 1.0f || sample_uv.y > 1.0f) continue;

        float sample_depth = load_position(c, sdx, sdy).w;
        q = unpack_reservoir(&P->reservoir_buffer[scx + (int32_t)render_size[0] * scy]);

        float depth_ratio = depth / sample_depth;
        if (depth_ratio < 0.9f || depth_ratio > 1.1f) continue;
        int normal_miss = dot3(s.visible_normal, q.s.visible_normal) < 0.866f;
        if (q.count < HK_F32_EPSILON || normal_miss) continue;
        v3 sample_direction = normalize3(sub3(xyz(q.s.sample_position), xyz(s.visible_position)));
        if (dot3(sample_direction, s.visible_normal) < 0.0f) continue;

        float tap_interval = hk_maxf(1.0f, py / (float)(SPATIAL_REUSE_TAPS + 1u));
        uint32_t tap_count = f2u32(py / tap_interval);
        int occluded = 0;
        float inv_len = 1.0f / sqrtf(dot2(offset, offset));
        v2 dir = V2(offset.x * inv_len, offset.y * inv_len);
        for (uint32_t j = 1u; j <= tap_count; j += 1u) {
            float tap_dist = (float)j * tap_interval;
            v2 tap_offset = V2(tap_dist * dir.x, tap_dist * dir.y);
            v2 tap_uv = V2(uv.x + tap_offset.x / (float)render_size[0], uv.y + tap_offset.y / (float)render_size[1]);
            int32_t tdx, tdy;
            jittered_deferred_coords(P, tap_uv, &tdx, &tdy);
            float tap_depth = load_position(c, tdx, tdy).w;
            float ref_depth = hk_mixf(depth, sample_depth, (float)j / (float)(tap_count + 1u));
            if (tap_depth > ref_depth + 0.00001f) {
                occluded = 1;
                break;
            }
        }
        if (occluded) continue;

        float jacobian = q.s.sample_position.w > 0.5f ? compute_jacobian(&q.s, &s) : 1.0f;
        if (P->emissive_lit) {
            merge_reservoir(&r, &q, lum3(xyz(q.s.radiance)) / jacobian);
        } else {
            v3 out_radiance = shading(P, view_direction, s.visible_normal, sample_direction, &surface, q.s.radiance);
            merge_reservoir(&r, &q, lum3(out_radiance) / jacobian);
        }
    }

    float m = (float)P->st->max_spatial_reuse_count;
    if (r.count > m) {
        r.w_sum *= m / r.count;
        r.w2_sum *= m / r.count;
        r.count = m;
    }
    v3 out_radiance = shading(P, view_direction, s.visible_normal,
                              normalize3(sub3(xyz(r.s.sample_position), xyz(s.visible_position))), &surface, r.s.radiance);
    float total_lum = P->emissive_lit ? r.count * lum3(xyz(r.s.radiance)) : r.count * lum3(out_radiance);
    r.w = total_lum > 0.0f ? r.w_sum / total_lum : 0.0f;
    r.lifetime += 1.0f;
    pack_reservoir(&r, &P->spatial_reservoir_buffer[idx]);
    if (use_spatial_variance) P->variance_texture[idx] = variance_of(&r);
    v3 out_color = scale3(out_radiance, r.w);
    if (P->render_emissive) out_color = add3(out_color, compute_emissive_radiance(surface.emissive));
    store_rgba16f(P->render_texture, (uint32_t)idx, V4(out_color.x, out_color.y, out_color.z, 1.0f));
}

/* ------------------------------------------------------------------ G-buffer (prepass.wgsl:84-100 via primary rays) */
static float ndc_depth(const float* view_proj, v3 p)
{
    v4 clip = mat4_mul(view_proj, V4(p.x, p.y, p.z, 1.0f));
    return clip.z / clip.w;
}
/* ---- G-buffer visibility: ordered closest-hit traversal (this build's primary-ray pass) ----
 * The reference rasterises the G-buffer (prepass.wgsl:84-100); this build traces one primary ray
 * per pixel instead, so its visibility rule is the build's own and is defined here, once, for
 * the oracle and for the HIP kernel (hk_device.h closest_hit_ordered), which must agree bit for
 * bit.  It walks the same flattened TLAS/BLAS (bvh 0.7.1 flatten: the subtree of an inner node
 * starts with the box node of its left child, whose subtree follows it; the box node of the
 * right child is at that box node's exit index) with the tests of light.wgsl:344-486:
 *   - a subtree starting at a leaf entry is a candidate: BLAS leaf -> slab test of its
 *     triangle's box (min/max of the 3 vertices), then Moller-Trumbore; TLAS leaf -> slab test of
 *     the instance's min/max, then the instance's BLAS from its position 0 (no root box test,
 *     as in the reference walk); a test passes iff its distance < best;
 *   - an inner subtree has two children (box node, subtree after it); a child is entered iff
 *     its box's slab distance t < best; with both entered, the smaller t first (left on ties)
 *     and the other is pushed with its t and dropped on pop if t >= best by then;
 *   - a triangle replaces the best hit iff d < best (the first found wins ties).
 * BLAS indices are mesh-local (offset by mesh.node[0], light.wgsl:404-405).  The stack never
 * holds more entries than TLAS depth + BLAS depth (HKO_GB_STACK, checked). */
#define HKO_GB_STACK 64
typedef struct { uint32_t node[HKO_GB_STACK]; float t[HKO_GB_STACK]; int sp; } GbStack;
static void gb_push(GbStack* s, uint32_t n, float t)
{
    if (s->sp >= HKO_GB_STACK) {
        fprintf(stderr, "hk_oracle: G-buffer traversal stack overflow (BVH deeper than %d)\n", HKO_GB_STACK);
        abort();
    }
    s->node[s->sp] = n;
    s->t[s->sp] = t;
    s->sp++;
}
/* pop the next entry above `base` whose t is still < best; returns 0 when none is left */
static int gb_pop(GbStack* s, int base, float best, uint32_t* n)
{
    while (s->sp > base) {
        s->sp--;
        if (s->t[s->sp] < best) {
            *n = s->node[s->sp];
            return 1;
        }
    }
    return 0;
}
/* the two children of the inner subtree at `p`: (box node, subtree start) pairs */
static void gb_children(const hk_node* nodes, uint32_t base, uint32_t p, uint32_t* lb, uint32_t* rb)
{
    *lb = p;
    *rb = base + nodes[p].exit_index;
}
static void gb_descend(GbStack* s, const Ray* ray, const hk_node* nodes, uint32_t base, uint32_t* p, float best,
                       int* go)
{
    uint32_t lb, rb;
    gb_children(nodes, base, *p, &lb, &rb);
    Aabb la = {ld3(nodes[lb].min), ld3(nodes[lb].max)}, ra = {ld3(nodes[rb].min), ld3(nodes[rb].max)};
    float tl = intersects_aabb(ray, la), tr = intersects_aabb(ray, ra);
    int hl = tl < best, hr = tr < best;
    *go = 1;
    if (hl && hr) {
        if (tr < tl) {
            gb_push(s, lb + 1, tl);
            *p = rb + 1;
        } else {
            gb_push(s, rb + 1, tr);
            *p = lb + 1;
        }
    } else if (hl) {
        *p = lb + 1;
    } else if (hr) {
        *p = rb + 1;
    } else {
        *go = 0;
    }
}
static void closest_bottom_ordered(const hko_ctx* c, GbStack* s, Hit* hit, const Ray* ray, const hk_mesh_index* mesh,
                                   uint32_t instance_index)
{
    const int sbase = s->sp;
    const uint32_t base = mesh->node[0];
    if (mesh->node[1] == 0) return;
    uint32_t p = base;
    for (;;) {
        HKO_STAT(3);
        const hk_node* node = &c->asset_nodes[p];
        int go = 0;
        if (node->entry_index >= HK_BVH_LEAF_FLAG) {
            uint32_t primitive_index = mesh->primitive + node->entry_index - HK_BVH_LEAF_FLAG;
            const hk_primitive_vertex* v = c->primitives[primitive_index].vertices;
            v3 a = ld3(v[0].position), e = ld3(v[1].position), d = ld3(v[2].position);
            Aabb box = {min3(a, min3(e, d)), max3(a, max3(e, d))};
            if (intersects_aabb(ray, box) < hit->intersection.distance) {
                HKO_STAT(4);
                Intersection is = intersects_triangle(ray, v);
                if (is.distance < hit->intersection.distance) {
                    hit->intersection = is;
                    hit->primitive_index = primitive_index;
                    hit->instance_index = instance_index;
                }
            }
        } else {
            gb_descend(s, ray, c->asset_nodes, base, &p, hit->intersection.distance, &go);
        }
        if (go) continue;
        if (!gb_pop(s, sbase, hit->intersection.distance, &p)) return;
    }
}
static Hit closest_hit_ordered(const hko_ctx* c, const Ray* ray)
{
    Hit hit;
    hit.intersection.uv = V2(0, 0);
    hit.intersection.distance = HK_F32_MAX;
    hit.instance_index = HK_U32_MAX;
    hit.primitive_index = HK_U32_MAX;
    if (c->n_instance_nodes == 0) return hit;
    GbStack s;
    s.sp = 0;
    uint32_t p = 0;
    for (;;) {
        HKO_STAT(1);
        const hk_node* node = &c->instance_nodes[p];
        int go = 0;
        if (node->entry_index >= HK_BVH_LEAF_FLAG) {
            uint32_t instance_index = node->entry_index - HK_BVH_LEAF_FLAG;
            const hk_instance* instance = &c->instances[instance_index];
            Aabb box = {ld3(instance->min), ld3(instance->max)};
            if (intersects_aabb(ray, box) < hit.intersection.distance) {
                Ray r;
                r.origin = instance_position_world_to_local(instance, ray->origin);
                r.direction = instance_direction_world_to_local(instance, ray->direction);
                r.inv_direction = inv3(r.direction);
                HKO_STAT(2);
                closest_bottom_ordered(c, &s, &hit, &r, &instance->mesh, instance_index);
            }
        } else {
            gb_descend(&s, ray, c->instance_nodes, 0, &p, hit.intersection.distance, &go);
        }
        if (go) continue;
        if (!gb_pop(&s, 0, hit.intersection.distance, &p)) return hit;
    }
}

/* the emitter BLAS walk with the ordered rule: closest_bottom_ordered from an empty stack; traced iff a
 * triangle replaced the empty hit (traverse_bottom's `intersected`) */
static int emitter_walk_ordered(const hko_ctx* c, Hit* hit, const Ray* ray, const hk_mesh_index* mesh)
{
    GbStack s;
    s.sp = 0;
    const uint32_t before = hit->primitive_index;
    const float d0 = hit->intersection.distance;
    const uint32_t inst = hit->instance_index;
    closest_bottom_ordered(c, &s, hit, ray, mesh, inst);
    return hit->intersection.distance < d0 || hit->primitive_index != before;
}

static v3 primary_direction(const hk_view* view, float px, float py, const uint32_t* size)
{
    float ndc_x = (px / (float)size[0]) * 2.0f - 1.0f;
    float ndc_y = 1.0f - (py / (float)size[1]) * 2.0f;
    v4 p = mat4_mul(view->inverse_view_proj, V4(ndc_x, ndc_y, 1.0f, 1.0f));
    v3 near = div3s(xyz(p), p.w);
    return normalize3(sub3(near, ld3(view->world_position)));
}
/* utils.wgsl:30-35 */
static v2 clip_to_uv(v4 clip)
{
    v2 uv = V2(clip.x / clip.w, clip.y / clip.w);
    uv = V2((uv.x + 1.0f) * 0.5f, (uv.y + 1.0f) * 0.5f);
    return V2(uv.x, 1.0f - uv.y);
}
/* Per-frame prepass state: the halton jitter in pixels (prepass.wgsl:30-38,52-54: jitter =
 * 2 h / viewport in NDC added to clip.xy with y flipped, so the point seen at pixel centre c is the
 * one that projects to c - h) and the motion-vector inputs. */
typedef struct {
    float jitter[2];
    int motion;                    /* camera or any instance moved: velocities are computed */
    const float* previous_view_proj;
} GbFrame;
static const float HALTON[8][4] = { /* view.rs:130-139 */
    {0.000000f, 0.000000f, 0.500000f, 0.333333f}, {0.250000f, 0.666667f, 0.750000f, 0.111111f},
    {0.125000f, 0.444444f, 0.625000f, 0.777778f}, {0.375000f, 0.222222f, 0.875000f, 0.555556f},
    {0.062500f, 0.888889f, 0.562500f, 0.037037f}, {0.312500f, 0.370370f, 0.812500f, 0.703704f},
    {0.187500f, 0.148148f, 0.687500f, 0.481481f}, {0.437500f, 0.814815f, 0.937500f, 0.259259f}};

/* frame_jitter (prepass.wgsl:30-38) */
static void frame_jitter(const hk_frame_inputs* in, float* jitter)
{
    jitter[0] = jitter[1] = 0.0f;
    if (in->jitter == HK_JITTER_TAA || in->jitter == HK_JITTER_TAA_SMAA) {
        uint32_t index = in->jitter == HK_JITTER_TAA_SMAA ? (in->frame_number >> 1) & 15u : in->frame_number & 15u;
        const float* h = HALTON[index >> 1];
        jitter[0] = (index & 1u) == 0u ? h[0] : h[2];
        jitter[1] = (index & 1u) == 0u ? h[1] : h[3];
    }
}

static void gbuffer_pixel(const hko_ctx* c, Counts* cnt, const hk_frame_inputs* in, const GbFrame* G, int32_t x,
                          int32_t y)
{
    size_t idx = (size_t)y * c->S[0] + (size_t)x;
    const hk_view* view = &in->view;
    Ray ray;
    ray.origin = ld3(view->world_position);
    ray.direction = primary_direction(view, ((float)x + 0.5f) - G->jitter[0], ((float)y + 0.5f) - G->jitter[1], c->S);
    ray.inv_direction = inv3(ray.direction);
    cnt->primary++;
    Counts dummy = {0, 0, 0};
    (void)dummy;
    Hit hit = closest_hit_ordered(c, &ray);
    float* gp = c->g_position + 4 * idx;
    float* gd = c->g_depth_gradient + 2 * idx;
    float* gi = c->g_instance_material + 2 * idx;
    float* gv = c->g_velocity_uv + 4 * idx;
    if (hit.instance_index == HK_U32_MAX) {
        memset(gp, 0, 16);
        c->g_normal[idx] = 0u;
        memset(gd, 0, 8);
        memset(gi, 0, 8);
        memset(gv, 0, 16);
        return;
    }
    HitInfo info = hit_info(c, &ray, &hit);
    v3 p = xyz(info.position);
    float depth = ndc_depth(view->view_proj, p);
    gp[0] = p.x; gp[1] = p.y; gp[2] = p.z; gp[3] = depth;
    c->g_normal[idx] = hk_pack4x8snorm(info.normal.x, info.normal.y, info.normal.z, 1.0f);
    /* depth derivatives: re-intersect the hit triangle's plane with the neighbour pixel rays */
    const hk_instance* instance = get_instance(c, hit.instance_index);
    const hk_primitive_vertex* tv = c->primitives[hit.primitive_index].vertices;
    v3 w0 = instance_position_local_to_world(instance, ld3(tv[0].position));
    v3 w1 = instance_position_local_to_world(instance, ld3(tv[1].position));
    v3 w2 = instance_position_local_to_world(instance, ld3(tv[2].position));
    v3 ng = cross3(sub3(w1, w0), sub3(w2, w0));
    float plane = dot3(sub3(p, ray.origin), ng);
    float grad[2];
    for (int k = 0; k < 2; ++k) {
        v3 d = primary_direction(view, ((float)x + 0.5f + (k == 0 ? 1.0f : 0.0f)) - G->jitter[0],
                                 ((float)y + 0.5f + (k == 1 ? 1.0f : 0.0f)) - G->jitter[1], c->S);
        float denom = dot3(d, ng);
        grad[k] = 0.0f;
        if (denom != 0.0f) {
            float t = plane / denom;
            v3 q = add3(ray.origin, scale3(d, t));
            grad[k] = ndc_depth(view->view_proj, q) - depth;
        }
    }
    gd[0] = grad[0]; gd[1] = grad[1];
    gi[0] = (float)hit.instance_index + 0.5f;
    gi[1] = (float)info.material_index + 0.5f;
    /* prepass.wgsl:49-50,96: the hit's object-space point (the barycentric combination of the
     * triangle, what the rasteriser interpolates) through this frame's and the previous frame's
     * model and view; exactly zero when nothing moved */
    gv[0] = 0.0f; gv[1] = 0.0f;
    if (G->motion) {
        v3 t0 = ld3(tv[0].position), t1 = ld3(tv[1].position), t2 = ld3(tv[2].position);
        v3 lp = add3(add3(t0, scale3(sub3(t1, t0), hit.intersection.uv.x)), scale3(sub3(t2, t0), hit.intersection.uv.y));
        v4 l4 = V4(lp.x, lp.y, lp.z, 1.0f);
        v4 wc = mat4_mul(instance->model, l4);
        v4 wp = mat4_mul(c->prev_models + 16 * (size_t)hit.instance_index, l4);
        v2 a = clip_to_uv(mat4_mul(view->view_proj, wc)), b = clip_to_uv(mat4_mul(G->previous_view_proj, wp));
        gv[0] = a.x - b.x;
        gv[1] = a.y - b.y;
    }
    gv[2] = info.uv.x; gv[3] = info.uv.y;
}

/* ------------------------------------------------------------------ denoise (denoise.wgsl) */
typedef struct {
    const hko_ctx* c;
    const hk_settings* st;
    uint32_t number;
    int level, firefly;
    const uint16_t* render;
    const float* variance;
    uint16_t* out;
} DPass;

static const float KERNEL[3][3] = {{0.0625f, 0.125f, 0.0625f}, {0.125f, 0.25f, 0.125f}, {0.0625f, 0.125f, 0.0625f}};

static inline v2 d_jittered_deferred_uv(const DPass* D, v2 uv)
{
    float tx = 1.0f / (float)D->c->S[0], ty = 1.0f / (float)D->c->S[1];
    float ratio = D->st->upscale_ratio - 1.0f;
    float j = (D->number & 1u) == 0u ? -0.5f : 0.5f;
    return V2(uv.x + (j * tx) * ratio, uv.y + (j * ty) * ratio);
}
static inline int uv_outside(v2 uv) { return uv.x < 0.0f || uv.y < 0.0f || uv.x > 1.0f || uv.y > 1.0f; }
static inline int any_nan_inf3(v3 v)
{
    int nan = (v.x != v.x) || (v.y != v.y) || (v.z != v.z);
    int inf = v.x > HK_F32_MAX || v.y > HK_F32_MAX || v.z > HK_F32_MAX;
    return nan || inf;
}

static void demodulation(const DPass* D, int32_t x, int32_t y)
{
    const hko_ctx* c = D->c;
    const uint32_t* size = c->s;
    uint32_t idx = (uint32_t)y * size[0] + (uint32_t)x;
    v2 uv = coords_to_uv(x, y, size);
    v2 duv = d_jittered_deferred_uv(D, uv);
    int32_t ax, ay, rx, ry;
    nearest_texel(duv, c->S, &ax, &ay);
    v3 albedo = xyz(load_rgba16f(c->albedo, (uint32_t)ay * c->S[0] + (uint32_t)ax));
    nearest_texel(uv, size, &rx, &ry);
    v3 irr = xyz(load_rgba16f(D->render, (uint32_t)ry * size[0] + (uint32_t)rx));
    irr = V3(albedo.x < 0.01f ? 0.0f : irr.x / albedo.x, albedo.y < 0.01f ? 0.0f : irr.y / albedo.y,
             albedo.z < 0.01f ? 0.0f : irr.z / albedo.z);
    store_rgba16f(c->internal[0], idx, V4(irr.x, irr.y, irr.z, 1.0f));

    static const int offs[9][2] = {{-1, -1}, {-1, 0}, {-1, 1}, {0, -1}, {0, 0}, {0, 1}, {1, -1}, {1, 0}, {1, 1}};
    float sum_variance = 0.0f;
    for (int k = 0; k < 9; ++k) {
        int ox = offs[k][0], oy = offs[k][1];
        v2 suv = V2(uv.x + (float)ox / (float)size[0], uv.y + (float)oy / (float)size[1]);
        if (uv_outside(suv)) continue;
        int32_t vx, vy;
        nearest_texel(suv, size, &vx, &vy);
        float variance = D->variance[(uint32_t)vy * size[0] + (uint32_t)vx];
        if (variance > HK_F32_MAX) continue;
        sum_variance += KERNEL[oy + 1][ox + 1] * hk_maxf(variance, 0.0f);
    }
    c->internal_variance[idx] = sum_variance;
}

static void denoise_pixel(const DPass* D, int32_t x, int32_t y)
{
    const hko_ctx* c = D->c;
    const uint32_t* size = c->s;
    uint32_t idx = (uint32_t)y * size[0] + (uint32_t)x;
    const uint16_t* input = c->internal[D->level];
    uint16_t* output = D->level == 3 ? D->out : c->internal[D->level + 1];
    int32_t step = 8 >> D->level;
    v2 uv = coords_to_uv(x, y, size);
    v2 duv = d_jittered_deferred_uv(D, uv);
    int32_t gx, gy;
    nearest_texel(duv, c->S, &gx, &gy);
    float depth = load_position(c, gx, gy).w;
    v2 depth_gradient = load_depth_gradient(c, gx, gy);
    v3 normal = normalize3(load_normal(c, gx, gy));
    float instance = load_instance_material(c, gx, gy).x;
    if (depth < HK_F32_EPSILON) {
        store_rgba16f(output, idx, V4(0, 0, 0, 0));
        return;
    }
    float variance = c->internal_variance[idx];
    v3 irradiance = xyz(load_rgba16f(input, idx));
    float k11 = KERNEL[1][1];
    v3 sum_irradiance = scale3(irradiance, k11);
    float sum_w = k11;
    if (any_nan_inf3(irradiance)) {
        irradiance = V3(0, 0, 0);
        sum_irradiance = V3(0, 0, 0);
        sum_w = 0.0f;
    }
    float lum = lum3(irradiance);
    float ff_m1 = 0.0f, ff_m2 = 0.0f, ff_count = 0.0f;
    static const int offs[8][2] = {{-1, -1}, {0, -1}, {1, -1}, {-1, 0}, {1, 0}, {-1, 1}, {0, 1}, {1, 1}};
    for (int k = 0; k < 8; ++k) {
        int ox = offs[k][0], oy = offs[k][1];
        int32_t sx = x + ox * step, sy = y + oy * step;
        v2 suv = coords_to_uv(sx, sy, size);
        v2 sduv = d_jittered_deferred_uv(D, suv);
        if (uv_outside(suv)) continue;
        v3 irr = xyz(load_rgba16f(input, (uint32_t)sy * size[0] + (uint32_t)sx));
        if (any_nan_inf3(irr)) continue;
        int32_t tx, ty;
        nearest_texel(sduv, c->S, &tx, &ty);
        v3 sample_normal = normalize3(load_normal(c, tx, ty));
        float sample_depth = load_position(c, tx, ty).w;
        float sample_instance = load_instance_material(c, tx, ty).x;
        float sample_luminance = lum3(irr);
        float w_normal = hk_pow16(hk_maxf(0.0f, dot3(normal, sample_normal)));
        float w_depth = hk_exp((-hk_absf(depth - sample_depth)) /
                               (hk_absf(dot2(depth_gradient, V2((float)ox, (float)oy))) + 0.01f));
        float w_instance = hk_maxf(0.0f, 1.0f - hk_absf(instance - sample_instance));
        float w_luminance = hk_exp((-hk_absf(lum - sample_luminance)) / (4.0f * hk_pow(variance, 0.25f) + 0.001f));
        float w = hk_clampf(((w_normal * w_depth) * w_instance) * w_luminance, 0.0f, 1.0f) * KERNEL[oy + 1][ox + 1];
        sum_irradiance = add3(sum_irradiance, scale3(irr, w));
        sum_w += w;
        if (D->firefly) {
            ff_m1 += sample_luminance;
            ff_m2 += sample_luminance * sample_luminance;
            ff_count += 1.0f;
        }
    }
    irradiance = sum_w < 0.0001f ? V3(0, 0, 0) : div3s(sum_irradiance, sum_w);
    if (D->firefly) {
        float ff_mean = ff_m1 / ff_count;
        float ff_var = ff_m2 / ff_count - ff_mean * ff_mean;
        if (lum > ff_mean + 3.0f * sqrtf(ff_var)) irradiance = scale3(irradiance, ff_mean / lum);
    }
    v4 color = V4(irradiance.x, irradiance.y, irradiance.z, 1.0f);
    if (D->level == 3) {
        v4 albedo = load_rgba16f(c->albedo, (uint32_t)gy * c->S[0] + (uint32_t)gx);
        color = V4(color.x * albedo.x, color.y * albedo.y, color.z * albedo.z, color.w * albedo.w);
    }
    store_rgba16f(output, idx, color);
}

/* ------------------------------------------------------------------ API */
static void* xdup(const hk_array* a, size_t elem)
{
    size_t n = a->count ? a->count : 1;
    void* p = calloc(n, elem);
    if (a->count && a->data) memcpy(p, a->data, a->count * elem);
    return p;
}

hko_ctx* hko_create(const hk_scene_desc* sc, const uint8_t* noise, uint32_t width, uint32_t height, float ratio,
                    int threads)
{
    hko_ctx* c = (hko_ctx*)calloc(1, sizeof(hko_ctx));
    c->vertices = (hk_vertex*)xdup(&sc->vertices, sizeof(hk_vertex)); c->n_vertices = sc->vertices.count;
    c->primitives = (hk_primitive*)xdup(&sc->primitives, sizeof(hk_primitive)); c->n_primitives = sc->primitives.count;
    c->asset_nodes = (hk_node*)xdup(&sc->asset_nodes, sizeof(hk_node)); c->n_asset_nodes = sc->asset_nodes.count;
    c->alias_table = (hk_alias_entry*)xdup(&sc->alias_table, sizeof(hk_alias_entry)); c->n_alias = sc->alias_table.count;
    c->instances = (hk_instance*)xdup(&sc->instances, sizeof(hk_instance)); c->n_instances = sc->instances.count;
    c->instance_nodes = (hk_node*)xdup(&sc->instance_nodes, sizeof(hk_node)); c->n_instance_nodes = sc->instance_nodes.count;
    c->materials = (hk_material*)xdup(&sc->materials, sizeof(hk_material)); c->n_materials = sc->materials.count;
    c->emissive_nodes = (hk_node*)xdup(&sc->emissive_nodes, sizeof(hk_node)); c->n_emissive_nodes = sc->emissive_nodes.count;
    c->emissives = (hk_emissive*)xdup(&sc->emissives, sizeof(hk_emissive)); c->n_emissives = sc->emissives.count;
    c->prev_models = (float*)calloc((size_t)(c->n_instances ? c->n_instances : 1) * 16, sizeof(float));
    for (uint32_t i = 0; i < c->n_instances; ++i) memcpy(c->prev_models + 16 * (size_t)i, c->instances[i].model, 64);
    if (noise) memcpy(c->noise, noise, sizeof(c->noise));
    if (ratio < 1.0f) ratio = 1.0f;
    if (ratio > 2.0f) ratio = 2.0f;
    c->ratio = ratio;
    c->S[0] = width;
    c->S[1] = height;
    c->s[0] = (uint32_t)ceilf((1.0f / ratio) * (float)width);
    c->s[1] = (uint32_t)ceilf((1.0f / ratio) * (float)height);
    c->threads = threads;
    c->band_y0 = 0;
    c->band_y1 = (int32_t)height;
    c->band_x0 = 0;
    c->band_x1 = (int32_t)width;
    size_t S = (size_t)width * height, s = (size_t)c->s[0] * c->s[1];
    c->g_position = (float*)calloc(S * 4, sizeof(float));
    c->g_normal = (uint32_t*)calloc(S, sizeof(uint32_t));
    c->g_depth_gradient = (float*)calloc(S * 2, sizeof(float));
    c->g_instance_material = (float*)calloc(S * 2, sizeof(float));
    c->g_velocity_uv = (float*)calloc(S * 4, sizeof(float));
    c->g_prev_position = (float*)calloc(S * 4, sizeof(float));
    c->g_prev_velocity_uv = (float*)calloc(S * 4, sizeof(float));
    c->albedo = (uint16_t*)calloc(S * 4, sizeof(uint16_t));
    for (int i = 0; i < 3; ++i) {
        c->variance[i] = (float*)calloc(s, sizeof(float));
        c->render[i] = (uint16_t*)calloc(s * 4, sizeof(uint16_t));
        c->denoised[i] = (uint16_t*)calloc(s * 4, sizeof(uint16_t));
    }
    for (int i = 0; i < HK_RESERVOIR_BUFFERS; ++i) c->reservoirs[i] = (hk_packed_reservoir*)calloc(S, sizeof(hk_packed_reservoir));
    for (int i = 0; i < 4; ++i) c->internal[i] = (uint16_t*)calloc(s * 4, sizeof(uint16_t));
    c->internal_variance = (float*)calloc(s, sizeof(float));
    c->tone_buf[0] = (uint16_t*)calloc(s * 4, sizeof(uint16_t));
    c->tone_buf[1] = (uint16_t*)calloc(s * 4, sizeof(uint16_t));
    c->tone = c->tone_buf[0];
    return c;
}

int hko_set_textures(hko_ctx* c, const hk_texture* t, uint32_t count)
{
    free(c->tex_desc); free(c->texels);
    c->tex_desc = NULL; c->texels = NULL; c->n_textures = 0;
    if (count == 0) return 0;
    uint64_t total = 0;
    c->tex_desc = (hk_texture_desc*)calloc(count, sizeof(hk_texture_desc));
    for (uint32_t i = 0; i < count; ++i) {
        hk_texture_desc d = {(uint32_t)total, t[i].width, t[i].height, t[i].format, t[i].address_u, t[i].address_v,
                             t[i].filter, 0u};
        c->tex_desc[i] = d;
        total += (uint64_t)t[i].width * t[i].height;
    }
    c->texels = (uint32_t*)malloc(total * 4 + 4);
    for (uint32_t i = 0; i < count; ++i)
        memcpy(c->texels + c->tex_desc[i].offset, t[i].rgba8, (size_t)t[i].width * t[i].height * 4);
    hk_texture_build_lut(c->tex_lut);
    c->n_textures = count;
    return 0;
}
void hko_sample_texture(const hko_ctx* c, uint32_t id, const float* uv, uint32_t n, float* out)
{
    for (uint32_t i = 0; i < n; ++i)
        hk_sample_texture(c->tex_desc + id, c->texels, c->tex_lut, uv[2 * i], uv[2 * i + 1], out + 4 * i);
}

void hko_destroy(hko_ctx* c)
{
    if (!c) return;
    free(c->vertices); free(c->primitives); free(c->asset_nodes); free(c->alias_table); free(c->instances);
    free(c->instance_nodes); free(c->materials); free(c->emissive_nodes); free(c->emissives);
    free(c->prev_models);
    free(c->tex_desc); free(c->texels);
    free(c->g_position); free(c->g_normal); free(c->g_depth_gradient); free(c->g_instance_material); free(c->g_velocity_uv);
    free(c->albedo);
    for (int i = 0; i < 3; ++i) { free(c->variance[i]); free(c->render[i]); free(c->denoised[i]); }
    for (int i = 0; i < HK_RESERVOIR_BUFFERS; ++i) free(c->reservoirs[i]);
    for (int i = 0; i < 4; ++i) free(c->internal[i]);
    free(c->internal_variance); free(c->tone_buf[0]); free(c->tone_buf[1]);
    free(c->g_prev_position); free(c->g_prev_velocity_uv);
    free(c->upscale); free(c->taa_buf[0]); free(c->taa_buf[1]);
    free(c);
}

static void add_counts(hko_ctx* c, const Counts* k)
{
#pragma omp critical(hko_counts)
    {
        c->counters.traverse_top += k->top;
        c->counters.traverse_emitter += k->emitter;
        c->counters.primary += k->primary;
    }
}

#define HKO_THREADS(c) num_threads((c)->threads > 0 ? (c)->threads : omp_get_max_threads())
#ifndef _OPENMP
static int omp_get_max_threads(void) { return 1; }
#endif

/* row y is computed (hko_set_stripes; every row otherwise) */
static inline int row_on(const hko_ctx* c, int32_t y)
{
    return c->stripe_n < 2 || (y / 8) % c->stripe_n == c->stripe_k;
}

static void set_head(hko_ctx* c, uint32_t frame_number)
{
    c->head = frame_number & 1u;
    c->tone = c->tone_buf[c->head];
}

void hko_render_gbuffer(hko_ctx* c, const hk_frame_inputs* in)
{
    /* a new frame: this frame's planes replace the previous ones (prepass.rs:309-317) */
    float* t = c->g_position;
    c->g_position = c->g_prev_position;
    c->g_prev_position = t;
    t = c->g_velocity_uv;
    c->g_velocity_uv = c->g_prev_velocity_uv;
    c->g_prev_velocity_uv = t;
    set_head(c, in->frame_number);
    GbFrame G;
    frame_jitter(in, G.jitter);
    G.previous_view_proj = in->has_previous_view ? in->previous_view_proj : in->view.view_proj;
    G.motion = memcmp(G.previous_view_proj, in->view.view_proj, 64) != 0;
    for (uint32_t i = 0; i < c->n_instances && !G.motion; ++i)
        G.motion = memcmp(c->prev_models + 16 * (size_t)i, c->instances[i].model, 64) != 0;
#pragma omp parallel HKO_THREADS(c)
    {
        Counts k = {0, 0, 0};
#pragma omp for schedule(dynamic, 4)
        for (int32_t y = c->band_y0; y < c->band_y1; ++y)
            {
                if (!row_on(c, y)) continue;
                for (int32_t x = c->band_x0; x < (c->band_x1 < (int32_t)c->S[0] ? c->band_x1 : (int32_t)c->S[0]); ++x) gbuffer_pixel(c, &k, in, &G, x, y);
            }
        add_counts(c, &k);
    }
    /* this frame's models are the next frame's previous ones */
    for (uint32_t i = 0; i < c->n_instances; ++i) memcpy(c->prev_models + 16 * (size_t)i, c->instances[i].model, 64);
}

/* replace the scene arrays (hk_update_instances / a host rebuild); the previous models stay */
void hko_set_scene(hko_ctx* c, const hk_scene_desc* sc)
{
    free(c->vertices); free(c->primitives); free(c->asset_nodes); free(c->alias_table); free(c->instances);
    free(c->instance_nodes); free(c->materials); free(c->emissive_nodes); free(c->emissives);
    uint32_t old_n = c->n_instances;
    c->vertices = (hk_vertex*)xdup(&sc->vertices, sizeof(hk_vertex)); c->n_vertices = sc->vertices.count;
    c->primitives = (hk_primitive*)xdup(&sc->primitives, sizeof(hk_primitive)); c->n_primitives = sc->primitives.count;
    c->asset_nodes = (hk_node*)xdup(&sc->asset_nodes, sizeof(hk_node)); c->n_asset_nodes = sc->asset_nodes.count;
    c->alias_table = (hk_alias_entry*)xdup(&sc->alias_table, sizeof(hk_alias_entry)); c->n_alias = sc->alias_table.count;
    c->instances = (hk_instance*)xdup(&sc->instances, sizeof(hk_instance)); c->n_instances = sc->instances.count;
    c->instance_nodes = (hk_node*)xdup(&sc->instance_nodes, sizeof(hk_node)); c->n_instance_nodes = sc->instance_nodes.count;
    c->materials = (hk_material*)xdup(&sc->materials, sizeof(hk_material)); c->n_materials = sc->materials.count;
    c->emissive_nodes = (hk_node*)xdup(&sc->emissive_nodes, sizeof(hk_node)); c->n_emissive_nodes = sc->emissive_nodes.count;
    c->emissives = (hk_emissive*)xdup(&sc->emissives, sizeof(hk_emissive)); c->n_emissives = sc->emissives.count;
    if (old_n != c->n_instances) { /* a different instance set: no history */
        free(c->prev_models);
        c->prev_models = (float*)calloc((size_t)(c->n_instances ? c->n_instances : 1) * 16, sizeof(float));
        for (uint32_t i = 0; i < c->n_instances; ++i) memcpy(c->prev_models + 16 * (size_t)i, c->instances[i].model, 64);
    }
}

typedef enum { K_DIRECT, K_INDIRECT, K_SPATIAL } Kind;

static void run_pass(hko_ctx* c, const Pass* P, Kind kind)
{
#pragma omp parallel HKO_THREADS(c)
    {
        Counts k = {0, 0, 0};
#pragma omp for schedule(dynamic, 4)
        for (int32_t y = c->band_y0; y < (c->band_y1 < (int32_t)c->s[1] ? c->band_y1 : (int32_t)c->s[1]); ++y)
        {
            if (!row_on(c, y)) continue;
            for (int32_t x = c->band_x0; x < (c->band_x1 < (int32_t)c->s[0] ? c->band_x1 : (int32_t)c->s[0]); ++x) {
#ifdef HKO_STATS
                hko_npix = c->s[0] * c->s[1];
                hko_pixel = (int32_t)(x + (int32_t)c->s[0] * y);
                hko_pass = kind == K_INDIRECT ? 2 : (P->emissive_lit ? 1 : 0);
                if (kind == K_SPATIAL) hko_pixel = -1;
#endif
                if (kind == K_DIRECT) direct_lit(P, &k, x, y);
                else if (kind == K_INDIRECT) indirect_lit_ambient(P, &k, x, y);
                else spatial_reuse(P, x, y);
            }
        }
#ifdef HKO_STATS
        hko_pixel = -1;
#endif
        add_counts(c, &k);
    }
}

/* LightNode::run (light.rs:590-702) */
void hko_render_frame(hko_ctx* c, const hk_settings* st, const hk_frame_inputs* in)
{
    set_head(c, in->frame_number);
    Pass P;
    memset(&P, 0, sizeof(P));
    P.c = c;
    P.st = st;
    P.in = in;
    P.number = in->frame_number;
    /* full-screen albedo over S */
#pragma omp parallel for schedule(static) HKO_THREADS(c)
    for (int32_t y = c->band_y0; y < c->band_y1; ++y)
        {
            if (!row_on(c, y)) continue;
            for (int32_t x = c->band_x0; x < (c->band_x1 < (int32_t)c->S[0] ? c->band_x1 : (int32_t)c->S[0]); ++x) full_screen_albedo(&P, x, y);
        }

    uint32_t current = P.number % 2u, previous = 1u - current;
    static const int pairs[3][2] = {{0, 4}, {2, 4}, {6, 8}};
    for (int ch = 0; ch < 3; ++ch) {
        Pass Q = P;
        Q.previous_reservoir_buffer = c->reservoirs[current + pairs[ch][0]];
        Q.reservoir_buffer = c->reservoirs[previous + pairs[ch][0]];
        Q.previous_spatial_reservoir_buffer = c->reservoirs[current + pairs[ch][1]];
        Q.spatial_reservoir_buffer = c->reservoirs[previous + pairs[ch][1]];
        Q.variance_texture = c->variance[ch];
        Q.render_texture = c->render[ch];
        if (ch == 0) {
            Q.render_emissive = 1;
            run_pass(c, &Q, K_DIRECT);
        } else if (ch == 1) {
            Q.emissive_lit = 1;
            run_pass(c, &Q, K_DIRECT);
            if (st->emissive_spatial_reuse) run_pass(c, &Q, K_SPATIAL);
        } else {
            Q.multiple_bounces = st->indirect_bounces >= 2u;
            run_pass(c, &Q, K_INDIRECT);
            if (st->indirect_spatial_reuse) {
                Q.multiple_bounces = 0;
                run_pass(c, &Q, K_SPATIAL);
            }
        }
    }
}

/* PostProcessNode::run denoise block (post_process.rs:1190-1224) */
void hko_denoise(hko_ctx* c, const hk_settings* st, const hk_frame_inputs* in)
{
    if (!st->denoise) return;
    int channels = st->indirect_bounces == 0u ? 2 : 3;
    for (int ch = 0; ch < channels; ++ch) {
        DPass D;
        D.c = c;
        D.st = st;
        D.number = in->frame_number;
        D.firefly = ch >= 1;
        D.render = c->render[ch];
        D.variance = c->variance[ch];
        D.out = c->denoised[ch];
        D.level = 0;
#pragma omp parallel for schedule(static) HKO_THREADS(c)
        for (int32_t y = c->band_y0; y < (c->band_y1 < (int32_t)c->s[1] ? c->band_y1 : (int32_t)c->s[1]); ++y)
            {
                if (!row_on(c, y)) continue;
                for (int32_t x = c->band_x0; x < (c->band_x1 < (int32_t)c->s[0] ? c->band_x1 : (int32_t)c->s[0]); ++x) demodulation(&D, x, y);
            }
        for (int level = 0; level < 4; ++level) {
            D.level = level;
#pragma omp parallel for schedule(static) HKO_THREADS(c)
            for (int32_t y = c->band_y0; y < (c->band_y1 < (int32_t)c->s[1] ? c->band_y1 : (int32_t)c->s[1]); ++y)
                {
                    if (!row_on(c, y)) continue;
                    for (int32_t x = c->band_x0; x < (c->band_x1 < (int32_t)c->s[0] ? c->band_x1 : (int32_t)c->s[0]); ++x) denoise_pixel(&D, x, y);
                }
        }
    }
}

/* tone_mapping.wgsl:21-32 */
void hko_tone_sum(hko_ctx* c, const hk_settings* st)
{
    const uint16_t* d = st->denoise ? c->denoised[0] : c->render[0];
    const uint16_t* e = st->denoise ? c->denoised[1] : c->render[1];
    const uint16_t* i = st->indirect_bounces == 0u ? NULL : (st->denoise ? c->denoised[2] : c->render[2]);
    size_t n = (size_t)c->s[0] * c->s[1];
#pragma omp parallel for schedule(static) HKO_THREADS(c)
    for (long long p = 0; p < (long long)n; ++p) {
        if (!row_on(c, (int32_t)(p / (long long)c->s[0]))) continue;
        v4 col = load_rgba16f(d, (uint32_t)p);
        v4 ec = load_rgba16f(e, (uint32_t)p);
        col = V4(col.x + ec.x, col.y + ec.y, col.z + ec.z, col.w + ec.w);
        if (i) {
            v4 ic = load_rgba16f(i, (uint32_t)p);
            col = V4(col.x + ic.x, col.y + ic.y, col.z + ic.z, col.w + ic.w);
        }
        v3 cc = max3(xyz(col), V3(0.0039f, 0.0039f, 0.0039f));
        float l_old = lum3(cc);
        float l_new = l_old / (1.0f + l_old);
        cc = scale3(cc, l_new / l_old);
        v4 out = col.w > 0.0f ? V4(cc.x, cc.y, cc.z, col.w)
                              : V4(st->clear_color[0], st->clear_color[1], st->clear_color[2], st->clear_color[3]);
        store_rgba16f(c->tone, (uint32_t)p, out);
    }
}

/* post_process.rs:1236-1276: SMAA TU4x then TAA Jasmine (include/hk_post.h, shared with the GPU) */
static hk_pp_tex pp_tex(const void* d, uint32_t w, uint32_t h, uint32_t f16, uint32_t comps)
{
    hk_pp_tex t;
    t.data = d, t.w = w, t.h = h, t.f16 = f16, t.comps = comps;
    return t;
}
void hko_post_process(hko_ctx* c, const hk_settings* st, const hk_frame_inputs* in)
{
    set_head(c, in->frame_number);
    const uint32_t head = c->head;
    float scale = 1.0f / c->ratio;
    hk_pp_frame F;
    F.number = in->frame_number;
    for (int k = 0; k < 4; ++k) F.clear_color[k] = st->clear_color[k];
    F.upscale_ratio = c->ratio;
    hk_pp_inputs I;
    const uint32_t S0 = c->S[0], S1 = c->S[1];
    I.position = pp_tex(c->g_position, S0, S1, 0, 4);
    I.previous_position = pp_tex(c->g_prev_position, S0, S1, 0, 4);
    I.velocity_uv = pp_tex(c->g_velocity_uv, S0, S1, 0, 4);
    I.previous_velocity_uv = pp_tex(c->g_prev_velocity_uv, S0, S1, 0, 4);
    I.instance_material = pp_tex(c->g_instance_material, S0, S1, 0, 2);
    hk_pp_tex taa_input = pp_tex(c->tone_buf[head], c->s[0], c->s[1], 1, 4);
    if (st->upscale == 0u) {
        scale *= 2.0f;
        const uint32_t U0 = (uint32_t)ceilf((float)S0 * scale), U1 = (uint32_t)ceilf((float)S1 * scale);
        if (!c->upscale || c->upscale_wh[0] != U0 || c->upscale_wh[1] != U1) {
            free(c->upscale);
            c->upscale = (uint16_t*)calloc((size_t)U0 * U1 * 4, sizeof(uint16_t));
            c->upscale_wh[0] = U0, c->upscale_wh[1] = U1;
        }
        I.render = pp_tex(c->tone_buf[head], c->s[0], c->s[1], 1, 4);
        I.previous_render = pp_tex(c->tone_buf[1u - head], c->s[0], c->s[1], 1, 4);
        I.output.data = c->upscale, I.output.w = U0, I.output.h = U1;
#pragma omp parallel for schedule(static) HKO_THREADS(c)
        for (int32_t y = 0; y < (int32_t)c->s[1]; ++y)
            for (int32_t x = c->band_x0; x < (c->band_x1 < (int32_t)c->s[0] ? c->band_x1 : (int32_t)c->s[0]); ++x) hk_pp_smaa_tu4x(&F, &I, x, y);
#pragma omp parallel for schedule(static) HKO_THREADS(c)
        for (int32_t y = 0; y < (int32_t)c->s[1]; ++y)
            for (int32_t x = c->band_x0; x < (c->band_x1 < (int32_t)c->s[0] ? c->band_x1 : (int32_t)c->s[0]); ++x) hk_pp_smaa_extrapolate(&I.output, x, y);
        taa_input = pp_tex(c->upscale, U0, U1, 1, 4);
    }
    if (st->taa == 0u) {
        const uint32_t T0 = (uint32_t)ceilf((float)S0 * scale), T1 = (uint32_t)ceilf((float)S1 * scale);
        if (!c->taa_buf[0] || c->taa_wh[0] != T0 || c->taa_wh[1] != T1) {
            for (int k = 0; k < 2; ++k) {
                free(c->taa_buf[k]);
                c->taa_buf[k] = (uint16_t*)calloc((size_t)T0 * T1 * 4, sizeof(uint16_t));
            }
            c->taa_wh[0] = T0, c->taa_wh[1] = T1;
        }
        I.render = taa_input;
        I.previous_render = pp_tex(c->taa_buf[1u - head], T0, T1, 1, 4);
        I.output.data = c->taa_buf[head], I.output.w = T0, I.output.h = T1;
#pragma omp parallel for schedule(static) HKO_THREADS(c)
        for (int32_t y = 0; y < (int32_t)T1; ++y)
            for (int32_t x = 0; x < (int32_t)T0; ++x) hk_pp_taa(&F, &I, x, y);
    }
}

void* hko_output(hko_ctx* c, int id, uint32_t* w, uint32_t* h, uint32_t* bpp)
{
    uint32_t W = c->s[0], H = c->s[1], B = 8;
    void* p = NULL;
    switch (id) {
    case HK_OUT_ALBEDO: p = c->albedo; W = c->S[0]; H = c->S[1]; break;
    case HK_OUT_VARIANCE_DIRECT: case HK_OUT_VARIANCE_EMISSIVE: case HK_OUT_VARIANCE_INDIRECT:
        p = c->variance[id - HK_OUT_VARIANCE_DIRECT]; B = 4; break;
    case HK_OUT_RENDER_DIRECT: case HK_OUT_RENDER_EMISSIVE: case HK_OUT_RENDER_INDIRECT:
        p = c->render[id - HK_OUT_RENDER_DIRECT]; break;
    case HK_OUT_DENOISED_DIRECT: case HK_OUT_DENOISED_EMISSIVE: case HK_OUT_DENOISED_INDIRECT:
        p = c->denoised[id - HK_OUT_DENOISED_DIRECT]; break;
    case HK_OUT_TONE_MAPPED: p = c->tone; break;
    case HK_OUT_UPSCALED: p = c->upscale; W = c->upscale_wh[0]; H = c->upscale_wh[1]; break;
    case HK_OUT_TAA: p = c->taa_buf[c->head]; W = c->taa_wh[0]; H = c->taa_wh[1]; break;
    case HK_OUT_GBUF_POSITION: p = c->g_position; W = c->S[0]; H = c->S[1]; B = 16; break;
    case HK_OUT_GBUF_NORMAL: p = c->g_normal; W = c->S[0]; H = c->S[1]; B = 4; break;
    case HK_OUT_GBUF_DEPTH_GRADIENT: p = c->g_depth_gradient; W = c->S[0]; H = c->S[1]; B = 8; break;
    case HK_OUT_GBUF_INSTANCE_MATERIAL: p = c->g_instance_material; W = c->S[0]; H = c->S[1]; B = 8; break;
    case HK_OUT_GBUF_VELOCITY_UV: p = c->g_velocity_uv; W = c->S[0]; H = c->S[1]; B = 16; break;
    case HK_OUT_DENOISE_INTERNAL_VARIANCE: p = c->internal_variance; B = 4; break;
    default: return NULL;
    }
    if (w) *w = W;
    if (h) *h = H;
    if (bpp) *bpp = B;
    return p;
}

hk_packed_reservoir* hko_reservoirs(hko_ctx* c, int id, uint32_t* count)
{
    if (id < 0 || id >= HK_RESERVOIR_BUFFERS) return NULL;
    if (count) *count = c->S[0] * c->S[1];
    return c->reservoirs[id];
}

void hko_set_band(hko_ctx* c, int32_t y0, int32_t rows, int32_t halo)
{
    int32_t a = y0 - halo, b = y0 + rows + halo;
    c->band_y0 = a < 0 ? 0 : a;
    c->band_y1 = b > (int32_t)c->S[1] ? (int32_t)c->S[1] : b;
}

/* a 2-D tile (hk_resize_tile): columns [x0, x0 + cols) of rows [y0, y0 + rows), plus halo on every side */
void hko_set_tile(hko_ctx* c, int32_t x0, int32_t cols, int32_t y0, int32_t rows, int32_t halo)
{
    hko_set_band(c, y0, rows, halo);
    int32_t a = x0 - halo, b = x0 + cols + halo;
    c->band_x0 = a < 0 ? 0 : a;
    c->band_x1 = b > (int32_t)c->S[0] ? (int32_t)c->S[0] : b;
}

void hko_set_stripes(hko_ctx* c, int32_t rank, int32_t world)
{
    c->stripe_n = world;
    c->stripe_k = rank;
}

void hko_counters(hko_ctx* c, hk_counters* out) { *out = c->counters; }
void hko_set_light_walk(hko_ctx* c, int mode)
{
    c->light_walk = mode;
    memset(c->walk_checked, 0, sizeof(c->walk_checked));
    memset(c->walk_differ, 0, sizeof(c->walk_differ));
}
void hko_light_walk_stats(const hko_ctx* c, unsigned long long* out)
{
    out[0] = c->walk_checked[0];
    out[1] = c->walk_differ[0];
    out[2] = c->walk_checked[1];
    out[3] = c->walk_differ[1];
}
void hko_reset_counters(hko_ctx* c) { memset(&c->counters, 0, sizeof(c->counters)); }

void hko_trace(hko_ctx* c, const float* rays, const float* max_distance, const float* early_distance,
               const uint32_t* exclude_instance, uint32_t n, void* hits)
{
#pragma omp parallel for schedule(static) HKO_THREADS(c)
    for (long long i = 0; i < (long long)n; ++i) {
        Counts k = {0, 0, 0};
#ifdef HKO_STATS
        hko_ray_steps = 0;
#endif
        Ray ray;
        ray.origin = ld3(rays + 6 * i);
        ray.direction = ld3(rays + 6 * i + 3);
        ray.inv_direction = inv3(ray.direction);
        Hit h = traverse_top(c, &k, &ray, max_distance ? max_distance[i] : HK_F32_MAX,
                             early_distance ? early_distance[i] : 0.0f,
                             exclude_instance ? exclude_instance[i] : DONT_EXCLUDE);
        uint32_t* o = (uint32_t*)hits + 5 * i;
        o[0] = hk_f2u(h.intersection.uv.x);
        o[1] = hk_f2u(h.intersection.uv.y);
        o[2] = hk_f2u(h.intersection.distance);
        o[3] = h.instance_index;
        o[4] = h.primitive_index;
#ifdef HKO_STATS
        if (hko_steps_out) hko_steps_out[i] = hko_ray_steps;
#endif
    }
}

/* hko_trace's closest-hit rays (no early exit, nothing excluded) with the ordered rule: 5 words per ray as hko_trace */
void hko_trace_ordered(hko_ctx* c, const float* rays, uint32_t n, void* hits)
{
#pragma omp parallel for schedule(static) HKO_THREADS(c)
    for (long long i = 0; i < (long long)n; ++i) {
        Ray ray;
        ray.origin = ld3(rays + 6 * i);
        ray.direction = ld3(rays + 6 * i + 3);
        ray.inv_direction = inv3(ray.direction);
        Hit h = closest_hit_ordered(c, &ray);
        uint32_t* o = (uint32_t*)hits + 5 * i;
        o[0] = hk_f2u(h.intersection.uv.x);
        o[1] = hk_f2u(h.intersection.uv.y);
        o[2] = hk_f2u(h.intersection.distance);
        o[3] = h.instance_index;
        o[4] = h.primitive_index;
    }
}

/* Primary rays of frame `in` (jittered as the G-buffer pass) walked two ways: the G-buffer's
 * ordered closest-hit walk and the reference-order traverse_top (light.wgsl:400-486, no early
 * exit).  out = 6 words per pixel: (instance, primitive, distance bits) of each walk. */
void hko_primary_hits(hko_ctx* c, const hk_frame_inputs* in, uint32_t* out)
{
    float jitter[2];
    frame_jitter(in, jitter);
#pragma omp parallel for schedule(dynamic, 4) HKO_THREADS(c)
    for (long long y = 0; y < (long long)c->S[1]; ++y)
        for (uint32_t x = 0; x < c->S[0]; ++x) {
            Ray ray;
            ray.origin = ld3(in->view.world_position);
            ray.direction = primary_direction(&in->view, ((float)x + 0.5f) - jitter[0],
                                              ((float)y + 0.5f) - jitter[1], c->S);
            ray.inv_direction = inv3(ray.direction);
            Counts k = {0, 0, 0};
            Hit a = closest_hit_ordered(c, &ray);
            Hit b = traverse_top(c, &k, &ray, HK_F32_MAX, 0.0f, DONT_EXCLUDE);
            uint32_t* o = out + 6 * ((size_t)y * c->S[0] + x);
            o[0] = a.instance_index; o[1] = a.primitive_index; o[2] = hk_f2u(a.intersection.distance);
            o[3] = b.instance_index; o[4] = b.primitive_index; o[5] = hk_f2u(b.intersection.distance);
        }
}

/* ---- KAT exports ---- */
float hko_intersects_aabb(const float* o, const float* inv, const float* mn, const float* mx)
{
    Ray r;
    r.origin = ld3(o);
    r.direction = V3(0, 0, 0);
    r.inv_direction = ld3(inv);
    Aabb a = {ld3(mn), ld3(mx)};
    return intersects_aabb(&r, a);
}
void hko_intersects_triangle(const float* o, const float* d, const float* v0, const float* v1, const float* v2_,
                             float* out)
{
    Ray r;
    r.origin = ld3(o);
    r.direction = ld3(d);
    r.inv_direction = inv3(r.direction);
    hk_primitive_vertex tri[3];
    memcpy(tri[0].position, v0, 12);
    memcpy(tri[1].position, v1, 12);
    memcpy(tri[2].position, v2_, 12);
    Intersection is = intersects_triangle(&r, tri);
    out[0] = is.uv.x;
    out[1] = is.uv.y;
    out[2] = is.distance;
}
/* fields: count, w, w_sum, w2_sum, lifetime, radiance[4], random[4], vis_pos[4], vis_n[3],
 *         vis_instance, sample_pos[4], sample_n[3]  (29 floats) -> unpacked in same order */
void hko_pack_reservoir_roundtrip(const float* f, hk_packed_reservoir* packed, float* u)
{
    Reservoir r;
    memset(&r, 0, sizeof(r));
    r.count = f[0]; r.w = f[1]; r.w_sum = f[2]; r.w2_sum = f[3]; r.lifetime = f[4];
    r.s.radiance = V4(f[5], f[6], f[7], f[8]);
    r.s.random = V4(f[9], f[10], f[11], f[12]);
    r.s.visible_position = V4(f[13], f[14], f[15], f[16]);
    r.s.visible_normal = V3(f[17], f[18], f[19]);
    r.s.visible_instance = (uint32_t)f[20];
    r.s.sample_position = V4(f[21], f[22], f[23], f[24]);
    r.s.sample_normal = V3(f[25], f[26], f[27]);
    pack_reservoir(&r, packed);
    Reservoir q = unpack_reservoir(packed);
    u[0] = q.count; u[1] = q.w; u[2] = q.w_sum; u[3] = q.w2_sum; u[4] = q.lifetime;
    u[5] = q.s.radiance.x; u[6] = q.s.radiance.y; u[7] = q.s.radiance.z; u[8] = q.s.radiance.w;
    u[9] = q.s.random.x; u[10] = q.s.random.y; u[11] = q.s.random.z; u[12] = q.s.random.w;
    u[13] = q.s.visible_position.x; u[14] = q.s.visible_position.y; u[15] = q.s.visible_position.z; u[16] = q.s.visible_position.w;
    u[17] = q.s.visible_normal.x; u[18] = q.s.visible_normal.y; u[19] = q.s.visible_normal.z;
    u[20] = (float)q.s.visible_instance;
    u[21] = q.s.sample_position.x; u[22] = q.s.sample_position.y; u[23] = q.s.sample_position.z; u[24] = q.s.sample_position.w;
    u[25] = q.s.sample_normal.x; u[26] = q.s.sample_normal.y; u[27] = q.s.sample_normal.z;
}
/* hk_unpack_unorm16_fast / hk_unpack_snorm8_fast (the device kernels' divide-free decodes) against
 * the divisions over their whole input domains: the number of codes whose bits differ */
uint32_t hko_unpack_fast_mismatches(void)
{
    uint32_t bad = 0;
    for (uint32_t v = 0; v < 65536u; ++v)
        if (hk_f2u(hk_unpack_unorm16_fast(v)) != hk_f2u(hk_unpack_unorm16(v))) ++bad;
    for (uint32_t v = 0; v < 256u; ++v) {
        if (hk_f2u(hk_unpack_snorm8_fast(v << 8, 1)) != hk_f2u(hk_unpack_snorm8(v << 8, 1))) ++bad;
        if (hk_f2u(hk_unorm8_fast(v)) != hk_f2u((float)v / 255.0f)) ++bad;
    }
    return bad;
}
/* The branchy forms hk_math.h's hk_exp2 / hk_log2 / hk_sincos had through round 4 (branch-free since round 5; the
 * Horner steps are HK_MAD in both forms): the
 * count of inputs, over every stride-th of the 2^32 bit patterns (stride 1: all of them, ~50 s on 8
 * cores; 0 and 0 when last run), where the current form's bits differ from these (NaN payloads included) */
static float exp2_branchy(float x)
{
    if (x != x) return x;
    if (x >= 128.0f) return hk_u2f(0x7F800000u);
    if (x < -151.0f) return 0.0f;
    float n = rintf(x);
    float f = x - n;
    float p = 1.5252733804059840e-05f;
    p = HK_MAD(p, f, 1.5403530393381608e-04f);
    p = HK_MAD(p, f, 1.3333558146428443e-03f);
    p = HK_MAD(p, f, 9.6181291076284772e-03f);
    p = HK_MAD(p, f, 5.5504108664821580e-02f);
    p = HK_MAD(p, f, 2.4022650695910071e-01f);
    p = HK_MAD(p, f, 6.9314718055994531e-01f);
    p = HK_MAD(p, f, 1.0f);
    int32_t ni = (int32_t)n;
    if (ni >= -126) return p * hk_u2f((uint32_t)(ni + 127) << 23);
    return (p * hk_u2f((uint32_t)(ni + 64 + 127) << 23)) * hk_u2f((uint32_t)(-64 + 127) << 23);
}
static float log2_branchy(float x)
{
    if (x != x) return x;
    if (x < 0.0f) return hk_u2f(0x7FC00000u);
    if (x == 0.0f) return hk_u2f(0xFF800000u);
    if (x == hk_u2f(0x7F800000u)) return x;
    int32_t e = 0;
    if (x < 1.17549435e-38f) { x = x * 8388608.0f; e = -23; }
    uint32_t u = hk_f2u(x);
    e += (int32_t)((u >> 23) & 0xFF) - 127;
    float m = hk_u2f((u & 0x007FFFFFu) | 0x3F800000u);
    if (m > 1.41421356f) { m = m * 0.5f; e += 1; }
    float s = (m - 1.0f) / (m + 1.0f);
    float s2 = s * s;
    float p = 0.11111111111111111f;
    p = HK_MAD(p, s2, 0.14285714285714285f);
    p = HK_MAD(p, s2, 0.2f);
    p = HK_MAD(p, s2, 0.33333333333333333f);
    p = HK_MAD(p, s2, 1.0f);
    float lm = (p * s) * 2.8853900817779268f;
    return (float)e + lm;
}
/* hk_exp_weight against hk_exp over every stride-th input x <= 0 (0 for NaN and where hk_exp is subnormal) */
unsigned long long hko_exp_weight_mismatches(uint32_t stride)
{
    unsigned long long bad = 0;
    const long long n = ((1ll << 32) + stride - 1) / stride;
#pragma omp parallel for schedule(static) reduction(+ : bad)
    for (long long k = 0; k < n; ++k) {
        const float x = hk_u2f((uint32_t)(k * (long long)stride));
        if (x > 0.0f) continue;  /* the weights' arguments: <= 0 or NaN */
        const float a = hk_exp_weight(x), b = hk_exp(x);
        /* equal bits, or 0 where hk_exp is below the normal range (flushed) */
        const int ok = x != x ? a == 0.0f : (hk_f2u(a) == hk_f2u(b) || (a == 0.0f && b < 1.17549435e-38f));
        if (!ok) ++bad;
    }
    return bad;
}
static void sincos_branchy(float x, float* s, float* c)
{
    if (x != x || hk_absf(x) == hk_u2f(0x7F800000u)) {
        *s = hk_u2f(0x7FC00000u);
        *c = *s;
        return;
    }
    float k = rintf(x * 0.63661977236758134f);
    float r = x - k * 1.5703125f;
    r = r - k * 4.837512969970703125e-4f;
    r = r - k * 7.54978995489188216e-8f;
    int32_t q = ((int32_t)k) & 3;
    float sk = hk_sin_kernel(r);
    float ck = hk_cos_kernel(r);
    if (q == 0) { *s = sk; *c = ck; }
    else if (q == 1) { *s = ck; *c = -sk; }
    else if (q == 2) { *s = -sk; *c = -ck; }
    else { *s = -ck; *c = sk; }
}
void hko_math_form_mismatches(uint32_t stride, unsigned long long* out)
{
    unsigned long long be = 0, bl = 0, bs = 0;
    const long long n = ((1ll << 32) + stride - 1) / stride;
#pragma omp parallel for schedule(static) reduction(+ : be, bl, bs)
    for (long long k = 0; k < n; ++k) {
        const float x = hk_u2f((uint32_t)(k * (long long)stride));
        if (hk_f2u(hk_exp2(x)) != hk_f2u(exp2_branchy(x))) ++be;
        if (hk_f2u(hk_log2(x)) != hk_f2u(log2_branchy(x))) ++bl;
        /* sincos: inputs below 2^31 pi/2 in magnitude, where the branchy form's (int32_t)k is defined */
        if (hk_absf(x) < 3.3e9f || x != x || hk_absf(x) == hk_u2f(0x7F800000u)) {
            float s0, c0, s1, c1;
            hk_sincos(x, &s0, &c0);
            sincos_branchy(x, &s1, &c1);
            if (hk_f2u(s0) != hk_f2u(s1) || hk_f2u(c0) != hk_f2u(c1)) ++bs;
        }
    }
    out[0] = be;
    out[1] = bl;
    out[2] = bs;
}
float hko_pow(float x, float y) { return hk_pow(x, y); }
float hko_pow_int(float x, int n) { return n == 2 ? hk_pow2(x) : (n == 5 ? hk_pow5(x) : hk_pow16(x)); }
float hko_exp2(float x) { return hk_exp2(x); }
float hko_log2(float x) { return hk_log2(x); }
float hko_sin(float x) { return hk_sin(x); }
float hko_cos(float x) { return hk_cos(x); }
uint32_t hko_f32_to_f16(float x) { return hk_f32_to_f16(x); }
void hko_f32_to_f16_array(const float* in, size_t n, uint16_t* out)
{
#pragma omp parallel for schedule(static)
    for (long i = 0; i < (long)n; ++i) out[i] = (uint16_t)hk_f32_to_f16(in[i]);
}
uint32_t hko_hash(uint32_t x) { return hk_hash(x); }
