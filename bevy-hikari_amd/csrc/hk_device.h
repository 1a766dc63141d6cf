// hk_device.h — device-side building blocks of the gfx950 integrator.
//
// Semantics follow src/shaders/light.wgsl / denoise.wgsl exactly (same operation order,
// same IEEE single rounding, transcendentals from include/hk_math.h, compiled with
// -ffp-contract=off) so that results are bit-identical to the CPU oracle.  The memory
// layout is MI355X-first instead of the reference's:
//   * reservoirs are stored as 4 SoA planes of 16-byte chunks (plane k = bytes 16k..16k+15
//     of every PackedReservoir), so a wave reads/writes 4 x 1 KiB fully coalesced;
//   * G-buffer / render targets are row-major planes (one per texture);
//   * scene records keep the std430 boundary layout (they are L2/MALL resident) and are
//     fetched with 16-byte vector loads.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hk_math.h"
#include "../../include/hk_types.h"
#include "../../include/hikari_amd.h"
#include "../../include/hk_texture.h"

namespace hk {

// ------------------------------------------------------------------ vectors
struct f2 {
    float x, y;
};
struct f3 {
    float x, y, z;
};
struct f4 {
    float x, y, z, w;
};
#define HKD __device__ __forceinline__
HKD f2 mk2(float x, float y) { return f2{x, y}; }
HKD f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
HKD f4 mk4(float x, float y, float z, float w) { return f4{x, y, z, w}; }
HKD f3 xyz(f4 a) { return mk3(a.x, a.y, a.z); }
HKD f3 operator+(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
HKD f3 operator-(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
HKD f3 operator*(f3 a, f3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
HKD f3 operator*(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
HKD f3 operator/(f3 a, float s) { return mk3(a.x / s, a.y / s, a.z / s); }
HKD float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
HKD float dot(f2 a, f2 b) { return a.x * b.x + a.y * b.y; }
HKD f3 cross(f3 a, f3 b) { return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
HKD float length(f3 a) { return sqrtf(dot(a, a)); }
HKD f3 vmin(f3 a, f3 b) { return mk3(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)); }
HKD f3 vmax(f3 a, f3 b) { return mk3(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)); }
HKD f3 mix(f3 a, f3 b, float t)
{
    float it = 1.0f - t;
    return mk3(a.x * it + b.x * t, a.y * it + b.y * t, a.z * it + b.z * t);
}
// 1 / d with the IEEE quotient's bits (checked for every f32 on the GPU by
// test_fast_reciprocal_is_exact): v_rcp_f32 (within 1 ulp) plus FMA residual corrections where
// neither d nor 1/d is near the denormal range; the IEEE divide sequence elsewhere (0, inf, NaN,
// |d| outside [2^-125, 2^125]).  Half the instructions of the divide.
// The corrected estimate is computed unconditionally and the divide only behind a branch that waves skip when
// none of their lanes needs it (one exec-mask region instead of an if / else pair).
HKD bool rcp_fast_ok(float d)
{
    const float a = fabsf(d);
    return a >= 0x1p-125f && a <= 0x1p125f;
}
HKD float rcp_fast(float d)
{
    const float r = __builtin_amdgcn_rcpf(d);
    return fmaf(fmaf(-d, r, 1.0f), r, r);
}
HKD float rcp_exact(float d)
{
    float r = rcp_fast(d);
    if (__builtin_expect(!rcp_fast_ok(d), 0)) r = 1.0f / d;
    return r;
}
// three reciprocals with one rare-path branch: where the fast result is exact it equals the IEEE quotient, so the
// branch may divide all three components
HKD f3 inv(f3 d)
{
    f3 r = mk3(rcp_fast(d.x), rcp_fast(d.y), rcp_fast(d.z));
    const bool ok = (int)rcp_fast_ok(d.x) & (int)rcp_fast_ok(d.y) & (int)rcp_fast_ok(d.z);
    if (__builtin_expect(!ok, 0)) r = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    return r;
}
HKD f3 normalize(f3 a) { return a * rcp_exact(sqrtf(dot(a, a))); }
HKD float sum4(f4 a) { return ((a.x + a.y) + a.z) + a.w; }
HKD float lum(f3 c) { return hk_luminance(c.x, c.y, c.z); }
HKD f3 ld3(const float* p) { return mk3(p[0], p[1], p[2]); }

HKD uint32_t f2u32(float x)
{
    if (!(x > 0.0f)) return 0u;
    if (x >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)x;
}
HKD int32_t f2i32(float x)
{
    if (x != x) return 0;
    if (x >= 2147483648.0f) return 0x7FFFFFFF;
    if (x <= -2147483648.0f) return (int32_t)0x80000000u;
    return (int32_t)x;
}
HKD uint32_t umod(uint32_t a, uint32_t b) { return b ? a % b : 0u; }

HKD f4 mat4_mul(const float* m, f4 v)
{
    f4 r;
    r.x = ((m[0] * v.x + m[4] * v.y) + m[8] * v.z) + m[12] * v.w;
    r.y = ((m[1] * v.x + m[5] * v.y) + m[9] * v.z) + m[13] * v.w;
    r.z = ((m[2] * v.x + m[6] * v.y) + m[10] * v.z) + m[14] * v.w;
    r.w = ((m[3] * v.x + m[7] * v.y) + m[11] * v.z) + m[15] * v.w;
    return r;
}

// ------------------------------------------------------------------ constants (light.wgsl:226-256)
constexpr float RAY_BIAS = 0.02f;
constexpr float DISTANCE_MAX = 65535.0f;
constexpr float MAX_VARIANCE = 10.0f;
constexpr uint32_t DONT_EXCLUDE = 0xFFFFFFFFu;
constexpr uint32_t DONT_SAMPLE_EMISSIVE = 0x80000000u;

// ------------------------------------------------------------------ kernel parameter blocks
// Scene arrays in Scene declaration order: vertices, primitives, asset_nodes, alias_table,
// instances, instance_nodes, materials, emissive_nodes, emissives, blas_wide, tlas_wide.
constexpr int SCENE_ARRAYS = 11;
struct Scene {
    const hk_vertex* vertices;
    const hk_primitive* primitives;
    const hk_node* asset_nodes;
    const hk_alias_entry* alias_table;
    const hk_instance* instances;
    const hk_node* instance_nodes;
    const hk_material* materials;
    const hk_node* emissive_nodes;
    const hk_emissive* emissives;
    uint32_t n_instances, n_instance_nodes, n_materials, n_emissive_nodes;
    // G-buffer traversal layout (k_build_wide): per subtree start, both child boxes + starts
    const float4* blas_wide;
    const float4* tlas_wide;
    // byte sizes of the arrays above, in declaration order (LDS staging, stage_scene)
    uint32_t bytes[SCENE_ARRAYS];
    // material textures (hk_texture_upload; n_textures = 0: the NO_TEXTURE pipeline)
    const hk_texture_desc* textures;
    const uint32_t* texels;
    const float* texture_lut;
    uint32_t n_textures;
};

// ------------------------------------------------------------------ LDS scene staging
// Small scenes (cornell: ~9.5 KB of scene arrays) are copied into LDS by every workgroup of a
// traversal kernel, so each dependent node / triangle / instance load of a walk is an LDS read
// (~50 cycles) instead of an L2 hit (~200).  A plan lists the arrays a kernel reads.
constexpr uint32_t LDS_SCENE_MAX = 32768;
enum : int { PLAN_LIGHT = 0, PLAN_GBUFFER = 1 };
__host__ __device__ constexpr bool plan_has(int plan, int k)
{
    return plan == PLAN_LIGHT ? k < 9 : (k == 0 || k == 1 || k == 4 || k == 9 || k == 10);
}
__host__ __device__ inline uint32_t stage_bytes(const uint32_t* bytes, int plan)
{
    uint32_t total = 0;
    for (int k = 0; k < 11; ++k)
        if (plan_has(plan, k)) total += (bytes[k] + 15u) & ~15u;
    return total;
}

// Frame-uniform + view + lights constants (view.rs:105-123, mesh_view_bindings.wgsl).
struct Frame {
    uint32_t number;
    uint32_t direct_validate_interval, emissive_validate_interval;
    uint32_t max_temporal_reuse_count, max_spatial_reuse_count;
    uint32_t indirect_bounces, temporal_reuse;
    float max_reservoir_lifetime, max_indirect_luminance, upscale_ratio;
    float cos_solar_angle;  // cos(frame.solar_angle), computed once per frame with hk_cos
    float clear_color[4];
    float view_world_position[3];
    float view_proj_z[3];   // view_proj[0].z, [1].z, [2].z (orthographic view vector)
    int orthographic;       // view.projection[3].w == 1.0
    float directional_color[3];
    float direction_to_light[3];
    float ambient_color[3];
    // sizes: S = deferred (physical), s = integrator; band = rows [row0, row0+rows) of the
    // global frame held in the local buffers (whole frame: 0, H)
    uint32_t S[2], s[2];
    int32_t S_row0, S_rows;  // deferred-plane band
    int32_t s_row0, s_rows;  // integrator-plane band
    // launch window (win_rows > 0): this launch covers only the local plane rows
    // [win_row0, win_row0 + win_rows) — a band's passes shrink their halo rows pass by pass
    // (hk_runtime.hip pass_window); 0: the whole plane
    int32_t win_row0, win_rows;
    // column window of a 2-D tile (hk_resize_tile; win_cols > 0): the launch covers only global columns
    // [win_col0, win_col0 + win_cols) of the full-width planes; 0: every column
    int32_t win_col0, win_cols;
    int32_t count_y0, count_y1;    // global integrator rows whose rays are counted (the band's own rows)
    int32_t count_x0, count_x1;    // ... and columns (a tile's own columns; the whole width otherwise)
    int32_t count_Sy0, count_Sy1;  // the same for the full-resolution G-buffer rows
    // interleaved stripes (stripe_n >= 2): the local planes hold the STRIPE_H-row stripes
    // k, k + n, k + 2n, ... of the frame (stripe_k = k) instead of one contiguous band; only for
    // passes without neighbour reads (no halo), see hk_resize_striped
    int32_t stripe_n, stripe_k;
    // host-evaluated constants (same IEEE expressions, so bit-identical to computing them here)
    float inv_S[2];                // 1 / S (jittered_uv texel size)
    float inv_s[2];                // RN(1 / s): div_by() reciprocals of the integrator size
    // spatial_reuse per-neighbour constants [EMISSIVE_LIT][i - 1] (light.wgsl:1568-1600):
    // py = sqrt(i / COUNT) * RANGE, tap_interval = max(1, py / 5), tap_count = u32(py / tap_interval)
    float sp_py[2][16];
    float sp_tap_interval[2][16];
    uint32_t sp_tap_count[2][16];
    float sp_tap_t[7][6];          // [tap_count][j] = j / (tap_count + 1), the depth-march mix weight
};

// Row-major planes of the deferred (G-buffer) textures, band-local.
struct GBuffer {
    float4* position;
    uint32_t* normal;
    float2* depth_gradient;
    float2* instance_material;
    float4* velocity_uv;
};

// Reservoir buffer of N 64-byte PackedReservoir records, as 16-byte chunks in SoA order: 4 planes of
// N chunks (chunk k of record i at k * N + i: a wave's 64 consecutive records are one 1-KiB coalesced
// load per chunk; the reference's AoS order measured slower).
struct ResBuf {
    uint4* base;
    uint32_t n;  // records
};
__host__ __device__ __forceinline__ uint32_t res_chunk(const ResBuf& b, uint32_t k, uint32_t i) { return k * b.n + i; }

struct Counters {
    unsigned long long* top;
    unsigned long long* emitter;
    unsigned long long* primary;
    // persistent-wave tile claims (k_indirect_persist): PERSIST_KINDS blocks of PERSIST_LINES 128-B lines,
    // zero between launches
    unsigned long long* persist;
};
constexpr uint32_t PERSIST_SHARDS = 8;               // claim counters per block (one per XCD of the round-robin)
constexpr uint32_t PERSIST_LINE = 16;                // u64 per 128-B line
constexpr uint32_t PERSIST_LINES = PERSIST_SHARDS + 1;  // + the exit counter
constexpr uint32_t PERSIST_KINDS = 4;

template <int PLAN>
HKD Scene stage_scene(const Scene& g, uint32_t* lds)
{
    const uint32_t* src[SCENE_ARRAYS] = {
        (const uint32_t*)g.vertices,       (const uint32_t*)g.primitives, (const uint32_t*)g.asset_nodes,
        (const uint32_t*)g.alias_table,    (const uint32_t*)g.instances,  (const uint32_t*)g.instance_nodes,
        (const uint32_t*)g.materials,      (const uint32_t*)g.emissive_nodes, (const uint32_t*)g.emissives,
        (const uint32_t*)g.blas_wide,      (const uint32_t*)g.tlas_wide};
    uint32_t* dst[SCENE_ARRAYS];
    uint4* const lds4 = reinterpret_cast<uint4*>(lds);  // (hk_lds_scene is 16-byte aligned)
    // The plan's arrays as one list of 16-byte chunks (array k at chunk off4[k], its last chunk rounded up: the
    // bytes read past an array's end lie in the same 16-byte block of its own allocation, and no reader looks at
    // them in LDS), copied four chunks per thread per iteration with the four loads issued before any store
    // (cornell: 12 KiB, ~770 chunks, one iteration).
    uint32_t off4[SCENE_ARRAYS];
    uint32_t total = 0;
#pragma unroll
    for (int k = 0; k < SCENE_ARRAYS; ++k) {
        off4[k] = total;
        dst[k] = reinterpret_cast<uint32_t*>(lds4 + total);
        if (plan_has(PLAN, k)) total += (g.bytes[k] + 15u) >> 4;
    }
    if (total > 0u) {
        for (uint32_t c0 = threadIdx.x; c0 < total; c0 += 4u * blockDim.x) {
            uint4 v[4];
            uint32_t cs[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t c = min(c0 + (uint32_t)j * blockDim.x, total - 1u);
                const uint4* p = nullptr;
#pragma unroll
                for (int k = 0; k < SCENE_ARRAYS; ++k)
                    if (plan_has(PLAN, k) && c >= off4[k]) p = reinterpret_cast<const uint4*>(src[k]) + (c - off4[k]);
                v[j] = *p;
                cs[j] = c;
            }
            // (unconditional: a clamped chunk is the last one, stored again with the same bits)
#pragma unroll
            for (int j = 0; j < 4; ++j) lds4[cs[j]] = v[j];
        }
    }
    __syncthreads();
    Scene s = g;
    if (plan_has(PLAN, 0)) s.vertices = (const hk_vertex*)dst[0];
    if (plan_has(PLAN, 1)) s.primitives = (const hk_primitive*)dst[1];
    if (plan_has(PLAN, 2)) s.asset_nodes = (const hk_node*)dst[2];
    if (plan_has(PLAN, 3)) s.alias_table = (const hk_alias_entry*)dst[3];
    if (plan_has(PLAN, 4)) s.instances = (const hk_instance*)dst[4];
    if (plan_has(PLAN, 5)) s.instance_nodes = (const hk_node*)dst[5];
    if (plan_has(PLAN, 6)) s.materials = (const hk_material*)dst[6];
    if (plan_has(PLAN, 7)) s.emissive_nodes = (const hk_node*)dst[7];
    if (plan_has(PLAN, 8)) s.emissives = (const hk_emissive*)dst[8];
    if (plan_has(PLAN, 9)) s.blas_wide = (const float4*)dst[9];
    if (plan_has(PLAN, 10)) s.tlas_wide = (const float4*)dst[10];
    return s;
}

// ------------------------------------------------------------------ division by a frame size
// x / d for a per-frame constant divisor d (an image dimension) with r = RN(1/d) from the host:
// q0 = x r, one correction brings q1 within 1 ulp of x / d, a second one (Markstein: r is the
// correctly rounded reciprocal, q1 is within 1 ulp) rounds correctly — the same bits as the IEEE
// divide for every x with a normal quotient (checked exhaustively over 2^31 patterns per divisor
// by test_fast_division_by_frame_size_is_exact).  Signed zero kept.
HKD float div_by(float x, float d, float r)
{
    const float q0 = x * r;
    const float e0 = fmaf(-q0, d, x);
    const float q1 = fmaf(e0, r, q0);
    const float e1 = fmaf(-q1, d, x);
    const float q2 = fmaf(e1, r, q1);
    return x == 0.0f ? x * r : q2;
}

// ------------------------------------------------------------------ f16 (hardware)
// v_cvt_f16_f32 rounds to nearest-even with f16 denormals kept (default MODE), which is the
// IEEE conversion hk_f32_to_f16 restates in software for the oracle; v_cvt_f32_f16 is exact.
// Both directions are inline asm so the optimiser cannot fold them into neighbouring f32
// arithmetic (f16 narrowing of fpext'd operands, v_fma_mix* selection): every value is rounded
// to f32 first and then to f16, as the reference's f32 shader math + pack2x16float does.
HKD uint32_t f16_bits(float f) { return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)f); }
HKD float f16_val(uint32_t h)
{
    float r;
    asm("v_cvt_f32_f16 %0, %1" : "=v"(r) : "v"(h));
    return r;
}
// asm as well: a plain fptrunc(fmul(a, b)) is selected as v_fma_mixlo_f16, which rounds the
// exact product once to f16 instead of to f32 then f16 (the reference's two roundings).
HKD uint32_t pack2x16float(float a, float b)
{
    uint32_t r;
    asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
HKD float unpack_lo16float(uint32_t v) { return f16_val(v); }
HKD float unpack_hi16float(uint32_t v)
{
    float r;
    asm("v_cvt_f32_f16_sdwa %0, %1 src0_sel:WORD_1" : "=v"(r) : "v"(v));
    return r;
}

// ------------------------------------------------------------------ texel access
HKD void store_rgba16f(uint2* tex, int32_t idx, f4 c)
{
    tex[idx] = make_uint2(pack2x16float(c.x, c.y), pack2x16float(c.z, c.w));
}
HKD f4 load_rgba16f(const uint2* tex, int32_t idx)
{
    uint2 v = tex[idx];
    return mk4(unpack_lo16float(v.x), unpack_hi16float(v.x), unpack_lo16float(v.y), unpack_hi16float(v.y));
}

// Deferred-texture addressing: frame-OOB -> 0 (textureLoad robustness); in-frame rows outside
// the band are clamped into it (those values only feed discarded halo pixels).
// the launch's columns [win_x0, win_x1(width)) (the column window of a tile, or the whole plane width)
HKD int32_t win_x0(const Frame& F) { return F.win_cols > 0 ? F.win_col0 : 0; }
HKD int32_t win_x1(const Frame& F, uint32_t width) { return F.win_cols > 0 ? F.win_col0 + F.win_cols : (int32_t)width; }
// the pixel's rays count towards this context's counters (its own rows and columns: halo pixels are another
// context's)
HKD bool counted(const Frame& F, int32_t x, int32_t y)
{
    return y >= F.count_y0 && y < F.count_y1 && x >= F.count_x0 && x < F.count_x1;
}
HKD bool in_frame(int32_t x, int32_t y, const uint32_t* size)
{
    return x >= 0 && y >= 0 && (uint32_t)x < size[0] && (uint32_t)y < size[1];
}
constexpr int32_t STRIPE_H = 8;  // rows per interleaved stripe (one wave tile high)
// local plane row of global row y: band offset, or the stripe map; rows this context does not
// hold clamp into the local plane (they only feed discarded halo pixels / motion edges)
HKD int32_t local_row(const Frame& F, int32_t y, int32_t row0)
{
    if (F.stripe_n >= 2) {
        const int32_t t = y / STRIPE_H;
        return (t / F.stripe_n) * STRIPE_H + (y - t * STRIPE_H);
    }
    return y - row0;
}
// global row of local plane row ly
HKD int32_t global_row(const Frame& F, int32_t ly, int32_t row0)
{
    if (F.stripe_n >= 2) {
        const int32_t t = ly / STRIPE_H;
        return (t * F.stripe_n + F.stripe_k) * STRIPE_H + (ly - t * STRIPE_H);
    }
    return row0 + ly;
}
HKD int32_t band_index(const Frame& F, int32_t x, int32_t y, uint32_t width, int32_t row0, int32_t rows)
{
    int32_t ly = local_row(F, y, row0);
    ly = ly < 0 ? 0 : (ly >= rows ? rows - 1 : ly);
    return x + (int32_t)width * ly;
}
HKD f4 load_position(const Frame& F, const GBuffer& G, int32_t x, int32_t y)
{
    if (!in_frame(x, y, F.S)) return mk4(0, 0, 0, 0);
    float4 p = G.position[band_index(F, x, y, F.S[0], F.S_row0, F.S_rows)];
    return mk4(p.x, p.y, p.z, p.w);
}
HKD float load_depth(const Frame& F, const GBuffer& G, int32_t x, int32_t y)
{
    if (!in_frame(x, y, F.S)) return 0.0f;
    return G.position[band_index(F, x, y, F.S[0], F.S_row0, F.S_rows)].w;
}
HKD f3 load_normal(const Frame& F, const GBuffer& G, int32_t x, int32_t y)
{
    if (!in_frame(x, y, F.S)) return mk3(0, 0, 0);
    uint32_t n = G.normal[band_index(F, x, y, F.S[0], F.S_row0, F.S_rows)];
    return mk3(hk_unpack_snorm8_fast(n, 0), hk_unpack_snorm8_fast(n, 1), hk_unpack_snorm8_fast(n, 2));
}
HKD f2 load_instance_material(const Frame& F, const GBuffer& G, int32_t x, int32_t y)
{
    if (!in_frame(x, y, F.S)) return mk2(0, 0);
    float2 v = G.instance_material[band_index(F, x, y, F.S[0], F.S_row0, F.S_rows)];
    return mk2(v.x, v.y);
}
HKD f4 load_velocity_uv(const Frame& F, const GBuffer& G, int32_t x, int32_t y)
{
    if (!in_frame(x, y, F.S)) return mk4(0, 0, 0, 0);
    float4 v = G.velocity_uv[band_index(F, x, y, F.S[0], F.S_row0, F.S_rows)];
    return mk4(v.x, v.y, v.z, v.w);
}
HKD f2 load_depth_gradient(const Frame& F, const GBuffer& G, int32_t x, int32_t y)
{
    if (!in_frame(x, y, F.S)) return mk2(0, 0);
    float2 v = G.depth_gradient[band_index(F, x, y, F.S[0], F.S_row0, F.S_rows)];
    return mk2(v.x, v.y);
}
// integrator-plane (s) index of an in-frame pixel
HKD int32_t s_index(const Frame& F, int32_t x, int32_t y) { return band_index(F, x, y, F.s[0], F.s_row0, F.s_rows); }
// s_index of the passes that read neighbours (spatial reuse, the denoiser), which never run on interleaved stripes
// (hk_render_frame / hk_denoise reject them): the row-band map alone
HKD int32_t rb_index(const Frame& F, int32_t x, int32_t y)
{
    int32_t ly = y - F.s_row0;
    ly = ly < 0 ? 0 : (ly >= F.s_rows ? F.s_rows - 1 : ly);
    return x + (int32_t)F.s[0] * ly;
}

HKD f2 coords_to_uv(int32_t x, int32_t y, const uint32_t* size)
{
    return mk2(((float)x + 0.5f) / (float)size[0], ((float)y + 0.5f) / (float)size[1]);
}
// coords_to_uv on the integrator grid with div_by (same bits as the IEEE divide)
HKD f2 coords_to_uv_s(const Frame& F, int32_t x, int32_t y)
{
    return mk2(div_by((float)x + 0.5f, (float)F.s[0], F.inv_s[0]), div_by((float)y + 0.5f, (float)F.s[1], F.inv_s[1]));
}
// light.wgsl:1007-1017 (jitter 0.25) / denoise.wgsl:37-41 (jitter 0.5)
HKD f2 jittered_uv(const Frame& F, f2 uv, float amount)
{
    float tx = F.inv_S[0], ty = F.inv_S[1];  // 1 / S, evaluated on the host
    float ratio = F.upscale_ratio - 1.0f;
    float j = (F.number & 1u) == 0u ? -amount : amount;
    return mk2(uv.x + (j * tx) * ratio, uv.y + (j * ty) * ratio);
}
HKD void jittered_coords(const Frame& F, f2 uv, int32_t& x, int32_t& y)
{
    f2 d = jittered_uv(F, uv, 0.25f);
    x = f2i32(d.x * (float)F.S[0]);
    y = f2i32(d.y * (float)F.S[1]);
}
HKD void nearest_texel(f2 uv, const uint32_t* size, int32_t& x, int32_t& y)
{
    int32_t ix = f2i32(floorf(uv.x * (float)size[0]));
    int32_t iy = f2i32(floorf(uv.y * (float)size[1]));
    x = ix < 0 ? 0 : (ix > (int32_t)size[0] - 1 ? (int32_t)size[0] - 1 : ix);
    y = iy < 0 ? 0 : (iy > (int32_t)size[1] - 1 ? (int32_t)size[1] - 1 : iy);
}

// ------------------------------------------------------------------ reservoirs (light.wgsl:45-223)
struct Sample {
    f4 radiance;
    f4 random;
    f4 visible_position;
    f3 visible_normal;
    uint32_t visible_instance;
    f4 sample_position;
    f3 sample_normal;
};
struct Reservoir {
    Sample s;
    float count, lifetime, w, w_sum, w2_sum;
};
HKD Sample zero_sample()
{
    Sample s;
    s.radiance = s.random = s.visible_position = s.sample_position = mk4(0, 0, 0, 0);
    s.visible_normal = s.sample_normal = mk3(0, 0, 0);
    s.visible_instance = 0u;
    return s;
}
HKD Reservoir zero_reservoir()
{
    Reservoir r;
    r.s = zero_sample();
    r.count = r.lifetime = r.w = r.w_sum = r.w2_sum = 0.0f;
    return r;
}

HKD Reservoir unpack_reservoir(uint4 c0, uint4 c1, uint4 c2, uint4 c3)
{
    Reservoir r;
    r.count = unpack_lo16float(c3.z);
    r.w = unpack_hi16float(c3.z);
    r.w_sum = unpack_lo16float(c3.w);
    r.w2_sum = unpack_hi16float(c3.w);
    r.s.radiance = mk4(unpack_lo16float(c0.x), unpack_hi16float(c0.x), unpack_lo16float(c0.y),
                       unpack_hi16float(c0.y));
    r.s.random = mk4(hk_unpack_unorm16_fast(c0.z), hk_unpack_unorm16_fast(c0.z >> 16), hk_unpack_unorm16_fast(c0.w),
                     hk_unpack_unorm16_fast(c0.w >> 16));
    r.s.visible_position = mk4(__uint_as_float(c1.x), __uint_as_float(c1.y), __uint_as_float(c1.z), __uint_as_float(c1.w));
    uint32_t vn = c3.x;
    r.s.visible_normal = normalize(mk3(hk_unpack_snorm8_fast(vn, 0), hk_unpack_snorm8_fast(vn, 1), hk_unpack_snorm8_fast(vn, 2)));
    r.lifetime = 127.0f * (1.0f + hk_unpack_snorm8_fast(vn, 3));
    uint32_t sn = c3.y;
    r.s.sample_position = mk4(__uint_as_float(c2.x), __uint_as_float(c2.y), __uint_as_float(c2.z), hk_unpack_snorm8_fast(sn, 3));
    r.s.sample_normal = normalize(mk3(hk_unpack_snorm8_fast(sn, 0), hk_unpack_snorm8_fast(sn, 1), hk_unpack_snorm8_fast(sn, 2)));
    r.s.visible_instance = f2u32(__uint_as_float(c2.w));
    return r;
}
HKD Reservoir load_res(const ResBuf& b, int32_t i)
{
    const uint4* p = b.base;
    const uint32_t u = (uint32_t)i;
    return unpack_reservoir(p[res_chunk(b, 0, u)], p[res_chunk(b, 1, u)], p[res_chunk(b, 2, u)], p[res_chunk(b, 3, u)]);
}
HKD void pack_res(const Reservoir& r, uint4& c0, uint4& c1, uint4& c2, uint4& c3)
{
    c3.z = pack2x16float(r.count, r.w);
    c3.w = pack2x16float(r.w_sum, r.w2_sum);
    c0.x = pack2x16float(r.s.radiance.x, r.s.radiance.y);
    c0.y = pack2x16float(r.s.radiance.z, r.s.radiance.w);
    c0.z = hk_pack2x16unorm(r.s.random.x, r.s.random.y);
    c0.w = hk_pack2x16unorm(r.s.random.z, r.s.random.w);
    c1 = make_uint4(__float_as_uint(r.s.visible_position.x), __float_as_uint(r.s.visible_position.y),
                    __float_as_uint(r.s.visible_position.z), __float_as_uint(r.s.visible_position.w));
    c2 = make_uint4(__float_as_uint(r.s.sample_position.x), __float_as_uint(r.s.sample_position.y),
                    __float_as_uint(r.s.sample_position.z), __float_as_uint((float)r.s.visible_instance));
    c3.x = hk_pack4x8snorm(r.s.visible_normal.x, r.s.visible_normal.y, r.s.visible_normal.z, div_by(r.lifetime, 127.0f, HK_INV_127) - 1.0f);  // div_by: exact for 127 (test_fast_division_by_frame_size_is_exact)
    c3.y = hk_pack4x8snorm(r.s.sample_normal.x, r.s.sample_normal.y, r.s.sample_normal.z, r.s.sample_position.w);
}
HKD void store_res(const ResBuf& b, int32_t i, const Reservoir& r)
{
    uint4 c0, c1, c2, c3;
    pack_res(r, c0, c1, c2, c3);
    uint4* p = b.base;
    const uint32_t u = (uint32_t)i;
    p[res_chunk(b, 0, u)] = c0;
    p[res_chunk(b, 1, u)] = c1;
    p[res_chunk(b, 2, u)] = c2;
    p[res_chunk(b, 3, u)] = c3;
}

// Spatial view planes (ChannelArgs::view): spatial reuse reads a neighbour's record for its rejection
// tests and its merge only (light.wgsl:1598-1642), so the temporal pass also stores, from the same packed
// words it writes into `cur`:
//   plane 0: sample_position xyz (c2.xyz) | the visible normal's snorm8 bytes (c3.x bits 0-23), bit 24:
//            q.s.sample_position.w > 0.5 (the jacobian's condition, c3.y byte 3), bit 25: !(q.count < eps)
//   plane 1: radiance (c0.xy, f16 x 4) | (count, w) (c3.z) | fract(dot(random, 1)) of the packed random
//            (c0.zw decoded), the value update_reservoir compares (light.wgsl:155)
//   plane 2: visible_position xyz (c1.xyz) | the sample normal's snorm8 word (c3.y)
// Every field is the bits, or the exact value, spatial reuse would derive from the packed record, so the
// results are unchanged; a tested neighbour costs one 16-B gather instead of two and a merged one two or
// three instead of four.
constexpr uint32_t VIEW_HIT = 1u << 24, VIEW_COUNT = 1u << 25;
// (the three chunks of a pixel in one 64-byte line instead of three planes measured slower: DESIGN §4)
constexpr uint32_t VIEW_PLANES = 3u;  // uint4 chunks allocated per pixel
HKD uint32_t view_at(uint32_t view_n, uint32_t plane, uint32_t u) { return plane * view_n + u; }
HKD void store_res_view(const ResBuf& b, uint4* view, uint32_t view_n, int32_t i, const Reservoir& r)
{
    uint4 c0, c1, c2, c3;
    pack_res(r, c0, c1, c2, c3);
    uint4* p = b.base;
    const uint32_t u = (uint32_t)i;
    p[res_chunk(b, 0, u)] = c0;
    p[res_chunk(b, 1, u)] = c1;
    p[res_chunk(b, 2, u)] = c2;
    p[res_chunk(b, 3, u)] = c3;
    if (!view) return;
    const uint32_t flags = (hk_unpack_snorm8_fast(c3.y, 3) > 0.5f ? VIEW_HIT : 0u) |
                           (!(unpack_lo16float(c3.z) < HK_F32_EPSILON) ? VIEW_COUNT : 0u);
    const float rand = hk_fract(((hk_unpack_unorm16_fast(c0.z) + hk_unpack_unorm16_fast(c0.z >> 16)) +
                                 hk_unpack_unorm16_fast(c0.w)) + hk_unpack_unorm16_fast(c0.w >> 16));
    view[view_at(view_n, 0u, u)] = make_uint4(c2.x, c2.y, c2.z, (c3.x & 0x00FFFFFFu) | flags);
    // spatial reuse reads plane 1 only behind VIEW_COUNT and plane 2 only behind VIEW_HIT (plane 0 of the
    // same frame), so a chunk whose flag is clear is never read and its store is skipped
    if (flags & VIEW_COUNT) view[view_at(view_n, 1u, u)] = make_uint4(c0.x, c0.y, c3.z, __float_as_uint(rand));
    if (flags & VIEW_HIT) view[view_at(view_n, 2u, u)] = make_uint4(c1.x, c1.y, c1.z, c3.y);
}

HKD void set_reservoir(Reservoir& r, const Sample& s, float w_new)
{
    r.count = 1.0f;
    r.lifetime = 0.0f;
    r.w_sum = w_new;
    r.w2_sum = w_new * w_new;
    r.s = s;
}
HKD void update_reservoir(Reservoir& r, const Sample& s, float w_new)
{
    r.w_sum += w_new;
    r.w2_sum += w_new * w_new;
    r.count = r.count + 1.0f;
    float rand = hk_fract(sum4(s.random));
    if (rand < w_new / r.w_sum) r.s = s;
}
HKD void merge_reservoir(Reservoir& r, const Reservoir& other, float p)
{
    float count = r.count;
    update_reservoir(r, other.s, (p * other.w) * other.count);
    r.count = count + other.count;
}
HKD bool uv_inside_open(f2 uv) { return fabsf(uv.x - 0.5f) < 0.5f && fabsf(uv.y - 0.5f) < 0.5f; }
HKD bool uv_inside_closed(f2 uv) { return fabsf(uv.x - 0.5f) <= 0.5f && fabsf(uv.y - 0.5f) <= 0.5f; }

HKD Reservoir load_previous(const Frame& F, const ResBuf& b, f2 uv)
{
    if (uv_inside_open(uv)) {
        int32_t x = f2i32(uv.x * (float)F.s[0]);
        int32_t y = f2i32(uv.y * (float)F.s[1]);
        return load_res(b, s_index(F, x, y));
    }
    return zero_reservoir();
}

HKD bool check_previous_reservoir(Reservoir& r, const Sample& s)
{
    float depth_ratio = r.s.visible_position.w / s.visible_position.w;
    depth_ratio = depth_ratio < 1.0f ? 1.0f / depth_ratio : depth_ratio;
    bool depth_miss = depth_ratio > 1.05f * (1.0f + 0.5f * s.random.x);
    bool instance_miss = r.s.visible_instance != s.visible_instance;
    bool normal_miss = dot(s.visible_normal, r.s.visible_normal) < 0.9f;
    if (depth_miss || normal_miss || instance_miss) {
        r = zero_reservoir();
        return false;
    }
    return true;
}
// load_previous + check_previous_reservoir read in two steps (the light passes' register peaks): the record's
// index and the words the check reads — chunk 3 (count, weights, visible normal, lifetime), the depth word of
// chunk 1 and the instance word of chunk 2 — first; the whole record later, with previous_record(), where the pass
// needs its sample.  The passes do not write their previous temporal buffer, so the second read returns the same
// bits: previous_record(previous_head(F, b, uv, s)) == the reservoir check_previous_reservoir leaves in
// load_previous(F, b, uv), and `kept` is its result.
struct PrevHead {
    int32_t index;  // load_previous's record; -1: outside the frame (the zero reservoir, which the check rejects)
    bool kept;      // check_previous_reservoir passed (otherwise the reservoir is the zero reservoir)
    float count, lifetime, w_sum, w2_sum;
};
HKD PrevHead previous_head(const Frame& F, const ResBuf& b, f2 uv, const Sample& s)
{
    PrevHead h;
    h.index = -1;
    h.kept = false;
    h.count = h.lifetime = h.w_sum = h.w2_sum = 0.0f;
    if (uv_inside_open(uv)) h.index = s_index(F, f2i32(uv.x * (float)F.s[0]), f2i32(uv.y * (float)F.s[1]));
    if (h.index >= 0) {
        const uint32_t u = (uint32_t)h.index;
        const uint4 c3 = b.base[res_chunk(b, 3u, u)];
        const float depth = __uint_as_float(b.base[res_chunk(b, 1u, u)].w);
        const uint32_t instance = f2u32(__uint_as_float(b.base[res_chunk(b, 2u, u)].w));
        const f3 normal = normalize(mk3(hk_unpack_snorm8_fast(c3.x, 0), hk_unpack_snorm8_fast(c3.x, 1), hk_unpack_snorm8_fast(c3.x, 2)));
        // check_previous_reservoir on the decoded fields
        float depth_ratio = depth / s.visible_position.w;
        depth_ratio = depth_ratio < 1.0f ? 1.0f / depth_ratio : depth_ratio;
        const bool depth_miss = depth_ratio > 1.05f * (1.0f + 0.5f * s.random.x);
        const bool instance_miss = instance != s.visible_instance;
        const bool normal_miss = dot(s.visible_normal, normal) < 0.9f;
        h.kept = !(depth_miss || normal_miss || instance_miss);
        if (h.kept) {
            h.count = unpack_lo16float(c3.z);
            h.w_sum = unpack_lo16float(c3.w);
            h.w2_sum = unpack_hi16float(c3.w);
            h.lifetime = 127.0f * (1.0f + hk_unpack_snorm8_fast(c3.x, 3));
        }
    }
    return h;
}
HKD Reservoir previous_record(const ResBuf& b, const PrevHead& h)
{
    return h.kept ? load_res(b, h.index) : zero_reservoir();
}
// the scatter of a rejected previous reservoir (light.wgsl:1092-1095, 1453-1457): the zero reservoir, at the
// previous uv's pixel when that uv is inside the frame
HKD void scatter_rejected(const Frame& F, const ResBuf& prev_spatial, f2 uv, const PrevHead& h)
{
    if (!h.kept && uv_inside_closed(uv))
        store_res(prev_spatial, s_index(F, f2i32(uv.x * (float)F.s[0]), f2i32(uv.y * (float)F.s[1])), zero_reservoir());
}
HKD void temporal_restir(Reservoir& r, const Sample& s, float w_new, uint32_t max_sample_count)
{
    update_reservoir(r, s, w_new);
    float m = (float)max_sample_count;
    if (r.count > m) {
        r.w_sum *= m / r.count;
        r.w2_sum *= m / r.count;
        r.count = m;
    }
}
HKD float variance_of(const Reservoir& r)
{
    float variance = r.w2_sum / r.count - hk_pow2(r.w_sum / r.count);
    variance = r.count < 1.0f ? variance : variance / r.count;
    return fminf(variance, MAX_VARIANCE);
}

// ------------------------------------------------------------------ tracing (light.wgsl:259-533)
struct Ray {
    f3 origin, direction, inv_direction;
};
struct Hit {
    f2 uv;
    float distance;
    uint32_t instance_index, primitive_index;
};
struct HitInfo {
    f4 position;
    f3 normal;
    f2 uv;
    uint32_t instance_index, material_index;
};
struct LightCandidate {
    f3 direction;
    float max_distance, min_distance;
    uint32_t emissive_instance;
    float p;
};
struct Surface {
    f4 base_color, emissive;
    float reflectance, metallic, roughness, occlusion;
};

HKD float intersects_aabb(const Ray& ray, f3 mn, f3 mx)
{
    f3 t1 = (mn - ray.origin) * ray.inv_direction;
    f3 t2 = (mx - ray.origin) * ray.inv_direction;
    float t_min = fminf(t1.x, t2.x);
    float t_max = fmaxf(t1.x, t2.x);
    t_min = fmaxf(t_min, fminf(t1.y, t2.y));
    t_max = fminf(t_max, fmaxf(t1.y, t2.y));
    t_min = fmaxf(t_min, fminf(t1.z, t2.z));
    t_max = fminf(t_max, fmaxf(t1.z, t2.z));
    return (t_max >= t_min && t_max >= 0.0f) ? t_min : HK_F32_MAX;
}

// Möller–Trumbore as light.wgsl:364-398; returns distance (F32_MAX on miss) and uv.
// Written without early returns: every value is computed and the result selected at the end (the values of the
// reference's early exits are the selects' other arms), so a wave whose lanes leave at different tests runs one
// straight sequence instead of three exec-mask regions.
HKD float intersects_triangle(const Ray& ray, f3 p0, f3 p1, f3 p2, f2& uv_out)
{
    f3 ab = p1 - p0;
    f3 ac = p2 - p0;
    f3 u_vec = cross(ray.direction, ac);
    float det = dot(ab, u_vec);
    const bool parallel = fabsf(det) < HK_F32_EPSILON;
    float inv_det = rcp_exact(det);
    f3 ao = ray.origin - p0;
    float u = dot(ao, u_vec) * inv_det;
    const bool u_miss = u < 0.0f || u > 1.0f;
    f3 v_vec = cross(ao, ab);
    float v = dot(ray.direction, v_vec) * inv_det;
    float distance = dot(ac, v_vec) * inv_det;
    uv_out = parallel ? mk2(0.0f, 0.0f) : mk2(u, u_miss ? 0.0f : v);
    if (parallel || u_miss || v < 0.0f || u + v > 1.0f) return HK_F32_MAX;
    return distance > HK_F32_EPSILON ? distance : HK_F32_MAX;
}

HKD void load_node(const hk_node* nodes, uint32_t i, f3& mn, uint32_t& entry, f3& mx, uint32_t& exit)
{
    const float4* p = reinterpret_cast<const float4*>(nodes + i);
    float4 a = p[0], b = p[1];
    mn = mk3(a.x, a.y, a.z);
    entry = __float_as_uint(a.w);
    mx = mk3(b.x, b.y, b.z);
    exit = __float_as_uint(b.w);
}
HKD void load_triangle(const hk_primitive* prims, uint32_t i, f3& a, f3& b, f3& c)
{
    const float4* p = reinterpret_cast<const float4*>(prims + i);
    float4 x = p[0], y = p[1], z = p[2];
    a = mk3(x.x, x.y, x.z);
    b = mk3(y.x, y.y, y.z);
    c = mk3(z.x, z.y, z.z);
}


// One iteration of the skip-pointer walk covering up to STEPS consecutive visits: node p and,
// while the visited node is an inner node whose box passes, its subtree start (the next node of
// the flattened array, bvh flatten).  All STEPS nodes are loaded and tested up front with the
// same hit distance (no leaf work happens between such visits).  Returns the node the walk visits
// next; `leaf_pass`/`leaf_entry` report the leaf reached in this iteration, if its box passed.
constexpr int WALK_STEPS = 2;  // visits per walk iteration (3 and 4 measured slower)
template <int STEPS>
HKD uint32_t walk_step(const hk_node* nodes, uint32_t index, uint32_t count, const Ray& tr, float distance,
                       bool& leaf_pass, uint32_t& leaf_entry)
{
    uint32_t entry[STEPS], exit[STEPS];
    f3 mn[STEPS], mx[STEPS];
    bool pass[STEPS];
#pragma unroll
    for (int k = 0; k < STEPS; ++k) {
        const uint32_t i = index + (uint32_t)k < count ? index + (uint32_t)k : index;  // in range; used only when visited
        load_node(nodes, i, mn[k], entry[k], mx[k], exit[k]);
    }
#pragma unroll
    for (int k = 0; k < STEPS; ++k) pass[k] = intersects_aabb(tr, mn[k], mx[k]) < distance;
    leaf_pass = false;
    leaf_entry = entry[0];
    uint32_t next = 0u;
    bool open = true;  // visits so far were passing inner nodes
#pragma unroll
    for (int k = 0; k < STEPS; ++k) {
        if (open) {
            if (entry[k] >= HK_BVH_LEAF_FLAG) {
                leaf_pass = pass[k];
                leaf_entry = entry[k];
                next = exit[k];
                open = false;
            } else if (!pass[k]) {
                next = exit[k];
                open = false;
            } else {
                next = entry[k];  // == index + k + 1, visited in this iteration if k + 1 < STEPS
            }
        }
    }
    return next;
}

// light.wgsl:400-440 — stackless skip-pointer BLAS walk (reference visit order).
HKD bool traverse_bottom(const Scene& sc, Hit& hit, const Ray& ray, uint32_t node_offset, uint32_t node_count,
                         uint32_t prim_offset, float early_distance)
{
    bool intersected = false;
    uint32_t index = 0u;
    // up to WALK_STEPS visits per iteration (walk_step), as in traverse_top below
    const hk_node* nodes = sc.asset_nodes + node_offset;
    while (index < node_count) {
        bool leaf_pass;
        uint32_t leaf_entry;
        const uint32_t next = walk_step<WALK_STEPS>(nodes, index, node_count, ray, hit.distance, leaf_pass, leaf_entry);
        if (leaf_pass) {
            uint32_t primitive_index = prim_offset + leaf_entry - HK_BVH_LEAF_FLAG;
            f3 a, b, c;
            load_triangle(sc.primitives, primitive_index, a, b, c);
            f2 uv;
            float d = intersects_triangle(ray, a, b, c, uv);
            if (d < hit.distance) {
                hit.distance = d;
                hit.uv = uv;
                hit.primitive_index = primitive_index;
                intersected = true;
                if (d < early_distance) return intersected;
            }
        }
        index = next;
    }
    return intersected;
}

HKD f3 world_to_local_point(const hk_instance& in, f3 p)
{
    const float* m = in.inverse_transpose_model;  // inverse_model = transpose(itm)
    float x = ((m[0] * p.x + m[1] * p.y) + m[2] * p.z) + m[3] * 1.0f;
    float y = ((m[4] * p.x + m[5] * p.y) + m[6] * p.z) + m[7] * 1.0f;
    float z = ((m[8] * p.x + m[9] * p.y) + m[10] * p.z) + m[11] * 1.0f;
    float w = ((m[12] * p.x + m[13] * p.y) + m[14] * p.z) + m[15] * 1.0f;
    if (w == 1.0f) return mk3(x, y, z);  // x / 1 == x exactly: skips three IEEE divides (affine transforms)
    return mk3(x / w, y / w, z / w);
}
HKD f3 world_to_local_dir(const hk_instance& in, f3 p)
{
    const float* m = in.inverse_transpose_model;
    float x = ((m[0] * p.x + m[1] * p.y) + m[2] * p.z) + m[3] * 0.0f;
    float y = ((m[4] * p.x + m[5] * p.y) + m[6] * p.z) + m[7] * 0.0f;
    float z = ((m[8] * p.x + m[9] * p.y) + m[10] * p.z) + m[11] * 0.0f;
    return mk3(x, y, z);
}
HKD f3 local_to_world_point(const hk_instance& in, f3 p)
{
    f4 r = mat4_mul(in.model, mk4(p.x, p.y, p.z, 1.0f));
    if (r.w == 1.0f) return mk3(r.x, r.y, r.z);  // exact, as in world_to_local_point
    return mk3(r.x / r.w, r.y / r.w, r.z / r.w);
}
HKD f3 local_to_world_normal(const hk_instance& in, f3 n)
{
    const float* m = in.inverse_transpose_model;
    f3 r;
    r.x = (m[0] * n.x + m[4] * n.y) + m[8] * n.z;
    r.y = (m[1] * n.x + m[5] * n.y) + m[9] * n.z;
    r.z = (m[2] * n.x + m[6] * n.y) + m[10] * n.z;
    return normalize(r);
}

// light.wgsl:442-486 with light.wgsl:400-440 inlined — the same two-level skip-pointer walk
// (every node, box test and triangle in the reference's visit order, so the hit and the early
// exits are identical) run as ONE loop in which each iteration advances a lane by one node,
// whether that lane is in the TLAS or in an instance's BLAS.  The nested form (a TLAS loop whose
// instance leaves run a BLAS loop) serialises a wave: lanes reach instance leaves in different
// TLAS iterations, so the BLAS loops of a wave's lanes run one after the other while the other
// lanes wait.  Here all lanes share every iteration's node load and slab test; only the leaf
// work (instance entry, triangle test) diverges.  Cornell 1080p: direct 0.185 -> 0.168 ms,
// indirect 0.311 -> 0.286 ms; scene 1080p emissive 0.476 -> 0.421 ms.
// Lane-efficiency instrumentation (experiment builds only, EXTRA=-DHK_LANE_STATS): every iteration
// of a traverse_top walk adds the wave's active lanes (its first active lane counts for the wave), so
// sum(active) / (64 x sum(iterations)) is the fraction of SIMD lanes doing walk work, idle lanes of
// the wave (walks already ended, lanes with no ray) included.
// Slot 0: the traverse_top walks; slots 1-4: the stages of spatial reuse's neighbour loop (k_spatial: a neighbour
// tested, a depth-march tap, the record tests, the shade / jacobian / merge), each tick at a stage's entry, so
// active / (64 x iterations) of a slot is the fraction of the wave's lanes that do that stage's work when it runs.
constexpr int LANE_SLOTS = 5;
#ifdef HK_LANE_STATS
extern __device__ unsigned long long hk_lane_stats_dev[2 * LANE_SLOTS];
template <int SLOT = 0>
struct LaneStats {
    unsigned long long act = 0, its = 0;
    HKD void tick()
    {
        const unsigned long long m = __ballot(1);
        if ((uint32_t)__builtin_ctzll(m) == (threadIdx.x & 63u)) {
            act += (unsigned long long)__builtin_popcountll(m);
            its += 1;
        }
    }
    HKD ~LaneStats()
    {
        if (its) {
            atomicAdd(&hk_lane_stats_dev[2 * SLOT], act);
            atomicAdd(&hk_lane_stats_dev[2 * SLOT + 1], its);
        }
    }
};
#define HK_LANE_STATS_DECL LaneStats<0> lane_stats_
#define HK_LANE_STATS_TICK lane_stats_.tick()
#define HK_STAGE_STATS_DECL LaneStats<1> stage1_; LaneStats<2> stage2_; LaneStats<3> stage3_; LaneStats<4> stage4_
#define HK_STAGE_TICK(k) stage##k##_.tick()
#else
#define HK_LANE_STATS_DECL
#define HK_LANE_STATS_TICK
#define HK_STAGE_STATS_DECL
#define HK_STAGE_TICK(k)
#endif

// Several visits per iteration where the order allows it (walk_step): an inner child-box node p
// that passes is always followed by node p + 1 (its subtree start, bvh flatten), tested with the
// same hit distance, so one iteration tests p and — while the visited nodes are passing inner
// nodes — p + 1, p + 2, ... too, from consecutive node loads.  At most one of them is a leaf,
// whose work (triangle test / instance entry) then follows.  Same visits, tests and results as
// one node per iteration (WALK_STEPS 2: cornell 1080p 0.619 -> 0.604 ms/frame).
HKD Hit traverse_top(const Scene& sc, const Ray& ray, float max_distance, float early_distance, uint32_t exclude)
{
    Hit hit;
    hit.uv = mk2(0.0f, 0.0f);
    hit.distance = max_distance;
    hit.instance_index = HK_U32_MAX;
    hit.primitive_index = HK_U32_MAX;
    // The walk in progress — the TLAS, or the BLAS of the instance being visited — as one set of registers (its
    // nodes, length, position and ray), switched when the walk enters or leaves an instance, so that an iteration
    // selects nothing between the two levels' states.
    const hk_node* nodes = sc.instance_nodes;
    uint32_t count = sc.n_instance_nodes, index = 0u;
    Ray tr = ray;                       // the current walk's ray (the instance-local ray inside a BLAS)
    uint32_t top = 0u;                  // the TLAS walk's next node while a BLAS is walked
    uint32_t prim_offset = 0u, cur_instance = 0u;
    bool in_bottom = false, intersected = false;
    HK_LANE_STATS_DECL;
    while (index < count) {
        HK_LANE_STATS_TICK;
        // BLAS leaves carry their triangle's box (k_fill_blas_leaves, light.wgsl:411-413), TLAS
        // leaves their instance's min/max (k_fill_tlas_leaves, light.wgsl:456-457); the leaf this
        // iteration reaches (if any) and the node after it
        bool leaf_pass;
        uint32_t leaf_entry;
        index = walk_step<WALK_STEPS>(nodes, index, count, tr, hit.distance, leaf_pass, leaf_entry);
        if (in_bottom) {
            bool stop = false;
            if (leaf_pass) {
                const uint32_t primitive_index = prim_offset + leaf_entry - HK_BVH_LEAF_FLAG;
                f3 a, b, c;
                load_triangle(sc.primitives, primitive_index, a, b, c);
                f2 uv;
                const float d = intersects_triangle(tr, a, b, c, uv);
                if (d < hit.distance) {
                    hit.distance = d;
                    hit.uv = uv;
                    hit.primitive_index = primitive_index;
                    intersected = true;
                    stop = d < early_distance;  // traverse_bottom's early return
                }
            }
            if (stop || index >= count) {  // back in traverse_top after traverse_bottom
                in_bottom = false;
                nodes = sc.instance_nodes;
                count = sc.n_instance_nodes;
                index = top;
                tr = ray;
                if (intersected) {
                    hit.instance_index = cur_instance;
                    if (hit.distance < early_distance) return hit;
                }
            }
        } else {
            const uint32_t instance_index = leaf_entry - HK_BVH_LEAF_FLAG;
            if (leaf_pass && instance_index != exclude) {
                const hk_instance& in = sc.instances[instance_index];
                const uint32_t bot_count = in.mesh.node[1];
                prim_offset = in.mesh.primitive;
                cur_instance = instance_index;
                intersected = false;
                if (bot_count > 0u) {  // traverse_bottom over an empty range does nothing
                    in_bottom = true;
                    top = index;
                    nodes = sc.asset_nodes + in.mesh.node[0];
                    count = bot_count;
                    index = 0u;
                    tr.origin = world_to_local_point(in, ray.origin);
                    tr.direction = world_to_local_dir(in, ray.direction);
                    tr.inv_direction = inv(tr.direction);
                }
            }
        }
    }
    return hit;
}

// ------------------------------------------------------------------ G-buffer visibility
// Ordered closest-hit traversal, the build's own primary-visibility rule (the reference
// rasterises the G-buffer); defined in oracle/hk_oracle.c (closest_hit_ordered) and reproduced
// here step for step.  Wide entry of a subtree start p (4 x float4, one 64-byte line):
//   inner: (left box min, left target), (left box max, right target),
//          (right box min, -), (right box max, -)      [targets mesh-local for BLAS]
//   leaf:  (leaf box min, entry = payload | LEAF), (leaf box max, U32_MAX)
// A target is the child's subtree start, or LEAF | payload when the child is a single leaf whose
// box equals the child box (k_build_wide): its box test is then the descent's / pop's comparison.
// Leaf boxes are the triangle's / instance's box, as the reference walk tests them.
constexpr int GB_STACK = 64;
// Stack entries (node, entry distance) live in the workgroup's LDS (entry-major, one uint2 per thread
// per level: conflict-free): all of them when the scene's stack bound is <= GB_STACK_LDS (SHALLOW,
// exactly that many levels), otherwise the first GB_DEEP_LDS, deeper ones in private scratch.
constexpr int GB_STACK_LDS = 16;
// a deeper scene's stack: its first GB_DEEP_LDS levels in LDS, the rest in private scratch
constexpr int GB_DEEP_LDS = 8;
// SHALLOW: the scene's stack bound fits the LDS levels (hk_runtime gb_stack_need), so there is no
// private overflow array (no scratch allocation for the kernel's waves)
// LVL: the LDS levels of a deep scene's stack (the rest in scratch)
template <bool SHALLOW, int LVL = GB_STACK_LDS>
struct GbStackT {
    uint2* lds;  // [LVL][blockDim.x], or null
    uint32_t node[SHALLOW ? 1 : GB_STACK - LVL];
    float t[SHALLOW ? 1 : GB_STACK - LVL];
    int sp;
    HKD void push(uint32_t n, float tt)
    {
        if (SHALLOW || (lds && sp < LVL)) lds[sp * 256 + threadIdx.x] = make_uint2(n, __float_as_uint(tt));
        else {
            const int k = lds ? sp - LVL : sp;
            node[k] = n;
            t[k] = tt;
        }
        sp++;
    }
    HKD void top(uint32_t& n, float& tt) const
    {
        if (SHALLOW || (lds && sp < LVL)) {
            const uint2 e = lds[sp * 256 + threadIdx.x];
            n = e.x;
            tt = __uint_as_float(e.y);
        } else {
            const int k = lds ? sp - LVL : sp;
            n = node[k];
            tt = t[k];
        }
    }
};
template <class GbStack>
HKD bool gb_pop(GbStack& s, int base, float best, uint32_t& n)
{
    while (s.sp > base) {
        s.sp--;
        uint32_t m;
        float tt;
        s.top(m, tt);
        if (tt < best) {
            n = m;
            return true;
        }
    }
    return false;
}
// one inner step: enter the nearer passing child, push the farther; false if neither passes
template <class GbStack>
HKD bool gb_descend(GbStack& s, const Ray& ray, float4 a, float4 b, float4 c, float4 d, float best, uint32_t& p)
{
    const float tl = intersects_aabb(ray, mk3(a.x, a.y, a.z), mk3(b.x, b.y, b.z));
    const float tr = intersects_aabb(ray, mk3(c.x, c.y, c.z), mk3(d.x, d.y, d.z));
    const uint32_t ls = __float_as_uint(a.w), rs = __float_as_uint(b.w);
    const bool hl = tl < best, hr = tr < best;
    if (hl && hr) {
        const bool right_first = tr < tl;
        s.push(right_first ? ls : rs, right_first ? tl : tr);
        p = right_first ? rs : ls;
        return true;
    }
    if (hl) {
        p = ls;
        return true;
    }
    if (hr) {
        p = rs;
        return true;
    }
    return false;
}
// The same walk with the TLAS and BLAS steps in one loop (as traverse_top): each iteration
// visits one wide entry of the lane's current level, so a wave's lanes do not wait for each
// other's BLAS walks.  Identical visits, pushes, pops and hit updates per lane.
template <bool SHALLOW = false, int LVL = GB_STACK_LDS>
HKD Hit closest_hit_ordered(const Scene& sc, const Ray& ray, uint2* lds_stack = nullptr)
{
    Hit hit;
    hit.uv = mk2(0.0f, 0.0f);
    hit.distance = HK_F32_MAX;
    hit.instance_index = HK_U32_MAX;
    hit.primitive_index = HK_U32_MAX;
    if (sc.n_instance_nodes == 0u) return hit;
    GbStackT<SHALLOW, LVL> s;
    s.sp = 0;
    s.lds = lds_stack;
    uint32_t p = 0u;          // subtree start of the current level (mesh-local in a BLAS)
    bool in_bottom = false;
    int sbase = 0;            // stack floor of the BLAS walk
    uint32_t bbase = 0u, prim_offset = 0u, cur = 0u;
    Ray local = ray;
    for (;;) {
        const Ray& r = in_bottom ? local : ray;
        // p: a wide entry, or (LEAF | payload) for a leaf child whose box is its parent entry's child
        // box (k_build_wide): that box test already passed, at the descent or at the pop
        uint32_t entry = p;
        bool pass = true, go = false;
        float4 a, b;
        const float4* w = nullptr;
        if (p < HK_BVH_LEAF_FLAG) {
            w = in_bottom ? sc.blas_wide + 4u * (size_t)(bbase + p) : sc.tlas_wide + 4u * (size_t)p;
            a = w[0];
            b = w[1];
            // a leaf entry (single-leaf tree root) has w[1].w == U32_MAX; an inner entry's a.w is its
            // left target, which may itself be (LEAF | payload)
            entry = __float_as_uint(b.w) == HK_U32_MAX ? __float_as_uint(a.w) : 0u;
            if (entry >= HK_BVH_LEAF_FLAG) pass = intersects_aabb(r, mk3(a.x, a.y, a.z), mk3(b.x, b.y, b.z)) < hit.distance;
        }
        if (entry >= HK_BVH_LEAF_FLAG) {
            if (pass) {
                if (in_bottom) {
                    const uint32_t primitive_index = prim_offset + entry - HK_BVH_LEAF_FLAG;
                    f3 t0, t1, t2;
                    load_triangle(sc.primitives, primitive_index, t0, t1, t2);
                    f2 uv;
                    const float dd = intersects_triangle(local, t0, t1, t2, uv);
                    if (dd < hit.distance) {
                        hit.distance = dd;
                        hit.uv = uv;
                        hit.primitive_index = primitive_index;
                        hit.instance_index = cur;
                    }
                } else {
                    const uint32_t instance_index = entry - HK_BVH_LEAF_FLAG;
                    const hk_instance& in = sc.instances[instance_index];
                    if (in.mesh.node[1] != 0u) {  // closest_bottom_ordered of an empty mesh returns at once
                        local.origin = world_to_local_point(in, ray.origin);
                        local.direction = world_to_local_dir(in, ray.direction);
                        local.inv_direction = inv(local.direction);
                        bbase = in.mesh.node[0];
                        prim_offset = in.mesh.primitive;
                        cur = instance_index;
                        sbase = s.sp;
                        in_bottom = true;
                        p = 0u;
                        go = true;
                    }
                }
            }
        } else {
            go = gb_descend(s, r, a, b, w[2], w[3], hit.distance, p);
        }
        if (!go) {
            if (in_bottom) {
                go = gb_pop(s, sbase, hit.distance, p);
                if (!go) in_bottom = false;  // the BLAS walk returned: continue the TLAS walk
            }
            if (!go && !gb_pop(s, 0, hit.distance, p)) return hit;
        }
    }
}

HKD const hk_instance& get_instance(const Scene& sc, uint32_t i) { return sc.instances[i < sc.n_instances ? i : sc.n_instances - 1]; }
HKD const hk_material& get_material(const Scene& sc, uint32_t i) { return sc.materials[i < sc.n_materials ? i : sc.n_materials - 1]; }

HKD HitInfo empty_hit_info(f3 position, f3 direction)
{
    HitInfo info;
    info.instance_index = HK_U32_MAX;
    info.material_index = HK_U32_MAX;
    f3 p = position + direction * DISTANCE_MAX;
    info.position = mk4(p.x, p.y, p.z, 0.0f);
    info.normal = mk3(0, 0, 0);
    info.uv = mk2(0, 0);
    return info;
}
HKD HitInfo hit_info(const Scene& sc, const Ray& ray, const Hit& hit)
{
    HitInfo info;
    info.instance_index = hit.instance_index;
    info.material_index = HK_U32_MAX;
    info.normal = mk3(0, 0, 0);
    info.uv = mk2(0, 0);
    if (hit.instance_index != HK_U32_MAX) {
        const hk_instance& in = get_instance(sc, hit.instance_index);
        const hk_primitive& pr = sc.primitives[hit.primitive_index];
        const hk_vertex& v0 = sc.vertices[in.mesh.vertex + pr.vertices[0].index];
        const hk_vertex& v1 = sc.vertices[in.mesh.vertex + pr.vertices[1].index];
        const hk_vertex& v2 = sc.vertices[in.mesh.vertex + pr.vertices[2].index];
        f2 uv = hit.uv;
        info.uv = mk2((v0.u + uv.x * (v1.u - v0.u)) + uv.y * (v2.u - v0.u),
                      (v0.v + uv.x * (v1.v - v0.v)) + uv.y * (v2.v - v0.v));
        f3 n0 = ld3(v0.normal), n1 = ld3(v1.normal), n2 = ld3(v2.normal);
        f3 n = (n0 + (n1 - n0) * uv.x) + (n2 - n0) * uv.y;
        info.normal = local_to_world_normal(in, n);
        f3 p = ray.origin + ray.direction * hit.distance;
        info.position = mk4(p.x, p.y, p.z, 1.0f);
        info.material_index = in.material;
    } else {
        f3 p = ray.origin + ray.direction * DISTANCE_MAX;
        info.position = mk4(p.x, p.y, p.z, 0.0f);
    }
    return info;
}
HKD void occlude_hit_info(const Ray& ray, const Hit& hit, HitInfo& info)
{
    if (hit.instance_index != HK_U32_MAX) {
        info.instance_index = hit.instance_index;
        info.material_index = HK_U32_MAX;
        f3 p = ray.origin + ray.direction * hit.distance;
        info.position = mk4(p.x, p.y, p.z, 1.0f);
        info.normal = mk3(0, 0, 0);
    }
}

// ------------------------------------------------------------------ sampling (light.wgsl:537-708)
HKD f4 sample_cosine_hemisphere(f2 rand)
{
    float r = sqrtf(rand.x);
    float theta = (2.0f * HK_PI) * rand.y;
    float sn, cs;
    hk_sincos(theta, &sn, &cs);
    f2 t = mk2(r * cs, r * sn);
    float z = sqrtf(1.0f - dot(t, t));
    return mk4(t.x, t.y, z, (2.0f * HK_INV_TAU) * z);
}
HKD f4 sample_uniform_cone(f2 rand, float cos_angle)
{
    float z = 1.0f - (1.0f - cos_angle) * rand.x;
    float theta = HK_TAU * rand.y;
    float r = sqrtf(1.0f - z * z);
    float sn, cs;
    hk_sincos(theta, &sn, &cs);
    return mk4(r * cs, r * sn, z, HK_INV_TAU / (1.0f - cos_angle));
}
HKD void normal_basis(f3 n, f3& t, f3& b)
{
    float sg = n.z > 0.0f ? 1.0f : (n.z < 0.0f ? -1.0f : 0.0f);
    float s = fminf(sg * 2.0f + 1.0f, 1.0f);
    float u = -1.0f / (s + n.z);
    float v = (n.x * n.y) * u;
    t = mk3(1.0f + ((s * n.x) * n.x) * u, s * v, -s * n.x);
    b = mk3(v, s + (n.y * n.y) * u, -n.y);
}
HKD f3 basis_mul(f3 t, f3 b, f3 n, f3 d) { return (t * d.x + b * d.y) + n * d.z; }
HKD f3 emissive_radiance(f4 e) { return xyz(e) * (255.0f * e.w); }

// select_light_candidate (light.wgsl:599-708) in two halves around its emitter BLAS walk, so that a kernel
// can run the walks of a whole workgroup as one compacted batch between them (k_direct_fused_w4's CW
// variant): light_pick_begin runs everything before the walk (directional cone sample, light-BVH reservoir
// pick, alias-table triangle sample, the ray towards the sampled point in world and emitter-local space),
// light_pick_end everything after it.  select_light_candidate = begin, the walk, end: the same statements
// in the same order.
struct LightPick {
    LightCandidate cand;
    f3 rand_direction;
    Ray ray;    // world: biased origin, direction towards the sampled point (inv_direction unused)
    Ray local;  // the emitter instance's local ray of the walk
    uint32_t picked;  // emissive record of the pick
    float count;
    bool emitter;     // an emitter was picked (light_pick_end must run)
    bool walk;        // ... and the walk runs (the sampled direction faces the normal)
};
template <bool COUNT>
HKD void light_pick_begin(const Scene& sc, const Frame& F, f4 rand, f3 position, f3 normal, uint32_t instance,
                          HitInfo& info, uint32_t& n_emitter, LightPick& L)
{
    LightCandidate& candidate = L.cand;
    candidate.max_distance = HK_F32_MAX;
    candidate.min_distance = DISTANCE_MAX;
    candidate.emissive_instance = DONT_SAMPLE_EMISSIVE;
    f3 cone = ld3(F.direction_to_light);
    f3 bt, bb;
    normal_basis(cone, bt, bb);
    f3 rand_direction = basis_mul(bt, bb, cone, xyz(sample_uniform_cone(mk2(rand.z, rand.w), F.cos_solar_angle)));
    L.rand_direction = rand_direction;
    candidate.direction = rand_direction;
    candidate.p = 1.0f;
    info = empty_hit_info(position, rand_direction);
    L.emitter = L.walk = false;
    if (instance == DONT_SAMPLE_EMISSIVE) return;

    uint32_t picked = 0u;
    float count = 0.0f;
    uint32_t index = 0u;
    float rand_1d = rand.x;
    while (index < sc.n_emissive_nodes) {
        f3 mn, mx;
        uint32_t entry, exit;
        load_node(sc.emissive_nodes, index, mn, entry, mx, exit);
        if (entry >= HK_BVH_LEAF_FLAG) {
            uint32_t ei = entry - HK_BVH_LEAF_FLAG;
            const hk_emissive& cur = sc.emissives[ei];
            f3 ep = ld3(cur.position);
            float rad = cur.radius;
            f3 emn = mk3(ep.x - rad, ep.y - rad, ep.z - rad), emx = mk3(ep.x + rad, ep.y + rad, ep.z + rad);
            bool inside = (position.x > emn.x && position.y > emn.y && position.z > emn.z) &&
                          (position.x < emx.x && position.y < emx.y && position.z < emx.z);
            if (instance != cur.instance && inside) {
                rand_1d = hk_fract(rand_1d + HK_GOLDEN_RATIO);
                count += 1.0f;
                if (rand_1d < 1.0f / count) {
                    candidate.emissive_instance = cur.instance;
                    picked = ei;
                }
            }
            index = exit;
        } else {
            bool inside = (position.x > mn.x && position.y > mn.y && position.z > mn.z) &&
                          (position.x < mx.x && position.y < mx.y && position.z < mx.z);
            index = inside ? entry : exit;
        }
    }
    L.picked = picked;
    L.count = count;
    if (candidate.emissive_instance != DONT_SAMPLE_EMISSIVE) {
        L.emitter = true;
        const hk_emissive& emissive = sc.emissives[picked];
        uint32_t len = emissive.alias_table[1];
        uint32_t alias_index = f2u32(rand.x * (float)len);
        if (alias_index > len - 1u) alias_index = len - 1u;
        hk_alias_entry ae = sc.alias_table[emissive.alias_table[0] + alias_index];
        uint32_t primitive_index = rand.y < ae.prob ? ae.index : alias_index;
        const hk_instance& ein = get_instance(sc, candidate.emissive_instance);
        f3 v0, v1, v2;
        load_triangle(sc.primitives, ein.mesh.primitive + primitive_index, v0, v1, v2);
        float srx = sqrtf(rand.z);
        f2 b = mk2(1.0f - srx, rand.w * srx);
        f3 p = local_to_world_point(ein, (v0 * b.x + v1 * b.y) + v2 * ((1.0f - b.x) - b.y));

        Ray& ray = L.ray;
        ray.origin = position + normal * RAY_BIAS;
        ray.direction = normalize(p - position);
        ray.inv_direction = mk3(0, 0, 0);
        Ray& r = L.local;
        r.origin = world_to_local_point(ein, ray.origin);
        r.direction = world_to_local_dir(ein, ray.direction);
        r.inv_direction = inv(r.direction);
        candidate.direction = ray.direction;
        if (dot(candidate.direction, normal) > 0.0f) {
            if (COUNT) n_emitter++;
            L.walk = true;
        }
    }
}
// the walk of L (traverse_bottom over the picked emitter's BLAS, closest hit): hit starts empty
HKD bool light_pick_walk(const Scene& sc, const LightPick& L, Hit& hit)
{
    hit.uv = mk2(0, 0);
    hit.distance = HK_F32_MAX;
    hit.instance_index = HK_U32_MAX;
    hit.primitive_index = HK_U32_MAX;
    if (!L.walk) return false;
    const hk_instance& ein = get_instance(sc, L.cand.emissive_instance);
    return traverse_bottom(sc, hit, L.local, ein.mesh.node[0], ein.mesh.node[1], ein.mesh.primitive, 0.0f);
}
// after the walk (traced: it ran and hit; hit: its result); only when L.emitter
HKD void light_pick_end(const Scene& sc, LightPick& L, f3 position, Hit hit, bool traced, HitInfo& info)
{
    LightCandidate& candidate = L.cand;
    const hk_emissive& emissive = sc.emissives[L.picked];
    const Ray& ray = L.ray;
    if (traced) {
        hit.instance_index = emissive.instance;
        info = hit_info(sc, ray, hit);
        candidate.max_distance = hit.distance;
        candidate.min_distance = hit.distance - 0.1f;
        f3 delta = xyz(info.position) - position;
        candidate.p = dot(delta, delta) / fabsf(dot(ray.direction, info.normal) * emissive.surface_area);
        candidate.p = candidate.p / L.count;
    } else {
        info = empty_hit_info(ray.origin, ray.direction);
        candidate.emissive_instance = DONT_SAMPLE_EMISSIVE;
        candidate.direction = L.rand_direction;
        candidate.p = 1.0f;
    }
}
template <bool COUNT>
HKD LightCandidate select_light_candidate(const Scene& sc, const Frame& F, f4 rand, f3 position, f3 normal,
                                          uint32_t instance, HitInfo& info, uint32_t& n_emitter)
{
    LightPick L;
    light_pick_begin<COUNT>(sc, F, rand, position, normal, instance, info, n_emitter, L);
    if (L.emitter) {
        Hit hit;
        const bool traced = light_pick_walk(sc, L, hit);
        light_pick_end(sc, L, position, hit, traced, info);
    }
    return L.cand;
}

// ------------------------------------------------------------------ shading (light.wgsl:714-908 + Bevy PBR)
HKD f3 calculate_view(const Frame& F, f4 world_position)
{
    if (F.orthographic) return normalize(ld3(F.view_proj_z));
    return normalize(ld3(F.view_world_position) - xyz(world_position));
}
// light.wgsl:729-794: NO_TEXTURE variant when the scene has no textures, otherwise each material
// texture id != U32_MAX modulates its factor with textureSampleLevel(.., uv, 0) (hk_texture.h)
HKD f4 sample_material_texture(const Scene& sc, uint32_t id, f2 uv)
{
    float t[4];
    hk_sample_texture(sc.textures + id, sc.texels, sc.texture_lut, uv.x, uv.y, t);
    return mk4(t[0], t[1], t[2], t[3]);
}
HKD bool has_texture(const Scene& sc, uint32_t id) { return id != HK_U32_MAX && id < sc.n_textures; }
HKD Surface retreive_surface(const Scene& sc, uint32_t material_index, f2 uv)
{
    const hk_material& m = get_material(sc, material_index);
    Surface s;
    s.base_color = mk4(m.base_color[0], m.base_color[1], m.base_color[2], m.base_color[3]);
    s.emissive = mk4(m.emissive[0], m.emissive[1], m.emissive[2], m.emissive[3]);
    s.metallic = m.metallic;
    s.occlusion = 1.0f;
    if (sc.n_textures) {
        if (has_texture(sc, m.base_color_texture)) {
            f4 t = sample_material_texture(sc, m.base_color_texture, uv);
            s.base_color = mk4(s.base_color.x * t.x, s.base_color.y * t.y, s.base_color.z * t.z, s.base_color.w * t.w);
        }
        if (has_texture(sc, m.emissive_texture)) {
            f4 t = sample_material_texture(sc, m.emissive_texture, uv);
            s.emissive = mk4(s.emissive.x * t.x, s.emissive.y * t.y, s.emissive.z * t.z, s.emissive.w * t.w);
        }
        if (has_texture(sc, m.metallic_roughness_texture))
            s.metallic = s.metallic * sample_material_texture(sc, m.metallic_roughness_texture, uv).x;
        if (has_texture(sc, m.occlusion_texture)) s.occlusion = sample_material_texture(sc, m.occlusion_texture, uv).x;
    }
    float pr = hk_clampf(m.perceptual_roughness, 0.089f, 1.0f);
    s.roughness = pr * pr;
    s.reflectance = m.reflectance;
    return s;
}
HKD f4 retreive_emissive(const Scene& sc, uint32_t material_index, f2 uv)
{
    const hk_material& m = get_material(sc, material_index);
    f4 e = mk4(m.emissive[0], m.emissive[1], m.emissive[2], m.emissive[3]);
    if (sc.n_textures && has_texture(sc, m.emissive_texture)) {
        f4 t = sample_material_texture(sc, m.emissive_texture, uv);
        e = mk4(e.x * t.x, e.y * t.y, e.z * t.z, e.w * t.w);
    }
    return e;
}
HKD float F_Schlick(float f0, float f90, float VoH) { return f0 + (f90 - f0) * hk_pow5(1.0f - VoH); }
HKD f3 F_Schlick_vec(f3 f0, float f90, float VoH)
{
    float k = hk_pow5(1.0f - VoH);
    return mk3(f0.x + (f90 - f0.x) * k, f0.y + (f90 - f0.y) * k, f0.z + (f90 - f0.z) * k);
}
HKD f3 EnvBRDFApprox(f3 f0, float pr, float NoV)
{
    float rx = pr * -1.0f + 1.0f;
    float ry = pr * -0.0275f + 0.0425f;
    float rz = pr * -0.572f + 1.04f;
    float rw = pr * 0.022f + -0.04f;
    float a004 = fminf(rx * rx, hk_exp2(-9.28f * NoV)) * rx + ry;
    float ABx = -1.04f * a004 + rz;
    float ABy = 1.04f * a004 + rw;
    return mk3(f0.x * ABx + ABy, f0.y * ABx + ABy, f0.z * ABx + ABy);
}
// shading() (light.wgsl:869-888) split into the part that depends only on (V, N, surface) —
// evaluated once per pixel — and the per-light part.  Every expression is the one lit()/
// ambient() evaluate (Bevy PBR), in the same order, so results are bit-identical
// to calling shading() each time; spatial reuse calls it up to 18 times per pixel.
struct ShadeCtx {
    f3 V, N, F0, diffuse_color, ambient;
    float roughness, NdotV, pow5_view, smith_view;
};
HKD ShadeCtx shade_ctx(const Frame& F, f3 V, f3 N, const Surface& s)
{
    ShadeCtx c;
    c.V = V;
    c.N = N;
    f3 base = xyz(s.base_color);
    float f0s = ((0.16f * s.reflectance) * s.reflectance) * (1.0f - s.metallic);
    c.F0 = mk3(f0s + base.x * s.metallic, f0s + base.y * s.metallic, f0s + base.z * s.metallic);
    c.diffuse_color = base * (1.0f - s.metallic);
    c.roughness = s.roughness;
    c.NdotV = fmaxf(dot(N, V), 0.0001f);
    c.pow5_view = hk_pow5(1.0f - c.NdotV);  // F_Schlick(1, f90, NdotV) of Fd_Burley
    float a2 = s.roughness * s.roughness;
    c.smith_view = sqrtf((c.NdotV - a2 * c.NdotV) * c.NdotV + a2);  // lambdaV's root
    // ambient() (light.wgsl:820-833)
    f3 da = EnvBRDFApprox(c.diffuse_color, 1.0f, c.NdotV);
    f3 sa = EnvBRDFApprox(c.F0, s.roughness, c.NdotV);
    c.ambient = ((da + sa) * s.occlusion) * ld3(F.ambient_color);
    return c;
}
HKD f3 shade(const ShadeCtx& c, f3 L, f4 in_radiance)
{
    // lit() (light.wgsl:796-818)
    f3 H = normalize(L + c.V);
    float NoL = hk_saturate(dot(c.N, L));
    float NoH = hk_saturate(dot(c.N, H));
    float LoH = hk_saturate(dot(L, H));
    float roughness = c.roughness;
    float f90 = 0.5f + ((2.0f * roughness) * LoH) * LoH;
    float fd = (F_Schlick(1.0f, f90, NoL) * (1.0f + (f90 - 1.0f) * c.pow5_view)) * (1.0f / HK_PI);
    f3 diffuse = c.diffuse_color * fd;
    float one_minus = 1.0f - NoH * NoH;
    float a = NoH * roughness;
    float k = roughness / (one_minus + a * a);
    float D = (k * k) * (1.0f / HK_PI);
    float a2 = roughness * roughness;
    float lambdaV = NoL * c.smith_view;
    float lambdaL = c.NdotV * sqrtf((NoL - a2 * NoL) * NoL + a2);
    float Vis = 0.5f / (lambdaV + lambdaL);
    float fr90 = hk_saturate(dot(c.F0, mk3(16.5f, 16.5f, 16.5f)));
    f3 Fr = F_Schlick_vec(c.F0, fr90, LoH);
    f3 specular_light = Fr * ((1.0f * D) * Vis);
    f3 lit_radiance = ((specular_light + diffuse) * xyz(in_radiance)) * NoL;
    return mix(lit_radiance, c.ambient, 1.0f - in_radiance.w);
}
HKD f3 shading(const Frame& F, f3 V, f3 N, f3 L, const Surface& s, f4 in_radiance)
{
    return shade(shade_ctx(F, V, N, s), L, in_radiance);
}
// light.wgsl:835-867
HKD f4 input_radiance(const Scene& sc, const Frame& F, const Ray& ray, const HitInfo& info, bool sample_directional,
                      uint32_t sample_emissive, bool sample_ambient)
{
    f3 radiance = mk3(0, 0, 0);
    float amb = 0.0f;
    if (info.instance_index == HK_U32_MAX) {
        bool hit_directional = dot(ray.direction, ld3(F.direction_to_light)) >= F.cos_solar_angle;
        if (sample_directional && hit_directional) {
            radiance = ld3(F.directional_color);
            amb = 0.0f;
        } else {
            radiance = sample_ambient ? ld3(F.ambient_color) : mk3(0, 0, 0);
            amb = 1.0f;
        }
    } else if (sample_emissive == info.instance_index) {
        radiance = emissive_radiance(retreive_emissive(sc, info.material_index, info.uv));
    }
    return mk4(radiance.x, radiance.y, radiance.z, 1.0f - amb);
}
HKD f3 env_brdf(f3 V, f3 N, const Surface& s)
{
    f3 base = xyz(s.base_color);
    float NdotV = fmaxf(dot(N, V), 0.0001f);
    float f0s = ((0.16f * s.reflectance) * s.reflectance) * (1.0f - s.metallic);
    f3 F0 = mk3(f0s + base.x * s.metallic, f0s + base.y * s.metallic, f0s + base.z * s.metallic);
    f3 diffuse_color = base * (1.0f - s.metallic);
    return (EnvBRDFApprox(diffuse_color, 1.0f, NdotV) + EnvBRDFApprox(F0, s.roughness, NdotV)) * s.occlusion;
}
HKD float compute_jacobian(const Sample& q, const Sample& r)
{
    f3 normal = q.sample_normal;
    float c1 = fabsf(dot(normalize(xyz(r.visible_position) - xyz(q.sample_position)), normal));
    float c2 = fabsf(dot(normalize(xyz(q.visible_position) - xyz(q.sample_position)), normal));
    float term_1 = c1 / fmaxf(0.0001f, c2);
    float num = length(xyz(q.visible_position) - xyz(q.sample_position));
    num *= num;
    float denom = length(xyz(r.visible_position) - xyz(q.sample_position));
    denom *= denom;
    float term_2 = num / fmaxf(denom, 0.0001f);
    return hk_clampf(term_1 * term_2, 1.0f, 50.0f);
}

// blue noise (light.wgsl:1075-1079): nearest + repeat => texel ((x + n) & 63, (y + n) & 63)
HKD uchar4 noise_texel(const uchar4* noise, uint32_t number, int32_t x, int32_t y)
{
    uint32_t id = number & 15u;
    uint32_t tx = ((uint32_t)x + number) & 63u, ty = ((uint32_t)y + number) & 63u;
    return noise[(id * 64u + ty) * 64u + tx];
}
HKD f4 noise_of(uchar4 t, uint32_t number)
{
    float fn = (float)number * HK_GOLDEN_RATIO;
    return mk4(hk_fract(hk_unorm8_fast(t.x) + fn), hk_fract(hk_unorm8_fast(t.y) + fn), hk_fract(hk_unorm8_fast(t.z) + fn),
               hk_fract(hk_unorm8_fast(t.w) + fn));
}
HKD f4 noise_random(const uchar4* noise, uint32_t number, int32_t x, int32_t y)
{
    uint32_t id = number & 15u;
    uint32_t tx = ((uint32_t)x + number) & 63u, ty = ((uint32_t)y + number) & 63u;
    uchar4 t = noise[(id * 64u + ty) * 64u + tx];
    float fn = (float)number * HK_GOLDEN_RATIO;
    return mk4(hk_fract(hk_unorm8_fast(t.x) + fn), hk_fract(hk_unorm8_fast(t.y) + fn), hk_fract(hk_unorm8_fast(t.z) + fn),
               hk_fract(hk_unorm8_fast(t.w) + fn));
}

// Ray counters are sharded: COUNTER_SHARDS 64-byte lines per counter, each wave adds its
// wave-reduced count to the line of its workgroup's shard.  A single shared word would
// serialise tens of thousands of same-address atomics per kernel at the memory side.
constexpr uint32_t COUNTER_SHARDS = 1024;
constexpr uint32_t COUNTER_STRIDE = 8;  // u64 per shard line (64 B)
HKD void wave_count(unsigned long long* dst, uint32_t v)
{
    unsigned long long s = v;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    uint32_t shard = ((blockIdx.x + blockIdx.y * gridDim.x) * 4u + (threadIdx.x >> 6)) % COUNTER_SHARDS;
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(dst + (size_t)shard * COUNTER_STRIDE, s);
}

}  // namespace hk
