// hk_kernels.hip — gfx950 kernels of the integrator and denoiser.
//
// Entry point map (reference -> kernel):
//   light.wgsl:1019 full_screen_albedo          -> k_albedo
//   light.wgsl:1044 direct_lit (+RENDER_EMISSIVE / +EMISSIVE_LIT) -> k_direct<EMISSIVE_LIT, RENDER_EMISSIVE>
//   light.wgsl:1263 indirect_lit_ambient (+MULTIPLE_BOUNCES)      -> k_indirect<MULTI>
//   light.wgsl:1503 spatial_reuse (+EMISSIVE_LIT)                 -> k_spatial<EMISSIVE_LIT>
//   denoise.wgsl:135 demodulation (x3 channels)                   -> k_demod3<C>
//   denoise.wgsl:215 denoise (DENOISE_LEVEL_0..3, FIREFLY) x3 ch  -> k_denoise3<C, LEVEL>
//   tone_mapping.wgsl:21 tone_mapping                             -> k_tone
//   prepass.wgsl:84-100 (raster G-buffer)                         -> k_gbuffer (primary rays)
//   light.wgsl:442 traverse_top                                   -> k_trace
//
// Launch shape: 256-thread workgroups covering a 16x16 pixel tile, each wave an 8x8
// sub-tile (the reference's workgroup footprint), so rays of one wave stay coherent.
#include <stdlib.h>
#include <mutex>

#include "hk_device.h"
#include "hk_launch.h"

namespace hk {

#ifdef HK_LANE_STATS
__device__ unsigned long long hk_lane_stats_dev[2 * LANE_SLOTS];
#endif
// lane statistics of every slot (LaneStats) since the last call (builds with -DHK_LANE_STATS; false otherwise)
bool lane_stats_take(unsigned long long out[2 * LANE_SLOTS], hipStream_t st)
{
#ifdef HK_LANE_STATS
    unsigned long long zero[2 * LANE_SLOTS] = {};
    if (hipStreamSynchronize(st) != hipSuccess) return false;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hk_lane_stats_dev), sizeof(zero)) != hipSuccess) return false;
    return hipMemcpyToSymbol(HIP_SYMBOL(hk_lane_stats_dev), zero, sizeof(zero)) == hipSuccess;
#else
    (void)st;
    for (int k = 0; k < 2 * LANE_SLOTS; ++k) out[k] = 0;
    return false;
#endif
}

// workgroup -> 16x16 tile -> pixel (global coordinates).  Tile orders:
// RASTER: blockIdx in raster order; workgroups are dealt round-robin over the 8 XCDs, so every
//   XCD works on the same band of the frame at once and per-region cost differences (sky vs.
//   geometry, lit vs. shadowed) are spread evenly.  The traversal kernels use it (an XCD-stripe
//   order measured 20% slower on cornell 1080p: the XCD holding the expensive stripe finishes last).
// XCD_RASTER: the bijective XCD-stripe order (cdna_hip_programming.md T1): workgroup L runs on XCD
//   L % 8 and each XCD gets a contiguous range of tiles in raster order, so neighbour taps hit its
//   own L2 (demodulation, tone mapping).
// XCD_STRIPS: as XCD_RASTER over tiles enumerated in vertical strips STRIP_TILES wide (raster
//   inside a strip).  The ~100 workgroups in flight on one XCD then cover a compact 2-D region, so
//   spatial reuse's 16 neighbour reservoirs (+/- 20 px) stay in that XCD's 4 MiB L2; in raster
//   order their +/- 20-row window of reservoirs (~7 MB at 1080p) does not fit it.  The a-trous
//   levels use it too (city 4K: 0.529 -> 0.436 ms per level).
enum TileOrder : int { RASTER = 0, XCD_RASTER = 1, XCD_STRIPS = 2 };
constexpr uint32_t STRIP_TILES = 16;  // 8 / 32 / 64 measured slower
template <int ORDER>
HKD void tile_coords_at(uint32_t bx, uint32_t by, uint32_t gx, uint32_t gy, uint32_t& tx, uint32_t& ty)
{
    const uint32_t L = bx + by * gx;
    if (ORDER == RASTER) {
        tx = bx;
        ty = by;
        return;
    }
    const uint32_t n = gx * gy;
    const uint32_t xcd = L & 7u, i = L >> 3, q = n >> 3, r = n & 7u;
    const uint32_t tile = (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + i;
    if (ORDER == XCD_RASTER) {
        tx = tile % gx;
        ty = tile / gx;
        return;
    }
    const uint32_t per_strip = STRIP_TILES * gy;  // every strip but the last is full width
    const uint32_t strip = tile / per_strip, k = tile - strip * per_strip;
    const uint32_t sw = min(STRIP_TILES, gx - strip * STRIP_TILES);
    ty = k / sw;
    tx = strip * STRIP_TILES + (k - ty * sw);
}
template <int ORDER>
HKD void tile_coords(uint32_t& tx, uint32_t& ty)
{
    tile_coords_at<ORDER>(blockIdx.x, blockIdx.y, gridDim.x, gridDim.y, tx, ty);
}
// the pixel of this thread in tile (bx, by) of a gx x gy tile grid (tile_pixel: the launch's own grid)
template <int ORDER = RASTER>
HKD bool tile_pixel_at(const Frame& F, uint32_t width, int32_t row0, int32_t rows, uint32_t bx, uint32_t by, uint32_t gx,
                       uint32_t gy, int32_t& x, int32_t& y)
{
    uint32_t tx, ty;
    tile_coords_at<ORDER>(bx, by, gx, gy, tx, ty);
    uint32_t t = threadIdx.x;
    uint32_t w = t >> 6, lane = t & 63u;
    x = win_x0(F) + (int32_t)(tx * 16u + (w & 1u) * 8u + (lane & 7u));
    const int32_t w0 = F.win_rows > 0 ? F.win_row0 : 0;
    const int32_t w1 = F.win_rows > 0 ? F.win_row0 + F.win_rows : rows;
    int32_t ly = w0 + (int32_t)(ty * 16u + (w >> 1) * 8u + (lane >> 3));
    y = global_row(F, ly, row0);
    return x < win_x1(F, width) && ly < w1;
}
template <int ORDER = RASTER>
HKD bool tile_pixel(const Frame& F, uint32_t width, int32_t row0, int32_t rows, int32_t& x, int32_t& y)
{
    return tile_pixel_at<ORDER>(F, width, row0, rows, blockIdx.x, blockIdx.y, gridDim.x, gridDim.y, x, y);
}

// origin (global coordinates, contiguous bands) of this workgroup's tile
template <int ORDER = RASTER>
HKD void tile_origin(const Frame& F, int32_t row0, int32_t& x0, int32_t& y0)
{
    uint32_t tx, ty;
    tile_coords<ORDER>(tx, ty);
    x0 = win_x0(F) + (int32_t)(tx * 16u);
    y0 = row0 + (F.win_rows > 0 ? F.win_row0 : 0) + (int32_t)(ty * 16u);
}
constexpr int SPATIAL_ORDER = XCD_STRIPS;  // spatial reuse: neighbour reservoirs +/- 20 px in one XCD's L2
constexpr int TRACE_ORDER = RASTER;        // G-buffer and light-pass kernels
constexpr int DENOISE_ORDER = XCD_STRIPS;  // the a-trous levels (taps up to 8 px away): city 4K 0.529 -> 0.436 ms per level

// ------------------------------------------------------------------ G-buffer
HKD f3 primary_direction(const ViewArgs& V, float px, float py, const uint32_t* size)
{
    float ndc_x = (px / (float)size[0]) * 2.0f - 1.0f;
    float ndc_y = 1.0f - (py / (float)size[1]) * 2.0f;
    f4 p = mat4_mul(V.inverse_view_proj, mk4(ndc_x, ndc_y, 1.0f, 1.0f));
    f3 nearp = mk3(p.x / p.w, p.y / p.w, p.z / p.w);
    return normalize(nearp - ld3(V.world_position));
}
HKD float ndc_depth(const float* vp, f3 p)
{
    f4 c = mat4_mul(vp, mk4(p.x, p.y, p.z, 1.0f));
    return c.z / c.w;
}
// utils.wgsl:30-35
HKD f2 clip_to_uv(f4 clip)
{
    f2 uv = mk2(clip.x / clip.w, clip.y / clip.w);
    uv = mk2((uv.x + 1.0f) * 0.5f, (uv.y + 1.0f) * 0.5f);
    return mk2(uv.x, 1.0f - uv.y);
}
// prepass.wgsl:49-50,96: the hit's object-space point p (the triangle's barycentric combination,
// what the rasteriser interpolates) through this frame's model and view and the previous ones
HKD f2 motion_vector(const ViewArgs& V, const hk_instance& in, uint32_t instance, f3 t0, f3 t1, f3 t2, f2 bary)
{
    const f3 lp = (t0 + (t1 - t0) * bary.x) + (t2 - t0) * bary.y;
    const f4 l4 = mk4(lp.x, lp.y, lp.z, 1.0f);
    const f4 wc = mat4_mul(in.model, l4);
    const f4 wp = mat4_mul(V.previous_models + 16u * (size_t)instance, l4);
    const f2 a = clip_to_uv(mat4_mul(V.view_proj, wc));
    const f2 b = clip_to_uv(mat4_mul(V.previous_view_proj, wp));
    return mk2(a.x - b.x, a.y - b.y);
}

extern __shared__ __attribute__((aligned(16))) uint32_t hk_lds_scene[];  // 16-byte aligned: stage_scene copies uint4

// full_screen_albedo (light.wgsl:1019-1042) of one deferred pixel from the G-buffer values as
// they are stored (snorm8 normal, f32 position, material id and uv): k_albedo, and fused into
// k_gbuffer, which has them in registers.
HKD f4 albedo_of(const Frame& F, const Scene& sc, f4 pd, uint32_t packed_normal, float material_f, f2 uv)
{
    if (pd.w < HK_F32_EPSILON) return mk4(0, 0, 0, 0);
    const f3 normal = mk3(hk_unpack_snorm8_fast(packed_normal, 0), hk_unpack_snorm8_fast(packed_normal, 1),
                          hk_unpack_snorm8_fast(packed_normal, 2));
    const Surface surface = retreive_surface(sc, f2u32(material_f), uv);
    const f3 view_direction = calculate_view(F, mk4(pd.x, pd.y, pd.z, 1.0f));
    const f3 a = env_brdf(view_direction, normal, surface);
    return mk4(a.x, a.y, a.z, 1.0f);
}

// albedo != null: the frame's full_screen_albedo is written here too (hk_render_frame skips it)
template <bool LDS, bool SHALLOW, int LVL = GB_STACK_LDS>
__global__ __launch_bounds__(256) void k_gbuffer(FrameArgs A, ViewArgs V, uint2* albedo)
{
    // The traversal stack's LDS levels, in the launch's dynamic LDS (entry-major, [level][256]): every
    // level of the scene's stack bound for SHALLOW (launch_gbuffer sizes it: a shallow scene's
    // workgroups then take less LDS and more of them fit a CU), the first LVL otherwise.  The
    // scene-staged variant (LDS) puts a shallow scene's stack after the staged arrays (small frames:
    // launch_gbuffer) and a deep one in scratch.
    uint2* gb_lds_stack = reinterpret_cast<uint2*>(hk_lds_scene);
    if constexpr (LDS) gb_lds_stack = SHALLOW ? reinterpret_cast<uint2*>(hk_lds_scene + stage_bytes(A.sc.bytes, PLAN_GBUFFER) / 4u) : nullptr;
    Scene sc;
    if constexpr (LDS) sc = stage_scene<PLAN_GBUFFER>(A.sc, hk_lds_scene);
    else sc = A.sc;
    int32_t x, y;
    bool active = tile_pixel<TRACE_ORDER>(A.F, A.F.S[0], A.F.S_row0, A.F.S_rows, x, y);
    uint32_t n_primary = 0;
    if (active) {
        n_primary = 1;
        int32_t idx = band_index(A.F, x, y, A.F.S[0], A.F.S_row0, A.F.S_rows);
        Ray ray;
        ray.origin = ld3(V.world_position);
        ray.direction = primary_direction(V, ((float)x + 0.5f) - V.jitter[0], ((float)y + 0.5f) - V.jitter[1], A.F.S);
        ray.inv_direction = inv(ray.direction);
        Hit hit = closest_hit_ordered<SHALLOW, LVL>(sc, ray, gb_lds_stack);
        if (hit.instance_index == HK_U32_MAX) {
            // a miss stores constant zeros: skipped when this slot already holds them (V.bg)
            bool stored = false;
            if (V.bg) {
                const uint32_t m = V.bg[idx];
                stored = (m & V.bg_need) != 0u;
                if (!stored) V.bg[idx] = (uint8_t)(m | V.bg_need);
            }
            if (!stored) {
                A.G.position[idx] = make_float4(0, 0, 0, 0);
                A.G.normal[idx] = 0u;
                A.G.depth_gradient[idx] = make_float2(0, 0);
                A.G.instance_material[idx] = make_float2(0, 0);
                A.G.velocity_uv[idx] = make_float4(0, 0, 0, 0);
                if (albedo) store_rgba16f(albedo, idx, mk4(0, 0, 0, 0));
            }
        } else {
            if (V.bg && V.bg[idx]) V.bg[idx] = 0;
            HitInfo info = hit_info(sc, ray, hit);
            f3 p = xyz(info.position);
            float depth = ndc_depth(V.view_proj, p);
            A.G.position[idx] = make_float4(p.x, p.y, p.z, depth);
            const uint32_t packed_normal = hk_pack4x8snorm(info.normal.x, info.normal.y, info.normal.z, 1.0f);
            A.G.normal[idx] = packed_normal;
            if (albedo)
                store_rgba16f(albedo, idx,
                              albedo_of(A.F, A.sc, mk4(p.x, p.y, p.z, depth), packed_normal,
                                        (float)info.material_index + 0.5f, info.uv));
            const hk_instance& in = get_instance(sc, hit.instance_index);
            f3 t0, t1, t2;
            load_triangle(sc.primitives, hit.primitive_index, t0, t1, t2);
            f3 w0 = local_to_world_point(in, t0), w1 = local_to_world_point(in, t1), w2 = local_to_world_point(in, t2);
            f3 ng = cross(w1 - w0, w2 - w0);
            float plane = dot(p - ray.origin, ng);
            float grad[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                f3 d = primary_direction(V, ((float)x + 0.5f + (k == 0 ? 1.0f : 0.0f)) - V.jitter[0],
                                         ((float)y + 0.5f + (k == 1 ? 1.0f : 0.0f)) - V.jitter[1], A.F.S);
                float denom = dot(d, ng);
                grad[k] = 0.0f;
                if (denom != 0.0f) {
                    float t = plane / denom;
                    grad[k] = ndc_depth(V.view_proj, ray.origin + d * t) - depth;
                }
            }
            A.G.depth_gradient[idx] = make_float2(grad[0], grad[1]);
            A.G.instance_material[idx] = make_float2((float)hit.instance_index + 0.5f, (float)info.material_index + 0.5f);
            f2 velocity = mk2(0.0f, 0.0f);  // exactly what motion_vector gives when nothing moved
            if (V.motion) velocity = motion_vector(V, in, hit.instance_index, t0, t1, t2, hit.uv);
            A.G.velocity_uv[idx] = make_float4(velocity.x, velocity.y, info.uv.x, info.uv.y);
        }
    }
    if (y < A.F.count_Sy0 || y >= A.F.count_Sy1 || x < A.F.count_x0 || x >= A.F.count_x1) n_primary = 0;
    wave_count(A.cnt.primary, n_primary);
}

// ------------------------------------------------------------------ albedo (light.wgsl:1019-1042)
__global__ __launch_bounds__(256) void k_albedo(FrameArgs A, uint2* albedo)
{
    int32_t x, y;
    if (!tile_pixel<TRACE_ORDER>(A.F, A.F.S[0], A.F.S_row0, A.F.S_rows, x, y)) return;
    const int32_t idx = band_index(A.F, x, y, A.F.S[0], A.F.S_row0, A.F.S_rows);
    const f4 pd = load_position(A.F, A.G, x, y);
    if (pd.w < HK_F32_EPSILON) {
        store_rgba16f(albedo, idx, mk4(0, 0, 0, 0));
        return;
    }
    const f4 velocity_uv = load_velocity_uv(A.F, A.G, x, y);
    store_rgba16f(albedo, idx, albedo_of(A.F, A.sc, pd, A.G.normal[idx], load_instance_material(A.F, A.G, x, y).y,
                                         mk2(velocity_uv.z, velocity_uv.w)));
}

// ------------------------------------------------------------------ direct_lit (light.wgsl:1044-1261)
// VALIDATE: 0 = the host knows this frame is not a validation frame of the pass (frame.number %
// validate_interval != 0, light.wgsl:1096,1149), so the validation block is compiled out — it holds
// the register peak (the reservoir stays live across its two walks: 142 -> 116 VGPRs for the emissive
// pass, 3 -> 4 waves per SIMD) — and the candidate block always runs; 1 = the general body.
// The G-buffer texels and the blue-noise sample a direct-light pass reads for its pixel
// (light.wgsl:1052-1090).  Loaded once per thread: the fused launch runs both passes of the pixel
// from one copy (the passes store only reservoir / render / variance planes, never the G-buffer),
// where each pass loading its own would issue a second round of dependent loads after the first
// pass's stores.  A background pixel (depth < epsilon) reads its position texel only.
struct DirectPixel {
    int32_t idx;
    f2 uv;
    f4 pd, velocity_uv, random;
    f3 normal;
    f2 imf;
};
// A light pass's G-buffer texels and blue-noise texel for its pixel, loaded together at the kernel's start: before
// the workgroup's scene staging, their latency overlaps the staging copy instead of following its barrier; without
// staging, they are one round trip instead of the position's followed by the rest once the pixel is known to be
// covered.  The loads the pass makes anyway (load_position / load_normal / load_instance_material /
// load_velocity_uv at the jittered coordinates, noise_random's texel), so the values are the same; a background
// pixel reads them too.
struct PixelTexels {
    float4 pd, vel;
    float2 imf;
    uint32_t normal;
    uchar4 noise;
};
HKD PixelTexels load_pixel_texels(const FrameArgs& A, int32_t x, int32_t y)
{
    const Frame& F = A.F;
    PixelTexels t;
    int32_t dx, dy;
    jittered_coords(F, coords_to_uv(x, y, F.s), dx, dy);
    if (in_frame(dx, dy, F.S)) {
        const int32_t i = band_index(F, dx, dy, F.S[0], F.S_row0, F.S_rows);
        t.pd = A.G.position[i];
        t.vel = A.G.velocity_uv[i];
        t.imf = A.G.instance_material[i];
        t.normal = A.G.normal[i];
    } else {
        t.pd = t.vel = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        t.imf = make_float2(0.0f, 0.0f);
        t.normal = 0u;
    }
    t.noise = noise_texel(A.noise, F.number, x, y);
    return t;
}
HKD f3 texel_normal(uint32_t n) { return mk3(hk_unpack_snorm8_fast(n, 0), hk_unpack_snorm8_fast(n, 1), hk_unpack_snorm8_fast(n, 2)); }
HKD DirectPixel direct_pixel_of(const FrameArgs& A, int32_t x, int32_t y, const PixelTexels& t)
{
    const Frame& F = A.F;
    DirectPixel p;
    p.idx = s_index(F, x, y);
    p.uv = coords_to_uv(x, y, F.s);
    p.pd = mk4(t.pd.x, t.pd.y, t.pd.z, t.pd.w);
    p.normal = mk3(0, 0, 0);
    p.imf = mk2(0, 0);
    p.velocity_uv = p.random = mk4(0, 0, 0, 0);
    if (p.pd.w >= HK_F32_EPSILON) {
        p.normal = texel_normal(t.normal);
        p.imf = mk2(t.imf.x, t.imf.y);
        p.velocity_uv = mk4(t.vel.x, t.vel.y, t.vel.z, t.vel.w);
        p.random = noise_of(t.noise, F.number);
    }
    return p;
}
HKD DirectPixel load_direct_pixel(const FrameArgs& A, int32_t x, int32_t y)
{
    const Frame& F = A.F;
    DirectPixel p;
    p.idx = s_index(F, x, y);
    p.uv = coords_to_uv(x, y, F.s);
    int32_t dx, dy;
    jittered_coords(F, p.uv, dx, dy);
    p.pd = load_position(F, A.G, dx, dy);
    p.normal = mk3(0, 0, 0);
    p.imf = mk2(0, 0);
    p.velocity_uv = p.random = mk4(0, 0, 0, 0);
    if (p.pd.w >= HK_F32_EPSILON) {
        p.normal = load_normal(F, A.G, dx, dy);
        p.imf = load_instance_material(F, A.G, dx, dy);
        p.velocity_uv = load_velocity_uv(F, A.G, dx, dy);
        p.random = noise_random(A.noise, F.number, x, y);
    }
    return p;
}

// Validation blocks park the reservoir in LDS across their walks (PARK): the block needs the
// whole reservoir after the shadow walk (light.wgsl:1130-1150), and held in registers through
// select_light_candidate's emitter walk and traverse_top it sets the kernel's register peak
// (143-147 VGPRs, 3 waves per SIMD).  Each thread writes its 28 words to its own LDS column before
// the walks and reads them back after; the compiler barriers keep the registers dead in between.
constexpr int PARK_WORDS = 39;  // the reservoir (28) + the sample's radiance / sample point (11): 39 KiB per
                                // workgroup, so 4 workgroups (4 waves per SIMD) fit a CU's 160 KiB
#define HK_PARK_FIELDS(X)                                                                                                  \
    X(0, s.radiance.x) X(1, s.radiance.y) X(2, s.radiance.z) X(3, s.radiance.w) X(4, s.random.x) X(5, s.random.y)         \
    X(6, s.random.z) X(7, s.random.w) X(8, s.visible_position.x) X(9, s.visible_position.y) X(10, s.visible_position.z)   \
    X(11, s.visible_position.w) X(12, s.visible_normal.x) X(13, s.visible_normal.y) X(14, s.visible_normal.z)             \
    X(16, s.sample_position.x) X(17, s.sample_position.y) X(18, s.sample_position.z) X(19, s.sample_position.w)           \
    X(20, s.sample_normal.x) X(21, s.sample_normal.y) X(22, s.sample_normal.z) X(23, count) X(24, lifetime) X(25, w)      \
    X(26, w_sum) X(27, w2_sum)
HKD void park_reservoir(float* lds, const Reservoir& r)
{
    const uint32_t t = threadIdx.x;
#define HK_PARK_ST(k, f) lds[(k) * 256 + t] = r.f;
    HK_PARK_FIELDS(HK_PARK_ST)
#undef HK_PARK_ST
    lds[15 * 256 + t] = __uint_as_float(r.s.visible_instance);
    __asm__ volatile("" ::: "memory");
}
HKD Reservoir unpark_reservoir(const float* lds)
{
    const uint32_t t = threadIdx.x;
    Reservoir r;
#define HK_PARK_LD(k, f) r.f = lds[(k) * 256 + t];
    HK_PARK_FIELDS(HK_PARK_LD)
#undef HK_PARK_LD
    r.s.visible_instance = __float_as_uint(lds[15 * 256 + t]);
    return r;
}
HKD void park_sample(float* lds, const Sample& s)
{
    const uint32_t t = threadIdx.x;
    const float v[11] = {s.radiance.x, s.radiance.y, s.radiance.z, s.radiance.w, s.sample_position.x, s.sample_position.y,
                         s.sample_position.z, s.sample_position.w, s.sample_normal.x, s.sample_normal.y, s.sample_normal.z};
#pragma unroll
    for (int k = 0; k < 11; ++k) lds[(28 + k) * 256 + t] = v[k];
    __asm__ volatile("" ::: "memory");
}
HKD void unpark_sample(const float* lds, Sample& s)
{
    const uint32_t t = threadIdx.x;
    float v[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) v[k] = lds[(28 + k) * 256 + t];
    s.radiance = mk4(v[0], v[1], v[2], v[3]);
    s.sample_position = mk4(v[4], v[5], v[6], v[7]);
    s.sample_normal = mk3(v[8], v[9], v[10]);
}
HKD float* park_area()
{
    __shared__ float park[PARK_WORDS * 256];
    return park;
}

// direct_lit (light.wgsl:1044-1261) in three parts, so that a kernel can run the candidate block's emitter
// walk for a whole workgroup at once between them (k_direct_fused_w4's CW variant): direct_begin runs the
// pass up to that walk (or the whole background pixel), direct_candidate the rest of the candidate block
// from the walk's result, direct_finish the validation block and the stores.  direct_body = the three with
// the walk in between: the same statements in the same order.
struct DirectState {
    Sample s;
    Reservoir r;
    HitInfo info;
    Ray ray;
    LightPick L;
    f4 position;
    f2 previous_uv;
    bool cand_block;  // the candidate block runs (light.wgsl:1096-1107)
};
template <bool EMISSIVE_LIT, bool RENDER_EMISSIVE, bool VALIDATE>
HKD bool direct_begin(const FrameArgs& A, const Scene& sc, const ChannelArgs& C, const DirectPixel& P, DirectState& D,
                      uint32_t& n_emitter)
{
    const Frame& F = A.F;
    const int32_t idx = P.idx;
    const f2 uv = P.uv;
    f4 pd = P.pd;
    D.position = mk4(pd.x, pd.y, pd.z, 1.0f);
    float depth = pd.w;
    Sample& s = D.s;
    s = zero_sample();
    if (depth < HK_F32_EPSILON) {
        Reservoir r = zero_reservoir();
        set_reservoir(r, s, 0.0f);
        store_res(C.cur, idx, r);
        // direct_lit (light.wgsl:1063-1071) also stores this zero reservoir into the spatial pair,
        // which it shares with the emissive pass (light.rs:518-546); the emissive pass, always run
        // next in the frame, stores the same bits at the same two addresses after every direct_lit
        // store of the frame, so the direct pass's two stores are dead and are skipped
        if (EMISSIVE_LIT) {
            store_res(C.spatial, idx, r);
            store_res(C.prev_spatial, idx, r);
        }
        C.variance[idx] = 0.0f;
        store_rgba16f(C.render, idx, mk4(0, 0, 0, 0));
        D.cand_block = false;
        return false;
    }
    f3 normal = P.normal;
    uint32_t im_x = f2u32(P.imf.x);
    f4 velocity_uv = P.velocity_uv;

    s.random = P.random;
    s.visible_position = mk4(D.position.x, D.position.y, D.position.z, depth);
    s.visible_normal = normal;
    s.visible_instance = im_x;

    D.ray.origin = D.ray.direction = D.ray.inv_direction = mk3(0, 0, 0);
    D.info = empty_hit_info(mk3(0, 0, 0), mk3(0, 0, 0));

    f2 juv = jittered_uv(F, uv, 0.25f);
    D.previous_uv = mk2(juv.x - velocity_uv.x, juv.y - velocity_uv.y);
    // (the whole previous record is read here, before the walks, which hide its latency: read in two steps as in
    // k_indirect's tail — previous_head before the walks, previous_record after them — the fused kernel needs 97
    // instead of 113 VGPRs but the second read lands on the critical path: cornell 0.181 -> 0.194 ms, city 4K
    // 1.337 -> 1.432 ms, profiles/r04/c9)
    Reservoir& r = D.r;
    r = load_previous(F, C.prev, D.previous_uv);
    if (!check_previous_reservoir(r, s) && uv_inside_closed(D.previous_uv)) {
        int32_t px = f2i32(D.previous_uv.x * (float)F.s[0]);
        int32_t py = f2i32(D.previous_uv.y * (float)F.s[1]);
        store_res(C.prev_spatial, s_index(F, px, py), r);
    }

    const uint32_t validate_interval = EMISSIVE_LIT ? F.emissive_validate_interval : F.direct_validate_interval;
    const uint32_t select_light_instance = EMISSIVE_LIT ? im_x : DONT_SAMPLE_EMISSIVE;
    D.cand_block = !VALIDATE || umod(F.number, validate_interval) != 0u || r.count < 4.0f;
    if (D.cand_block)
        light_pick_begin<true>(sc, F, s.random, xyz(s.visible_position), s.visible_normal, select_light_instance, D.info,
                               n_emitter, D.L);
    return true;
}
// the candidate block after its emitter walk (hit, traced: light_pick_walk's result), up to its shadow walk:
// returns whether the shadow ray (D.ray, cand's distances) is traced
template <bool EMISSIVE_LIT>
HKD bool direct_candidate_a(const Scene& sc, const DirectPixel& P, DirectState& D, const Hit& walk_hit, bool traced,
                            uint32_t& n_top)
{
    Sample& s = D.s;
    if (D.L.emitter) light_pick_end(sc, D.L, xyz(s.visible_position), walk_hit, traced, D.info);
    const LightCandidate& cand = D.L.cand;
    const f3 normal = P.normal;
    Ray& ray = D.ray;
    ray.origin = xyz(D.position) + normal * RAY_BIAS;
    ray.direction = cand.direction;
    ray.inv_direction = inv(ray.direction);
    bool trace = dot(cand.direction, normal) > 0.0f && cand.p > 0.0f;
    if (EMISSIVE_LIT) trace = trace && cand.emissive_instance != DONT_SAMPLE_EMISSIVE;
    if (trace) n_top++;
    return trace;
}
// ... and after the shadow walk (hit: its result, when traced)
template <bool EMISSIVE_LIT>
HKD void direct_candidate_b(const FrameArgs& A, const Scene& sc, DirectState& D, bool trace, const Hit& hit)
{
    const Frame& F = A.F;
    Sample& s = D.s;
    const LightCandidate& cand = D.L.cand;
    const Ray& ray = D.ray;
    if (trace) {
        occlude_hit_info(ray, hit, D.info);
        s.radiance = EMISSIVE_LIT ? input_radiance(sc, F, ray, D.info, false, cand.emissive_instance, false)
                                  : input_radiance(sc, F, ray, D.info, true, DONT_SAMPLE_EMISSIVE, false);
    }
    s.sample_position = D.info.position;
    s.sample_normal = D.info.normal;
    float w_new = cand.p > 0.0f ? lum(xyz(s.radiance)) / cand.p : 0.0f;
    temporal_restir(D.r, s, w_new, F.max_temporal_reuse_count);
}
template <bool EMISSIVE_LIT>
HKD void direct_candidate(const FrameArgs& A, const Scene& sc, const DirectPixel& P, DirectState& D, const Hit& walk_hit,
                          bool traced, uint32_t& n_top)
{
    const bool trace = direct_candidate_a<EMISSIVE_LIT>(sc, P, D, walk_hit, traced, n_top);
    Hit hit;
    if (trace) hit = traverse_top(sc, D.ray, D.L.cand.max_distance, D.L.cand.min_distance, D.L.cand.emissive_instance);
    direct_candidate_b<EMISSIVE_LIT>(A, sc, D, trace, hit);
}

// PARK: 0 = the validation block keeps the reservoir in registers, 1 = parks it in a static LDS array,
// 2 = in the launch's dynamic LDS (k_light_merged: the direct and indirect workgroups share one buffer)
template <bool EMISSIVE_LIT, bool RENDER_EMISSIVE, bool VALIDATE = true, int PARK = 0>
HKD void direct_finish(const FrameArgs& A, const Scene& sc, const ChannelArgs& C, const DirectPixel& P, DirectState& D,
                       uint32_t& n_top, uint32_t& n_emitter, Surface* surface_out = nullptr,
                       const Surface* surface_in = nullptr)
{
    const Frame& F = A.F;
    const int32_t idx = P.idx;
    const f4 position = D.position;
    Sample& s = D.s;
    Reservoir& r = D.r;
    HitInfo& info = D.info;
    Ray& ray = D.ray;
    const f2 previous_uv = D.previous_uv;
    const uint32_t im_x = f2u32(P.imf.x), im_y = f2u32(P.imf.y);
    const f4 velocity_uv = P.velocity_uv;
    const uint32_t validate_interval = EMISSIVE_LIT ? F.emissive_validate_interval : F.direct_validate_interval;
    const uint32_t select_light_instance = EMISSIVE_LIT ? im_x : DONT_SAMPLE_EMISSIVE;

    if (VALIDATE && umod(F.number, validate_interval) == 0u) {
        float* lds = nullptr;
        if constexpr (PARK) {
            lds = PARK == 2 ? reinterpret_cast<float*>(hk_lds_scene) : park_area();
            park_sample(lds, s);
            park_reservoir(lds, r);
        }
        LightCandidate cand;
        {
            const Reservoir rv = PARK ? unpark_reservoir(lds) : r;  // the fields the walks need
            cand = select_light_candidate<true>(sc, F, rv.s.random, xyz(rv.s.visible_position), rv.s.visible_normal,
                                                select_light_instance, info, n_emitter);
            ray.origin = xyz(s.visible_position) + s.visible_normal * RAY_BIAS;
            ray.direction = normalize(xyz(rv.s.sample_position) - xyz(s.visible_position));
            ray.inv_direction = inv(ray.direction);
        }
        // (r.s.visible_normal for the trace test below comes back with the reservoir)
        f4 validate_radiance = mk4(0, 0, 0, 0);
        bool trace;
        if constexpr (PARK) {
            const f3 vn = mk3(lds[12 * 256 + threadIdx.x], lds[13 * 256 + threadIdx.x], lds[14 * 256 + threadIdx.x]);
            trace = dot(cand.direction, vn) > 0.0f && cand.p > 0.0f;
        } else {
            trace = dot(cand.direction, r.s.visible_normal) > 0.0f && cand.p > 0.0f;
        }
        if (EMISSIVE_LIT) trace = trace && cand.emissive_instance != DONT_SAMPLE_EMISSIVE;
        if constexpr (PARK) __asm__ volatile("" ::: "memory");
        if (trace) {
            n_top++;
            Hit hit = traverse_top(sc, ray, cand.max_distance, cand.min_distance, cand.emissive_instance);
            occlude_hit_info(ray, hit, info);
            validate_radiance = EMISSIVE_LIT ? input_radiance(sc, F, ray, info, false, cand.emissive_instance, false)
                                             : input_radiance(sc, F, ray, info, true, DONT_SAMPLE_EMISSIVE, false);
        }
        if constexpr (PARK) {
            __asm__ volatile("" ::: "memory");
            r = unpark_reservoir(lds);
            unpark_sample(lds, s);
        }
        if (r.count >= 4.0f) {
            s.random = r.s.random;
            s.sample_position = info.position;
            s.sample_normal = info.normal;
            s.radiance = validate_radiance;
        }
        float ratio = lum(xyz(validate_radiance)) / fmaxf(lum(xyz(r.s.radiance)), 0.0001f);
        if (ratio > 1.25f || ratio < 0.8f) {
            if (uv_inside_closed(previous_uv)) {
                int32_t px = f2i32(previous_uv.x * (float)F.s[0]);
                int32_t py = f2i32(previous_uv.y * (float)F.s[1]);
                store_res(C.prev_spatial, s_index(F, px, py), r);
            }
            float w_new = cand.p > 0.0f ? lum(xyz(s.radiance)) / cand.p : 0.0f;
            set_reservoir(r, s, w_new);
        }
    }

    float total_lum = r.count * lum(xyz(r.s.radiance));
    r.w = total_lum > 0.0f ? r.w_sum / total_lum : 0.0f;
    r.s.visible_position = s.visible_position;
    r.s.visible_normal = s.visible_normal;
    r.lifetime += 1.0f;
    C.variance[idx] = variance_of(r);
    if (F.temporal_reuse > 0u) store_res(C.cur, idx, r);

    Surface surface = surface_in ? *surface_in : retreive_surface(sc, im_y, mk2(velocity_uv.z, velocity_uv.w));
    if (surface_out) *surface_out = surface;
    f3 view_direction = calculate_view(F, position);
    f3 out = shading(F, view_direction, r.s.visible_normal, normalize(xyz(r.s.sample_position) - xyz(r.s.visible_position)),
                     surface, r.s.radiance);
    out = out * r.w;
    if (RENDER_EMISSIVE) out = out + emissive_radiance(surface.emissive);
    store_rgba16f(C.render, idx, mk4(out.x, out.y, out.z, 1.0f));
}


template <bool EMISSIVE_LIT, bool RENDER_EMISSIVE, bool VALIDATE = true, int PARK = 0>
HKD void direct_body(const FrameArgs& A, const Scene& sc, const ChannelArgs& C, const DirectPixel P, uint32_t& n_top,
                     uint32_t& n_emitter, Surface* surface_out = nullptr, const Surface* surface_in = nullptr)
{
    DirectState D;
    if (!direct_begin<EMISSIVE_LIT, RENDER_EMISSIVE, VALIDATE>(A, sc, C, P, D, n_emitter)) return;
    if (D.cand_block) {
        Hit hit;
        bool traced = false;
        if (D.L.emitter) traced = light_pick_walk(sc, D.L, hit);
        direct_candidate<EMISSIVE_LIT>(A, sc, P, D, hit, traced, n_top);
    }
    direct_finish<EMISSIVE_LIT, RENDER_EMISSIVE, VALIDATE, PARK>(A, sc, C, P, D, n_top, n_emitter, surface_out, surface_in);
}

// Background store elision (ChannelArgs::bg).  A background pixel (G-buffer depth 0, or every
// pixel of an indirect pass with no bounces) stores the same constant words on every frame: the
// zero reservoir into the pass's temporal buffer and both spatial buffers, variance 0 and a zero
// render texel (light.wgsl:1063-1071, 1283-1290).  The mask byte says which physical targets got
// those words on an earlier frame and have not been written since; targets that all have are not
// stored again — every buffer still ends the frame with the reference's bits.  A covered pixel
// writes other values, so it clears its byte.  When the channel's spatial reuse runs, it rewrites
// the spatial buffer with a repacked copy of the temporal record (light.wgsl:1566-1574: other
// bits for the zero normal), so the pair alternates between two words and is stored every frame
// (bg_need without BG_PAIR).  The runtime resets the mask whenever anything else may have written
// these targets (a launch without the mask, reservoir uploads, reallocation, another pass window).
enum BgElide : uint32_t { BG_STORE = 0, BG_SKIP_OWN = 1, BG_SKIP_ALL = 2 };
constexpr uint32_t BG_PAIR = 16u;
HKD uint32_t bg_elide(const ChannelArgs& C, int32_t idx, bool background)
{
    if (!C.bg) return BG_STORE;
    const uint32_t m = C.bg[idx];
    if (!background) {
        if (m) C.bg[idx] = 0;
        return BG_STORE;
    }
    const uint32_t own = C.bg_need & 15u, pair = C.bg_need & BG_PAIR;
    const uint32_t nm = (m & 15u) | own | pair;
    if (nm != m) C.bg[idx] = (uint8_t)nm;
    if ((m & own) != own) return BG_STORE;
    return (pair && (m & BG_PAIR)) ? BG_SKIP_ALL : BG_SKIP_OWN;
}
HKD Reservoir background_reservoir()
{
    Reservoir r = zero_reservoir();
    set_reservoir(r, zero_sample(), 0.0f);
    return r;
}

// The separate direct_lit / emissive launches share the pair's mask (ChannelArgs::bg of both):
// direct_lit, first on the stream, only reads it (its targets are among the bits); the emissive
// pass, which stores after it into the spatial pair, updates it for both.  Both classify a pixel
// from the same G-buffer texel, so they agree on which pixels are background.
template <bool EMISSIVE_LIT, bool RENDER_EMISSIVE, bool VALIDATE>
HKD void direct_pass(const FrameArgs& A, const Scene& sc, const ChannelArgs& C, int32_t x, int32_t y, uint32_t& n_top,
                     uint32_t& n_emitter, const PixelTexels* tex = nullptr)
{
    const DirectPixel P = tex ? direct_pixel_of(A, x, y, *tex) : load_direct_pixel(A, x, y);
    const bool background = P.pd.w < HK_F32_EPSILON;
    if constexpr (!EMISSIVE_LIT) {
        if (C.bg && background && (C.bg[P.idx] & (C.bg_need & 15u)) == (C.bg_need & 15u)) return;
    } else {
        const uint32_t bg = bg_elide(C, P.idx, background);
        if (bg == BG_SKIP_ALL) return;
        if (bg == BG_SKIP_OWN) {
            const Reservoir z = background_reservoir();
            store_res(C.spatial, P.idx, z);
            store_res(C.prev_spatial, P.idx, z);
            return;
        }
    }
    direct_body<EMISSIVE_LIT, RENDER_EMISSIVE, VALIDATE>(A, sc, C, P, n_top, n_emitter);
}

template <bool EMISSIVE_LIT, bool RENDER_EMISSIVE, bool LDS, bool VALIDATE>
__global__ __launch_bounds__(256) void k_direct(FrameArgs A, ChannelArgs C)
{
    int32_t x, y;
    const bool active = tile_pixel<TRACE_ORDER>(A.F, A.F.s[0], A.F.s_row0, A.F.s_rows, x, y);
    PixelTexels tex;
    if (active) tex = load_pixel_texels(A, x, y);
    Scene sc;
    if constexpr (LDS) sc = stage_scene<PLAN_LIGHT>(A.sc, hk_lds_scene);
    else sc = A.sc;
    uint32_t n_top = 0, n_emitter = 0;
    if (active) direct_pass<EMISSIVE_LIT, RENDER_EMISSIVE, VALIDATE>(A, sc, C, x, y, n_top, n_emitter, &tex);
    if (!counted(A.F, x, y)) n_top = n_emitter = 0;
    wave_count(A.cnt.top, n_top);
    wave_count(A.cnt.emitter, n_emitter);
}

// direct_lit alone (no emissive sampling) fits 128 VGPRs with at most a few scratch words: the
// same body with 4 waves per SIMD for the separate-launch path (bands / stripes) when the grid
// has enough waves to use them (>= 400 K pixels): cornell 2-way stripe 0.348 -> 0.328 ms/frame,
// 4-way 0.192 -> 0.187; an 8-way stripe (259 K pixels, about one wave per slot) 0.1455 -> 0.1474
// (the threshold is LaunchOpts::direct_w4_min_px)
template <bool LDS, bool VALIDATE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_direct_lit_w4(FrameArgs A, ChannelArgs C)
{
    int32_t x, y;
    const bool active = tile_pixel<TRACE_ORDER>(A.F, A.F.s[0], A.F.s_row0, A.F.s_rows, x, y);
    PixelTexels tex;
    if (active) tex = load_pixel_texels(A, x, y);
    Scene sc;
    if constexpr (LDS) sc = stage_scene<PLAN_LIGHT>(A.sc, hk_lds_scene);
    else sc = A.sc;
    uint32_t n_top = 0, n_emitter = 0;
    if (active) direct_pass<false, true, VALIDATE>(A, sc, C, x, y, n_top, n_emitter, &tex);
    if (!counted(A.F, x, y)) n_top = n_emitter = 0;
    wave_count(A.cnt.top, n_top);
    wave_count(A.cnt.emitter, n_emitter);
}

// direct_lit then the emissive pass in one launch, each thread running both passes for its pixel
// in the reference's pass order.  Both passes store into the spatial reservoir pair they share
// only at their own pixel when the reprojection is the identity (zero velocity at upscale ratio
// 1: the G-buffer of k_gbuffer), so per-thread program order is the reference's pass order for
// every stored word; the runtime uses it only then.  One launch and one tail instead of two.
template <bool LDS, bool VD, bool VE>
__global__ __launch_bounds__(256) void k_direct_fused(FrameArgs A, ChannelArgs C0, ChannelArgs C1)
{
    int32_t x, y;
    const bool active = tile_pixel<TRACE_ORDER>(A.F, A.F.s[0], A.F.s_row0, A.F.s_rows, x, y);
    PixelTexels tex;
    if (active) tex = load_pixel_texels(A, x, y);  // in flight during the staging
    Scene sc;
    if constexpr (LDS) sc = stage_scene<PLAN_LIGHT>(A.sc, hk_lds_scene);
    else sc = A.sc;
    uint32_t n_top = 0, n_emitter = 0;
    if (active) {
        const DirectPixel P = direct_pixel_of(A, x, y, tex);
        const uint32_t bg = bg_elide(C0, P.idx, P.pd.w < HK_F32_EPSILON);
        if (bg == BG_SKIP_OWN) {  // the emissive pass's stores into the spatial pair (direct_body)
            const Reservoir z = background_reservoir();
            store_res(C1.spatial, P.idx, z);
            store_res(C1.prev_spatial, P.idx, z);
        } else if (bg == BG_STORE) {
            // the pixel's surface (same material and uv in both passes) is fetched once
            Surface surface;
            direct_body<false, true, VD, !LDS>(A, sc, C0, P, n_top, n_emitter, &surface);
            direct_body<true, false, VE, !LDS>(A, sc, C1, P, n_top, n_emitter, nullptr, &surface);
        }
    }
    if (!counted(A.F, x, y)) n_top = n_emitter = 0;
    wave_count(A.cnt.top, n_top);
    wave_count(A.cnt.emitter, n_emitter);
}

// The fused launch on frames that are not emissive-validation frames, held to 4 waves per SIMD
// (128 VGPRs): without the emissive validation block the body needs 117-137 VGPRs (the direct
// validation block on every third frame), a few of which then spill.
// With the validation blocks parked in LDS (non-LDS-scene variants) the emissive
// validation frames take this 4-wave kernel too (VE).
template <bool LDS, bool VD, bool VE = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_direct_fused_w4(FrameArgs A, ChannelArgs C0,
                                                                                                   ChannelArgs C1)
{
    int32_t x, y;
    const bool active = tile_pixel<TRACE_ORDER>(A.F, A.F.s[0], A.F.s_row0, A.F.s_rows, x, y);
    PixelTexels tex;
    if (active) tex = load_pixel_texels(A, x, y);  // in flight during the staging
    Scene sc;
    if constexpr (LDS) sc = stage_scene<PLAN_LIGHT>(A.sc, hk_lds_scene);
    else sc = A.sc;
    uint32_t n_top = 0, n_emitter = 0;
    if (active) {
        const DirectPixel P = direct_pixel_of(A, x, y, tex);
        const uint32_t bg = bg_elide(C0, P.idx, P.pd.w < HK_F32_EPSILON);
        if (bg == BG_SKIP_OWN) {  // the emissive pass's stores into the spatial pair (direct_body)
            const Reservoir z = background_reservoir();
            store_res(C1.spatial, P.idx, z);
            store_res(C1.prev_spatial, P.idx, z);
        } else if (bg == BG_STORE) {
            // the pixel's surface (same material and uv in both passes) is fetched once
            Surface surface;
            direct_body<false, true, VD, !LDS>(A, sc, C0, P, n_top, n_emitter, &surface);
            direct_body<true, false, VE, !LDS>(A, sc, C1, P, n_top, n_emitter, nullptr, &surface);
        }
    }
    if (!counted(A.F, x, y)) n_top = n_emitter = 0;
    wave_count(A.cnt.top, n_top);
    wave_count(A.cnt.emitter, n_emitter);
}

// Emitter walks of a workgroup as one compacted batch (the CW variant of the fused launch).  In city the
// emissive pass picks an emitter for ~3 of 4 covered pixels: mostly the small lamp meshes (a 3-visit BLAS
// walk) and for ~13 % the emissive sphere (13-180 visits).  A wave runs the walk until its longest lane
// ends, so the one or two sphere walkers in most waves kept the whole wave in the walk: SIMD lane efficiency
// 0.14 (tools/walk_lanes.py, oracle statistics of city frames).  Here the workgroup's walk requests are
// written to LDS, queued long walks first (emitter BLAS with more than CW_LONG_NODES nodes) then short ones,
// and thread t runs queue entry t: the long walks of the 4 waves share one or two waves (model: 0.35).  A
// walk's result does not depend on the thread that runs it, so the results are those of the per-pixel walk.
constexpr uint32_t CW_LONG_NODES = 16u;
// LDS of a compacted batch: 9 rows of one word per thread (a request: local origin 3, direction 3, BLAS node
// offset, node count, primitive offset; then the result over it) and a row for the queue.  With the direct
// validation block (VD) these are rows of its park columns: a thread writes its own column's request only
// after its own park ended, and the queue / results only after the batch's first barrier, which every
// thread reaches after its park ended; the per-wave counts have their own array (written before it).
constexpr int CW_WORDS = 10;
static_assert(CW_WORDS <= PARK_WORDS, "the batch rows fit the park columns");
HKD float* cw_area()
{
    __shared__ float cw[CW_WORDS * 256];
    return cw;
}
// every thread of the workgroup calls this at the same point (barriers); need = the thread's pixel walks
HKD bool compact_emitter_walks(const Scene& sc, float* lds, const LightPick& L, bool need, Hit& hit)
{
    uint32_t* const queue = reinterpret_cast<uint32_t*>(lds + 9 * 256);
    __shared__ uint32_t wave_counts[8];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    uint32_t node_offset = 0u, node_count = 0u;
    if (need) {
        const hk_instance& ein = get_instance(sc, L.cand.emissive_instance);
        node_offset = ein.mesh.node[0];
        node_count = ein.mesh.node[1];
        lds[0 * 256 + t] = L.local.origin.x;
        lds[1 * 256 + t] = L.local.origin.y;
        lds[2 * 256 + t] = L.local.origin.z;
        lds[3 * 256 + t] = L.local.direction.x;
        lds[4 * 256 + t] = L.local.direction.y;
        lds[5 * 256 + t] = L.local.direction.z;
        lds[6 * 256 + t] = __uint_as_float(node_offset);
        lds[7 * 256 + t] = __uint_as_float(node_count);
        lds[8 * 256 + t] = __uint_as_float(ein.mesh.primitive);
    }
    const bool lng = need && node_count > CW_LONG_NODES;
    const uint64_t m_long = __ballot(lng), m_short = __ballot(need && !lng);
    if (lane == 0u) {
        wave_counts[2u * w] = (uint32_t)__popcll(m_long);
        wave_counts[2u * w + 1u] = (uint32_t)__popcll(m_short);
    }
    __syncthreads();
    uint32_t n_long = 0u, n_short = 0u, below_long = 0u, below_short = 0u;
#pragma unroll
    for (uint32_t k = 0; k < 4u; ++k) {
        const uint32_t a = wave_counts[2u * k], b = wave_counts[2u * k + 1u];
        below_long += k < w ? a : 0u;
        below_short += k < w ? b : 0u;
        n_long += a;
        n_short += b;
    }
    if (need) {
        const uint64_t below = (1ull << lane) - 1ull;
        const uint32_t pos = lng ? below_long + (uint32_t)__popcll(m_long & below)
                                 : n_long + below_short + (uint32_t)__popcll(m_short & below);
        queue[pos] = t;
    }
    __syncthreads();
    if (t < n_long + n_short) {
        const uint32_t o = queue[t];
        Ray r;
        r.origin = mk3(lds[0 * 256 + o], lds[1 * 256 + o], lds[2 * 256 + o]);
        r.direction = mk3(lds[3 * 256 + o], lds[4 * 256 + o], lds[5 * 256 + o]);
        r.inv_direction = inv(r.direction);
        Hit h;
        h.uv = mk2(0, 0);
        h.distance = HK_F32_MAX;
        h.instance_index = HK_U32_MAX;
        h.primitive_index = HK_U32_MAX;
        const bool traced = traverse_bottom(sc, h, r, __float_as_uint(lds[6 * 256 + o]), __float_as_uint(lds[7 * 256 + o]),
                                            __float_as_uint(lds[8 * 256 + o]), 0.0f);
        // the result over the request's own slots (read only by this thread)
        lds[0 * 256 + o] = h.uv.x;
        lds[1 * 256 + o] = h.uv.y;
        lds[2 * 256 + o] = h.distance;
        lds[3 * 256 + o] = __uint_as_float(h.primitive_index);
        lds[4 * 256 + o] = traced ? 1.0f : 0.0f;
    }
    __syncthreads();
    hit.uv = mk2(0, 0);
    hit.distance = HK_F32_MAX;
    hit.instance_index = HK_U32_MAX;
    hit.primitive_index = HK_U32_MAX;
    if (!need) return false;
    hit.uv = mk2(lds[0 * 256 + t], lds[1 * 256 + t]);
    hit.distance = lds[2 * 256 + t];
    hit.primitive_index = __float_as_uint(lds[3 * 256 + t]);
    return lds[4 * 256 + t] != 0.0f;
}

// Shadow walks (traverse_top any-hit) of a workgroup as one compacted batch: the lanes that trace a shadow
// ray are a scattered subset of the workgroup (cornell: the direct_lit pass's lanes that face the light,
// the indirect pass's bounces that hit a surface and pick a light), and a wave with a few of them runs the
// walk for all 64 lanes.  Requests go to LDS (origin, direction, max / early distance, excluded instance),
// packed in pixel order, and thread t runs request t (model: cornell direct_lit 0.31 -> 0.53 of the lanes
// busy, indirect emissive shadows 0.25 -> 0.41; tools/walk_lanes.py).  The walk's result depends only on
// the request, so it is the per-pixel walk's.
// (LDS: the rows of compact_emitter_walks, cw_area / park columns)
HKD bool compact_top_walks(const Scene& sc, float* lds, bool need, const Ray& ray, float max_distance, float early_distance,
                           uint32_t exclude, Hit& hit)
{
    uint32_t* const ct_queue = reinterpret_cast<uint32_t*>(lds + 9 * 256);
    __shared__ uint32_t ct_counts[4];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    if (need) {
        lds[0 * 256 + t] = ray.origin.x;
        lds[1 * 256 + t] = ray.origin.y;
        lds[2 * 256 + t] = ray.origin.z;
        lds[3 * 256 + t] = ray.direction.x;
        lds[4 * 256 + t] = ray.direction.y;
        lds[5 * 256 + t] = ray.direction.z;
        lds[6 * 256 + t] = max_distance;
        lds[7 * 256 + t] = early_distance;
        lds[8 * 256 + t] = __uint_as_float(exclude);
    }
    const uint64_t m = __ballot(need);
    if (lane == 0u) ct_counts[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t n = 0u, below = 0u;
#pragma unroll
    for (uint32_t k = 0; k < 4u; ++k) {
        const uint32_t a = ct_counts[k];
        below += k < w ? a : 0u;
        n += a;
    }
    if (need) ct_queue[below + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = t;
    __syncthreads();
    if (t < n) {
        const uint32_t o = ct_queue[t];
        Ray r;
        r.origin = mk3(lds[0 * 256 + o], lds[1 * 256 + o], lds[2 * 256 + o]);
        r.direction = mk3(lds[3 * 256 + o], lds[4 * 256 + o], lds[5 * 256 + o]);
        r.inv_direction = inv(r.direction);
        const Hit h = traverse_top(sc, r, lds[6 * 256 + o], lds[7 * 256 + o], __float_as_uint(lds[8 * 256 + o]));
        lds[0 * 256 + o] = h.uv.x;
        lds[1 * 256 + o] = h.uv.y;
        lds[2 * 256 + o] = h.distance;
        lds[3 * 256 + o] = __uint_as_float(h.instance_index);
        lds[4 * 256 + o] = __uint_as_float(h.primitive_index);
    }
    __syncthreads();
    if (!need) return false;
    hit.uv = mk2(lds[0 * 256 + t], lds[1 * 256 + t]);
    hit.distance = lds[2 * 256 + t];
    hit.instance_index = __float_as_uint(lds[3 * 256 + t]);
    hit.primitive_index = __float_as_uint(lds[4 * 256 + t]);
    return true;
}

// k_direct_fused_w4 on the frames that validate neither pass's emitter picks (VE false) with the emissive
// pass's emitter walks compacted per workgroup (compact_emitter_walks).  Every thread reaches the barriers:
// the pixel's work is predicated, not returned from.  The walk requests live in the direct validation
// block's park columns when that block runs (VD: a thread's own column, written after its own block ended)
// or in their own LDS array.
template <bool VD, bool SHADOW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_direct_fused_cw(FrameArgs A, ChannelArgs C0,
                                                                                                   ChannelArgs C1)
{
    const Scene& sc = A.sc;
    float* lds = VD ? park_area() : cw_area();
    int32_t x, y;
    uint32_t n_top = 0, n_emitter = 0;
    const bool on = tile_pixel<TRACE_ORDER>(A.F, A.F.s[0], A.F.s_row0, A.F.s_rows, x, y);
    DirectPixel P;
    uint32_t bg = BG_SKIP_ALL;
    if (on) {
        P = direct_pixel_of(A, x, y, load_pixel_texels(A, x, y));
        bg = bg_elide(C0, P.idx, P.pd.w < HK_F32_EPSILON);
        if (bg == BG_SKIP_OWN) {  // the emissive pass's stores into the spatial pair (direct_body)
            const Reservoir z = background_reservoir();
            store_res(C1.spatial, P.idx, z);
            store_res(C1.prev_spatial, P.idx, z);
        }
    }
    const bool work = on && bg == BG_STORE;
    Surface surface;
    DirectState D;
    bool lit = false;
    if constexpr (SHADOW) {
        // direct_lit with its candidate block's shadow walk compacted (its validation block, every
        // direct_validate_interval-th frame, walks per pixel)
        bool cand = false, trace = false;
        if (work) {
            lit = direct_begin<false, true, VD>(A, sc, C0, P, D, n_emitter);
            cand = lit && D.cand_block;
            Hit none;
            if (cand) trace = direct_candidate_a<false>(sc, P, D, none, false, n_top);
        }
        Hit sh;
        compact_top_walks(sc, lds, trace, D.ray, D.L.cand.max_distance, D.L.cand.min_distance, D.L.cand.emissive_instance, sh);
        if (cand) direct_candidate_b<false>(A, sc, D, trace, sh);
        if (lit) direct_finish<false, true, VD, 1>(A, sc, C0, P, D, n_top, n_emitter, &surface);
        lit = false;
        if (work) lit = direct_begin<true, false, false>(A, sc, C1, P, D, n_emitter);
    } else if (work) {
        direct_body<false, true, VD, 1>(A, sc, C0, P, n_top, n_emitter, &surface);
        lit = direct_begin<true, false, false>(A, sc, C1, P, D, n_emitter);
    }
    Hit hit;
    const bool traced = compact_emitter_walks(sc, lds, D.L, lit && D.L.walk, hit);
    if constexpr (SHADOW) {
        bool trace = false;
        if (lit) trace = direct_candidate_a<true>(sc, P, D, hit, traced, n_top);
        Hit sh;
        compact_top_walks(sc, lds, trace, D.ray, D.L.cand.max_distance, D.L.cand.min_distance, D.L.cand.emissive_instance, sh);
        if (lit) {
            direct_candidate_b<true>(A, sc, D, trace, sh);
            direct_finish<true, false, false, 0>(A, sc, C1, P, D, n_top, n_emitter, nullptr, &surface);
        }
    } else if (lit) {
        direct_candidate<true>(A, sc, P, D, hit, traced, n_top);
        direct_finish<true, false, false, 0>(A, sc, C1, P, D, n_top, n_emitter, nullptr, &surface);
    }
    if (!counted(A.F, x, y)) n_top = n_emitter = 0;
    wave_count(A.cnt.top, n_top);
    wave_count(A.cnt.emitter, n_emitter);
}

// ------------------------------------------------------------------ indirect_lit_ambient (light.wgsl:1263-1498)
// The pass runs either as one megakernel (IND_ALL: one thread per pixel, start to end) or as the
// wavefront pipeline of config 5 (WfArgs below): IND_GEN (the dead-pixel stores; live pixels go to a
// compacted queue), IND_TRACE (the cosine bounce's closest hit, stored as an SoA hit record, keyed
// by the hit's material), IND_SHADE (in material order: the rest of the pass from the stored hit).
// The stages run the same statements in the same order for a pixel, so results are identical.
enum IndStage : int { IND_ALL = 0, IND_GEN = 1, IND_TRACE = 2, IND_SHADE = 3 };
HKD void wf_store_hit(const WfArgs& W, int32_t idx, const Hit& h)
{
    W.hit[idx] = make_uint4(h.instance_index, h.primitive_index, __float_as_uint(h.uv.x), __float_as_uint(h.uv.y));
    W.hit_t[idx] = h.distance;
}
HKD Hit wf_load_hit(const WfArgs& W, int32_t idx)
{
    const uint4 v = W.hit[idx];
    Hit h;
    h.instance_index = v.x;
    h.primitive_index = v.y;
    h.uv = mk2(__uint_as_float(v.z), __uint_as_float(v.w));
    h.distance = W.hit_t[idx];
    return h;
}
// indirect_lit_ambient's one-bounce path (light.wgsl:1300-1394 with indirect_bounces 1) in pieces around its
// two walks, so that a kernel can run the shadow walks of a workgroup as one compacted batch (k_indirect's CS
// variant): bounce_ray builds the cosine bounce, bounce_hit_a runs everything from the bounce's hit to the
// shadow ray (hit_info, the hit's surface, select_light_candidate), bounce_hit_b everything after the shadow
// walk.  indirect_body runs them with the walks in between: the same statements in the same order.
struct BounceState {
    Sample s;
    Ray ray;
    HitInfo info;
    Surface surface;
    LightCandidate cand;
    bool hit, sample_directional;
};
HKD f4 bounce_ray(BounceState& B)
{
    const Sample& s = B.s;
    f4 rs = sample_cosine_hemisphere(mk2(s.random.x, s.random.y));
    B.ray.origin = xyz(s.visible_position) + s.visible_normal * RAY_BIAS;
    f3 bt, bb;
    normal_basis(s.visible_normal, bt, bb);
    B.ray.direction = basis_mul(bt, bb, s.visible_normal, xyz(rs));
    B.ray.inv_direction = inv(B.ray.direction);
    return rs;
}
// returns whether the shadow ray (B.ray, B.cand's distances and instance) is traced
HKD bool bounce_hit_a(const Scene& sc, const Frame& F, BounceState& B, const Hit& hit, uint32_t& n_top, uint32_t& n_emitter)
{
    Sample& s = B.s;
    HitInfo& info = B.info;
    info = hit_info(sc, B.ray, hit);
    s.sample_position = info.position;
    s.sample_normal = info.normal;
    B.hit = hit.instance_index != HK_U32_MAX;
    if (!B.hit) return false;
    B.surface = retreive_surface(sc, info.material_index, info.uv);
    B.surface.roughness = 1.0f;
    B.cand = select_light_candidate<true>(sc, F, s.random, xyz(s.sample_position), s.sample_normal, info.instance_index,
                                          info, n_emitter);
    B.sample_directional = B.cand.emissive_instance == DONT_SAMPLE_EMISSIVE;
    if (!(dot(B.cand.direction, s.sample_normal) > 0.0f && B.cand.p > 0.0f)) return false;
    B.ray.origin = xyz(s.sample_position) + s.sample_normal * RAY_BIAS;
    B.ray.direction = B.cand.direction;
    B.ray.inv_direction = inv(B.ray.direction);
    n_top++;
    return true;
}
HKD void bounce_hit_b(const Scene& sc, const Frame& F, BounceState& B, bool shadow, const Hit& sh)
{
    Sample& s = B.s;
    if (B.hit) {
        if (shadow) {
            occlude_hit_info(B.ray, sh, B.info);
            f4 in_rad = input_radiance(sc, F, B.ray, B.info, B.sample_directional, B.cand.emissive_instance, false);
            f3 out = shading(F, normalize(xyz(s.visible_position) - xyz(s.sample_position)), s.sample_normal,
                             B.ray.direction, B.surface, in_rad);
            out = out / B.cand.p;
            s.radiance = mk4(s.radiance.x + out.x, s.radiance.y + out.y, s.radiance.z + out.z, s.radiance.w + 1.0f);
        }
    } else {
        f3 out = xyz(input_radiance(sc, F, B.ray, B.info, false, DONT_SAMPLE_EMISSIVE, true));
        s.radiance = mk4(s.radiance.x + out.x, s.radiance.y + out.y, s.radiance.z + out.z, s.radiance.w + 0.0f);
    }
}

// The pass up to the one-bounce path's shadow walk (I.shadow: whether it is traced; the multiple-bounce
// path runs its whole loop here).  Returns false when the pixel's pass ends here: a background pixel (its
// stores done), the IND_GEN / IND_TRACE stages (*ret: their result).
// The pixel's G-buffer and blue-noise fields, kept in LDS through the walks by the tile kernels (k_indirect,
// k_light_merged): indirect_end reads them back from there instead of from global memory (one thread's slot,
// struct-of-arrays so that a wave's 16-byte accesses are conflict-free)
struct IndStash {
    float4 pd[256];     // position, depth
    float4 vel[256];    // velocity, uv
    float4 rnd[256];    // s.random
    float4 nrm[256];    // normalize(normal), visible instance (bits)
    uint32_t im_y[256]; // material
};
struct IndirectState {
    BounceState B;
    int32_t x, y, idx;
    f2 uv;
    f4 position, velocity_uv;
    uint32_t im_y;
    float pdf;
    bool shadow;
};
template <bool MULTI, int STAGE = IND_ALL>
HKD bool indirect_begin(const FrameArgs& A, const Scene& sc, const ChannelArgs& C, int32_t x, int32_t y, uint32_t& n_top,
                        uint32_t& n_emitter, const WfArgs* W, uint32_t* key, IndirectState& I, bool& ret,
                        IndStash* stash = nullptr, const PixelTexels* tex = nullptr)
{
    static_assert(!MULTI || STAGE == IND_ALL, "the wavefront stages cover one bounce");
    I.shadow = false;
    ret = false;
    const Frame& F = A.F;
    const int32_t idx = s_index(F, x, y);
    const f2 uv = coords_to_uv(x, y, F.s);
    int32_t dx, dy;
    jittered_coords(F, uv, dx, dy);
    f4 pd = tex ? mk4(tex->pd.x, tex->pd.y, tex->pd.z, tex->pd.w) : load_position(F, A.G, dx, dy);
    f4 position = mk4(pd.x, pd.y, pd.z, 1.0f);
    float depth = pd.w;
    Sample s = zero_sample();
    Reservoir r = zero_reservoir();
    const bool background = F.indirect_bounces == 0u || depth < HK_F32_EPSILON;
    uint32_t bg = BG_STORE;
    if constexpr (STAGE == IND_ALL || STAGE == IND_GEN) bg = bg_elide(C, idx, background);
    if (background) {
        if constexpr (STAGE == IND_ALL || STAGE == IND_GEN) {
            if (bg != BG_SKIP_ALL) {
                store_res(C.spatial, idx, r);
                store_res(C.prev_spatial, idx, r);
            }
            if (bg == BG_STORE) {
                store_res(C.cur, idx, r);
                C.variance[idx] = 0.0f;
                store_rgba16f(C.render, idx, mk4(0, 0, 0, 0));
            }
        }
        return false;
    }
    if constexpr (STAGE == IND_GEN) {
        ret = true;
        return false;
    }
    f3 normal = normalize(tex ? texel_normal(tex->normal) : load_normal(F, A.G, dx, dy));
    f2 imf = tex ? mk2(tex->imf.x, tex->imf.y) : load_instance_material(F, A.G, dx, dy);
    uint32_t im_x = f2u32(imf.x), im_y = f2u32(imf.y);
    f4 velocity_uv = tex ? mk4(tex->vel.x, tex->vel.y, tex->vel.z, tex->vel.w) : load_velocity_uv(F, A.G, dx, dy);

    s.random = tex ? noise_of(tex->noise, F.number) : noise_random(A.noise, F.number, x, y);
    s.visible_position = mk4(position.x, position.y, position.z, depth);
    s.visible_normal = normal;
    s.visible_instance = im_x;
    if (stash) {
        const uint32_t t = threadIdx.x;
        stash->pd[t] = make_float4(pd.x, pd.y, pd.z, pd.w);
        stash->vel[t] = make_float4(velocity_uv.x, velocity_uv.y, velocity_uv.z, velocity_uv.w);
        stash->rnd[t] = make_float4(s.random.x, s.random.y, s.random.z, s.random.w);
        stash->nrm[t] = make_float4(normal.x, normal.y, normal.z, __uint_as_float(im_x));
        stash->im_y[t] = im_y;
    }

    Ray ray;
    HitInfo info;
    float pdf = 0.0f;
    Surface surface;

    if (MULTI) {
        Sample bs = s;
        f3 ct = mk3(1.0f, 1.0f, 1.0f);
        for (uint32_t n = 0u; n < F.indirect_bounces && (ct.x > 0.01f || ct.y > 0.01f || ct.z > 0.01f); n += 1u) {
            f4 rs = sample_cosine_hemisphere(mk2(bs.random.x, bs.random.y));
            ray.origin = xyz(bs.visible_position) + bs.visible_normal * RAY_BIAS;
            f3 bt, bb;
            normal_basis(bs.visible_normal, bt, bb);
            ray.direction = basis_mul(bt, bb, bs.visible_normal, xyz(rs));
            ray.inv_direction = inv(ray.direction);
            n_top++;
            Hit hit = traverse_top(sc, ray, HK_F32_MAX, 0.0f, DONT_EXCLUDE);
            info = hit_info(sc, ray, hit);
            if (n == 0u) {
                s.sample_position = info.position;
                s.sample_normal = info.normal;
                pdf = rs.w;
            }
            bs.sample_position = info.position;
            bs.sample_normal = info.normal;
            if (hit.instance_index != HK_U32_MAX) {
                f3 out = mk3(0, 0, 0);
                surface = retreive_surface(sc, info.material_index, info.uv);
                surface.roughness = 1.0f;
                LightCandidate cand = select_light_candidate<true>(sc, F, bs.random, xyz(bs.sample_position),
                                                                   bs.sample_normal, info.instance_index, info, n_emitter);
                bool sample_directional = cand.emissive_instance == DONT_SAMPLE_EMISSIVE;
                f3 bvd = normalize(xyz(bs.visible_position) - xyz(bs.sample_position));
                if (dot(cand.direction, bs.sample_normal) > 0.0f && cand.p > 0.0f) {
                    ray.origin = xyz(bs.sample_position) + bs.sample_normal * RAY_BIAS;
                    ray.direction = cand.direction;
                    ray.inv_direction = inv(ray.direction);
                    n_top++;
                    Hit sh = traverse_top(sc, ray, cand.max_distance, cand.min_distance, cand.emissive_instance);
                    occlude_hit_info(ray, sh, info);
                    f4 in_rad = input_radiance(sc, F, ray, info, sample_directional, cand.emissive_instance, false);
                    out = shading(F, bvd, bs.sample_normal, ray.direction, surface, in_rad);
                    out = out / cand.p;
                    if (n > 0u) out = rs.w < 0.01f ? mk3(0, 0, 0) : out / rs.w;
                    float ol = lum(out);
                    if (ol > F.max_indirect_luminance) out = (out * F.max_indirect_luminance) / ol;
                    f3 add = ct * out;
                    s.radiance = mk4(s.radiance.x + add.x, s.radiance.y + add.y, s.radiance.z + add.z, s.radiance.w + 1.0f);
                }
                ct = ct * env_brdf(bvd, bs.sample_normal, surface);
                float fn = (float)F.number * HK_GOLDEN_RATIO;
                bs.random = mk4(hk_fract(bs.random.x + fn), hk_fract(bs.random.y + fn), hk_fract(bs.random.z + fn),
                                hk_fract(bs.random.w + fn));
                bs.visible_position = bs.sample_position;
                bs.visible_normal = bs.sample_normal;
            } else {
                f3 out = xyz(input_radiance(sc, F, ray, info, false, DONT_SAMPLE_EMISSIVE, true));
                f3 add = ct * out;
                s.radiance = mk4(s.radiance.x + add.x, s.radiance.y + add.y, s.radiance.z + add.z, s.radiance.w + 0.0f);
                break;
            }
        }
    } else {
        BounceState B;
        B.s = s;
        B.ray = ray;
        Hit hit;
        const f4 rs = bounce_ray(B);
        if constexpr (STAGE == IND_SHADE) {
            hit = wf_load_hit(*W, idx);
        } else {
            n_top++;
            hit = traverse_top(sc, B.ray, HK_F32_MAX, 0.0f, DONT_EXCLUDE);
        }
        if constexpr (STAGE == IND_TRACE) {
            wf_store_hit(*W, idx, hit);
            *key = hit.instance_index != HK_U32_MAX ? min(get_instance(sc, hit.instance_index).material, W->bins - 2u) : W->bins - 1u;
            ret = true;
            return false;
        }
        pdf = rs.w;
        I.shadow = bounce_hit_a(sc, F, B, hit, n_top, n_emitter);
        I.B = B;
    }
    if (MULTI) I.B.s = s;
    I.x = x;
    I.y = y;
    I.idx = idx;
    I.uv = uv;
    I.position = position;
    I.velocity_uv = velocity_uv;
    I.im_y = im_y;
    I.pdf = pdf;
    return true;
}
// the rest of the pass after the shadow walk (sh: its result when I.shadow)
template <bool MULTI>
HKD void indirect_end(const FrameArgs& A, const Scene& sc, const ChannelArgs& C, IndirectState& I, const Hit& sh,
                      const IndStash* stash = nullptr)
{
    const Frame& F = A.F;
    if (!MULTI) bounce_hit_b(sc, F, I.B, I.shadow, sh);
    Sample& s = I.B.s;
    if (stash) {
        // the same fields from the thread's LDS slot (indirect_begin wrote them): no global round trip in the tail
        __asm__ volatile("" ::: "memory");
        const uint32_t t = threadIdx.x;
        const float4 pd = stash->pd[t], nv = stash->nrm[t], vel = stash->vel[t], rnd = stash->rnd[t];
        s.visible_position = mk4(pd.x, pd.y, pd.z, pd.w);
        s.visible_normal = mk3(nv.x, nv.y, nv.z);
        s.visible_instance = __float_as_uint(nv.w);
        s.random = mk4(rnd.x, rnd.y, rnd.z, rnd.w);
        I.position = mk4(pd.x, pd.y, pd.z, 1.0f);
        I.velocity_uv = mk4(vel.x, vel.y, vel.z, vel.w);
        I.im_y = stash->im_y[t];
    } else {
        // The pixel's G-buffer and blue-noise fields read again here — the same texels, so the same bits — behind
        // a compiler barrier, instead of being held in registers through both walks: with the previous record
        // read in two steps below, the pass's register peak (this tail) falls from 105 to 94 VGPRs, 4 -> 5 waves
        // per SIMD.  Cornell 1080p k_indirect 0.225 -> 0.211 ms, frame 0.408 -> 0.396 ms; city 4K 0.632 -> 0.607 ms
        // (profiles/r04/c7).
        __asm__ volatile("" ::: "memory");
        int32_t dx, dy;
        jittered_coords(F, I.uv, dx, dy);
        const f4 pd = load_position(F, A.G, dx, dy);
        s.visible_position = pd;
        s.visible_normal = normalize(load_normal(F, A.G, dx, dy));
        const f2 imf = load_instance_material(F, A.G, dx, dy);
        s.visible_instance = f2u32(imf.x);
        s.random = noise_random(A.noise, F.number, I.x, I.y);
        I.position = mk4(pd.x, pd.y, pd.z, 1.0f);
        I.velocity_uv = load_velocity_uv(F, A.G, dx, dy);
        I.im_y = f2u32(imf.y);
    }
    const int32_t idx = I.idx;
    const f2 uv = I.uv;
    const f4 position = I.position, velocity_uv = I.velocity_uv;
    const uint32_t im_y = I.im_y;
    const float pdf = I.pdf;
    Reservoir r;
    Surface surface;

    // load_previous + check_previous_reservoir + temporal_restir (light.wgsl:1460-1478) with the previous record
    // read in two steps: first the words the check and the merge weights read (chunk 3, the depth word of chunk 1,
    // the instance word of chunk 2), then — only when update_reservoir keeps the previous sample — the whole
    // record again.  C.prev is not written by this pass, so the second read returns the same bits: the same
    // reservoir, without the previous sample's registers live next to the new sample's shading.
    f2 juv = jittered_uv(F, uv, 0.25f);
    f2 previous_uv = mk2(juv.x - velocity_uv.x, juv.y - velocity_uv.y);
    const PrevHead ph = previous_head(F, C.prev, previous_uv, s);
    scatter_rejected(F, C.prev_spatial, previous_uv, ph);
    float r_count = ph.count, r_lifetime = ph.lifetime, r_w_sum = ph.w_sum, r_w2_sum = ph.w2_sum;
    surface = retreive_surface(sc, im_y, mk2(velocity_uv.z, velocity_uv.w));
    f3 view_direction = calculate_view(F, position);
    f3 sample_radiance = shading(F, view_direction, s.visible_normal,
                                 normalize(xyz(s.sample_position) - xyz(s.visible_position)), surface, s.radiance);
    float w_new = pdf > 0.0f ? lum(sample_radiance) / pdf : 0.0f;
    // temporal_restir: update_reservoir, then the clamp to max_temporal_reuse_count
    r_w_sum += w_new;
    r_w2_sum += w_new * w_new;
    r_count = r_count + 1.0f;
    const bool take = hk_fract(sum4(s.random)) < w_new / r_w_sum;
    {
        const float m = (float)F.max_temporal_reuse_count;
        if (r_count > m) {
            r_w_sum *= m / r_count;
            r_w2_sum *= m / r_count;
            r_count = m;
        }
    }
    if (take) r.s = s;
    else r.s = previous_record(C.prev, ph).s;
    r.count = r_count;
    r.lifetime = r_lifetime;
    r.w_sum = r_w_sum;
    r.w2_sum = r_w2_sum;
    f3 out = shading(F, view_direction, r.s.visible_normal, normalize(xyz(r.s.sample_position) - xyz(r.s.visible_position)),
                     surface, r.s.radiance);
    float total_lum = r.count * lum(out);
    r.w = total_lum > 0.0f ? r.w_sum / total_lum : 0.0f;
    r.s.visible_position = s.visible_position;
    r.s.visible_normal = s.visible_normal;
    r.lifetime += 1.0f;
    C.variance[idx] = variance_of(r);
    if (F.temporal_reuse > 0u) store_res_view(C.cur, C.view, C.view_n, idx, r);
    f3 o = out * r.w;
    store_rgba16f(C.render, idx, mk4(o.x, o.y, o.z, 1.0f));
}
// returns (IND_GEN) whether the pixel traces a bounce; (IND_TRACE) the hit's material bin in *key
template <bool MULTI, int STAGE = IND_ALL>
HKD bool indirect_body(const FrameArgs& A, const Scene& sc, const ChannelArgs& C, int32_t x, int32_t y, uint32_t& n_top,
                       uint32_t& n_emitter, const WfArgs* W = nullptr, uint32_t* key = nullptr, IndStash* stash = nullptr,
                       const PixelTexels* tex = nullptr)
{
    IndirectState I;
    bool ret;
    if (!indirect_begin<MULTI, STAGE>(A, sc, C, x, y, n_top, n_emitter, W, key, I, ret, stash, tex)) return ret;
    Hit sh;
    if (!MULTI && I.shadow)
        sh = traverse_top(sc, I.B.ray, I.B.cand.max_distance, I.B.cand.min_distance, I.B.cand.emissive_instance);
    indirect_end<MULTI>(A, sc, C, I, sh, stash);
    return true;
}

// CS: the one-bounce path's shadow walks compacted per workgroup (compact_top_walks; option compact_shadow)
template <bool MULTI, bool LDS, bool CS = false>
__global__ __launch_bounds__(256) void k_indirect(FrameArgs A, ChannelArgs C)
{
    int32_t x, y;
    const bool active = tile_pixel<TRACE_ORDER>(A.F, A.F.s[0], A.F.s_row0, A.F.s_rows, x, y);
    // The one-bounce variant without LDS staging (scene, city) loads all of its pixel's texels up front: one round
    // trip instead of the position's followed by the rest once the pixel is known to be covered (city 4K 0.536 ->
    // 0.497 ms, scene 0.251 -> 0.243, profiles/r06/c13).  The staged variant (cornell) does not: the texels live
    // across the staging took it 92 -> 99 VGPRs, 5 -> 4 waves per SIMD (0.178 -> 0.192 ms), and the position + noise
    // texels alone (95 VGPRs) measured 0.181.  The multi-bounce variants (no BASELINE config) keep their own loads.
    constexpr bool PRE = !MULTI && !LDS && !CS;
    PixelTexels tex;
    if (PRE && active) tex = load_pixel_texels(A, x, y);
    Scene sc = A.sc;
    if constexpr (LDS) {
        sc = stage_scene<PLAN_LIGHT>(A.sc, hk_lds_scene);
    }
    uint32_t n_top = 0, n_emitter = 0;
    if constexpr (CS && !MULTI) {
        IndirectState I;
        bool ret = false;
        const bool live = active && indirect_begin<false>(A, sc, C, x, y, n_top, n_emitter, nullptr, nullptr, I, ret);
        Hit sh;
        compact_top_walks(sc, cw_area(), live && I.shadow, I.B.ray, I.B.cand.max_distance, I.B.cand.min_distance,
                          I.B.cand.emissive_instance, sh);
        if (live) indirect_end<false>(A, sc, C, I, sh);
    } else if (active) {
        // the pixel's fields through the walks in LDS (IndStash): k_indirect alone city 4K 0.590 -> 0.558 ms, scene
        // 1080p 0.268 -> 0.259, cornell 1080p 0.180 -> 0.179 (17 KiB per workgroup; still 5 waves per SIMD)
        __shared__ IndStash stash;
        indirect_body<MULTI>(A, sc, C, x, y, n_top, n_emitter, nullptr, nullptr, &stash, PRE ? &tex : nullptr);
    }
    if (!counted(A.F, x, y)) n_top = n_emitter = 0;
    wave_count(A.cnt.top, n_top);
    wave_count(A.cnt.emitter, n_emitter);
}

// ------------------------------------------------------------------ persistent waves (the north star's layout)
// Option persistent_indirect = 1 (hk_set_option): a light pass as persistent waves instead of one workgroup per 16x16 tile.  The grid is what
// the GPU holds resident (occupancy x CUs); each wave claims 8x8-pixel tiles one at a time from a claim
// counter (workgroup b uses counter b % 8 — the XCD the round-robin dispatch puts it on — and counter k hands
// out tiles k, k + 8, k + 16, ... in raster order), runs the unchanged per-pixel body on the tile's 64 pixels
// and exits once its counter is exhausted.  Every wave makes exactly one failing claim, so every wave
// reaches the exit; the last wave out (an exit counter) zeroes the block for the next launch.  Workgroups
// stage the scene into LDS once instead of once per tile, and waves whose tiles are cheap (background) take
// more of them.  The per-pixel code is the tile kernel's, so every stored word is unchanged.
enum PersistKind : uint32_t { PERSIST_INDIRECT = 0, PERSIST_DIRECT = 1 };
template <class Body>
HKD void persist_tiles(const FrameArgs& A, uint32_t kind, Body body)
{
    const Frame& F = A.F;
    const int32_t w0 = F.win_rows > 0 ? F.win_row0 : 0;
    const int32_t w1 = F.win_rows > 0 ? F.win_row0 + F.win_rows : F.s_rows;
    const int32_t c0 = win_x0(F), c1 = win_x1(F, F.s[0]);
    const uint32_t tiles_x = (uint32_t)(c1 - c0 + 7) >> 3;
    const uint32_t n = tiles_x * ((uint32_t)(w1 - w0 + 7) >> 3);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t shards = gridDim.x < PERSIST_SHARDS ? gridDim.x : PERSIST_SHARDS, shard = blockIdx.x % shards;
    unsigned long long* block = A.cnt.persist + (size_t)kind * PERSIST_LINES * PERSIST_LINE;
    for (;;) {
        uint32_t k = 0;
        if (lane == 0) k = (uint32_t)atomicAdd(block + shard * PERSIST_LINE, 1ull);
        k = __shfl(k, 0, 64);
        const uint32_t t = shard + shards * k;
        if (t >= n) break;
        const uint32_t ty = t / tiles_x, tx = t - ty * tiles_x;
        const int32_t x = c0 + (int32_t)(tx * 8u + (lane & 7u));
        const int32_t ly = w0 + (int32_t)(ty * 8u + (lane >> 3));
        body(x, global_row(F, ly, F.s_row0), x < c1 && ly < w1);
    }
    if (lane == 0) {
        __threadfence();
        unsigned int* exited = reinterpret_cast<unsigned int*>(block + PERSIST_SHARDS * PERSIST_LINE);
        if (atomicAdd(exited, 1u) == gridDim.x * 4u - 1u) {  // every other wave has made its last claim
            for (uint32_t k = 0; k < PERSIST_SHARDS; ++k) atomicExch(block + k * PERSIST_LINE, 0ull);
            atomicExch(exited, 0u);
        }
    }
}
template <bool MULTI, bool LDS>
__global__ __launch_bounds__(256) void k_indirect_persist(FrameArgs A, ChannelArgs C)
{
    Scene sc = A.sc;
    if constexpr (LDS) sc = stage_scene<PLAN_LIGHT>(A.sc, hk_lds_scene);
    uint32_t n_top = 0, n_emitter = 0;
    persist_tiles(A, PERSIST_INDIRECT, [&](int32_t x, int32_t y, bool active) {
        uint32_t t = 0, e = 0;
        if (active) indirect_body<MULTI>(A, sc, C, x, y, t, e);
        if (counted(A.F, x, y)) {
            n_top += t;
            n_emitter += e;
        }
    });
    wave_count(A.cnt.top, n_top);
    wave_count(A.cnt.emitter, n_emitter);
}

// The fused direct/emissive pass and the one-bounce indirect pass in ONE launch.  They read the same
// G-buffer and write disjoint buffers (reservoirs 0-5 and the direct / emissive planes, reservoirs 6-9
// and the indirect planes: light.rs:518-546), so their workgroups are independent and are interleaved
// in one grid — blockIdx.z 0: a direct tile, 1: the indirect tile — instead of the indirect pass
// running on a side stream joined by events.  Each CU then mixes both kinds of work and the frame has
// no cross-stream dependency: cornell 8-way stripe ....  Same per-pixel code as
// k_direct_fused_w4 / k_indirect, so the results are identical.  The direct role parks its validation
// state in the dynamic LDS buffer the indirect role stages the scene into (PARK 2): one buffer of
// max(park, scene) bytes per workgroup, as each kernel alone needs.
template <bool VD, bool VE, bool LDS_I>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_light_merged(FrameArgs A, ChannelArgs C0,
                                                                                                ChannelArgs C1, ChannelArgs C2)
{
    // gridDim.z == 2: every direct workgroup (z = 0) is dispatched before the indirect ones
    const bool zsplit = gridDim.z == 2u;
    const uint32_t bx = zsplit ? blockIdx.x : blockIdx.x >> 1, gx = zsplit ? gridDim.x : gridDim.x >> 1;
    int32_t x, y;
    uint32_t n_top = 0, n_emitter = 0;
    const bool active = tile_pixel_at<TRACE_ORDER>(A.F, A.F.s[0], A.F.s_row0, A.F.s_rows, bx, blockIdx.y, gx, gridDim.y, x, y);
    if (zsplit ? blockIdx.z == 1u : (blockIdx.x & 1u) != 0u) {
        Scene sc = A.sc;
        if constexpr (LDS_I) sc = stage_scene<PLAN_LIGHT>(A.sc, hk_lds_scene);
        // the IndStash in the launch's dynamic LDS after the staged scene, within the direct role's park area on
        // validation frames (launch_light_merged sizes the buffer); a static one cost the merged grid a wave per SIMD
        // (cornell 4-way stripe 0.138 -> 0.159 ms, profiles/r05/c26)
        IndStash* stash = reinterpret_cast<IndStash*>(hk_lds_scene + (LDS_I ? stage_bytes(A.sc.bytes, PLAN_LIGHT) / 4u : 0u));
        if (active) indirect_body<false>(A, sc, C2, x, y, n_top, n_emitter, nullptr, nullptr, stash);
    } else if (active) {
        const Scene& sc = A.sc;
        // (its own loads: the texel preload here measured 0-1 % slower on the cornell 2- to 8-way stripes, r06/c16-c17)
        const DirectPixel P = load_direct_pixel(A, x, y);
        const uint32_t bg = bg_elide(C0, P.idx, P.pd.w < HK_F32_EPSILON);
        if (bg == BG_SKIP_OWN) {  // the emissive pass's stores into the spatial pair (direct_body)
            const Reservoir z = background_reservoir();
            store_res(C1.spatial, P.idx, z);
            store_res(C1.prev_spatial, P.idx, z);
        } else if (bg == BG_STORE) {
            Surface surface;
            direct_body<false, true, VD, 2>(A, sc, C0, P, n_top, n_emitter, &surface);
            direct_body<true, false, VE, 2>(A, sc, C1, P, n_top, n_emitter, nullptr, &surface);
        }
    }
    if (!counted(A.F, x, y)) n_top = n_emitter = 0;
    wave_count(A.cnt.top, n_top);
    wave_count(A.cnt.emitter, n_emitter);
}

// ------------------------------------------------------------------ wavefront indirect pass (config 5)
// BASELINE configs[4] asks for wavefront, material-sorted shading.  The megakernel k_indirect runs
// one thread per pixel from the G-buffer to the stored reservoir; lanes of sky pixels idle through
// the bounce walk and a wave's lanes hit unrelated materials.  Here the pass is five launches:
//   k_wf_gen      per 16x16 tile: dead pixels (sky, bounces 0) do their stores; live pixels are
//                 compacted into queue1 (wave64 ballot + prefix popcount inside the workgroup, one
//                 atomic per workgroup on its segment's counter)
//   k_wf_trace    per 256 queue1 entries: the cosine bounce's closest hit (traverse_top), written
//                 as an SoA hit record; the hit's material bin goes to keys[] and the segment's
//                 histogram (one atomic per wave and distinct bin)
//   k_wf_scan     one workgroup: bin totals, their exclusive prefix sum, each segment's offset in
//                 each bin -> bin write cursors
//   k_wf_scatter  per 256 queue1 entries: pixels into queue2 grouped by bin (per wave and bin one
//                 atomic on the segment's cursor, ranks from the ballot)
//   k_wf_shade    per 256 queue2 entries, in bin order: hit_info, surface fetch, NEE (light-BVH pick,
//                 emitter BLAS walk, shadow any-hit) and the temporal ReSTIR tail
// A pixel executes the statements of indirect_body in the same order (the stages stop / resume at
// the bounce hit), so every stored word equals the megakernel's.  Grids are sized for the largest
// queue; workgroups past the live count exit at once.  Atomics on one shared word (a queue cursor
// or the hottest bin) serialise at the L2, so every counter is split over WF_SEGS segments.
HKD uint32_t wave_rank(uint64_t m) { return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)); }
HKD uint32_t wf_pack(int32_t x, int32_t ly) { return (uint32_t)x | ((uint32_t)ly << 16); }
HKD void wf_unpack(const Frame& F, uint32_t p, int32_t& x, int32_t& y)
{
    x = (int32_t)(p & 0xFFFFu);
    y = global_row(F, (int32_t)(p >> 16), F.s_row0);
}
// per wave: for each distinct key among the active lanes, one atomicAdd of its lane count on
// base[key]; returns the lane's slot (base + rank among the lanes with its key)
HKD uint32_t wf_bin_slot(uint32_t* base, bool active, uint32_t key)
{
    uint64_t left = __ballot(active);
    uint32_t slot = 0;
    while (left) {
        const uint32_t leader = (uint32_t)__builtin_ctzll(left);
        const uint32_t k = __shfl(key, (int)leader, 64);
        const uint64_t same = __ballot(active && key == k);
        uint32_t b = 0;
        if ((threadIdx.x & 63u) == leader) b = atomicAdd(base + k, (uint32_t)__builtin_popcountll(same));
        b = __shfl(b, (int)leader, 64);
        if (active && key == k) slot = b + wave_rank(same);
        left &= ~same;
    }
    return slot;
}
// the queue1 entry of this thread for the per-entry kernels: workgroup b -> segment b % WF_SEGS,
// entries 256 (b / WF_SEGS) .. of that segment; false past the segment's live count
HKD bool wf_entry(const WfArgs& W, uint32_t& seg, uint32_t& i)
{
    seg = blockIdx.x % WF_SEGS;
    i = (blockIdx.x / WF_SEGS) * 256u + threadIdx.x;
    return i < W.ctl[seg];
}

__global__ __launch_bounds__(256) void k_wf_gen(FrameArgs A, ChannelArgs C, WfArgs W)
{
    __shared__ uint32_t wave_n[4], wg_base;
    int32_t x, y;
    uint32_t n_top = 0, n_emitter = 0;
    bool live = false;
    if (tile_pixel<TRACE_ORDER>(A.F, A.F.s[0], A.F.s_row0, A.F.s_rows, x, y))
        live = indirect_body<false, IND_GEN>(A, A.sc, C, x, y, n_top, n_emitter);
    const uint64_t m = __ballot(live);
    const uint32_t wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 0u) wave_n[wave] = (uint32_t)__builtin_popcountll(m);
    __syncthreads();
    // tiles dealt round-robin over the segments: the workgroups in flight (neighbouring tiles) append
    // to different counters (contiguous runs of tiles per segment measured slower: city 4K 16 spp
    // 121.1 -> 124.9 ms, the concurrent workgroups then share one counter); a segment's entries
    // stay grouped by tile, so a wave of a bin still holds one tile's pixels
    const uint32_t tile = blockIdx.x + blockIdx.y * gridDim.x, seg = tile % WF_SEGS;
    if (threadIdx.x == 0) {
        const uint32_t total = wave_n[0] + wave_n[1] + wave_n[2] + wave_n[3];
        wg_base = total ? atomicAdd(&W.ctl[seg], total) : 0u;
    }
    __syncthreads();
    uint32_t off = wg_base;
    for (uint32_t k = 0; k < wave; ++k) off += wave_n[k];
    if (live) W.queue1[seg * W.seg_cap + off + wave_rank(m)] = wf_pack(x, local_row(A.F, y, A.F.s_row0));
}

template <bool LDS>
__global__ __launch_bounds__(256) void k_wf_trace(FrameArgs A, ChannelArgs C, WfArgs W)
{
    uint32_t seg, i;
    const bool valid = wf_entry(W, seg, i);
    if ((blockIdx.x / WF_SEGS) * 256u >= W.ctl[seg]) return;  // the whole workgroup is past the count
    // the queued pixel's texels first (every queued pixel is covered: one round trip, before any staging)
    int32_t x = 0, y = 0;
    PixelTexels tex;
    if (valid) {
        wf_unpack(A.F, W.queue1[seg * W.seg_cap + i], x, y);
        tex = load_pixel_texels(A, x, y);
    }
    Scene sc;
    if constexpr (LDS) sc = stage_scene<PLAN_LIGHT>(A.sc, hk_lds_scene);
    else sc = A.sc;
    uint32_t n_top = 0, n_emitter = 0, key = 0;
    if (valid) {
        indirect_body<false, IND_TRACE>(A, sc, C, x, y, n_top, n_emitter, &W, &key, nullptr, &tex);
        if (!counted(A.F, x, y)) n_top = 0;
        W.keys[seg * W.seg_cap + i] = key;
    }
    (void)wf_bin_slot(W.ctl + WF_CTL_HIST + seg * W.bins, valid, key);  // the segment's histogram
    wave_count(A.cnt.top, n_top);
}

__global__ __launch_bounds__(256) void k_wf_scan(WfArgs W)
{
    __shared__ uint32_t part[256];
    const uint32_t bins = W.bins, t = threadIdx.x;
    const uint32_t per = (bins + 255u) / 256u, b0 = t * per, b1 = min(bins, b0 + per);
    const uint32_t* hist = W.ctl + WF_CTL_HIST;
    uint32_t* cursor = W.ctl + WF_CTL_HIST + WF_SEGS * bins;
    uint32_t sum = 0;
    for (uint32_t b = b0; b < b1; ++b)
        for (uint32_t g = 0; g < WF_SEGS; ++g) sum += hist[g * bins + b];
    part[t] = sum;
    __syncthreads();
    if (t == 0) {
        uint32_t acc = 0;
        for (uint32_t k = 0; k < 256u; ++k) {
            const uint32_t v = part[k];
            part[k] = acc;
            acc += v;
        }
        W.ctl[WF_SEGS] = acc;  // all live pixels
    }
    __syncthreads();
    uint32_t acc = part[t];
    for (uint32_t b = b0; b < b1; ++b)
        for (uint32_t g = 0; g < WF_SEGS; ++g) {
            cursor[g * bins + b] = acc;
            acc += hist[g * bins + b];
        }
}

__global__ __launch_bounds__(256) void k_wf_scatter(WfArgs W)
{
    uint32_t seg, i;
    const bool valid = wf_entry(W, seg, i);
    if ((blockIdx.x / WF_SEGS) * 256u >= W.ctl[seg]) return;
    const uint32_t key = valid ? W.keys[seg * W.seg_cap + i] : 0u;
    const uint32_t slot = wf_bin_slot(W.ctl + WF_CTL_HIST + WF_SEGS * W.bins + seg * W.bins, valid, key);
    if (valid) W.queue2[slot] = W.queue1[seg * W.seg_cap + i];
}

template <bool LDS>
__global__ __launch_bounds__(256) void k_wf_shade(FrameArgs A, ChannelArgs C, WfArgs W)
{
    const uint32_t n = W.ctl[WF_SEGS];
    if (blockIdx.x * 256u >= n) return;
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    // the queued pixel's texels first (as k_wf_trace)
    int32_t x = 0, y = 0;
    PixelTexels tex;
    if (i < n) {
        wf_unpack(A.F, W.queue2[i], x, y);
        tex = load_pixel_texels(A, x, y);
    }
    Scene sc;
    if constexpr (LDS) sc = stage_scene<PLAN_LIGHT>(A.sc, hk_lds_scene);
    else sc = A.sc;
    uint32_t n_top = 0, n_emitter = 0;
    if (i < n) {
        indirect_body<false, IND_SHADE>(A, sc, C, x, y, n_top, n_emitter, &W, nullptr, nullptr, &tex);
        if (!counted(A.F, x, y)) n_top = n_emitter = 0;
    }
    wave_count(A.cnt.top, n_top);
    wave_count(A.cnt.emitter, n_emitter);
}

// ------------------------------------------------------------------ spatial_reuse (light.wgsl:1500-1684)
// The reference's workgroup-shared copies (shared_reservoir/shared_depth) hold exactly the
// values the global path reads for in-tile neighbours, so every neighbour is read from the
// (L2-resident) reservoir planes directly.
// Depth window of spatial reuse: at upscale ratio 1 every neighbour and screen-space occlusion
// tap of a 16x16 tile lies within RANGE (20) + 2 pixels of it, so the workgroup stages that
// 60x60 window of G-buffer depth in LDS once (14 KiB) instead of ~80 scattered 16-byte position
// loads per pixel.  Values are load_depth() of the same coordinates (frame-OOB -> 0, band
// clamp), so results are unchanged; a coordinate outside the window reads global memory.
constexpr int32_t SP_HALO = 22, SP_WIN = 16 + 2 * SP_HALO;
struct DepthWin {
    const float* lds;  // null: no window (upscale ratio != 1)
    int32_t x0, y0;
};
// WINDOW: every coordinate the pass reads lies in the window — a neighbour is at most RANGE (20) px from its pixel
// (f2i32 truncates toward zero, never outward) and a march tap between the two, so it is within 20 + 1 px of the
// 16x16 tile and SP_HALO = 22 leaves a pixel to spare on each side — so the window is read without a bounds test
template <bool WINDOW>
HKD float win_depth(const Frame& F, const GBuffer& G, const DepthWin& W, int32_t x, int32_t y)
{
    if constexpr (WINDOW) return W.lds[(y - W.y0) * SP_WIN + (x - W.x0)];
    return load_depth(F, G, x, y);
}

// The reservoir being built is carried through the neighbour loop as (count, w_sum, w2_sum) plus
// the index of the record its sample came from (sel: a neighbour's index in `cur`, SEL_OWN or
// SEL_PREVIOUS); the selected sample is re-read from that record once, after the loop.  The
// records are not written by this pass (it writes C.spatial only), so the re-read returns the
// bits update_reservoir() would have copied (light.wgsl:138-151), and the 22 registers of a
// carried sample (plus the copy per merge) leave the loop.
constexpr int32_t SEL_OWN = -1, SEL_PREVIOUS = -2;

template <bool EMISSIVE_LIT, bool WINDOW, bool VIEW>
HKD void spatial_body(const FrameArgs& A, const ChannelArgs& C, int32_t x, int32_t y, const DepthWin& W)
{
    const Frame& F = A.F;
    constexpr uint32_t COUNT = EMISSIVE_LIT ? 8u : 16u;
    const int32_t idx = rb_index(F, x, y);
    const f2 uv = coords_to_uv(x, y, F.s);
    int32_t dx, dy;
    jittered_coords(F, uv, dx, dy);
    f4 pd = load_position(F, A.G, dx, dy);
    f4 position = mk4(pd.x, pd.y, pd.z, 1.0f);
    float depth = pd.w;
    if (depth < HK_F32_EPSILON) {
        // the temporal pass of this frame left its background record in C.cur at this pixel (it
        // classifies the pixel from the same G-buffer texel, over a window that contains this
        // pass's): the emissive pass's set_reservoir'd zero or the indirect pass's zero reservoir
        // (light.wgsl:1063-1071, 1283-1290), so the record is repacked from registers, not re-read
        {
            uint4 c0, c1, c2, c3;
            pack_res(EMISSIVE_LIT ? background_reservoir() : zero_reservoir(), c0, c1, c2, c3);
            store_res(C.spatial, idx, unpack_reservoir(c0, c1, c2, c3));
        }
        store_rgba16f(C.render, idx, mk4(0, 0, 0, 0));
        return;
    }
    const Reservoir own = load_res(C.cur, idx);
    const Sample& s = own.s;
    uint32_t im_y = f2u32(load_instance_material(F, A.G, dx, dy).y);
    f4 velocity_uv = load_velocity_uv(F, A.G, dx, dy);
    Surface surface = retreive_surface(A.sc, im_y, mk2(velocity_uv.z, velocity_uv.w));
    const bool use_spatial_variance = own.count <= 4.0f;
    f2 juv = jittered_uv(F, uv, 0.25f);
    f2 previous_uv = mk2(juv.x - velocity_uv.x, juv.y - velocity_uv.y);
    float lifetime_max = F.max_reservoir_lifetime <= 1.0f ? HK_F32_MAX : F.max_reservoir_lifetime;
    // r = the previous spatial reservoir (load_previous) or the pixel's own one
    const bool from_previous = own.lifetime <= lifetime_max;
    int32_t previous_index = -1;  // load_previous's record; -1: outside the frame (the zero reservoir)
    if (from_previous && uv_inside_open(previous_uv))
        previous_index = rb_index(F, f2i32(previous_uv.x * (float)F.s[0]), f2i32(previous_uv.y * (float)F.s[1]));
    float r_count = own.count, r_lifetime = own.lifetime, r_w_sum = own.w_sum, r_w2_sum = own.w2_sum;
    int32_t sel = SEL_OWN;
    if (from_previous) {
        sel = SEL_PREVIOUS;
        r_count = r_lifetime = r_w_sum = r_w2_sum = 0.0f;
        if (previous_index >= 0) {
            const uint4 p3 = C.prev_spatial.base[res_chunk(C.prev_spatial, 3u, (uint32_t)previous_index)];
            r_count = unpack_lo16float(p3.z);
            r_w_sum = unpack_lo16float(p3.w);
            r_w2_sum = unpack_hi16float(p3.w);
            r_lifetime = 127.0f * (1.0f + hk_unpack_snorm8_fast(p3.x, 3));
        }
    }
    f3 view_direction = calculate_view(F, position);
    const ShadeCtx sc = shade_ctx(F, view_direction, s.visible_normal, surface);
    // merge_reservoir(r, own, p) (light.wgsl:153-160)
    // rand: fract(dot(q.s.random, 1)), the value update_reservoir compares (light.wgsl:155)
    auto merge = [&](float p, float q_w, float q_count, float rand, int32_t q_sel) {
        const float w_new = (p * q_w) * q_count;
        r_w_sum += w_new;
        r_w2_sum += w_new * w_new;
        if (rand < w_new / r_w_sum) sel = q_sel;
        r_count = r_count + q_count;
    };
    if (EMISSIVE_LIT) {
        merge(lum(xyz(s.radiance)), own.w, own.count, hk_fract(sum4(s.random)), SEL_OWN);
    } else {
        f3 o = shade(sc, normalize(xyz(s.sample_position) - xyz(s.visible_position)), s.radiance);
        merge(lum(o), own.w, own.count, hk_fract(sum4(s.random)), SEL_OWN);
    }

    const float rf = hk_random_float(F.number);
    const float srand = sum4(s.random);
    const f3 s_visible = xyz(s.visible_position);
    const f3 s_normal = s.visible_normal;
    HK_STAGE_STATS_DECL;
    for (uint32_t i = 1u; i <= COUNT; i += 1u) {
        HK_STAGE_TICK(1);
        float px = HK_TAU * hk_fract(((float)i * HK_GOLDEN_RATIO + srand) + rf);
        const float py = F.sp_py[EMISSIVE_LIT][i - 1u];  // sqrt(i / COUNT) * RANGE
        float sn, cs;
        hk_sincos(px, &sn, &cs);
        f2 offset = mk2(py * cs, py * sn);
        int32_t scx = f2i32(offset.x + (float)x), scy = f2i32(offset.y + (float)y);
        int32_t sdx, sdy;
        if (WINDOW) {
            // upscale ratio 1 and s == S (the window variant): the uv bounds test is the integer
            // test (see k_denoise3), and jittered_coords(coords_to_uv(c)) == c: the jitter is
            // (j * tx) * 0 and u32((c + 0.5) / S * S) truncates back to c for c < 2^22
            if (scx < 0 || scy < 0 || scx >= (int32_t)F.s[0] || scy >= (int32_t)F.s[1]) continue;
            sdx = scx;
            sdy = scy;
        } else {
            f2 suv = coords_to_uv_s(F, scx, scy);
            if (suv.x < 0.0f || suv.y < 0.0f || suv.x > 1.0f || suv.y > 1.0f) continue;
            jittered_coords(F, suv, sdx, sdy);
        }
        float sample_depth = win_depth<WINDOW>(F, A.G, W, sdx, sdy);
        float depth_ratio = depth / sample_depth;
        if (depth_ratio < 0.9f || depth_ratio > 1.1f) continue;
        const int32_t nidx = rb_index(F, scx, scy);
        // (VIEW) the neighbour's view plane 0 is gathered before the march: the march's LDS and VALU work then
        // hides the gather's latency (a neighbour the march rejects has read 16 bytes for nothing)
        uint4 view0 = make_uint4(0u, 0u, 0u, 0u);
        if constexpr (VIEW) view0 = C.view[view_at(C.view_n, 0u, (uint32_t)nidx)];
        // the screen-space depth march first: it reads only the LDS depth window and rejects a third of
        // the neighbours (city 1080p: 35 %; the count / normal and direction tests below reject < 1 %),
        // so those never gather reservoir planes.  The rejection tests are pure, so their order does not
        // change which neighbours are merged.
        const float tap_interval = F.sp_tap_interval[EMISSIVE_LIT][i - 1u];  // max(1, py / 5)
        uint32_t tap_count = F.sp_tap_count[EMISSIVE_LIT][i - 1u];          // u32(py / tap_interval)
        bool occluded = false;
        float inv_len = 1.0f / sqrtf(dot(offset, offset));
        f2 dir = mk2(offset.x * inv_len, offset.y * inv_len);
        const float sx = (float)F.s[0], sy = (float)F.s[1];
        for (uint32_t j = 1u; j <= tap_count; j += 1u) {
            HK_STAGE_TICK(2);
            float tap_dist = (float)j * tap_interval;
            f2 tuv = mk2(uv.x + div_by(tap_dist * dir.x, sx, F.inv_s[0]), uv.y + div_by(tap_dist * dir.y, sy, F.inv_s[1]));
            int32_t tdx, tdy;
            if constexpr (WINDOW) {
                // ratio 1, s == S: jittered_coords(tuv) adds the jitter (j tx) * 0 = +-0 to tuv (never -0
                // itself: uv > 0 and an exact cancellation rounds to +0), so it is i32(tuv * S); tuv is
                // finite and within [-1, 2], where the plain conversion is f2i32's value
                tdx = (int32_t)(tuv.x * sx);
                tdy = (int32_t)(tuv.y * sy);
            } else {
                jittered_coords(F, tuv, tdx, tdy);
            }
            float tap_depth = win_depth<WINDOW>(F, A.G, W, tdx, tdy);
            // j / (tap_count + 1) from the host table (tap_count <= 5 for RANGE <= 20)
            const float t = tap_count < 7u && j < 6u ? F.sp_tap_t[tap_count][j] : (float)j / (float)(tap_count + 1u);
            float ref_depth = hk_mixf(depth, sample_depth, t);
            if (tap_depth > ref_depth + 0.00001f) {
                occluded = true;
                break;
            }
        }
        if (occluded) continue;
        HK_STAGE_TICK(3);
        // the neighbour's reservoir, its 16-byte planes loaded as the tests need them (the rejection
        // tests read plane 3 (count, normals) and plane 2 (sample position); planes 0-1 only for a
        // neighbour that is merged): the same values as load_res, fewer gathers for rejected ones
        // the neighbour's record: the view planes (VIEW, store_res_view) or the reservoir's own 16-byte
        // planes, loaded as the tests need them (rejection: plane 3 count / normal, plane 2 sample
        // position; merge: planes 0-1): the same values as load_res either way
        uint4 c3 = make_uint4(0u, 0u, 0u, 0u);
        uint32_t normal_word;
        bool count_ok;
        f3 q_sample;
        if constexpr (VIEW) {
            const uint4 a = view0;
            normal_word = a.w;
            count_ok = (a.w & VIEW_COUNT) != 0u;
            q_sample = mk3(__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z));
        } else {
            c3 = C.cur.base[res_chunk(C.cur, 3u, (uint32_t)nidx)];
            normal_word = c3.x;
            count_ok = !(unpack_lo16float(c3.z) < HK_F32_EPSILON);
        }
        const f3 q_normal = normalize(mk3(hk_unpack_snorm8_fast(normal_word, 0), hk_unpack_snorm8_fast(normal_word, 1),
                                          hk_unpack_snorm8_fast(normal_word, 2)));
        bool normal_miss = dot(s_normal, q_normal) < 0.866f;
        if (!count_ok || normal_miss) continue;
        if constexpr (!VIEW) {
            const uint4 c2 = C.cur.base[res_chunk(C.cur, 2u, (uint32_t)nidx)];
            q_sample = mk3(__uint_as_float(c2.x), __uint_as_float(c2.y), __uint_as_float(c2.z));
        }
        // normalize(q_sample - visible), its length kept for the jacobian below
        const f3 to_sample = q_sample - s_visible;
        const float to_sample_length = sqrtf(dot(to_sample, to_sample));
        f3 sample_direction = to_sample * rcp_exact(to_sample_length);
        if (dot(sample_direction, s_normal) < 0.0f) continue;
        HK_STAGE_TICK(4);

        // merge_reservoir(r, q, p / jacobian): the fields of q that the merge reads
        float q_w, q_count, q_rand;
        f4 q_radiance;
        bool hit;
        if constexpr (VIEW) {
            const uint4 b = C.view[view_at(C.view_n, 1u, (uint32_t)nidx)];
            q_radiance = mk4(unpack_lo16float(b.x), unpack_hi16float(b.x), unpack_lo16float(b.y), unpack_hi16float(b.y));
            q_count = unpack_lo16float(b.z);
            q_w = unpack_hi16float(b.z);
            q_rand = __uint_as_float(b.w);
            hit = (normal_word & VIEW_HIT) != 0u;
        } else {
            const uint4 c0 = C.cur.base[res_chunk(C.cur, 0u, (uint32_t)nidx)];
            q_radiance = mk4(unpack_lo16float(c0.x), unpack_hi16float(c0.x), unpack_lo16float(c0.y), unpack_hi16float(c0.y));
            q_count = unpack_lo16float(c3.z);
            q_w = unpack_hi16float(c3.z);
            q_rand = hk_fract(sum4(mk4(hk_unpack_unorm16_fast(c0.z), hk_unpack_unorm16_fast(c0.z >> 16),
                                       hk_unpack_unorm16_fast(c0.w), hk_unpack_unorm16_fast(c0.w >> 16))));
            hit = hk_unpack_snorm8_fast(c3.y, 3) > 0.5f;
        }
        float jacobian = 1.0f;
        if (hit) {
            // compute_jacobian(q.s, s) (light.wgsl:990-1004).  Its first vector, visible - q_sample,
            // is -to_sample exactly, so its normalisation is -sample_direction and its length is
            // to_sample_length, bit for bit (negation is exact; the squares are equal)
            uint4 c1;
            uint32_t sample_normal_word;
            if constexpr (VIEW) {
                c1 = C.view[view_at(C.view_n, 2u, (uint32_t)nidx)];
                sample_normal_word = c1.w;
            } else {
                c1 = C.cur.base[res_chunk(C.cur, 1u, (uint32_t)nidx)];
                sample_normal_word = c3.y;
            }
            const f3 q_visible = mk3(__uint_as_float(c1.x), __uint_as_float(c1.y), __uint_as_float(c1.z));
            const f3 normal = normalize(mk3(hk_unpack_snorm8_fast(sample_normal_word, 0), hk_unpack_snorm8_fast(sample_normal_word, 1),
                                            hk_unpack_snorm8_fast(sample_normal_word, 2)));
            const float c1_ = fabsf(dot(sample_direction, normal));
            const f3 back = q_visible - q_sample;
            const float back_length = sqrtf(dot(back, back));
            const float c2_ = fabsf(dot(back * rcp_exact(back_length), normal));
            const float term_1 = c1_ / fmaxf(0.0001f, c2_);
            const float num = back_length * back_length;
            const float denom = to_sample_length * to_sample_length;
            const float term_2 = num / fmaxf(denom, 0.0001f);
            jacobian = hk_clampf(term_1 * term_2, 1.0f, 50.0f);
        }
        if (EMISSIVE_LIT) {
            merge(lum(xyz(q_radiance)) / jacobian, q_w, q_count, q_rand, nidx);
        } else {
            f3 o = shade(sc, sample_direction, q_radiance);
            merge(lum(o) / jacobian, q_w, q_count, q_rand, nidx);
        }
    }
    // the selected sample, re-read from its record (see SEL_OWN above)
    Reservoir r;
    {
        ResBuf b = C.cur;
        int32_t at = sel >= 0 ? sel : idx;
        if (sel == SEL_PREVIOUS) {
            b = C.prev_spatial;
            at = previous_index;
        }
        if (at >= 0) {
            r = load_res(b, at);
        } else {
            r = zero_reservoir();
        }
        if (sel < 0) {  // r.s.visible_position / visible_normal = s's (light.wgsl:1563-1564)
            r.s.visible_position = s.visible_position;
            r.s.visible_normal = s.visible_normal;
        }
    }
    r.count = r_count;
    r.lifetime = r_lifetime;
    r.w_sum = r_w_sum;
    r.w2_sum = r_w2_sum;
    float m = (float)F.max_spatial_reuse_count;
    if (r.count > m) {
        r.w_sum *= m / r.count;
        r.w2_sum *= m / r.count;
        r.count = m;
    }
    f3 out = shade(sc, normalize(xyz(r.s.sample_position) - xyz(s.visible_position)), r.s.radiance);
    float total_lum = EMISSIVE_LIT ? r.count * lum(xyz(r.s.radiance)) : r.count * lum(out);
    r.w = total_lum > 0.0f ? r.w_sum / total_lum : 0.0f;
    r.lifetime += 1.0f;
    store_res(C.spatial, idx, r);
    if (use_spatial_variance) C.variance[idx] = variance_of(r);
    f3 oc = out * r.w;
    store_rgba16f(C.render, idx, mk4(oc.x, oc.y, oc.z, 1.0f));
}

template <bool EMISSIVE_LIT, bool WINDOW, bool VIEW>
HKD void spatial_kernel(const FrameArgs& A, const ChannelArgs& C)
{
    __shared__ float win[WINDOW ? SP_WIN * SP_WIN : 1];
    DepthWin W{nullptr, 0, 0};
    if (WINDOW) {
        int32_t x0, y0;
        tile_origin<SPATIAL_ORDER>(A.F, A.F.s_row0, x0, y0);
        W.x0 = x0 - SP_HALO;
        W.y0 = y0 - SP_HALO;
        // load_depth of the 3600 window texels, 15 per thread: all 15 loads issued before any LDS store (at
        // clamped coordinates, so none is conditional; outside the frame the value is then 0 as load_depth's),
        // instead of one load -> wait -> store round trip per texel
        // (the window variant runs on row bands, never on interleaved stripes: band_index is the band's row offset
        // and clamp; texel k = t + 256 j steps 4 rows and 16 columns per j)
        constexpr int32_t N = SP_WIN * SP_WIN, PER = (N + 255) / 256;
        static_assert(256 / SP_WIN == 4 && 256 % SP_WIN == 16, "window stepping");
        float v[PER];
        int32_t col = (int32_t)threadIdx.x % SP_WIN, row = (int32_t)threadIdx.x / SP_WIN;
        const int32_t S0 = (int32_t)A.F.S[0], S1 = (int32_t)A.F.S[1];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int32_t wx = W.x0 + col, wy = W.y0 + row;
            const int32_t cx = min(max(wx, 0), S0 - 1), cy = min(max(wy, 0), S1 - 1);
            int32_t ly = cy - A.F.S_row0;
            ly = ly < 0 ? 0 : (ly >= A.F.S_rows ? A.F.S_rows - 1 : ly);
            const float d = A.G.position[cx + S0 * ly].w;
            v[j] = in_frame(wx, wy, A.F.S) ? d : 0.0f;
            col += 16;
            row += 4;
            if (col >= SP_WIN) {
                col -= SP_WIN;
                row += 1;
            }
        }
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int32_t k = (int32_t)threadIdx.x + j * 256;
            if (j < PER - 1 || k < N) win[k] = v[j];
        }
        __syncthreads();
        W.lds = win;
    }
    int32_t x, y;
    if (tile_pixel<SPATIAL_ORDER>(A.F, A.F.s[0], A.F.s_row0, A.F.s_rows, x, y)) spatial_body<EMISSIVE_LIT, WINDOW, VIEW>(A, C, x, y, W);
}
// The window variant (upscale ratio 1) at 6 waves per SIMD: its neighbour loop fits 78 VGPRs without spilling once
// the window staging no longer holds 15 loads' worth of state per texel loop (city 4K 1.587 -> 1.481 ms, scene
// 0.489 -> 0.464 ms, profiles/r04/c15; the 14.4 KiB window allows 11 workgroups per CU).  The variant without the
// window (upscale ratio 2, host G-buffers) would spill there and keeps the compiler's choice.
template <bool EMISSIVE_LIT, bool VIEW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_spatial(FrameArgs A,
                                                                                                             ChannelArgs C)
{
    spatial_kernel<EMISSIVE_LIT, true, VIEW>(A, C);
}
template <bool EMISSIVE_LIT, bool VIEW>
__global__ __launch_bounds__(256) void k_spatial_nowin(FrameArgs A, ChannelArgs C)
{
    spatial_kernel<EMISSIVE_LIT, false, VIEW>(A, C);
}

// ------------------------------------------------------------------ denoise (denoise.wgsl)
__constant__ float KERNEL3[3][3] = {{0.0625f, 0.125f, 0.0625f}, {0.125f, 0.25f, 0.125f}, {0.0625f, 0.125f, 0.0625f}};

HKD bool uv_outside(f2 uv) { return uv.x < 0.0f || uv.y < 0.0f || uv.x > 1.0f || uv.y > 1.0f; }
// NaN or +inf in a component (denoise.wgsl's `any(isnan) || any(x > F32_MAX)` skip): one class test per
// component (v_cmp_class_f32: signalling / quiet NaN, +inf) instead of two compares
HKD bool bad3(f3 v)
{
    constexpr int NAN_PINF = 0x1 | 0x2 | 0x200;
    return __builtin_amdgcn_classf(v.x, NAN_PINF) || __builtin_amdgcn_classf(v.y, NAN_PINF) ||
           __builtin_amdgcn_classf(v.z, NAN_PINF);
}

// albedo plane is S-sized (band-local rows)
HKD f4 load_albedo(const Frame& F, const uint2* albedo, int32_t x, int32_t y)
{
    return load_rgba16f(albedo, band_index(F, x, y, F.S[0], F.S_row0, F.S_rows));
}

// Channel-fused denoiser.  The reference runs demodulation + 4 levels separately for each of the 3 channels
// (post_process.rs:1199-1223); channels are independent and share every geometry weight, so one launch per level
// processes all channels and computes the normal / depth / instance weights of each tap once.  Demodulation
// produces, with exactly the expressions denoise.wgsl evaluates per tap:
//   nd      (normalised normal, depth) of the pixel's deferred texel          — read at every tap
//   center  (depth gradient x, y, luminance denominator of channels 0, 1)     — read at the pixel only
//   den2    (luminance denominator of channel 2)                                — read at the pixel only
// and the level-0 input.  A level's input / output (the reference's internal textures, RGBA16F per channel)
// is kept as the three channels' RGB halves packed into 20 bytes plus the pixel's instance (alpha is never
// read): rgb[L] = r0 g0 | b0 r1 | g1 b1 | r2 g2, bi[L] = b2 | (instance bits); the halves are the f16 bits the
// reference stores (pack2x16float), so every value read back is unchanged.  The planes are private to
// hk_denoise (no output id reads them).
HKD void store_level(const DenoiseArgs& D, int level, int32_t idx, f3 c0, f3 c1, f3 c2, uint32_t inst_bits)
{
    D.rgb[level][idx] = make_uint4(pack2x16float(c0.x, c0.y), pack2x16float(c0.z, c1.x), pack2x16float(c1.y, c1.z),
                                   pack2x16float(c2.x, c2.y));
    D.bi[level][idx] = make_uint2(pack2x16float(c2.z, 0.0f), inst_bits);
}
// channel ch's RGB from a packed texel (ch: an unrolled loop's constant)
HKD f3 dn_rgb(int ch, uint4 rgb, uint2 bi)
{
    if (ch == 0) return mk3(unpack_lo16float(rgb.x), unpack_hi16float(rgb.x), unpack_lo16float(rgb.y));
    if (ch == 1) return mk3(unpack_hi16float(rgb.y), unpack_lo16float(rgb.z), unpack_hi16float(rgb.z));
    return mk3(unpack_lo16float(rgb.w), unpack_hi16float(rgb.w), unpack_lo16float(bi.x));
}

// The 3x3 variance blur's taps (denoise.wgsl:116-132) lie within 1 px of the pixel (nearest_texel of uv +- 1 / s is
// the neighbour, clamped into the frame), so each workgroup stages its 16x16 tile + 1 px of the channels' variance
// planes in LDS once (the values the taps would load: the same plane index) and the 27 taps of a pixel read LDS.
template <int C>
__global__ __launch_bounds__(256) void k_demod3(FrameArgs A, DenoiseArgs D)
{
    constexpr int32_t RW = 18, RS = 24;  // region width (tile + 1 px each side), row stride (an odd multiple of 8)
    __shared__ float s_var[C][RW * RS];
    const Frame& F = A.F;
    int32_t x0, y0;
    tile_origin<XCD_RASTER>(F, F.s_row0, x0, y0);
    // the pixel's own texels first (its deferred texel at the nearest texel of the jittered uv, albedo, the channels'
    // render texels), so that their latency overlaps the variance staging instead of following its barrier
    int32_t x, y;
    const bool active = tile_pixel<XCD_RASTER>(F, F.s[0], F.s_row0, F.s_rows, x, y);
    int32_t idx = 0;
    f2 uv = mk2(0, 0);
    uint32_t n_bits = 0u;
    float depth = 0.0f, inst = 0.0f;
    float2 grad = make_float2(0.0f, 0.0f);
    uint2 alb = make_uint2(0u, 0u), rtex[C];
    if (active) {
        idx = s_index(F, x, y);
        uv = coords_to_uv(x, y, F.s);
        f2 duv = jittered_uv(F, uv, 0.5f);
        int32_t ax, ay, rx, ry;
        nearest_texel(duv, F.S, ax, ay);
        // (ax, ay) is a nearest_texel: inside the frame, so the load_* bounds tests always pass; the texels are read
        // directly, without their branch regions, so all of them are in flight together (same texels, same values)
        const int32_t g = band_index(F, ax, ay, F.S[0], F.S_row0, F.S_rows);
        n_bits = A.G.normal[g];
        depth = A.G.position[g].w;
        grad = A.G.depth_gradient[g];
        inst = A.G.instance_material[g].x;
        alb = D.albedo[g];  // load_albedo(ax, ay): the same band index
        nearest_texel(uv, F.s, rx, ry);
        const int32_t ridx = s_index(F, rx, ry);
#pragma unroll
        for (int ch = 0; ch < C; ++ch) rtex[ch] = D.render[ch][ridx];
    }
    for (int32_t k = (int32_t)threadIdx.x; k < RW * RW; k += 256) {
        const int32_t ry = k / RW, rx = k - ry * RW;
        const int32_t vidx = rb_index(F, min(max(x0 - 1 + rx, 0), (int32_t)F.s[0] - 1), min(max(y0 - 1 + ry, 0), (int32_t)F.s[1] - 1));
#pragma unroll
        for (int ch = 0; ch < C; ++ch) s_var[ch][ry * RS + rx] = D.variance[ch][vidx];
    }
    __syncthreads();
    if (!active) return;
    {
        const uint32_t n = n_bits;
        const f3 normal = normalize(mk3(hk_unpack_snorm8_fast(n, 0), hk_unpack_snorm8_fast(n, 1), hk_unpack_snorm8_fast(n, 2)));
        D.nd[idx] = make_float4(normal.x, normal.y, normal.z, depth);  // denoise.wgsl:220-223, 197-200
    }
    f3 albedo = mk3(unpack_lo16float(alb.x), unpack_hi16float(alb.x), unpack_lo16float(alb.y));
    f3 out[3] = {mk3(0, 0, 0), mk3(0, 0, 0), mk3(0, 0, 0)};
    float den[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int ch = 0; ch < C; ++ch) {
        f3 irr = mk3(unpack_lo16float(rtex[ch].x), unpack_hi16float(rtex[ch].x), unpack_lo16float(rtex[ch].y));
        out[ch] = mk3(albedo.x < 0.01f ? 0.0f : irr.x / albedo.x, albedo.y < 0.01f ? 0.0f : irr.y / albedo.y,
                      albedo.z < 0.01f ? 0.0f : irr.z / albedo.z);
        float sum_variance = 0.0f;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int ox = k / 3 - 1, oy = k % 3 - 1;  // (-1,-1),(-1,0),(-1,1),(0,-1),...
            f2 suv = mk2(uv.x + (float)ox / (float)F.s[0], uv.y + (float)oy / (float)F.s[1]);
            // every tap read (nearest_texel clamps an outside tap into the frame), its term selected
            int32_t vx, vy;
            nearest_texel(suv, F.s, vx, vy);
            const float v = s_var[ch][(vy - y0 + 1) * RS + (vx - x0 + 1)];
            const float t = sum_variance + KERNEL3[oy + 1][ox + 1] * fmaxf(v, 0.0f);
            sum_variance = (uv_outside(suv) || v > HK_F32_MAX) ? sum_variance : t;
        }
        D.internal_variance[ch][idx] = sum_variance;
        // the levels' luminance-weight denominator (denoise.wgsl:56-60: strictness 4, exponent 0.25, eps 0.001) of
        // this pixel's variance, the same in every level: evaluated once here instead of once per level
        den[ch] = 4.0f * hk_pow(sum_variance, 0.25f) + 0.001f;
    }
    // internal0 = (irradiance / albedo, 1) per channel (denoise.wgsl:143-147), packed
    store_level(D, 0, idx, out[0], out[1], out[2], __float_as_uint(inst));
    D.center[idx] = make_float4(grad.x, grad.y, den[0], den[1]);
    if (C == 3) D.den2[idx] = den[2];
}

// One a-trous level (denoise.wgsl:215-319) with its inputs staged in LDS.  A workgroup's 256 pixels read their taps
// from a region around them that the workgroup copies once — each texel's (normal, depth), packed channels and
// instance, three coalesced 16 / 16 / 8-byte loads — and the taps then read LDS instead of gathering ~37 scattered
// texels per pixel through the caches.  Every value is the one a per-tap load would read (rb_index of the same
// coordinates) and the arithmetic per tap is the reference's, so the stored bits are those of the per-tap version:
// city 4K 0.417 -> 0.354 ms per level (profiles/r05/c3).
// The tile: TW columns x TH rows spaced RSP apart.  A level's taps are `step` px away, so at RSP = step a tile of
// rows y, y + step, ... reads only rows of its own residue class: the region is (TW + 2 step) x (TH + 2) texels.
// L0-L2 use 32 x 8 tiles at RSP = step (L0: 48 x 10 texels = 1.9x the tile instead of 32 x 32 = 4x for a 16x16
// tile; L1 1.6x instead of 2.25x; L2 1.4x instead of 1.6x) and L3 (step 1) a 16x16 tile (1.27x).  Row stride: an
// odd multiple of 8 texels, so the two 8-texel rows of a 16-lane LDS read phase fall in different halves of the
// banks.
template <int LEVEL>
struct DnRegion {
    static constexpr int32_t step = 8 >> LEVEL;
    static constexpr int32_t RSP = LEVEL < 3 ? step : 1;       // row spacing of the tile's pixels
    static constexpr int32_t TW = LEVEL < 3 ? 32 : 16;          // tile columns
    static constexpr int32_t TH = 256 / TW;                     // tile rows
    static constexpr int32_t RW = TW + 2 * step;                // region width
    static constexpr int32_t RH = TH + 2 * (step / RSP);        // region rows
    static constexpr int32_t STRIDE = (RW % 16 == 8) ? RW : (RW / 16) * 16 + (RW % 16 < 8 ? 8 : 24);
    static constexpr int32_t N = RH * STRIDE;
};
template <int LEVEL>
static dim3 level_tiles(uint32_t width, int32_t rows)
{
    using R = DnRegion<LEVEL>;
    const uint32_t block = (uint32_t)(R::TH * R::RSP);  // rows of one block of RSP tiles
    return dim3((width + R::TW - 1u) / R::TW, ((uint32_t)rows + block - 1u) / block * R::RSP, 1);
}
template <int C, int LEVEL>
__global__ __launch_bounds__(256) void k_denoise3(FrameArgs A, DenoiseArgs D)
{
    using R = DnRegion<LEVEL>;
    constexpr int32_t step = R::step, rstep = step / R::RSP;  // a tap's offset in region columns / rows
    __shared__ float4 s_nd[R::N];
    __shared__ uint4 s_rgb[R::N];
    __shared__ uint2 s_bi[R::N];
    const Frame& F = A.F;
    uint32_t tx, ty;
    tile_coords<DENOISE_ORDER>(tx, ty);
    const int32_t w0 = F.win_rows > 0 ? F.win_row0 : 0;
    const int32_t w1 = F.win_rows > 0 ? F.win_row0 + F.win_rows : F.s_rows;
    const int32_t x0 = win_x0(F) + (int32_t)tx * R::TW;
    // band row of the tile's first row: block ty / RSP, residue ty % RSP
    const int32_t ly0 = w0 + (int32_t)(ty / R::RSP) * R::TH * R::RSP + (int32_t)(ty % R::RSP);
    {
        const int32_t y0 = F.s_row0 + ly0;
        for (int32_t k = (int32_t)threadIdx.x; k < R::RW * R::RH; k += 256) {
            const int32_t ry = k / R::RW, rx = k - ry * R::RW;
            // out-of-frame texels are never tapped (the tap bounds test below); read at clamped coordinates
            const int32_t gx = min(max(x0 - step + rx, 0), (int32_t)F.s[0] - 1);
            const int32_t gy = min(max(y0 + (ry - rstep) * R::RSP, 0), (int32_t)F.s[1] - 1);
            const int32_t sidx = rb_index(F, gx, gy);
            const float4 nd = D.nd[sidx];
            const uint4 rgb = D.rgb[LEVEL][sidx];
            const uint2 bi = D.bi[LEVEL][sidx];
            const int32_t o = ry * R::STRIDE + rx;
            s_nd[o] = nd;
            s_rgb[o] = rgb;
            s_bi[o] = bi;
        }
    }
    __syncthreads();
    int32_t x, y;
    int32_t tc, tr;  // the pixel's tile column / row
    if constexpr (R::TW == 16) {  // 16x16: a wave per 8x8 quad (tile_pixel_at)
        const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
        tc = (int32_t)((w & 1u) * 8u + (lane & 7u));
        tr = (int32_t)((w >> 1) * 8u + (lane >> 3));
    } else {
        tc = (int32_t)(threadIdx.x % R::TW);
        tr = (int32_t)(threadIdx.x / R::TW);
    }
    x = x0 + tc;
    const int32_t ly = ly0 + tr * R::RSP;
    if (x >= win_x1(F, F.s[0]) || ly >= w1) return;
    y = global_row(F, ly, F.s_row0);
    const int32_t idx = rb_index(F, x, y);
    const int32_t oc = (tr + rstep) * R::STRIDE + (tc + step);  // the pixel in the region
    const float4 g0 = s_nd[oc];
    const uint2 cbi = s_bi[oc];
    const float depth = g0.w;
    if (depth < HK_F32_EPSILON) {
        if (LEVEL == 3) {
#pragma unroll
            for (int ch = 0; ch < C; ++ch) store_rgba16f(D.output[ch], idx, mk4(0, 0, 0, 0));
        } else {
            store_level(D, LEVEL + 1, idx, mk3(0, 0, 0), mk3(0, 0, 0), mk3(0, 0, 0), cbi.y);
        }
        return;
    }
    const float4 gc = D.center[idx];
    const f3 normal = mk3(g0.x, g0.y, g0.z);
    const float instance = __uint_as_float(cbi.y);
    const f2 depth_gradient = mk2(gc.x, gc.y);
    f3 sum_irr[C], irradiance[C];
    float sum_w[C], l0[C], lum_denom[C], lum_rcp[C], m1[C], m2[C], cnt[C];
    const uint4 crgb = s_rgb[oc];
#pragma unroll
    for (int ch = 0; ch < C; ++ch) {
        irradiance[ch] = dn_rgb(ch, crgb, cbi);
        sum_irr[ch] = irradiance[ch] * 0.25f;
        sum_w[ch] = 0.25f;
        if (bad3(irradiance[ch])) {
            irradiance[ch] = mk3(0, 0, 0);
            sum_irr[ch] = mk3(0, 0, 0);
            sum_w[ch] = 0.0f;
        }
        l0[ch] = lum(irradiance[ch]);
        lum_denom[ch] = ch == 0 ? gc.z : (ch == 1 ? gc.w : D.den2[idx]);  // k_demod3
        lum_rcp[ch] = rcp_exact(lum_denom[ch]);                           // == 1 / lum_denom (all inputs)
        m1[ch] = m2[ch] = cnt[ch] = 0.0f;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int kk = k < 4 ? k : k + 1;  // skip the centre
        const int ox = kk % 3 - 1, oy = kk / 3 - 1;  // (-1,-1),(0,-1),(1,-1),(-1,0),(1,0),(-1,1),(0,1),(1,1)
        const int32_t sx = x + ox * step, sy = y + oy * step;
        // uv_outside(coords_to_uv(s)) exactly: (sx + 0.5) / w < 0 iff sx < 0, and its rounding
        // exceeds 1 iff sx >= w (for w < 2^24 the quotient is >= 1 + 2^-13 or <= 1 - 2^-25)
        if (sx < 0 || sy < 0 || sx >= (int32_t)F.s[0] || sy >= (int32_t)F.s[1]) continue;
        const int32_t o = oc + oy * rstep * R::STRIDE + ox * step;
        const float4 t0 = s_nd[o];
        const uint4 trgb = s_rgb[o];
        const uint2 tbi = s_bi[o];
        const float si = __uint_as_float(tbi.y);
        const float w_normal = hk_pow16(fmaxf(0.0f, dot(normal, mk3(t0.x, t0.y, t0.z))));
        const float w_depth = hk_exp_weight((-fabsf(depth - t0.w)) / (fabsf(dot(depth_gradient, mk2((float)ox, (float)oy))) + 0.01f));
        const float w_instance = fmaxf(0.0f, 1.0f - fabsf(instance - si));
        const float w_geo = (w_normal * w_depth) * w_instance;
        const float kw = KERNEL3[oy + 1][ox + 1];
#pragma unroll
        for (int ch = 0; ch < C; ++ch) {
            f3 irr = dn_rgb(ch, trgb, tbi);
            if (bad3(irr)) continue;
            float sl = lum(irr);
            // x / lum_denom with the per-pixel reciprocal (div_by: the IEEE quotient for normal
            // results; lum_denom >= 0.001 and |x| <= 2 x 65504 for finite RGBA16F texels, and a
            // quotient below the normal range rounds exp() to 1 either way); hk_exp_weight: hk_exp's bits
            // for every argument a weight can take (<= 0, NaN clamped to 0 below)
            float w_lum = hk_exp_weight(div_by(-fabsf(l0[ch] - sl), lum_denom[ch], lum_rcp[ch]));
            float w = hk_clampf(w_geo * w_lum, 0.0f, 1.0f) * kw;
            sum_irr[ch] = sum_irr[ch] + irr * w;
            sum_w[ch] += w;
            if (ch >= 1) {  // FIREFLY_FILTERING on emissive and indirect (post_process.rs:1193-1197)
                m1[ch] += sl;
                m2[ch] += sl * sl;
                cnt[ch] += 1.0f;
            }
        }
    }
    f4 a = mk4(0, 0, 0, 0);
    if (LEVEL == 3) {
        int32_t gx, gy;
        nearest_texel(jittered_uv(F, coords_to_uv(x, y, F.s), 0.5f), F.S, gx, gy);
        a = load_albedo(F, D.albedo, gx, gy);
    }
    f3 res[3] = {mk3(0, 0, 0), mk3(0, 0, 0), mk3(0, 0, 0)};
#pragma unroll
    for (int ch = 0; ch < C; ++ch) {
        f3 ir = sum_w[ch] < 0.0001f ? mk3(0, 0, 0) : sum_irr[ch] / sum_w[ch];
        if (ch >= 1) {
            float mean = m1[ch] / cnt[ch];
            float var = m2[ch] / cnt[ch] - mean * mean;
            if (l0[ch] > mean + 3.0f * sqrtf(var)) ir = ir * (mean / l0[ch]);
        }
        if (LEVEL == 3) {  // the output texture: (ir, 1) x albedo
            store_rgba16f(D.output[ch], idx, mk4(ir.x * a.x, ir.y * a.y, ir.z * a.z, 1.0f * a.w));
        }
        res[ch] = ir;
    }
    if (LEVEL < 3) store_level(D, LEVEL + 1, idx, res[0], res[1], res[2], cbi.y);
}

// ------------------------------------------------------------------ tone mapping (tone_mapping.wgsl:21-32)
// one pixel's output texel from its direct, emissive and (has_i) indirect texels
HKD uint2 tone_texel(const Frame& F, uint2 dv, uint2 ev, uint2 iv, bool has_i)
{
    f4 c = mk4(unpack_lo16float(dv.x), unpack_hi16float(dv.x), unpack_lo16float(dv.y), unpack_hi16float(dv.y));
    const f4 e = mk4(unpack_lo16float(ev.x), unpack_hi16float(ev.x), unpack_lo16float(ev.y), unpack_hi16float(ev.y));
    c = mk4(c.x + e.x, c.y + e.y, c.z + e.z, c.w + e.w);
    if (has_i) {
        const f4 i = mk4(unpack_lo16float(iv.x), unpack_hi16float(iv.x), unpack_lo16float(iv.y), unpack_hi16float(iv.y));
        c = mk4(c.x + i.x, c.y + i.y, c.z + i.z, c.w + i.w);
    }
    f3 cc = vmax(xyz(c), mk3(0.0039f, 0.0039f, 0.0039f));
    float l_old = lum(cc);
    float l_new = l_old / (1.0f + l_old);
    cc = cc * (l_new / l_old);
    f4 o = c.w > 0.0f ? mk4(cc.x, cc.y, cc.z, c.w) : mk4(F.clear_color[0], F.clear_color[1], F.clear_color[2], F.clear_color[3]);
    return make_uint2(pack2x16float(o.x, o.y), pack2x16float(o.z, o.w));
}
__global__ __launch_bounds__(256) void k_tone(FrameArgs A, ToneArgs T)
{
    const Frame& F = A.F;
    int32_t x, y;
    if (!tile_pixel<XCD_RASTER>(F, F.s[0], F.s_row0, F.s_rows, x, y)) return;
    const int32_t idx = s_index(F, x, y);
    T.output[idx] = tone_texel(F, T.direct[idx], T.emissive[idx], T.indirect ? T.indirect[idx] : make_uint2(0u, 0u),
                               T.indirect != nullptr);
}
// The same over the launch window as runs of TONE_RUN pixels of a row (launch_tone, when the plane width and the
// window's columns are multiples of TONE_RUN): a texel depends on its own pixel only, so a thread takes TONE_RUN
// consecutive texels of each plane (16-byte loads) and a wave 64 x 8 x TONE_RUN bytes of contiguous plane, instead of
// an 8x8 tile whose rows are 64-byte half lines.  Run q of the window: local row ly0 + q / runs, columns
// x0 + TONE_RUN (q % runs) ...
constexpr int TONE_RUN = 2;  // 2: 0.0143 ms on cornell, 4: 0.0156, 8: 0.0204 (profiles/r06/c19)
__global__ __launch_bounds__(256) void k_tone_run(FrameArgs A, ToneArgs T, int32_t ly0, int32_t x0, uint32_t runs, uint32_t n)
{
    constexpr int V = TONE_RUN / 2;  // 16-byte vectors per plane
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (q >= n) return;
    const uint32_t r = q / runs;
    const int32_t idx = x0 + TONE_RUN * (int32_t)(q - r * runs) + (int32_t)A.F.s[0] * (ly0 + (int32_t)r);
    const uint4* d = reinterpret_cast<const uint4*>(T.direct + idx);
    const uint4* e = reinterpret_cast<const uint4*>(T.emissive + idx);
    const uint4* ip = reinterpret_cast<const uint4*>(T.indirect + idx);
    const bool has_i = T.indirect != nullptr;
    uint4 dv[V], ev[V], iv[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
        dv[k] = d[k];
        ev[k] = e[k];
        iv[k] = has_i ? ip[k] : make_uint4(0u, 0u, 0u, 0u);
    }
    const Frame& F = A.F;
    uint4* o = reinterpret_cast<uint4*>(T.output + idx);
#pragma unroll
    for (int k = 0; k < V; ++k) {
        const uint2 a = tone_texel(F, make_uint2(dv[k].x, dv[k].y), make_uint2(ev[k].x, ev[k].y), make_uint2(iv[k].x, iv[k].y), has_i);
        const uint2 b = tone_texel(F, make_uint2(dv[k].z, dv[k].w), make_uint2(ev[k].z, ev[k].w), make_uint2(iv[k].z, iv[k].w), has_i);
        o[k] = make_uint4(a.x, a.y, b.x, b.y);
    }
}

// ------------------------------------------------------------------ stand-alone ray query
__global__ __launch_bounds__(256) void k_trace(Scene sc, const float* rays, const float* max_d, const float* early_d,
                                               const uint32_t* excl, uint32_t n, uint32_t* hits, unsigned long long* top)
{
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t cnt = 0;
    if (i < n) {
        cnt = 1;
        Ray ray;
        ray.origin = ld3(rays + 6 * (size_t)i);
        ray.direction = ld3(rays + 6 * (size_t)i + 3);
        ray.inv_direction = inv(ray.direction);
        Hit h = traverse_top(sc, ray, max_d ? max_d[i] : HK_F32_MAX, early_d ? early_d[i] : 0.0f,
                             excl ? excl[i] : DONT_EXCLUDE);
        uint32_t* o = hits + 5 * (size_t)i;
        o[0] = __float_as_uint(h.uv.x);
        o[1] = __float_as_uint(h.uv.y);
        o[2] = __float_as_uint(h.distance);
        o[3] = h.instance_index;
        o[4] = h.primitive_index;
    }
    wave_count(top, cnt);
}

// ------------------------------------------------------------------ launchers
static dim3 tiles(uint32_t width, int32_t rows) { return dim3((width + 15u) / 16u, ((uint32_t)rows + 15u) / 16u, 1); }
// the pixels of the context's planes a launch-shape choice weighs: the band's rows, at a tile's window width
static double plane_px(const Frame& F) { return (double)(F.win_cols > 0 ? (uint32_t)F.win_cols : F.s[0]) * (double)F.s_rows; }
// the tile grid of a launch: its window's rows (Frame::win_rows), else the plane's
static dim3 tiles(const Frame& F, uint32_t width, int32_t rows)
{
    return tiles(F.win_cols > 0 ? (uint32_t)F.win_cols : width, F.win_rows > 0 ? F.win_rows : rows);
}

// LDS staging is used when the kernel's scene arrays fit LDS_SCENE_MAX and the kernel gains from
// it.  Measured on cornell 1080p (1 x MI355X): indirect 0.370 -> 0.317 ms; direct_lit even;
// direct_emissive 0.167 -> 0.183 ms and the G-buffer even, so those two stay on global loads
// (round 1, word-by-word staging; round 4: the fused direct launch stages, launch_direct_fused).
// Option lds_scene: 0 disables staging, 2 stages in every traversal kernel.
static uint32_t lds_plan_bytes(const FrameArgs& A, int plan, bool preferred)
{
    const int mode = A.opt.lds_scene;
    if (mode == 0 || (mode == 1 && !preferred)) return 0u;
    uint32_t b = stage_bytes(A.sc.bytes, plan);
    return b <= LDS_SCENE_MAX ? b : 0u;
}

void launch_gbuffer(const FrameArgs& A, const ViewArgs& V, uint2* albedo, uint32_t stack_need, hipStream_t st)
{
    const dim3 g = tiles(A.F, A.F.S[0], A.F.S_rows);
    constexpr uint32_t level_bytes = 256u * sizeof(uint2);  // one stack level of the workgroup
    // option gbuffer_stack_full: the shallow variant with all GB_STACK_LDS levels (the round-2 allocation)
    const bool full = A.opt.gbuffer_stack_full != 0;
    const bool shallow = stack_need <= (uint32_t)GB_STACK_LDS && !A.opt.gbuffer_deep;
    const uint32_t levels = full ? (uint32_t)GB_STACK_LDS : (stack_need ? stack_need : 1u);
    // A small frame (an 8- or 4-way stripe of 1080p: <= gbuffer_lds_max_px pixels, one dispatch round) is as long
    // as one wave's walk, a chain of dependent node loads: there the scene is staged in LDS with the stack after it
    // (cornell 8-way stripe ...).  A whole frame runs many rounds and stays on L2 node loads (round 1: even).
    const bool small = (double)(A.F.win_cols > 0 ? (uint32_t)A.F.win_cols : A.F.S[0]) *
                           (double)(A.F.win_rows > 0 ? A.F.win_rows : A.F.S_rows) <= A.opt.gbuffer_lds_max_px;
    const uint32_t scene = lds_plan_bytes(A, PLAN_GBUFFER, small);
    // (scene + stack within the LDS budget of a staged kernel)
    if (scene && shallow && scene + levels * level_bytes <= LDS_SCENE_MAX + 16384u)
        hipLaunchKernelGGL((k_gbuffer<true, true>), g, dim3(256), scene + levels * level_bytes, st, A, V, albedo);
    else if (scene) hipLaunchKernelGGL((k_gbuffer<true, false, 0>), g, dim3(256), scene, st, A, V, albedo);
    else if (shallow) {
        // pushes never exceed the bound (hk_runtime gb_stack_need: inner nodes on a TLAS + BLAS path)
        hipLaunchKernelGGL((k_gbuffer<false, true>), g, dim3(256), levels * level_bytes, st, A, V, albedo);
    } else {
        // a deep scene: GB_DEEP_LDS levels in LDS, the rest in scratch (8 levels: 16 KiB per workgroup,
        // 8 waves/SIMD instead of 5; city 4K G-buffer 0.388 -> 0.362 ms, 4 levels 0.374, scene 1080p
        // unchanged)
        hipLaunchKernelGGL((k_gbuffer<false, false, GB_DEEP_LDS>), g, dim3(256), (uint32_t)GB_DEEP_LDS * level_bytes, st, A,
                           V, albedo);
    }
}
void launch_albedo(const FrameArgs& A, uint2* albedo, hipStream_t st)
{
    hipLaunchKernelGGL(k_albedo, tiles(A.F, A.F.S[0], A.F.S_rows), dim3(256), 0, st, A, albedo);
}
// a validation frame of a direct-light pass: frame.number % interval == 0 (umod: interval 0 -> 0)
static bool validation_frame(uint32_t number, uint32_t interval) { return interval == 0u || number % interval == 0u; }
template <bool EL, bool RE, bool LDS>
static void launch_direct_v(const FrameArgs& A, const ChannelArgs& C, bool val, dim3 g, uint32_t lds, hipStream_t st)
{
    if (val) hipLaunchKernelGGL((k_direct<EL, RE, LDS, true>), g, dim3(256), lds, st, A, C);
    else hipLaunchKernelGGL((k_direct<EL, RE, LDS, false>), g, dim3(256), lds, st, A, C);
}
void launch_direct(const FrameArgs& A, const ChannelArgs& C, bool emissive_lit, hipStream_t st)
{
    dim3 g = tiles(A.F, A.F.s[0], A.F.s_rows);
    // staged since round 4 (stage_scene) on frames of >= direct_w4_min_px pixels: cornell 1080p under an orbiting
    // camera direct_lit 0.110 -> 0.098 ms, emissive 0.124 -> 0.109 ms, frame 0.457 -> 0.413 ms (profiles/r04/c22,
    // c23); a 256x256 frame (256 workgroups) lost 3 % with it (c23)
    const bool big = plane_px(A.F) >= A.opt.direct_w4_min_px;
    const uint32_t lds = lds_plan_bytes(A, PLAN_LIGHT, big);
    if (emissive_lit) {
        const bool val = validation_frame(A.F.number, A.F.emissive_validate_interval);
        if (lds) launch_direct_v<true, false, true>(A, C, val, g, lds, st);
        else launch_direct_v<true, false, false>(A, C, val, g, 0, st);
    } else {
        const bool val = validation_frame(A.F.number, A.F.direct_validate_interval);
        if (plane_px(A.F) >= A.opt.direct_w4_min_px) {
            if (lds) {
                if (val) hipLaunchKernelGGL((k_direct_lit_w4<true, true>), g, dim3(256), lds, st, A, C);
                else hipLaunchKernelGGL((k_direct_lit_w4<true, false>), g, dim3(256), lds, st, A, C);
            } else {
                if (val) hipLaunchKernelGGL((k_direct_lit_w4<false, true>), g, dim3(256), 0, st, A, C);
                else hipLaunchKernelGGL((k_direct_lit_w4<false, false>), g, dim3(256), 0, st, A, C);
            }
        } else if (lds) launch_direct_v<false, true, true>(A, C, val, g, lds, st);
        else launch_direct_v<false, true, false>(A, C, val, g, 0, st);
    }
}
template <bool LDS>
static void launch_fused_v(const FrameArgs& A, const ChannelArgs& C0, const ChannelArgs& C1, bool vd, bool ve, dim3 g,
                           uint32_t lds, hipStream_t st)
{
    const bool w4 = A.opt.fused_w4 != 0;
    if (!LDS && w4 && !ve && (A.opt.compact_emitter || A.opt.compact_shadow)) {
        // (compact_shadow implies the emitter compaction: one kernel variant per shadow choice)
        if (A.opt.compact_shadow) {
            if (vd) hipLaunchKernelGGL((k_direct_fused_cw<true, true>), g, dim3(256), lds, st, A, C0, C1);
            else hipLaunchKernelGGL((k_direct_fused_cw<false, true>), g, dim3(256), lds, st, A, C0, C1);
        } else if (vd) hipLaunchKernelGGL((k_direct_fused_cw<true, false>), g, dim3(256), lds, st, A, C0, C1);
        else hipLaunchKernelGGL((k_direct_fused_cw<false, false>), g, dim3(256), lds, st, A, C0, C1);
    } else if (!LDS && w4 && ve) {
        if (vd) hipLaunchKernelGGL((k_direct_fused_w4<LDS, true, true>), g, dim3(256), lds, st, A, C0, C1);
        else hipLaunchKernelGGL((k_direct_fused_w4<LDS, false, true>), g, dim3(256), lds, st, A, C0, C1);
    } else if (vd && ve) hipLaunchKernelGGL((k_direct_fused<LDS, true, true>), g, dim3(256), lds, st, A, C0, C1);
    else if (ve) hipLaunchKernelGGL((k_direct_fused<LDS, false, true>), g, dim3(256), lds, st, A, C0, C1);
    else if (w4 && vd) hipLaunchKernelGGL((k_direct_fused_w4<LDS, true>), g, dim3(256), lds, st, A, C0, C1);
    else if (w4) hipLaunchKernelGGL((k_direct_fused_w4<LDS, false>), g, dim3(256), lds, st, A, C0, C1);
    else if (vd) hipLaunchKernelGGL((k_direct_fused<LDS, true, false>), g, dim3(256), lds, st, A, C0, C1);
    else hipLaunchKernelGGL((k_direct_fused<LDS, false, false>), g, dim3(256), lds, st, A, C0, C1);
}
void launch_direct_fused(const FrameArgs& A, const ChannelArgs& C0, const ChannelArgs& C1, hipStream_t st)
{
    dim3 g = tiles(A.F, A.F.s[0], A.F.s_rows);
    // staged by default since the staging copies chunks with their loads in flight (stage_scene): cornell 1080p
    // 0.179 -> 0.154 ms, frame 0.363 -> 0.345 ms (profiles/r04/c15, option lds_scene = 2 then)
    const uint32_t lds = lds_plan_bytes(A, PLAN_LIGHT, true);
    const bool vd = validation_frame(A.F.number, A.F.direct_validate_interval);
    const bool ve = validation_frame(A.F.number, A.F.emissive_validate_interval);
    if (lds) launch_fused_v<true>(A, C0, C1, vd, ve, g, lds, st);
    else launch_fused_v<false>(A, C0, C1, vd, ve, g, 0, st);
}
// workgroups of a persistent launch: what the device holds resident of this kernel, at most one 8x8 tile per wave
static uint32_t persist_grid(const void* kernel, uint32_t lds, const Frame& F)
{
    // CU count and resident workgroups per CU, per (device, kernel, LDS bytes): queried once each.
    // Contexts of different devices may launch from different host threads, so the cache is keyed by
    // the current device and guarded.
    struct Occ {
        int dev;
        const void* kernel;
        uint32_t lds;
        int per_cu, cus;
    };
    static std::mutex mu;
    static Occ cache[32];
    static int cached = 0;
    int dev = 0;
    (void)hipGetDevice(&dev);
    int per_cu = -1, cus = 0;
    {
        std::lock_guard<std::mutex> lock(mu);
        for (int i = 0; i < cached; ++i)
            if (cache[i].dev == dev && cache[i].kernel == kernel && cache[i].lds == lds) {
                per_cu = cache[i].per_cu;
                cus = cache[i].cus;
            }
        if (per_cu < 0) {
            per_cu = 0;
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, lds);
            if (cached < 32) cache[cached++] = Occ{dev, kernel, lds, per_cu, cus};
        }
    }
    const int32_t rows = F.win_rows > 0 ? F.win_rows : F.s_rows;
    const uint32_t cols = F.win_cols > 0 ? (uint32_t)F.win_cols : F.s[0];
    const uint32_t tiles8 = ((cols + 7u) / 8u) * (((uint32_t)rows + 7u) / 8u);
    const uint32_t g = (uint32_t)(per_cu > 0 ? per_cu : 1) * (uint32_t)(cus > 0 ? cus : 1);
    const uint32_t need = (tiles8 + 3u) / 4u;
    return need < g ? (need > 0u ? need : 1u) : g;
}
void launch_indirect(const FrameArgs& A, const ChannelArgs& C, bool multi, hipStream_t st)
{
    dim3 g = tiles(A.F, A.F.s[0], A.F.s_rows);
    const uint32_t lds = lds_plan_bytes(A, PLAN_LIGHT, true);
    if (A.opt.persistent_indirect) {
#define HK_PERSIST_LAUNCH(M_, L_)                                                                                    \
    hipLaunchKernelGGL((k_indirect_persist<M_, L_>), dim3(persist_grid((const void*)k_indirect_persist<M_, L_>, lds, A.F)), \
                       dim3(256), lds, st, A, C)
        if (multi) {
            if (lds) HK_PERSIST_LAUNCH(true, true);
            else HK_PERSIST_LAUNCH(true, false);
        } else {
            if (lds) HK_PERSIST_LAUNCH(false, true);
            else HK_PERSIST_LAUNCH(false, false);
        }
#undef HK_PERSIST_LAUNCH
        return;
    }
    if (multi) {
        if (lds) hipLaunchKernelGGL((k_indirect<true, true>), g, dim3(256), lds, st, A, C);
        else hipLaunchKernelGGL((k_indirect<true, false>), g, dim3(256), 0, st, A, C);
    } else if (A.opt.compact_shadow) {
        if (lds) hipLaunchKernelGGL((k_indirect<false, true, true>), g, dim3(256), lds, st, A, C);
        else hipLaunchKernelGGL((k_indirect<false, false, true>), g, dim3(256), 0, st, A, C);
    } else {
        if (lds) hipLaunchKernelGGL((k_indirect<false, true>), g, dim3(256), lds, st, A, C);
        else hipLaunchKernelGGL((k_indirect<false, false>), g, dim3(256), 0, st, A, C);
    }
}
bool light_lds_direct(const FrameArgs& A) { return lds_plan_bytes(A, PLAN_LIGHT, false) != 0u; }
void launch_light_merged(const FrameArgs& A, const ChannelArgs& C0, const ChannelArgs& C1, const ChannelArgs& C2,
                         hipStream_t st)
{
    dim3 g = tiles(A.F, A.F.s[0], A.F.s_rows);
    // the direct workgroups are dispatched first (grid z 0, then the indirect ones at z 1): cornell 4-way stripe
    // 0.1453 -> 0.1412 ms/frame, 2- and 8-way even, against the indirect ones first (round 3's order, then 8-way
    // 0.1194 -> 0.1181 against even / odd blockIdx.x; profiles/r05/c16, c18)
    g.z = 2u;
    const uint32_t scene = lds_plan_bytes(A, PLAN_LIGHT, true);
    const bool vd = validation_frame(A.F.number, A.F.direct_validate_interval);
    const bool ve = validation_frame(A.F.number, A.F.emissive_validate_interval);
    const uint32_t park = (vd || ve) ? (uint32_t)(PARK_WORDS * 256 * sizeof(float)) : 0u;
    const uint32_t ind = scene + (uint32_t)sizeof(IndStash);  // the indirect role: staged scene + stash
    const uint32_t lds = ind > park ? ind : park;
#define HK_MERGED(VD_, VE_)                                                                                         \
    if (scene) hipLaunchKernelGGL((k_light_merged<VD_, VE_, true>), g, dim3(256), lds, st, A, C0, C1, C2);          \
    else hipLaunchKernelGGL((k_light_merged<VD_, VE_, false>), g, dim3(256), lds, st, A, C0, C1, C2);
    if (vd && ve) { HK_MERGED(true, true) }
    else if (vd) { HK_MERGED(true, false) }
    else if (ve) { HK_MERGED(false, true) }
    else { HK_MERGED(false, false) }
#undef HK_MERGED
}
void launch_indirect_wavefront(const FrameArgs& A, const ChannelArgs& C, const WfArgs& W, hipStream_t st)
{
    const dim3 g = tiles(A.F, A.F.s[0], A.F.s_rows);
    const uint32_t lds = lds_plan_bytes(A, PLAN_LIGHT, true);
    const dim3 per_seg(WF_SEGS * (W.seg_cap / 256u));      // every segment's entries, 256 per workgroup
    const dim3 all(((uint32_t)A.F.s[0] * (uint32_t)A.F.s_rows + 255u) / 256u);
    hipLaunchKernelGGL(k_wf_gen, g, dim3(256), 0, st, A, C, W);
    if (lds) hipLaunchKernelGGL(k_wf_trace<true>, per_seg, dim3(256), lds, st, A, C, W);
    else hipLaunchKernelGGL(k_wf_trace<false>, per_seg, dim3(256), 0, st, A, C, W);
    hipLaunchKernelGGL(k_wf_scan, dim3(1), dim3(256), 0, st, W);
    hipLaunchKernelGGL(k_wf_scatter, per_seg, dim3(256), 0, st, W);
    if (lds) hipLaunchKernelGGL(k_wf_shade<true>, all, dim3(256), lds, st, A, C, W);
    else hipLaunchKernelGGL(k_wf_shade<false>, all, dim3(256), 0, st, A, C, W);
}
void launch_spatial(const FrameArgs& A, const ChannelArgs& C, bool emissive_lit, hipStream_t st)
{
    dim3 g = tiles(A.F, A.F.s[0], A.F.s_rows);
    // the window assumes integrator pixels == deferred pixels (upscale ratio 1)
    const bool window = A.F.upscale_ratio == 1.0f && A.F.s[0] == A.F.S[0] && A.F.s[1] == A.F.S[1];
    // the view planes hold the indirect channel's records only (ChannelArgs::view)
    if (emissive_lit) {
        if (window) hipLaunchKernelGGL((k_spatial<true, false>), g, dim3(256), 0, st, A, C);
        else hipLaunchKernelGGL((k_spatial_nowin<true, false>), g, dim3(256), 0, st, A, C);
    } else if (C.view) {
        if (window) hipLaunchKernelGGL((k_spatial<false, true>), g, dim3(256), 0, st, A, C);
        else hipLaunchKernelGGL((k_spatial_nowin<false, true>), g, dim3(256), 0, st, A, C);
    } else {
        if (window) hipLaunchKernelGGL((k_spatial<false, false>), g, dim3(256), 0, st, A, C);
        else hipLaunchKernelGGL((k_spatial_nowin<false, false>), g, dim3(256), 0, st, A, C);
    }
}
void launch_demod(const FrameArgs& A, const DenoiseArgs& D, hipStream_t st)
{
    dim3 g = tiles(A.F, A.F.s[0], A.F.s_rows);
    if (D.channels == 3) hipLaunchKernelGGL(k_demod3<3>, g, dim3(256), 0, st, A, D);
    else hipLaunchKernelGGL(k_demod3<2>, g, dim3(256), 0, st, A, D);
}
template <int C, int LEVEL>
static void launch_level(const FrameArgs& A, const DenoiseArgs& D, hipStream_t st)
{
    const dim3 g = level_tiles<LEVEL>(A.F.win_cols > 0 ? (uint32_t)A.F.win_cols : A.F.s[0],
                                      A.F.win_rows > 0 ? A.F.win_rows : A.F.s_rows);
    hipLaunchKernelGGL((k_denoise3<C, LEVEL>), g, dim3(256), 0, st, A, D);
}
template <int C>
static void launch_level(const FrameArgs& A, const DenoiseArgs& D, int level, hipStream_t st)
{
    switch (level) {
    case 0: launch_level<C, 0>(A, D, st); break;
    case 1: launch_level<C, 1>(A, D, st); break;
    case 2: launch_level<C, 2>(A, D, st); break;
    default: launch_level<C, 3>(A, D, st); break;
    }
}
void launch_denoise(const FrameArgs& A, const DenoiseArgs& D, int level, hipStream_t st)
{
    if (D.channels == 3) launch_level<3>(A, D, level, st);
    else launch_level<2>(A, D, level, st);
}
void launch_tone(const FrameArgs& A, const ToneArgs& T, hipStream_t st)
{
    const Frame& F = A.F;
    const int32_t ly0 = F.win_rows > 0 ? F.win_row0 : 0, rows = F.win_rows > 0 ? F.win_rows : F.s_rows;
    const int32_t x0 = F.win_cols > 0 ? F.win_col0 : 0, cols = F.win_cols > 0 ? F.win_cols : (int32_t)F.s[0];
    if (F.s[0] % (uint32_t)TONE_RUN == 0u && x0 % TONE_RUN == 0 && cols % TONE_RUN == 0 && rows > 0 && cols > 0) {
        const uint32_t runs = (uint32_t)cols / (uint32_t)TONE_RUN, n = runs * (uint32_t)rows;
        hipLaunchKernelGGL(k_tone_run, dim3((n + 255u) / 256u), dim3(256), 0, st, A, T, ly0, x0, runs, n);
    } else {
        hipLaunchKernelGGL(k_tone, tiles(A.F, A.F.s[0], A.F.s_rows), dim3(256), 0, st, A, T);
    }
}
// ------------------------------------------------------------------ sub-frame accumulation
__global__ __launch_bounds__(256) void k_accumulate(const uint2* tone, float4* acc, uint32_t n, int reset)
{
    uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    f4 t = load_rgba16f(tone, (int32_t)i);
    float4 a = reset ? make_float4(0, 0, 0, 0) : acc[i];
    acc[i] = make_float4(a.x + t.x, a.y + t.y, a.z + t.z, a.w + t.w);
}
__global__ __launch_bounds__(256) void k_resolve(const float4* acc, uint32_t n, float count, uint2* out)
{
    uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    float4 a = acc[i];
    store_rgba16f(out, (int32_t)i, mk4(a.x / count, a.y / count, a.z / count, a.w / count));
}
void launch_accumulate(const uint2* tone, float4* acc, uint32_t n, int reset, hipStream_t st)
{
    if (n) hipLaunchKernelGGL(k_accumulate, dim3((n + 255u) / 256u), dim3(256), 0, st, tone, acc, n, reset);
}
void launch_resolve(const float4* acc, uint32_t n, float count, uint2* out, hipStream_t st)
{
    if (n) hipLaunchKernelGGL(k_resolve, dim3((n + 255u) / 256u), dim3(256), 0, st, acc, n, count, out);
}

// ------------------------------------------------------------------ scene preparation
// The reference's flattened leaves carry an empty AABB and the kernels recompute the box of the
// leaf's triangle / instance before testing it (light.wgsl:411-412, 456-457).  At upload the
// device copy of each leaf gets exactly that box (same vmin/vmax expression on the device, or
// the instance record's min/max), so the traversal reads it with the node and only fetches the
// 48-byte triangle / 176-byte instance once the box test has passed.  Same tests, same order.
__global__ __launch_bounds__(256) void k_fill_blas_leaves(hk_node* nodes, uint32_t n, const uint32_t* prim_offset,
                                                          const hk_primitive* prims)
{
    uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n || prim_offset[i] == HK_U32_MAX) return;
    hk_node& nd = nodes[i];
    if (nd.entry_index < HK_BVH_LEAF_FLAG) return;
    f3 a, b, c;
    load_triangle(prims, prim_offset[i] + nd.entry_index - HK_BVH_LEAF_FLAG, a, b, c);
    f3 mn = vmin(a, vmin(b, c)), mx = vmax(a, vmax(b, c));
    nd.min[0] = mn.x, nd.min[1] = mn.y, nd.min[2] = mn.z;
    nd.max[0] = mx.x, nd.max[1] = mx.y, nd.max[2] = mx.z;
}
__global__ __launch_bounds__(256) void k_fill_tlas_leaves(hk_node* nodes, uint32_t n, const hk_instance* inst,
                                                          uint32_t n_inst)
{
    uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    hk_node& nd = nodes[i];
    if (nd.entry_index < HK_BVH_LEAF_FLAG || nd.entry_index - HK_BVH_LEAF_FLAG >= n_inst) return;
    const hk_instance& in = inst[nd.entry_index - HK_BVH_LEAF_FLAG];
    for (int k = 0; k < 3; ++k) nd.min[k] = in.min[k], nd.max[k] = in.max[k];
}
// Wide entries for the G-buffer traversal (hk_device.h closest_hit_ordered), built from the
// prepared flat nodes: node_base/node_count = the owning mesh's node range (TLAS: 0, n).
__global__ __launch_bounds__(256) void k_build_wide(const hk_node* flat, uint32_t n, const uint32_t* node_base,
                                                    const uint32_t* node_count, float4* wide)
{
    uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= n) return;
    float4* w = wide + 4u * (size_t)p;
    const hk_node& f = flat[p];
    const uint32_t base = node_base ? node_base[p] : 0u, count = node_count ? node_count[p] : n;
    // leaf entry: (box min, payload | LEAF), (box max, U32_MAX); inner: see below (w[1].w != U32_MAX)
    w[0] = make_float4(f.min[0], f.min[1], f.min[2], __uint_as_float(f.entry_index));
    w[1] = make_float4(f.max[0], f.max[1], f.max[2], __uint_as_float(HK_U32_MAX));
    w[2] = make_float4(0, 0, 0, 0);
    w[3] = make_float4(0, 0, 0, 0);
    if (f.entry_index >= HK_BVH_LEAF_FLAG || base == HK_U32_MAX) return;
    // inner subtree starting at p: left box node p (subtree p+1), right box node q (subtree q+1).
    // A child subtree that is a single leaf whose box equals the child box (bitwise) is stored as
    // its payload (LEAF | payload): the walk's descent / pop comparison already is that leaf's
    // box test, so the leaf entry is not loaded.
    const uint32_t local = p - base, q_local = f.exit_index;
    if (q_local >= count) return;  // p is a right-child box node, never a subtree start
    const hk_node& g = flat[base + q_local];
    auto target = [&](const hk_node& child, uint32_t start) -> uint32_t {
        if (start >= count) return start;
        const hk_node& lf = flat[base + start];
        if (lf.entry_index < HK_BVH_LEAF_FLAG) return start;
        for (int k = 0; k < 3; ++k)
            if (__float_as_uint(lf.min[k]) != __float_as_uint(child.min[k]) ||
                __float_as_uint(lf.max[k]) != __float_as_uint(child.max[k]))
                return start;
        return lf.entry_index;
    };
    w[0].w = __uint_as_float(target(f, local + 1u));
    w[1].w = __uint_as_float(target(g, q_local + 1u));
    w[2] = make_float4(g.min[0], g.min[1], g.min[2], 0.0f);
    w[3] = make_float4(g.max[0], g.max[1], g.max[2], 0.0f);
}
void launch_build_wide(const hk_node* flat, uint32_t n, const uint32_t* node_base, const uint32_t* node_count,
                       float4* wide, hipStream_t st)
{
    if (n) hipLaunchKernelGGL(k_build_wide, dim3((n + 255u) / 256u), dim3(256), 0, st, flat, n, node_base, node_count,
                              wide);
}

// Leaf collapse of the device node copies for the light-pass walks.  bvh 0.7.1 flattens a leaf
// child into a child-box node p (the BVH's child AABB; entry p+1, exit q) followed by the leaf
// node p+1 (payload, exit q).  The reference tests p's box, then at p+1 the recomputed triangle /
// instance box (light.wgsl:411-413, 456-457) with the same ray and the same hit distance (nothing
// changes between the two visits).  Where the two boxes are bitwise identical the second test
// repeats the first, so p can take the leaf's payload (entry = LEAF | payload, same exit): one
// node visit per leaf instead of two, the same tests and results.  Two passes (decide, write) so
// no thread reads a node another thread rewrites.  The G-buffer wide layout is built before this.
__global__ __launch_bounds__(256) void k_collapse_decide(const hk_node* nodes, uint32_t n, const uint32_t* node_base,
                                                         const uint32_t* node_count, uint32_t* new_entry)
{
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= n) return;
    const hk_node nd = nodes[p];
    new_entry[p] = nd.entry_index;
    const uint32_t base = node_base ? node_base[p] : 0u, count = node_count ? node_count[p] : n;
    if (base == HK_U32_MAX || nd.entry_index >= HK_BVH_LEAF_FLAG || nd.entry_index >= count) return;
    const hk_node lf = nodes[base + nd.entry_index];
    if (lf.entry_index < HK_BVH_LEAF_FLAG || lf.exit_index != nd.exit_index) return;
    for (int k = 0; k < 3; ++k)
        if (__float_as_uint(lf.min[k]) != __float_as_uint(nd.min[k]) || __float_as_uint(lf.max[k]) != __float_as_uint(nd.max[k]))
            return;
    new_entry[p] = lf.entry_index;
}
__global__ __launch_bounds__(256) void k_collapse_write(hk_node* nodes, uint32_t n, const uint32_t* new_entry)
{
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p < n) nodes[p].entry_index = new_entry[p];
}
void launch_collapse_leaves(hk_node* nodes, uint32_t n, const uint32_t* node_base, const uint32_t* node_count,
                            uint32_t* scratch, hipStream_t st)
{
    if (!n) return;
    const dim3 g((n + 255u) / 256u);
    hipLaunchKernelGGL(k_collapse_decide, g, dim3(256), 0, st, nodes, n, node_base, node_count, scratch);
    hipLaunchKernelGGL(k_collapse_write, g, dim3(256), 0, st, nodes, n, scratch);
}

void launch_fill_leaves(hk_node* blas, uint32_t n_blas, const uint32_t* prim_offset, const hk_primitive* prims,
                        hk_node* tlas, uint32_t n_tlas, const hk_instance* inst, uint32_t n_inst, hipStream_t st)
{
    if (n_blas) hipLaunchKernelGGL(k_fill_blas_leaves, dim3((n_blas + 255u) / 256u), dim3(256), 0, st, blas, n_blas,
                                   prim_offset, prims);
    if (n_tlas) hipLaunchKernelGGL(k_fill_tlas_leaves, dim3((n_tlas + 255u) / 256u), dim3(256), 0, st, tlas, n_tlas,
                                   inst, n_inst);
}

// exhaustive check of div_by against the IEEE divide: x over bit patterns [lo, hi) with both signs
__global__ __launch_bounds__(256) void k_div_check(float d, float r, uint32_t lo, uint32_t hi,
                                                   unsigned long long* bad)
{
    uint32_t n = 0;
    for (uint64_t u = (uint64_t)lo + blockIdx.x * 256u + threadIdx.x; u < hi; u += (uint64_t)gridDim.x * 256u) {
        for (uint32_t sgn = 0; sgn < 2; ++sgn) {
            const float x = __uint_as_float((uint32_t)u | (sgn << 31));
            const float a = div_by(x, d, r), b = x / d;
            if (__float_as_uint(a) != __float_as_uint(b) && !(a != a && b != b)) n++;
        }
    }
    wave_count(bad, n);
}
void launch_div_check(float d, float r, uint32_t lo, uint32_t hi, unsigned long long* bad, hipStream_t st)
{
    hipLaunchKernelGGL(k_div_check, dim3(8192), dim3(256), 0, st, d, r, lo, hi, bad);
}
// exhaustive check of rcp_exact against the IEEE divide 1 / x over bit patterns [lo, hi), both signs
__global__ __launch_bounds__(256) void k_rcp_check(uint32_t lo, uint32_t hi, unsigned long long* bad)
{
    uint32_t n = 0;
    for (uint64_t u = (uint64_t)lo + blockIdx.x * 256u + threadIdx.x; u < hi; u += (uint64_t)gridDim.x * 256u) {
        for (uint32_t sgn = 0; sgn < 2; ++sgn) {
            const float x = __uint_as_float((uint32_t)u | (sgn << 31));
            const float a = rcp_exact(x), b = 1.0f / x;
            if (__float_as_uint(a) != __float_as_uint(b) && !(a != a && b != b)) n++;
        }
    }
    wave_count(bad, n);
}
void launch_rcp_check(uint32_t lo, uint32_t hi, unsigned long long* bad, hipStream_t st)
{
    hipLaunchKernelGGL(k_rcp_check, dim3(8192), dim3(256), 0, st, lo, hi, bad);
}

__global__ __launch_bounds__(256) void k_f16(const float* in, uint32_t n, uint16_t* out)
{
    uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) out[i] = (uint16_t)(pack2x16float(in[i], 0.0f) & 0xFFFFu);
}

void launch_f16(const float* in, uint32_t n, uint16_t* out, hipStream_t st)
{
    hipLaunchKernelGGL(k_f16, dim3((n + 255u) / 256u), dim3(256), 0, st, in, n, out);
}

void launch_trace(const Scene& sc, const float* rays, const float* max_d, const float* early_d, const uint32_t* excl,
                  uint32_t n, uint32_t* hits, unsigned long long* top, hipStream_t st)
{
    hipLaunchKernelGGL(k_trace, dim3((n + 255u) / 256u), dim3(256), 0, st, sc, rays, max_d, early_d, excl, n, hits, top);
}

}  // namespace hk
