// hk_launch.h — kernel argument blocks and launchers shared by hk_kernels.hip and the
// host runtime (hk_runtime.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hk_device.h"
#include "../../include/hk_post.h"

namespace hk {

// Kernel-variant choices of the launchers (host only; hk_set_option keys in parentheses).  They pick
// among bit-identical kernels, so they change speed, never results.
struct LaunchOpts {
    int lds_scene = 1;               // ("lds_scene") 0: no LDS scene staging, 1: where it measured faster, 2: every traversal kernel
    int gbuffer_stack_full = 0;      // ("gbuffer_stack_full") shallow G-buffer walk with all GB_STACK_LDS levels
    int gbuffer_deep = 0;            // ("gbuffer_deep") the deep-scene G-buffer variant on any scene
    double gbuffer_lds_max_px = 6e5; // ("gbuffer_lds_max_px") G-buffer with the scene and its stack in LDS up to this many pixels
    double direct_w4_min_px = 4e5;   // ("direct_w4_min_px") k_direct_lit_w4 from this many pixels up
    int fused_w4 = 1;                // ("fused_w4") the 4-wave fused direct/emissive variants
    int persistent_indirect = 0;     // ("persistent_indirect") k_indirect_persist (opt-in, measured slower)
    int compact_emitter = 0;         // ("compact_emitter") the fused launch's emitter walks compacted per workgroup
    int compact_shadow = 0;          // ("compact_shadow") shadow walks compacted per workgroup (fused launch, indirect)
};

struct FrameArgs {
    Scene sc;
    Frame F;
    GBuffer G;
    const uchar4* noise;  // 16 x 64 x 64 RGBA8
    Counters cnt;
    LaunchOpts opt;       // host-side launcher choices (not read by the kernels)
};

// One channel's bindings: group 5 (variance/render) + group 6 (reservoir pair) of light.rs:455-555.
struct ChannelArgs {
    ResBuf prev;          // previous_reservoir_buffer  (read)
    ResBuf cur;           // reservoir_buffer            (write)
    ResBuf prev_spatial;  // previous_spatial_reservoir_buffer
    ResBuf spatial;       // spatial_reservoir_buffer
    float* variance;
    uint2* render;
    // Background store elision (k_direct_fused / k_indirect only; nullptr elsewhere): one byte per
    // pixel recording which of the pass's physical targets already hold a background pixel's
    // constant zero words (bit r = reservoir parity r's temporal buffers, bit 2 + s = render /
    // variance slot s, bit 4 = both buffers of the spatial pair).  bg_need = the bits this frame's
    // stores target; when all are set the stores are skipped (same bits in every buffer).
    uint8_t* bg;
    uint32_t bg_need;
    // Spatial view planes (indirect channel; nullptr elsewhere): 3 planes of view_n 16-byte chunks holding
    // what spatial reuse reads from a NEIGHBOUR's temporal record, derived from the packed words this
    // frame's temporal pass stores into `cur` (store_res_view, hk_device.h).  Written by the indirect
    // temporal pass when non-null, read by k_spatial<false, ·, true>.
    uint4* view;
    uint32_t view_n;
};

// Wavefront indirect pass (config 5: material-sorted shading), see hk_kernels.hip k_wf_*.
// The live-pixel queue is split into WF_SEGS segments (tile t -> segment t % WF_SEGS, each with room
// for all its tiles' pixels) so that appends and the material histogram spread their atomics over
// WF_SEGS addresses.  ctl words: [s] live pixels of segment s, [WF_SEGS] all live pixels,
// [WF_CTL_HIST + s * bins + b] segment s's pixels in material bin b, then the same layout of bin
// write cursors.
constexpr uint32_t WF_SEGS = 64;
constexpr uint32_t WF_CTL_HIST = WF_SEGS + 16;
constexpr uint32_t WF_MAX_BINS = 4096;  // materials + 1 (misses); larger scenes use the megakernel
struct WfArgs {
    uint32_t* queue1;  // live pixels (x | local row << 16): segment s at [s * seg_cap, s * seg_cap + count)
    uint32_t* keys;    // material bin per queue1 slot
    uint32_t* queue2;  // all live pixels, grouped by material bin
    uint4* hit;        // per pixel (s plane): instance, primitive, u bits, v bits of the bounce hit
    float* hit_t;      // per pixel: its distance
    uint32_t* ctl;
    uint32_t bins;     // n_materials + 1
    uint32_t seg_cap;  // queue1 slots per segment: 256 x ceil(tiles / WF_SEGS)
};
constexpr uint32_t wf_ctl_words(uint32_t bins) { return WF_CTL_HIST + 2u * WF_SEGS * bins; }

struct ViewArgs {
    float world_position[3];
    float view_proj[16];
    float inverse_view_proj[16];
    // prepass.wgsl:30-54: the primary ray of pixel (x, y) goes through (x + 0.5 - jitter[0], y + 0.5 - jitter[1])
    float jitter[2];
    // motion vectors (prepass.wgsl:96): 0 = camera and every instance static this frame, so the
    // velocity is exactly zero and is not computed
    int motion;
    float previous_view_proj[16];
    const float* previous_models;  // 16 floats per instance: model at the previous k_gbuffer
    // background store elision (as ChannelArgs::bg): bit s = G-buffer slot s holds a miss pixel's
    // zero texels in every plane (position, normal, gradient, ids, velocity/uv, albedo); nullptr = off
    uint8_t* bg;
    uint32_t bg_need;
};

// All channels of one frame (post_process.rs:1199-1223 runs them one after another).
struct DenoiseArgs {
    int channels;            // 3, or 2 when indirect_bounces == 0 (post_process.rs:949-954)
    const uint2* albedo;     // S
    const uint2* render[3];  // s
    const float* variance[3];
    // a level's input (the reference's internal textures of the 3 channels, hk_kernels.hip store_level): RGB f16
    // halves packed r0 g0 | b0 r1 | g1 b1 | r2 g2, and b2 | instance bits
    uint4* rgb[4];
    uint2* bi[4];
    float* internal_variance[3];
    uint2* output[3];
    float4* nd;              // per pixel: (normalised normal, depth)
    float4* center;          // per pixel: (depth gradient x, y, luminance denominator of channels 0, 1)
    float* den2;             // per pixel: luminance denominator of channel 2
};

struct ToneArgs {
    const uint2* direct;
    const uint2* emissive;
    const uint2* indirect;  // may be null (indirect_bounces == 0)
    uint2* output;
};

// Dynamic instance update (hk_dynamic.hip): device buffers + scratch, sized by the runtime.
struct DynamicArgs {
    hk_instance* instances;
    uint32_t n_instances;
    const float* models;       // n x 16, column-major
    const float* local_aabbs;  // n x 6: local AABB center xyz, half extents xyz (Bevy Aabb)
    hk_node* tlas;             // 3n - 2 nodes
    hk_emissive* emissives;
    uint32_t n_emissives;
    const hk_material* materials;
    const hk_primitive* primitives;
    hk_alias_entry* alias;
    uint32_t n_alias;
    hk_node* lbvh;             // 3m - 2 nodes
    int buckets;
    // scratch
    float* areas;              // alias entries
    void* alias_work;          // 2 x alias entries x 8 B
    void* boxes;               // max(n, m) x 24 B
    uint32_t* idx;             // 2 x max(n, m)
    void* segments;            // 2 x max(n, m) x 12 B
    uint32_t* flags;           // [0] singular transform, [1] TLAS split levels (G-buffer stack bound)
};
void launch_dynamic_update(const DynamicArgs& D, hipStream_t st);

// Post-process (hk_post.hip over include/hk_post.h)
struct PostArgs {
    hk_pp_frame frame;
    hk_pp_inputs in;
};
void launch_smaa(const PostArgs& P, hipStream_t st);
void launch_smaa_extrapolate(const PostArgs& P, hipStream_t st);
void launch_taa(const PostArgs& P, hipStream_t st);

bool lane_stats_take(unsigned long long out[2 * LANE_SLOTS], hipStream_t st);
void launch_gbuffer(const FrameArgs& A, const ViewArgs& V, uint2* albedo, uint32_t stack_need, hipStream_t st);
void launch_direct_fused(const FrameArgs& A, const ChannelArgs& C0, const ChannelArgs& C1, hipStream_t st);
void launch_albedo(const FrameArgs& A, uint2* albedo, hipStream_t st);
void launch_direct(const FrameArgs& A, const ChannelArgs& C, bool emissive_lit, hipStream_t st);
void launch_indirect(const FrameArgs& A, const ChannelArgs& C, bool multi, hipStream_t st);
// the wavefront indirect pass (one bounce): gen + compaction, bounce trace, bin scan, scatter by
// material, material-sorted shade; W.ctl must be zeroed on `st` before
void launch_indirect_wavefront(const FrameArgs& A, const ChannelArgs& C, const WfArgs& W, hipStream_t st);
void launch_spatial(const FrameArgs& A, const ChannelArgs& C, bool emissive_lit, hipStream_t st);
// the direct-light passes stage the scene in LDS (HK_LDS_SCENE=2 with a small enough scene)
bool light_lds_direct(const FrameArgs& A);
// direct_lit + emissive (fused per pixel) and the one-bounce indirect pass in one launch (k_light_merged)
void launch_light_merged(const FrameArgs& A, const ChannelArgs& C0, const ChannelArgs& C1, const ChannelArgs& C2,
                         hipStream_t st);
void launch_demod(const FrameArgs& A, const DenoiseArgs& D, hipStream_t st);
void launch_denoise(const FrameArgs& A, const DenoiseArgs& D, int level, hipStream_t st);
void launch_tone(const FrameArgs& A, const ToneArgs& T, hipStream_t st);
void launch_collapse_leaves(hk_node* nodes, uint32_t n, const uint32_t* node_base, const uint32_t* node_count,
                            uint32_t* scratch, hipStream_t st);
void launch_fill_leaves(hk_node* blas, uint32_t n_blas, const uint32_t* prim_offset, const hk_primitive* prims,
                        hk_node* tlas, uint32_t n_tlas, const hk_instance* inst, uint32_t n_inst, hipStream_t st);
void launch_build_wide(const hk_node* flat, uint32_t n, const uint32_t* node_base, const uint32_t* node_count,
                       float4* wide, hipStream_t st);
void launch_accumulate(const uint2* tone, float4* acc, uint32_t n, int reset, hipStream_t st);
void launch_resolve(const float4* acc, uint32_t n, float count, uint2* out, hipStream_t st);
void launch_div_check(float d, float r, uint32_t lo, uint32_t hi, unsigned long long* bad, hipStream_t st);
void launch_rcp_check(uint32_t lo, uint32_t hi, unsigned long long* bad, hipStream_t st);
void launch_f16(const float* in, uint32_t n, uint16_t* out, hipStream_t st);
void launch_trace(const Scene& sc, const float* rays, const float* max_d, const float* early_d, const uint32_t* excl,
                  uint32_t n, uint32_t* hits, unsigned long long* top, hipStream_t st);

}  // namespace hk
