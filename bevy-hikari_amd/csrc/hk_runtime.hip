// hk_runtime.hip — host runtime behind the C ABI (include/hikari_amd.h).
//
// One hk_ctx per camera entity owns everything the reference keeps per view:
//   ReservoirCache (light.rs:342-363)        -> 10 SoA reservoir buffers in HBM
//   LightTextures (light.rs:297-383)          -> albedo (S), variance[3], render[3] (s)
//   PostProcessTextures denoise part (post_process.rs:710-714) -> internal[4] (packed: dn_rgb / dn_bi), internal variance,
//                                               denoised[3], tone-mapped output
//   group-2 scene buffers (mesh_material/mod.rs:488-598) -> device copies of the std430 arrays
// hk_render_frame issues the kernels in LightNode::run order (light.rs:646-699) and
// hk_denoise in PostProcessNode::run order (post_process.rs:1190-1224).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/hikari_amd.h"
#include "hk_launch.h"

using namespace hk;

namespace {
constexpr int32_t BAND_HALO = 40;  // >= 36 rows: 20 (spatial reuse) + 15 (a-trous) + 1 (variance blur)
// 3 counters (top, emitter, primary) x COUNTER_SHARDS lines of 64 B
constexpr size_t COUNTER_SPAN = (size_t)COUNTER_SHARDS * COUNTER_STRIDE;  // u64 per counter
constexpr size_t COUNTER_BYTES = 3 * COUNTER_SPAN * sizeof(unsigned long long);
constexpr size_t PERSIST_BYTES = (size_t)PERSIST_KINDS * PERSIST_LINES * PERSIST_LINE * sizeof(unsigned long long);

struct TimedLaunch {
    const char* name;
    hipEvent_t start, stop;
};

// Runtime options (hk_set_option / hk_get_option): each picks among schedules or kernel variants that
// produce the same bits, so they change speed only.  Read once per call from the context (no environment
// variables on the frame path); the defaults are the measured-fastest configuration.
enum Opt {
    OPT_PIPELINE_MIN_PX,     // frame pipelining (G-buffer / tail streams) from this many integrator pixels up
    OPT_PIPELINE_HEAVY_MIN_PX,  // ... and from this many up on frames with spatial reuse or the denoiser
    OPT_GBUFFER_PIPELINE,    // k_gbuffer of frame f on its own stream next to frame f-1's light passes
    OPT_TAIL_PIPELINE,       // denoise + tone-sum of frame f on their own stream next to frame f+1
    OPT_CHANNEL_STREAMS,     // the indirect chain on a side stream next to direct -> emissive
    OPT_FUSE,                // k_direct_fused when every reprojection is the identity
    OPT_FUSE_MIN_PX,         // ... from this many pixels up
    OPT_MERGE,               // k_light_merged: -1 auto (small unpipelined frames), 0 never, 1 whenever possible
    OPT_BG_ELISION,          // background store elision (bg_elide)
    OPT_SPATIAL_VIEW,        // spatial view planes written by the indirect temporal pass
    OPT_BAND_FULL_WINDOWS,   // every pass of a band on all its rows (no per-pass row windows)
    OPT_LEAF_COLLAPSE,       // leaf-collapsed node copies for the light walks (at scene upload / update)
    OPT_GBUFFER_REUSE,       // skip k_gbuffer when its slot already holds this frame's planes (static sub-frames)
    OPT_LDS_SCENE,           // LaunchOpts
    OPT_GBUFFER_STACK_FULL,
    OPT_GBUFFER_DEEP,
    OPT_GBUFFER_LDS_MAX_PX,
    OPT_DIRECT_W4_MIN_PX,
    OPT_FUSED_W4,
    OPT_PERSISTENT_INDIRECT,
    OPT_COMPACT_EMITTER,
    OPT_COMPACT_SHADOW,
    OPT_COUNT
};
struct OptDef {
    const char* key;
    double def, lo, hi;
};
constexpr OptDef OPTS[OPT_COUNT] = {
    {"pipeline_min_px", 1.2e6, 0.0, 1e12}, {"pipeline_heavy_min_px", 0.0, 0.0, 1e12},
    {"gbuffer_pipeline", 1, 0, 1},         {"tail_pipeline", 1, 0, 1},
    {"channel_streams", 1, 0, 1},          {"fuse", 1, 0, 1},              {"fuse_min_px", 1048576.0, 0.0, 1e12},
    {"merge", -1, -1, 1},                  {"bg_elision", 1, 0, 1},        {"spatial_view_planes", 1, 0, 1},
    {"band_full_windows", 0, 0, 1},        {"leaf_collapse", 1, 0, 1},     {"gbuffer_reuse", 1, 0, 1},
    {"lds_scene", 1, 0, 2},                {"gbuffer_stack_full", 0, 0, 1}, {"gbuffer_deep", 0, 0, 1},
    {"gbuffer_lds_max_px", 6e5, 0.0, 1e12},
    {"direct_w4_min_px", 4e5, 0.0, 1e12},  {"fused_w4", 1, 0, 1},          {"persistent_indirect", 0, 0, 1},
    {"compact_emitter", 0, 0, 1},          {"compact_shadow", 0, 0, 1},
};
}  // namespace

struct hk_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string error;
    double opt[OPT_COUNT];  // hk_set_option
    bool on(Opt o) const { return opt[o] != 0.0; }

    // scene
    void* buf[9] = {};
    uint32_t count[9] = {};
    hk_node* walk_nodes[2] = {nullptr, nullptr};  // BLAS / TLAS copies of the light walks (leaf-collapsed)
    uint32_t* collapse_scratch = nullptr;
    float4* blas_wide = nullptr;  // G-buffer traversal layout (k_build_wide)
    float4* tlas_wide = nullptr;
    uint32_t gb_stack_need = 0;   // TLAS + BLAS subtree depth bound of closest_hit_ordered
    bool heavy = false;           // the last hk_render_frame had spatial reuse or followed a denoised frame (pipeline_size)
    int dn_calls = 0;             // hk_denoise calls since the last hk_render_frame
    uint32_t gb_blas_depth = 0;   // BLAS part of it (the TLAS part changes with hk_update_instances)
    void* dyn_scratch = nullptr;  // hk_update_instances scratch (sized at upload)
    size_t dyn_bytes = 0;
    // GlobalTransformQueue[1] of every instance (transform.rs:32-44): the models as of the previous
    // k_gbuffer, read by its motion vectors; refreshed after a k_gbuffer that followed an update
    float* prev_models = nullptr;
    bool models_dirty = false;   // hk_update_instances ran since the last k_gbuffer
    bool velocity_zero = true;   // the current G-buffer's velocity plane is all zero (k_gbuffer, no motion)
    bool has_scene = false;
    uchar4* noise = nullptr;
    bool has_noise = false;
    // material textures (hk_texture_upload)
    hk_texture_desc* tex_desc = nullptr;
    uint32_t* texels = nullptr;
    float* tex_lut = nullptr;
    uint32_t n_textures = 0;

    // sizes
    uint32_t S[2] = {0, 0}, s[2] = {0, 0};
    float ratio = 1.0f;
    int32_t S_row0 = 0, S_rows = 0, s_row0 = 0, s_rows = 0;
    int32_t core_row0 = 0, core_rows = 0;
    int32_t halo = BAND_HALO;
    int32_t stripe_n = 0, stripe_k = 0;  // interleaved stripes (hk_resize_striped), stripe_n >= 2
    bool albedo_fresh = false;  // the albedo target matches the G-buffer (k_gbuffer wrote both)
    bool sized = false;

    // G-buffer (band-local, S-wide)
    float4* g_position = nullptr;
    uint32_t* g_normal = nullptr;
    float2* g_depth_gradient = nullptr;
    float2* g_instance_material = nullptr;
    float4* g_velocity_uv = nullptr;
    float4* g_prev_position = nullptr;    // the previous frame's planes (prepass.rs:309-317 swap)
    float4* g_prev_velocity_uv = nullptr;
    // the other slot of the planes k_gbuffer double-buffers (swapped with the current ones on each
    // hk_render_gbuffer, like position / velocity above) so a frame's G-buffer can be traced ahead
    uint32_t* g_prev_normal = nullptr;
    float2* g_prev_depth_gradient = nullptr;
    float2* g_prev_instance_material = nullptr;
    uint2* albedo_prev = nullptr;
    // G-buffer pipelining: k_gbuffer of frame f runs on gb_stream, next to frame f-1's light passes
    hipStream_t gb_stream = nullptr;
    hipEvent_t ev_gb_done = nullptr;            // after the latest k_gbuffer launch on gb_stream
    hipEvent_t ev_gb_call[2] = {nullptr, nullptr};  // caller stream at the entry of the last two pipelined calls
    hipEvent_t ev_post = nullptr;               // after a post-process read of the previous slot
    bool gb_pending = false;                    // a k_gbuffer launch was made on gb_stream
    bool gb_serial = true;                      // the next k_gbuffer runs in caller-stream order
    bool post_pending = false;
    bool gb_call_rec = false;                   // the last call recorded ev_gb_call (it was pipelined)
    uint32_t gb_calls = 0;
    // fork shortcut bookkeeping (pick / pick_frame, hk_render_frame): API calls outside the frame
    // sequence, the frame sequence's stream and its changes; at each hk_render_gbuffer entry (by call
    // parity) those counts; the latest k_gbuffer ran on gb_stream (gb_on_gs) after the caller stream at
    // the previous call's entry (gb_wait_*: the counts there) and after frame tail gb_tail_seq; the
    // previous hk_render_frame ran its indirect chain on the side stream only (rf_side_only)
    uint64_t other_picks = 0, frame_st_epoch = 0;
    hipStream_t frame_st = nullptr;
    uint64_t entry_other[2] = {0, 0}, entry_epoch[2] = {0, 0};
    bool gb_on_gs = false, gb_wait_valid = false, rf_side_only = false;
    uint64_t gb_wait_other = 0, gb_wait_epoch = 0, gb_tail_seq = 0;
    // hk_render_frame calls (rf_seq) and the latest one that recorded ev_rf (rf_rec_seq, with the counts
    // there); the ev_rf the open tail waited for (tail_rf), per G-buffer slot the one its last tail
    // waited for; per call parity, at hk_render_gbuffer's entry: the latest hk_render_frame and whether
    // only the frame sequence ran since it recorded ev_rf (entry_clean)
    uint64_t rf_seq = 0, rf_rec_seq = 0, rf_other = 0, rf_epoch = 0, tail_rf = 0;
    uint64_t gslot_rf[2] = {0, 0}, entry_rf[2] = {0, 0};
    bool entry_clean[2] = {false, false};
    // Frame-tail pipelining: the demodulation, a-trous levels and tone-sum of frame f run on
    // dn_stream next to frame f+1's light passes; render / variance are double-buffered for it.
    // Slot events: the latest tail work that read render slot r / G-buffer slot g.
    uint2* render_alt[3] = {};
    float* variance_alt[3] = {};
    hipStream_t dn_stream = nullptr;
    hipEvent_t ev_rf = nullptr;                 // caller stream, end of the latest hk_render_frame
    hipEvent_t ev_rslot[2] = {nullptr, nullptr};
    hipEvent_t ev_gslot[2] = {nullptr, nullptr};
    hipEvent_t ev_dn_last = nullptr;            // dn_stream, after its latest work
    bool rslot_rec[2] = {false, false}, gslot_rec[2] = {false, false};
    // tail_end calls so far, and the one that last recorded each slot event (0: none)
    uint64_t tail_seq = 0, rslot_seq[2] = {0, 0}, gslot_seq[2] = {0, 0};
    uint32_t rslot = 0, gslot = 0;              // current render / G-buffer slot
    bool dn_pending = false;                    // work was queued on dn_stream
    bool rf_swapped = false;                    // the latest hk_render_frame wrote the other render slot
    bool tail_open = false;                     // dn_stream already waits for that frame (ev_rf)
    uint32_t head = 0;                    // frame_number % 2 (PostProcessTextures.head)
    // channel fork-join: emissive and indirect passes on side streams next to direct_lit
    hipStream_t side[2] = {nullptr, nullptr};
    hipEvent_t ev_fork = nullptr, ev_join[2] = {nullptr, nullptr};
    // light targets
    uint2* albedo = nullptr;
    float* variance[3] = {};
    uint2* render[3] = {};
    uint4* reservoirs[HK_RESERVOIR_BUFFERS] = {};
    uint32_t res_n = 0;
    // background store elision masks (ChannelArgs::bg): [0] the fused direct/emissive pair, [1] the
    // indirect channel; valid = the mask describes the buffers' contents for pass window key
    uint8_t* bgmask[2] = {};
    bool bg_valid[2] = {false, false};
    // a band's per-channel row-window margins, sticky maxima since hk_resize (band_windows): -1 = none yet
    int32_t win_out = -1, win_emi = -1, win_ind = -1;
    // a 2-D tile's own columns (hk_resize_tile): global [core_col0, core_col0 + core_cols); 0 / S.x otherwise
    int32_t core_col0 = 0, core_cols = 0;
    int32_t bg_key[2][2] = {};
    uint8_t* gbmask = nullptr;  // the G-buffer's (ViewArgs::bg), per S pixel
    uint4* sp_view = nullptr;   // spatial view planes of the indirect channel (ChannelArgs::view), 3 x res_n
    bool gb_valid = false;
    int32_t gb_key[2] = {};
    // denoise
    uint4* dn_rgb[4] = {};        // a-trous level inputs, the 3 channels packed (DenoiseArgs::rgb / bi)
    uint2* dn_bi[4] = {};
    float* internal_variance[3] = {};
    float4* dn_nd = nullptr;      // (normal, depth) per pixel (k_demod3)
    float4* dn_center = nullptr;  // (depth gradient, luminance denominators of channels 0, 1) per pixel
    float* dn_den2 = nullptr;     // luminance denominator of channel 2 per pixel
    int last_denoised_channels = 3;
    uint2* denoised[3] = {};
    uint2* tone_buf[2] = {};      // tone_mapping_output[2], written at [head]
    uint2* upscale = nullptr;     // upscale_output[0] (SMAA TU4x), U = ceil(S * 2 / ratio)
    uint2* taa_buf[2] = {};       // taa_output[2]
    uint32_t upscale_wh[2] = {0, 0}, taa_wh[2] = {0, 0};
    float4* accum = nullptr;      // sub-frame accumulator (hk_accumulate), allocated on first use
    uint2* accum_out = nullptr;
    uint32_t accum_n = 0;
    // counters (top, emitter, primary)
    unsigned long long* counters = nullptr;
    unsigned long long* persist = nullptr;  // persistent-wave tile claim counters (Counters::persist)
    // wavefront indirect pass (hk_set_wavefront): queues, SoA hit records, control words
    bool wavefront = false;
    uint32_t* wf_queue1 = nullptr;
    uint32_t* wf_keys = nullptr;
    uint32_t* wf_queue2 = nullptr;
    uint4* wf_hit = nullptr;
    float* wf_hit_t = nullptr;
    uint32_t* wf_ctl = nullptr;
    uint32_t wf_seg_cap = 0;

    // reads of output planes on streams other than the frame sequence's (hk_copy_output_rows): the plane
    // and an event after the copy; the next write of that plane waits for it (ext_wait)
    std::vector<std::pair<const void*, hipEvent_t>> ext_reads;
    std::vector<hipEvent_t> ext_pool;
    hipEvent_t ev_frame_mark = nullptr;  // the frame stream's position, waited for by a foreign-stream copy
    // G-buffer reuse (option gbuffer_reuse): what produced the planes now in each G-buffer slot — the
    // view, jitter and band window of the k_gbuffer that wrote them and the input generation at that
    // time (bumped by every scene / texture / instance / size / host-plane / option change)
    struct GbSig {
        float view[3 + 16 + 16 + 16 + 2];
        int32_t win[2];
        uint64_t gen;
        bool valid;
    } gsig[2] = {};
    uint64_t gen = 1;
    uint64_t primary_reused = 0;  // primary rays of the skipped launches (since hk_reset_counters)

    // timing
    bool timing = false;
    uint32_t timing_every = 1;   // time frames with frame_number % timing_every == 0
    bool timing_frame = true;    // the current frame is one of them
    std::vector<TimedLaunch> pending;
    std::vector<hipEvent_t> event_pool;
    std::vector<std::string> timing_names;
    std::vector<double> timing_ms;
    std::vector<uint64_t> timing_n;
    // traverse_top lane statistics per timed launch name (instrumented builds, hk_lane_stats)
    std::vector<std::string> lane_names;
    std::vector<unsigned long long> lane_act, lane_its;
};

namespace {

int fail(hk_ctx* c, int code, const std::string& msg)
{
    if (c) c->error = msg;
    return code;
}

#define HK_HIP(c, expr)                                                                          \
    do {                                                                                         \
        hipError_t _e = (expr);                                                                  \
        if (_e != hipSuccess)                                                                    \
            return fail((c), HK_ERR_HIP, std::string(#expr " failed: ") + hipGetErrorString(_e)); \
    } while (0)

// Every API call that enqueues work resolves its stream here.  The frame sequence (hk_render_gbuffer,
// hk_render_frame, hk_denoise, hk_tone_sum) uses pick_frame; the count of the other calls and a change
// of the frame sequence's stream tell hk_render_frame what ran since k_gbuffer's wait point (the fork
// shortcut there).
hipStream_t pick(hk_ctx* c, void* stream)
{
    c->other_picks++;
    return stream ? (hipStream_t)stream : c->stream;
}
hipStream_t pick_frame(hk_ctx* c, void* stream)
{
    const hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    if (s != c->frame_st) {
        c->frame_st = s;
        c->frame_st_epoch++;
    }
    return s;
}


#define HK_TRY(expr)            \
    do {                        \
        int _r = (expr);        \
        if (_r != HK_OK) return _r; \
    } while (0)

// Work that reads G-buffer planes, counters or targets, or that changes the scene, first waits
// for any k_gbuffer launched ahead on gb_stream and any denoise / tone-sum queued on dn_stream
// (hipStreamWaitEvent: device-side, no host wait).
int gb_join(hk_ctx* c, hipStream_t st, bool with_denoise = true)
{
    if (c->gb_pending && hipStreamWaitEvent(st, c->ev_gb_done, 0) != hipSuccess)
        return fail(c, HK_ERR_HIP, "hipStreamWaitEvent(G-buffer) failed");
    if (with_denoise && c->dn_pending && hipStreamWaitEvent(st, c->ev_dn_last, 0) != hipSuccess)
        return fail(c, HK_ERR_HIP, "hipStreamWaitEvent(denoise) failed");
    return HK_OK;
}
// The next write of `plane` (nullptr: of any plane) waits on `st` for the foreign-stream copies that read it.
int ext_wait(hk_ctx* c, hipStream_t st, const void* plane)
{
    for (size_t k = 0; k < c->ext_reads.size();) {
        if (plane && c->ext_reads[k].first != plane) {
            ++k;
            continue;
        }
        if (hipStreamWaitEvent(st, c->ext_reads[k].second, 0) != hipSuccess)
            return fail(c, HK_ERR_HIP, "hipStreamWaitEvent(output read) failed");
        c->ext_pool.push_back(c->ext_reads[k].second);
        c->ext_reads[k] = c->ext_reads.back();
        c->ext_reads.pop_back();
    }
    return HK_OK;
}
// frame-tail work on dn_stream: it starts after the frame's hk_render_frame (ev_rf) and marks
// the render / G-buffer slots it read
int tail_begin(hk_ctx* c)
{
    if (!c->tail_open) {
        if (hipStreamWaitEvent(c->dn_stream, c->ev_rf, 0) != hipSuccess)
            return fail(c, HK_ERR_HIP, "hipStreamWaitEvent(frame) failed");
        c->tail_rf = c->rf_rec_seq;
    }
    c->tail_open = true;
    return HK_OK;
}
int tail_end(hk_ctx* c)
{
    if (hipEventRecord(c->ev_rslot[c->rslot], c->dn_stream) != hipSuccess ||
        hipEventRecord(c->ev_gslot[c->gslot], c->dn_stream) != hipSuccess ||
        hipEventRecord(c->ev_dn_last, c->dn_stream) != hipSuccess)
        return fail(c, HK_ERR_HIP, "hipEventRecord(frame tail) failed");
    c->rslot_rec[c->rslot] = c->gslot_rec[c->gslot] = true;
    c->tail_seq++;
    c->rslot_seq[c->rslot] = c->gslot_seq[c->gslot] = c->tail_seq;
    c->gslot_rf[c->gslot] = c->tail_rf;
    c->dn_pending = true;
    return HK_OK;
}
// Frame pipelining pays on large frames: on a small stripe of traversal + NEE alone (a 2- to 8-way split
// of 1080p: <= 1 Mpx, 0.1-0.25 ms frames) the cross-stream waits cost more than the overlap hides
// (cornell 8-way stripe 0.145 -> 0.172 ms), on a 1080p frame or a 4K band it gains.  A frame with spatial
// reuse or the denoiser (`heavy`: this frame's spatial settings, or hk_denoise in the previous frame) has a
// long G-buffer and tail to hide, and pipelines at every size: scene 1080p 2-way band 1.12 -> 0.92 ms,
// 8-way 0.50 -> 0.45, city 4K 8-way 0.90 -> 0.86 (profiles/r05/c21).  Only the schedule changes, never
// the results.
// (the pixels of the band's rows, at a 2-D tile's columns + halo: the work its launches cover)
double ctx_px(const hk_ctx* c)
{
    double cols = (double)c->s[0];
    if (c->core_cols > 0 && c->core_cols < (int32_t)c->S[0])
        cols = (double)(std::min((int32_t)c->s[0], c->core_col0 + c->core_cols + c->halo) - std::max(0, c->core_col0 - c->halo));
    return cols * (double)c->s_rows;
}
bool pipeline_size(const hk_ctx* c)
{
    const double px = ctx_px(c);
    return px >= c->opt[OPT_PIPELINE_MIN_PX] || (c->heavy && px >= c->opt[OPT_PIPELINE_HEAVY_MIN_PX]);
}
bool dn_pipeline_enabled(const hk_ctx* c) { return c->on(OPT_TAIL_PIPELINE) && pipeline_size(c); }
// the scene, sizes or G-buffer planes change on the caller's stream: the next k_gbuffer must run
// in caller-stream order (and a synchronous change waits for the one in flight)
int gb_serialize(hk_ctx* c, bool host_sync)
{
    c->gb_serial = true;
    if (host_sync && c->gb_stream && hipStreamSynchronize(c->gb_stream) != hipSuccess)
        return fail(c, HK_ERR_HIP, "hipStreamSynchronize(G-buffer stream) failed");
    if (host_sync && c->dn_stream && hipStreamSynchronize(c->dn_stream) != hipSuccess)
        return fail(c, HK_ERR_HIP, "hipStreamSynchronize(denoise stream) failed");
    return HK_OK;
}

template <typename T>
void release(T*& p)
{
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

void free_targets(hk_ctx* c)
{
    release(c->g_position);
    release(c->g_normal);
    release(c->g_depth_gradient);
    release(c->g_instance_material);
    release(c->g_velocity_uv);
    release(c->albedo);
    for (int i = 0; i < 3; ++i) {
        release(c->variance[i]);
        release(c->render[i]);
        release(c->variance_alt[i]);
        release(c->render_alt[i]);
        release(c->denoised[i]);
    }
    for (int i = 0; i < HK_RESERVOIR_BUFFERS; ++i) release(c->reservoirs[i]);
    for (int k = 0; k < 2; ++k) {
        release(c->bgmask[k]);
        c->bg_valid[k] = false;
    }
    release(c->gbmask);
    c->gb_valid = false;
    release(c->sp_view);
    for (int ch = 0; ch < 3; ++ch) {
        release(c->internal_variance[ch]);
    }
    for (int i = 0; i < 4; ++i) {
        release(c->dn_rgb[i]);
        release(c->dn_bi[i]);
    }
    release(c->dn_nd);
    release(c->dn_center);
    release(c->dn_den2);
    for (int k = 0; k < 2; ++k) {
        release(c->tone_buf[k]);
        release(c->taa_buf[k]);
    }
    release(c->upscale);
    release(c->g_prev_position);
    release(c->g_prev_velocity_uv);
    release(c->g_prev_normal);
    release(c->g_prev_depth_gradient);
    release(c->g_prev_instance_material);
    release(c->albedo_prev);
    c->gb_serial = true;
    c->gb_calls = 0;
    c->gb_on_gs = c->gb_wait_valid = c->rf_side_only = false;
    c->gb_call_rec = false;
    c->rf_swapped = c->tail_open = false;
    c->rslot_rec[0] = c->rslot_rec[1] = c->gslot_rec[0] = c->gslot_rec[1] = false;
    c->rslot_seq[0] = c->rslot_seq[1] = c->gslot_seq[0] = c->gslot_seq[1] = 0;
    c->gslot_rf[0] = c->gslot_rf[1] = 0;
    c->entry_clean[0] = c->entry_clean[1] = false;
    c->upscale_wh[0] = c->upscale_wh[1] = c->taa_wh[0] = c->taa_wh[1] = 0;
    release(c->accum);
    release(c->accum_out);
    c->accum_n = 0;
    release(c->wf_queue1);
    release(c->wf_keys);
    release(c->wf_queue2);
    release(c->wf_hit);
    release(c->wf_hit_t);
    release(c->wf_ctl);
    c->sized = false;
}

// the wavefront pass's buffers, allocated on first use after a resize (s-plane sized)
int ensure_wavefront(hk_ctx* c)
{
    if (c->wf_ctl) return HK_OK;
    const size_t n = (size_t)c->s[0] * (size_t)c->s_rows;
    const size_t tiles = (size_t)((c->s[0] + 15u) / 16u) * (size_t)(((uint32_t)c->s_rows + 15u) / 16u);
    c->wf_seg_cap = (uint32_t)(256u * ((tiles + WF_SEGS - 1u) / WF_SEGS));
    HK_HIP(c, hipMalloc(&c->wf_queue1, (size_t)WF_SEGS * c->wf_seg_cap * 4));
    HK_HIP(c, hipMalloc(&c->wf_keys, (size_t)WF_SEGS * c->wf_seg_cap * 4));
    HK_HIP(c, hipMalloc(&c->wf_queue2, n * 4));
    HK_HIP(c, hipMalloc(&c->wf_hit, n * sizeof(uint4)));
    HK_HIP(c, hipMalloc(&c->wf_hit_t, n * 4));
    HK_HIP(c, hipMalloc(&c->wf_ctl, (size_t)wf_ctl_words(WF_MAX_BINS) * 4));
    return HK_OK;
}

hipEvent_t take_event(hk_ctx* c)
{
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

// Launch wrapper: records HIP events around the kernel on its own stream when timing is on.
void lane_stats_account(hk_ctx* c, const char* name, hipStream_t st)
{
    unsigned long long v[2 * LANE_SLOTS];
    if (!lane_stats_take(v, st)) return;
    static const char* const stage[LANE_SLOTS] = {"", "/neighbour", "/march_tap", "/record_tests", "/merge"};
    for (int slot = 0; slot < LANE_SLOTS; ++slot) {
        if (!v[2 * slot + 1]) continue;
        const std::string key = std::string(name) + stage[slot];
        size_t k = 0;
        for (; k < c->lane_names.size(); ++k)
            if (c->lane_names[k] == key) break;
        if (k == c->lane_names.size()) {
            c->lane_names.push_back(key);
            c->lane_act.push_back(0);
            c->lane_its.push_back(0);
        }
        c->lane_act[k] += v[2 * slot];
        c->lane_its[k] += v[2 * slot + 1];
    }
}

template <typename F>
void timed(hk_ctx* c, const char* name, hipStream_t st, F&& launch)
{
#ifdef HK_LANE_STATS
    // instrumented build: attribute the walk statistics to this launch (serialises the streams)
    (void)hipDeviceSynchronize();
    unsigned long long drop[2 * LANE_SLOTS];
    (void)lane_stats_take(drop, st);
    launch();
    lane_stats_account(c, name, st);
    return;
#endif
    if (!c->timing || !c->timing_frame) {
        launch();
        return;
    }
    TimedLaunch t{name, take_event(c), take_event(c)};
    (void)hipEventRecord(t.start, st);
    launch();
    (void)hipEventRecord(t.stop, st);
    c->pending.push_back(t);
}

void flush_timing(hk_ctx* c)
{
    for (TimedLaunch& t : c->pending) {
        (void)hipEventSynchronize(t.stop);
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, t.start, t.stop);
        size_t k = 0;
        for (; k < c->timing_names.size(); ++k)
            if (c->timing_names[k] == t.name) break;
        if (k == c->timing_names.size()) {
            c->timing_names.push_back(t.name);
            c->timing_ms.push_back(0.0);
            c->timing_n.push_back(0);
        }
        c->timing_ms[k] += ms;
        c->timing_n[k] += 1;
        c->event_pool.push_back(t.start);
        c->event_pool.push_back(t.stop);
    }
    c->pending.clear();
}

FrameArgs frame_args(hk_ctx* c, const hk_settings* st, const hk_frame_inputs* in)
{
    FrameArgs A;
    std::memset(&A, 0, sizeof(A));
    A.sc.vertices = (const hk_vertex*)c->buf[0];
    A.sc.primitives = (const hk_primitive*)c->buf[1];
    A.sc.asset_nodes = c->walk_nodes[0];  // leaf-collapsed copies (launch_collapse_leaves)
    A.sc.alias_table = (const hk_alias_entry*)c->buf[3];
    A.sc.instances = (const hk_instance*)c->buf[4];
    A.sc.instance_nodes = c->walk_nodes[1];
    A.sc.materials = (const hk_material*)c->buf[6];
    A.sc.emissive_nodes = (const hk_node*)c->buf[7];
    A.sc.emissives = (const hk_emissive*)c->buf[8];
    A.sc.n_instances = c->count[4];
    A.sc.n_instance_nodes = c->count[5];
    A.sc.n_materials = c->count[6];
    A.sc.n_emissive_nodes = c->count[7];
    A.sc.blas_wide = c->blas_wide;
    A.sc.tlas_wide = c->tlas_wide;
    A.sc.textures = c->tex_desc;
    A.sc.texels = c->texels;
    A.sc.texture_lut = c->tex_lut;
    A.sc.n_textures = c->n_textures;
    {
        const size_t elem[9] = {sizeof(hk_vertex), sizeof(hk_primitive), sizeof(hk_node), sizeof(hk_alias_entry),
                                sizeof(hk_instance), sizeof(hk_node), sizeof(hk_material), sizeof(hk_node),
                                sizeof(hk_emissive)};
        for (int k = 0; k < 9; ++k) A.sc.bytes[k] = (uint32_t)std::min<size_t>((size_t)c->count[k] * elem[k], 0xFFFFFFF0u);
        A.sc.bytes[9] = (uint32_t)std::min<size_t>((size_t)c->count[2] * 64, 0xFFFFFFF0u);
        A.sc.bytes[10] = (uint32_t)std::min<size_t>((size_t)c->count[5] * 64, 0xFFFFFFF0u);
    }
    Frame& F = A.F;
    hk_settings def;
    hk_settings_default(&def);
    if (!st) st = &def;
    F.number = in ? in->frame_number : 0u;
    F.direct_validate_interval = st->direct_validate_interval;
    F.emissive_validate_interval = st->emissive_validate_interval;
    F.max_temporal_reuse_count = st->max_temporal_reuse_count;
    F.max_spatial_reuse_count = st->max_spatial_reuse_count;
    F.indirect_bounces = st->indirect_bounces;
    F.temporal_reuse = st->temporal_reuse;
    F.max_reservoir_lifetime = st->max_reservoir_lifetime;
    F.max_indirect_luminance = st->max_indirect_luminance;
    F.upscale_ratio = c->ratio;
    F.cos_solar_angle = hk_cos(st->solar_angle);  // same implementation as the device side
    for (int i = 0; i < 4; ++i) F.clear_color[i] = st->clear_color[i];
    if (in) {
        for (int i = 0; i < 3; ++i) {
            F.view_world_position[i] = in->view.world_position[i];
            F.view_proj_z[i] = in->view.view_proj[4 * i + 2];
            F.directional_color[i] = in->lights.directional_color[i];
            F.direction_to_light[i] = in->lights.direction_to_light[i];
            F.ambient_color[i] = in->lights.ambient_color[i];
        }
        F.orthographic = in->view.projection[15] == 1.0f;
    }
    F.S[0] = c->S[0];
    F.S[1] = c->S[1];
    F.inv_S[0] = 1.0f / (float)c->S[0];
    F.inv_S[1] = 1.0f / (float)c->S[1];
    for (int el = 0; el < 2; ++el) {
        const uint32_t count = el ? 8u : 16u;
        const float range = el ? 10.0f : 20.0f;
        for (uint32_t i = 1u; i <= 16u; ++i) {
            float py = i <= count ? std::sqrt((float)i / (float)count) * range : 0.0f;
            float interval = std::fmax(1.0f, py / 5.0f);
            float q = py / interval;
            F.sp_py[el][i - 1] = py;
            F.sp_tap_interval[el][i - 1] = interval;
            F.sp_tap_count[el][i - 1] = q > 0.0f ? (q >= 4294967296.0f ? 0xFFFFFFFFu : (uint32_t)q) : 0u;
        }
    }
    for (uint32_t tc = 0; tc < 7; ++tc)
        for (uint32_t j = 0; j < 6; ++j) F.sp_tap_t[tc][j] = (float)j / (float)(tc + 1u);
    F.inv_s[0] = 1.0f / (float)c->s[0];
    F.inv_s[1] = 1.0f / (float)c->s[1];
    F.s[0] = c->s[0];
    F.s[1] = c->s[1];
    F.S_row0 = c->S_row0;
    F.S_rows = c->S_rows;
    F.s_row0 = c->s_row0;
    F.s_rows = c->s_rows;
    F.count_y0 = c->s_row0 + c->core_row0;
    F.count_y1 = F.count_y0 + c->core_rows;
    // G-buffer rows: whole frame, or (ratio 1 bands) the same rows as the integrator
    F.count_Sy0 = c->S_row0 + c->core_row0;
    F.count_Sy1 = c->S_rows == (int32_t)c->S[1] && c->core_rows == (int32_t)c->s[1] ? (int32_t)c->S[1]
                                                                                      : F.count_Sy0 + c->core_rows;
    // columns: a tile's own (ratio 1, so the same for the G-buffer), every column otherwise
    const bool tile = c->core_cols > 0 && c->core_cols < (int32_t)c->S[0];
    F.count_x0 = tile ? c->core_col0 : 0;
    F.count_x1 = tile ? c->core_col0 + c->core_cols : INT32_MAX;
    F.win_col0 = F.win_cols = 0;
    F.stripe_n = c->stripe_n;
    F.stripe_k = c->stripe_k;
    if (c->stripe_n >= 2) {  // every local row is one of this context's own rows
        F.count_y0 = F.count_Sy0 = 0;
        F.count_y1 = (int32_t)c->s[1];
        F.count_Sy1 = (int32_t)c->S[1];
    }
    A.G.position = c->g_position;
    A.G.normal = c->g_normal;
    A.G.depth_gradient = c->g_depth_gradient;
    A.G.instance_material = c->g_instance_material;
    A.G.velocity_uv = c->g_velocity_uv;
    A.noise = c->noise;
    A.cnt.top = c->counters;
    A.cnt.emitter = c->counters + COUNTER_SPAN;
    A.cnt.primary = c->counters + 2 * COUNTER_SPAN;
    A.cnt.persist = c->persist;
    A.opt.lds_scene = (int)c->opt[OPT_LDS_SCENE];
    A.opt.gbuffer_stack_full = c->on(OPT_GBUFFER_STACK_FULL);
    A.opt.gbuffer_deep = c->on(OPT_GBUFFER_DEEP);
    A.opt.gbuffer_lds_max_px = c->opt[OPT_GBUFFER_LDS_MAX_PX];
    A.opt.direct_w4_min_px = c->opt[OPT_DIRECT_W4_MIN_PX];
    A.opt.fused_w4 = c->on(OPT_FUSED_W4);
    A.opt.persistent_indirect = c->on(OPT_PERSISTENT_INDIRECT);
    A.opt.compact_emitter = c->on(OPT_COMPACT_EMITTER);
    A.opt.compact_shadow = c->on(OPT_COMPACT_SHADOW);
    return A;
}

// Per-pass launch windows of a row band (hk_resize with a halo).  A band recomputes halo rows so
// that its own ("core") rows see exactly the inputs of a whole-frame render; each pass needs
// fewer of them than the one before it, counted back from the tone-sum (core rows only):
//   the a-trous levels L3..L0 read their input at +-1, 2, 4, 8 px (denoise.wgsl:101-114), so
//   L3, L2, L1, L0 run on core +-0, 1, 3, 7 rows and demodulation on +-15; its 3x3 variance blur
//   (denoise.wgsl:151-159) reads the light passes' render / variance at +-16 (OUT);
//   spatial reuse runs on core +-OUT and reads the temporal reservoirs and the G-buffer depth
//   within its RANGE (20 px indirect, 10 emissive: light.wgsl:1568-1600), so each channel's temporal
//   pass runs on core +-(OUT + its RANGE) — direct_lit has no spatial pass (light.rs:656-676), so the
//   direct / emissive launch needs only +-OUT when emissive spatial reuse is off — and the G-buffer on
//   core +-(OUT + 20).
// For a static camera every other read is the pixel's own (temporal reprojection is the
// identity), so the core rows stay bit-identical to the whole frame (test_gpu_row_bands_*),
// with 1.15x instead of 1.30x the work of an 8-way city 4K band.  Rows outside a pass's window
// keep stale values that no windowed pass reads; a settings change that widens a window (band_windows) takes the
// history of the rows it brings in from their owner bands (or zero-fills them) and keeps the window wide from
// then on.  Option band_full_windows: every pass on all rows.
constexpr int32_t DENOISE_OUT_REACH = 16, SPATIAL_RANGE = 20, EMISSIVE_SPATIAL_RANGE = 10;
constexpr int32_t GBUFFER_REACH = DENOISE_OUT_REACH + SPATIAL_RANGE;
// Only for a static frame: under camera or instance motion temporal reprojection reads the previous
// frame's reservoirs at other rows, so every pass runs on the whole band (velocity_zero is set by
// hk_render_gbuffer before its own window is taken, and cleared by a host G-buffer plane upload).
bool tile_columns(const hk_ctx* c) { return c->core_cols > 0 && c->core_cols < (int32_t)c->S[0]; }
bool band_windowed(const hk_ctx* c)
{
    return !(c->stripe_n >= 2 || (c->core_rows >= c->s_rows && !tile_columns(c)) || c->S_rows != c->s_rows ||
             !c->velocity_zero || c->on(OPT_BAND_FULL_WINDOWS));
}
// (a 2-D tile: the columns core +- margin as well; its planes are full width, so only the launches shrink)
FrameArgs pass_window(const hk_ctx* c, FrameArgs A, int32_t margin)
{
    if (!band_windowed(c)) return A;
    const int32_t lo = std::max(0, c->core_row0 - margin);
    const int32_t hi = std::min(c->s_rows, c->core_row0 + c->core_rows + margin);
    A.F.win_row0 = lo;
    A.F.win_rows = hi - lo;
    if (tile_columns(c)) {
        const int32_t c0 = std::max(0, c->core_col0 - margin);
        const int32_t c1 = std::min((int32_t)c->s[0], c->core_col0 + c->core_cols + margin);
        A.F.win_col0 = c0;
        A.F.win_cols = c1 - c0;
    }
    return A;
}
// option bg_elision = 0 switches background store elision off (the G-buffer's and the light passes'
// masks are both dropped while it is off)
bool bg_elision_off(const hk_ctx* c) { return !c->on(OPT_BG_ELISION); }
int32_t light_out_reach(const hk_settings* st) { return st->denoise ? DENOISE_OUT_REACH : 0; }
// The settings-dependent margins of a band's light-pass windows (pass_window) as sticky maxima: a
// setting turned on later (denoise, emissive or indirect spatial reuse) widens its channel's window, and the rows
// it brings in hold records no pass of this band has updated since it was sized (or since a motion frame ran
// every pass on the whole band).  A whole-frame render holds those rows' history — its temporal passes run on every
// pixel whatever the spatial flags (light.rs:656-699) — and so does the band whose core the rows belong to (its
// core rows equal the whole frame's).  window_growth lists the rows per reservoir buffer; the host copies them
// from their owners between frames (hk_band_window_grow, hk_reservoir_rows: bands.refill_windows), and the frame
// after that is bit-identical to a whole-frame render (test_gpu_row_bands_settings_toggle).  A window that grows
// without the refill (hk_render_frame first) has its new rows zero-filled instead, as hk_resize zero-fills the
// buffers (light.rs:355-358): exact again once the history has refilled.  The window never narrows.
struct WindowGrowth {
    int32_t want[3];                // the margins `st` needs: spatial pass (out), direct + emissive, indirect
    int32_t rows[HK_RESERVOIR_BUFFERS][2][2];  // per buffer, above / below the core: local rows [r0, r1) to fill
    bool grows, fill;               // some margin widens; its new rows need history (a windowed frame, not the first)
};
WindowGrowth window_growth(const hk_ctx* c, const hk_settings* st)
{
    WindowGrowth G{};
    const int32_t out = light_out_reach(st);
    G.want[0] = out;
    G.want[1] = out + (st->emissive_spatial_reuse ? EMISSIVE_SPATIAL_RANGE : 0);
    G.want[2] = out + (st->indirect_spatial_reuse ? SPATIAL_RANGE : 0);
    if (tile_columns(c)) {
        // a 2-D tile runs every channel on its widest window from the first frame (every setting on): its window
        // never grows, so a settings change needs no refill (the row bands' refill moves rows, not rectangles)
        G.want[0] = DENOISE_OUT_REACH;
        G.want[1] = DENOISE_OUT_REACH + EMISSIVE_SPATIAL_RANGE;
        G.want[2] = DENOISE_OUT_REACH + SPATIAL_RANGE;
    }
    const int32_t have[3] = {c->win_out, c->win_emi, c->win_ind};
    // the buffers whose records the group's window holds: spatial pairs 4/5, 8/9; direct + emissive 0-5; indirect 6-9
    static const uint32_t members[3] = {0x330u, 0x03Fu, 0x3C0u};
    const bool windowed = band_windowed(c);
    const int32_t core0 = c->core_row0, core1 = c->core_row0 + c->core_rows;
    for (int b = 0; b < HK_RESERVOIR_BUFFERS; ++b) {
        G.rows[b][0][0] = G.rows[b][1][0] = INT32_MAX;
        G.rows[b][0][1] = G.rows[b][1][1] = INT32_MIN;
    }
    for (int g = 0; g < 3; ++g) {
        const int32_t old = have[g], m = std::max(old, G.want[g]);
        if (m == old) continue;
        G.grows = true;
        if (old < 0 || !windowed) continue;  // zero-filled since hk_resize, or every row computed this frame
        G.fill = true;
        const int32_t span[2][2] = {{std::max(0, core0 - m), std::max(0, core0 - old)},
                                    {std::min(c->s_rows, core1 + old), std::min(c->s_rows, core1 + m)}};
        for (int b = 0; b < HK_RESERVOIR_BUFFERS; ++b) {
            if (!(members[g] >> b & 1u)) continue;
            // union over the groups: the rows between two groups' spans lie in the narrower group's old window,
            // which this band computed exactly, so they equal the owner's records as well
            for (int side = 0; side < 2; ++side) {
                if (span[side][1] <= span[side][0]) continue;
                G.rows[b][side][0] = std::min(G.rows[b][side][0], span[side][0]);
                G.rows[b][side][1] = std::max(G.rows[b][side][1], span[side][1]);
            }
        }
    }
    for (int b = 0; b < HK_RESERVOIR_BUFFERS; ++b)
        for (int side = 0; side < 2; ++side)
            if (G.rows[b][side][1] <= G.rows[b][side][0]) G.rows[b][side][0] = G.rows[b][side][1] = 0;
    return G;
}
void commit_growth(hk_ctx* c, const WindowGrowth& G)
{
    int32_t* have[3] = {&c->win_out, &c->win_emi, &c->win_ind};
    for (int g = 0; g < 3; ++g) *have[g] = std::max(*have[g], G.want[g]);
}
int band_windows(hk_ctx* c, const hk_settings* st, hipStream_t s)
{
    const WindowGrowth G = window_growth(c, st);
    if (!G.grows) return HK_OK;
    commit_growth(c, G);
    if (!G.fill) return HK_OK;
    const size_t w = c->s[0];
    for (int b = 0; b < HK_RESERVOIR_BUFFERS; ++b)
        for (int side = 0; side < 2; ++side) {
            const int32_t r0 = G.rows[b][side][0], r1 = G.rows[b][side][1];
            if (r1 <= r0) continue;
            for (uint32_t plane = 0; plane < 4; ++plane)
                HK_HIP(c, hipMemsetAsync(c->reservoirs[b] + (size_t)plane * c->res_n + (size_t)r0 * w, 0,
                                         (size_t)(r1 - r0) * w * sizeof(uint4), s));
        }
    c->bg_valid[0] = c->bg_valid[1] = false;  // the elision masks no longer describe the buffers
    return HK_OK;
}


// The primary rays a k_gbuffer launch over A counts (its active pixels on the rows it counts: k_gbuffer's
// n_primary), for the launches G-buffer reuse skips.
uint64_t gbuffer_primary_rays(const FrameArgs& A)
{
    const Frame& F = A.F;
    const int32_t w0 = F.win_rows > 0 ? F.win_row0 : 0, w1 = F.win_rows > 0 ? F.win_row0 + F.win_rows : F.S_rows;
    if (F.stripe_n >= 2) return (uint64_t)F.S[0] * (uint64_t)(w1 - w0);
    const int32_t lo = std::max(F.S_row0 + w0, F.count_Sy0), hi = std::min(F.S_row0 + w1, F.count_Sy1);
    const int32_t x0 = std::max(F.win_cols > 0 ? F.win_col0 : 0, F.count_x0);
    const int32_t x1 = std::min(F.win_cols > 0 ? F.win_col0 + F.win_cols : (int32_t)F.S[0], F.count_x1);
    return hi > lo && x1 > x0 ? (uint64_t)(x1 - x0) * (uint64_t)(hi - lo) : 0u;
}

int check_ready(hk_ctx* c, bool need_scene)
{
    if (!c) return HK_ERR_INVALID;
    if (!c->sized) return fail(c, HK_ERR_STATE, "hk_resize has not been called");
    if (need_scene && !c->has_scene) return fail(c, HK_ERR_STATE, "no scene uploaded (hk_scene_upload)");
    if (need_scene && !c->has_noise) return fail(c, HK_ERR_STATE, "no blue noise uploaded (hk_set_noise)");
    return HK_OK;
}

}  // namespace

extern "C" {

int hk_abi_version(void) { return HK_ABI_VERSION; }

void hk_settings_default(hk_settings* o)
{
    // HikariSettings::default() (lib.rs:435-455); upscale ratio defaults to SMAA_TU_2_0
    o->direct_validate_interval = 3;
    o->emissive_validate_interval = 5;
    o->max_temporal_reuse_count = 50;
    o->max_spatial_reuse_count = 800;
    o->max_reservoir_lifetime = 100.0f;
    o->solar_angle = 0.046f;
    o->indirect_bounces = 1;
    o->max_indirect_luminance = 10.0f;
    // Color::rgb(0.4, 0.4, 0.4) is sRGB; as linear RGBA
    float l = std::pow((0.4f + 0.055f) / 1.055f, 2.4f);
    o->clear_color[0] = o->clear_color[1] = o->clear_color[2] = l;
    o->clear_color[3] = 1.0f;
    o->temporal_reuse = 1;
    o->emissive_spatial_reuse = 0;
    o->indirect_spatial_reuse = 1;
    o->denoise = 1;
    o->taa = 0;
    o->upscale_ratio = 2.0f;
    o->upscale = 0;
}

int hk_create(int device, hk_ctx** out)
{
    if (!out) return HK_ERR_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return HK_ERR_NO_DEVICE;
    if (device < 0 || device >= n) return HK_ERR_INVALID;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return HK_ERR_HIP;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return HK_ERR_NO_DEVICE;
    hk_ctx* c = new hk_ctx();
    c->device = device;
    for (int k = 0; k < OPT_COUNT; ++k) c->opt[k] = OPTS[k].def;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->counters, COUNTER_BYTES) != hipSuccess || hipMemset(c->counters, 0, COUNTER_BYTES) != hipSuccess ||
        hipMalloc(&c->persist, PERSIST_BYTES) != hipSuccess || hipMemset(c->persist, 0, PERSIST_BYTES) != hipSuccess) {
        delete c;
        return HK_ERR_HIP;
    }
    // side[1] runs the indirect chain.  side[0] carries no work but is kept: streams are mapped
    // round-robin onto the process's hardware queues (GPU_MAX_HW_QUEUES = 4), and without it the
    // G-buffer / tail streams land on queues that serialise them behind the light passes
    // (cornell 1080p 0.601 -> 0.674 ms/frame measured without it)
    for (int k = 0; k < 2; ++k)
        if (hipStreamCreateWithFlags(&c->side[k], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_join[k], hipEventDisableTiming) != hipSuccess) {
            hk_destroy(c);
            return HK_ERR_HIP;
        }
    if (hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&c->gb_stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_gb_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_gb_call[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_gb_call[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_post, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&c->dn_stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_rf, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_rslot[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_rslot[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_gslot[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_gslot[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_dn_last, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_frame_mark, hipEventDisableTiming) != hipSuccess) {
        hk_destroy(c);
        return HK_ERR_HIP;
    }
    *out = c;
    return HK_OK;
}

void hk_destroy(hk_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->gb_stream) (void)hipStreamSynchronize(c->gb_stream);
    if (c->dn_stream) (void)hipStreamSynchronize(c->dn_stream);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    free_targets(c);
    for (int i = 0; i < 9; ++i) release(c->buf[i]);
    release(c->blas_wide);
    release(c->tlas_wide);
    release(c->walk_nodes[0]);
    release(c->walk_nodes[1]);
    release(c->collapse_scratch);
    release(c->dyn_scratch);
    release(c->prev_models);
    release(c->tex_desc);
    release(c->texels);
    release(c->tex_lut);
    release(c->noise);
    release(c->counters);
    release(c->persist);
    for (auto& t : c->pending) {
        c->event_pool.push_back(t.start);
        c->event_pool.push_back(t.stop);
    }
    for (hipEvent_t e : c->event_pool) (void)hipEventDestroy(e);
    for (auto& r : c->ext_reads) c->ext_pool.push_back(r.second);
    for (hipEvent_t e : c->ext_pool) (void)hipEventDestroy(e);
    if (c->ev_frame_mark) (void)hipEventDestroy(c->ev_frame_mark);
    for (int k = 0; k < 2; ++k) {
        if (c->side[k]) (void)hipStreamSynchronize(c->side[k]);
        if (c->side[k]) (void)hipStreamDestroy(c->side[k]);
        if (c->ev_join[k]) (void)hipEventDestroy(c->ev_join[k]);
    }
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    for (hipEvent_t e : {c->ev_gb_done, c->ev_gb_call[0], c->ev_gb_call[1], c->ev_post, c->ev_rf, c->ev_rslot[0],
                         c->ev_rslot[1], c->ev_gslot[0], c->ev_gslot[1], c->ev_dn_last})
        if (e) (void)hipEventDestroy(e);
    if (c->gb_stream && c->gb_stream != c->side[0]) (void)hipStreamDestroy(c->gb_stream);
    if (c->dn_stream && c->dn_stream != c->side[0]) (void)hipStreamDestroy(c->dn_stream);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* hk_last_error(const hk_ctx* c) { return c ? c->error.c_str() : "null context"; }

int hk_set_option(hk_ctx* c, const char* key, double value)
{
    if (!c || !key) return HK_ERR_INVALID;
    for (int k = 0; k < OPT_COUNT; ++k) {
        if (std::strcmp(OPTS[k].key, key) != 0) continue;
        if (!(value >= OPTS[k].lo && value <= OPTS[k].hi))
            return fail(c, HK_ERR_INVALID, std::string("option ") + key + " out of range");
        // every key but the pixel-count thresholds is an on/off switch or a mode: integers only
        if (!std::strstr(key, "_px") && value != std::floor(value))
            return fail(c, HK_ERR_INVALID, std::string("option ") + key + " takes an integer value");
        c->opt[k] = value;
        c->gen++;  // (G-buffer reuse: planes written under other options are not reused)
        if (k == OPT_BAND_FULL_WINDOWS) c->bg_valid[0] = c->bg_valid[1] = c->gb_valid = false;  // new windows
        return HK_OK;
    }
    return fail(c, HK_ERR_INVALID, std::string("unknown option ") + key);
}

int hk_get_option(const hk_ctx* c, const char* key, double* value)
{
    if (!c || !key || !value) return HK_ERR_INVALID;
    for (int k = 0; k < OPT_COUNT; ++k)
        if (std::strcmp(OPTS[k].key, key) == 0) {
            *value = c->opt[k];
            return HK_OK;
        }
    return HK_ERR_INVALID;
}

const char* hk_option_name(int index) { return index >= 0 && index < OPT_COUNT ? OPTS[index].key : nullptr; }

int hk_scene_upload(hk_ctx* c, const hk_scene_desc* d)
{
    if (!c || !d) return HK_ERR_INVALID;
    (void)hipSetDevice(c->device);
    HK_TRY(gb_serialize(c, true));
    const hk_array* arr[9] = {&d->vertices, &d->primitives, &d->asset_nodes, &d->alias_table, &d->instances,
                              &d->instance_nodes, &d->materials, &d->emissive_nodes, &d->emissives};
    const size_t elem[9] = {sizeof(hk_vertex), sizeof(hk_primitive), sizeof(hk_node), sizeof(hk_alias_entry),
                            sizeof(hk_instance), sizeof(hk_node), sizeof(hk_material), sizeof(hk_node),
                            sizeof(hk_emissive)};
    if (d->instances.count == 0 || d->materials.count == 0)
        return fail(c, HK_ERR_INVALID, "scene needs at least one instance and one material");
    c->gen++;
    for (int i = 0; i < 9; ++i)
        if (arr[i]->count && !arr[i]->data) return fail(c, HK_ERR_INVALID, "scene array with count but no data");
    HK_HIP(c, hipStreamSynchronize(c->stream));
    for (int i = 0; i < 9; ++i) {
        release(c->buf[i]);
        size_t bytes = (size_t)(arr[i]->count ? arr[i]->count : 1) * elem[i];
        HK_HIP(c, hipMalloc(&c->buf[i], bytes));
        HK_HIP(c, hipMemset(c->buf[i], 0, bytes));
        if (arr[i]->count) HK_HIP(c, hipMemcpy(c->buf[i], arr[i]->data, arr[i]->count * elem[i], hipMemcpyHostToDevice));
        c->count[i] = arr[i]->count;
    }
    // leaf boxes of the device node copies (see k_fill_blas_leaves) and the wide layout of the
    // G-buffer traversal: BLAS node -> primitive offset / node range of the mesh that owns it,
    // from the instances' mesh indices
    const uint32_t n_blas = d->asset_nodes.count, n_tlas = d->instance_nodes.count;
    std::vector<uint32_t> prim_offset(n_blas, HK_U32_MAX), node_base(n_blas, HK_U32_MAX), node_count(n_blas, 0);
    const hk_instance* inst = (const hk_instance*)d->instances.data;
    const hk_node* blas = (const hk_node*)d->asset_nodes.data;
    const hk_node* tlas = (const hk_node*)d->instance_nodes.data;
    for (uint32_t k = 0; k < d->instances.count; ++k) {
        const hk_mesh_index& m = inst[k].mesh;
        if ((size_t)m.node[0] + m.node[1] > n_blas) return fail(c, HK_ERR_INVALID, "instance mesh node range outside asset nodes");
        for (uint32_t j = 0; j < m.node[1]; ++j) {
            prim_offset[m.node[0] + j] = m.primitive;
            node_base[m.node[0] + j] = m.node[0];
            node_count[m.node[0] + j] = m.node[1];
        }
    }
    // stack bound of closest_hit_ordered: pushes along a path <= inner subtree starts on it
    auto depth = [](const hk_node* f, uint32_t count) {
        std::vector<uint32_t> dep(count + 1, 0);
        uint32_t best = 0;
        for (uint32_t p = count; p-- > 0;) {
            if (f[p].entry_index >= HK_BVH_LEAF_FLAG) continue;
            uint32_t q = f[p].exit_index;
            uint32_t dl = p + 1 < count ? dep[p + 1] : 0, dr = q < count && q + 1 < count ? dep[q + 1] : 0;
            dep[p] = 1 + (dl > dr ? dl : dr);
        }
        for (uint32_t p = 0; p < count; ++p) best = dep[p] > best ? dep[p] : best;
        return best;
    };
    uint32_t blas_depth = 0;
    for (uint32_t k = 0; k < d->instances.count; ++k) {
        const hk_mesh_index& m = inst[k].mesh;
        uint32_t dd = depth(blas + m.node[0], m.node[1]);
        blas_depth = dd > blas_depth ? dd : blas_depth;
    }
    c->gb_stack_need = depth(tlas, n_tlas) + blas_depth;
    c->gb_blas_depth = blas_depth;
    release(c->dyn_scratch);
    c->dyn_bytes = 0;
    uint32_t* d_aux = nullptr;
    HK_HIP(c, hipMalloc(&d_aux, (size_t)(n_blas ? n_blas : 1) * 12));
    if (n_blas) {
        HK_HIP(c, hipMemcpy(d_aux, prim_offset.data(), (size_t)n_blas * 4, hipMemcpyHostToDevice));
        HK_HIP(c, hipMemcpy(d_aux + n_blas, node_base.data(), (size_t)n_blas * 4, hipMemcpyHostToDevice));
        HK_HIP(c, hipMemcpy(d_aux + 2 * (size_t)n_blas, node_count.data(), (size_t)n_blas * 4, hipMemcpyHostToDevice));
    }
    launch_fill_leaves((hk_node*)c->buf[2], n_blas, d_aux, (const hk_primitive*)c->buf[1], (hk_node*)c->buf[5],
                       n_tlas, (const hk_instance*)c->buf[4], c->count[4], c->stream);
    HK_HIP(c, hipGetLastError());
    release(c->blas_wide);
    release(c->tlas_wide);
    release(c->walk_nodes[0]);
    release(c->walk_nodes[1]);
    release(c->collapse_scratch);
    HK_HIP(c, hipMalloc(&c->blas_wide, (size_t)(n_blas ? n_blas : 1) * 64));
    HK_HIP(c, hipMalloc(&c->tlas_wide, (size_t)(n_tlas ? n_tlas : 1) * 64));
    launch_build_wide((const hk_node*)c->buf[2], n_blas, d_aux + n_blas, d_aux + 2 * (size_t)n_blas, c->blas_wide,
                      c->stream);
    launch_build_wide((const hk_node*)c->buf[5], n_tlas, nullptr, nullptr, c->tlas_wide, c->stream);
    // the light walks' node copies, leaf-collapsed (k_collapse_decide); the arrays above stay as
    // uploaded (hk_read_scene_array, the wide layout and hk_update_instances read them)
    HK_HIP(c, hipMalloc(&c->walk_nodes[0], (size_t)(n_blas ? n_blas : 1) * sizeof(hk_node)));
    HK_HIP(c, hipMalloc(&c->walk_nodes[1], (size_t)(n_tlas ? n_tlas : 1) * sizeof(hk_node)));
    HK_HIP(c, hipMalloc(&c->collapse_scratch, (size_t)std::max<uint32_t>(1u, std::max(n_blas, n_tlas)) * 4));
    HK_HIP(c, hipMemcpyAsync(c->walk_nodes[0], c->buf[2], (size_t)n_blas * sizeof(hk_node), hipMemcpyDeviceToDevice,
                             c->stream));
    HK_HIP(c, hipMemcpyAsync(c->walk_nodes[1], c->buf[5], (size_t)n_tlas * sizeof(hk_node), hipMemcpyDeviceToDevice,
                             c->stream));
    if (c->on(OPT_LEAF_COLLAPSE)) {
        launch_collapse_leaves(c->walk_nodes[0], n_blas, d_aux + n_blas, d_aux + 2 * (size_t)n_blas, c->collapse_scratch,
                               c->stream);
        launch_collapse_leaves(c->walk_nodes[1], n_tlas, nullptr, nullptr, c->collapse_scratch, c->stream);
    }
    HK_HIP(c, hipGetLastError());
    // previous models = the uploaded ones (GlobalTransformQueue([matrix; 2]) for a new entity)
    release(c->prev_models);
    HK_HIP(c, hipMalloc(&c->prev_models, (size_t)d->instances.count * 64));
    HK_HIP(c, hipMemcpy2DAsync(c->prev_models, 64, (const char*)c->buf[4] + offsetof(hk_instance, model),
                               sizeof(hk_instance), 64, d->instances.count, hipMemcpyDeviceToDevice, c->stream));
    c->models_dirty = false;
    HK_HIP(c, hipStreamSynchronize(c->stream));
    release(d_aux);
    c->has_scene = true;
    return HK_OK;
}

int hk_update_instances(hk_ctx* c, const float* models, const float* local_aabbs, uint32_t count, void* stream)
{
    if (!c || !models || !local_aabbs) return HK_ERR_INVALID;
    if (!c->has_scene) return fail(c, HK_ERR_STATE, "no scene uploaded (hk_scene_upload)");
    if (count != c->count[4]) return fail(c, HK_ERR_INVALID, "hk_update_instances needs every instance, in upload order");
    if (c->count[5] != 3u * count - 2u || (c->count[8] && c->count[7] != 3u * c->count[8] - 2u))
        return fail(c, HK_ERR_STATE, "scene BVHs are not bvh-0.7.1 flattened (3n - 2 nodes); cannot rebuild");
    (void)hipSetDevice(c->device);
    hipStream_t st = pick(c, stream);
    HK_TRY(gb_join(c, st));
    HK_TRY(gb_serialize(c, false));
    c->gen++;
    const uint32_t n = count, m = c->count[8], n_alias = c->count[3];
    const uint32_t nm = n > m ? n : m;
    auto align = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t sz[] = {align((size_t)n * 64), align((size_t)n * 24), align((size_t)(n_alias ? n_alias : 1) * 4),
                         align((size_t)(n_alias ? n_alias : 1) * 16), align((size_t)nm * 24), align((size_t)nm * 8),
                         align((size_t)nm * 24), align((size_t)3 * n * 4), align(16)};
    size_t total = 0;
    for (size_t b : sz) total += b;
    if (c->dyn_bytes < total) {
        release(c->dyn_scratch);
        HK_HIP(c, hipMalloc(&c->dyn_scratch, total));
        c->dyn_bytes = total;
    }
    char* p = (char*)c->dyn_scratch;
    char* part[9];
    for (int k = 0; k < 9; ++k) {
        part[k] = p;
        p += sz[k];
    }
    HK_HIP(c, hipMemcpyAsync(part[0], models, (size_t)n * 64, hipMemcpyHostToDevice, st));
    HK_HIP(c, hipMemcpyAsync(part[1], local_aabbs, (size_t)n * 24, hipMemcpyHostToDevice, st));
    HK_HIP(c, hipMemsetAsync(part[8], 0, 16, st));
    DynamicArgs D;
    D.instances = (hk_instance*)c->buf[4];
    D.n_instances = n;
    D.models = (const float*)part[0];
    D.local_aabbs = (const float*)part[1];
    D.tlas = (hk_node*)c->buf[5];
    D.emissives = (hk_emissive*)c->buf[8];
    D.n_emissives = m;
    D.materials = (const hk_material*)c->buf[6];
    D.primitives = (const hk_primitive*)c->buf[1];
    D.alias = (hk_alias_entry*)c->buf[3];
    D.n_alias = n_alias;
    D.lbvh = (hk_node*)c->buf[7];
    D.buckets = 6;  // bvh 0.7.1 NUM_BUCKETS (hks_build default)
    D.areas = (float*)part[2];
    D.alias_work = part[3];
    D.boxes = part[4];
    D.idx = (uint32_t*)part[5];
    D.segments = part[6];
    D.flags = (uint32_t*)part[8];
    timed(c, "update_instances", st, [&] {
        launch_dynamic_update(D, st);
        // device-only derivatives of the TLAS: leaf boxes and the G-buffer wide layout
        launch_fill_leaves(nullptr, 0, nullptr, nullptr, (hk_node*)c->buf[5], c->count[5], (const hk_instance*)c->buf[4],
                           n, st);
        launch_build_wide((const hk_node*)c->buf[5], c->count[5], nullptr, nullptr, c->tlas_wide, st);
        (void)hipMemcpyAsync(c->walk_nodes[1], c->buf[5], (size_t)c->count[5] * sizeof(hk_node), hipMemcpyDeviceToDevice,
                             st);
        if (c->on(OPT_LEAF_COLLAPSE))
            launch_collapse_leaves(c->walk_nodes[1], c->count[5], nullptr, nullptr, c->collapse_scratch, st);
    });
    HK_HIP(c, hipGetLastError());
    uint32_t flags[2] = {0, 0};
    HK_HIP(c, hipMemcpyAsync(flags, part[8], 8, hipMemcpyDeviceToHost, st));
    HK_HIP(c, hipStreamSynchronize(st));
    if (flags[0]) return fail(c, HK_ERR_INVALID, "singular instance transform");
    c->gb_stack_need = flags[1] + c->gb_blas_depth;
    c->models_dirty = true;  // the next G-buffer reads the models before this update as the previous ones
    return HK_OK;
}

int hk_read_scene_array(hk_ctx* c, int array, void* dst, size_t bytes)
{
    if (!c || !dst || array < 0 || array > 8) return HK_ERR_INVALID;
    if (!c->has_scene) return fail(c, HK_ERR_STATE, "no scene uploaded (hk_scene_upload)");
    const size_t elem[9] = {sizeof(hk_vertex), sizeof(hk_primitive), sizeof(hk_node), sizeof(hk_alias_entry),
                            sizeof(hk_instance), sizeof(hk_node), sizeof(hk_material), sizeof(hk_node),
                            sizeof(hk_emissive)};
    const size_t have = (size_t)c->count[array] * elem[array];
    if (bytes < have) return fail(c, HK_ERR_INVALID, "destination too small");
    (void)hipSetDevice(c->device);
    HK_HIP(c, hipStreamSynchronize(c->stream));
    if (have) HK_HIP(c, hipMemcpy(dst, c->buf[array], have, hipMemcpyDeviceToHost));
    return HK_OK;
}

int hk_texture_upload(hk_ctx* c, const hk_texture* t, uint32_t count)
{
    if (!c || (count && !t)) return HK_ERR_INVALID;
    (void)hipSetDevice(c->device);
    HK_TRY(gb_serialize(c, true));
    std::vector<hk_texture_desc> desc(count);
    uint64_t total = 0;
    c->gen++;
    for (uint32_t i = 0; i < count; ++i) {
        if (!t[i].width || !t[i].height || !t[i].rgba8) return fail(c, HK_ERR_INVALID, "texture without texels");
        if (t[i].format > HK_TEXTURE_RGBA8_UNORM || t[i].address_u > HK_ADDRESS_MIRROR_REPEAT ||
            t[i].address_v > HK_ADDRESS_MIRROR_REPEAT || t[i].filter > HK_FILTER_LINEAR)
            return fail(c, HK_ERR_INVALID, "unknown texture format / address mode / filter");
        desc[i] = hk_texture_desc{(uint32_t)total, t[i].width, t[i].height, t[i].format, t[i].address_u,
                                  t[i].address_v, t[i].filter, 0u};
        total += (uint64_t)t[i].width * t[i].height;
        if (total > 0xFFFFFFFFull) return fail(c, HK_ERR_INVALID, "more than 2^32 texels");
    }
    HK_HIP(c, hipStreamSynchronize(c->stream));
    release(c->tex_desc);
    release(c->texels);
    c->n_textures = 0;
    if (count == 0) return HK_OK;
    if (!c->tex_lut) {
        float lut[512];
        hk_texture_build_lut(lut);
        HK_HIP(c, hipMalloc(&c->tex_lut, sizeof(lut)));
        HK_HIP(c, hipMemcpy(c->tex_lut, lut, sizeof(lut), hipMemcpyHostToDevice));
    }
    HK_HIP(c, hipMalloc(&c->tex_desc, count * sizeof(hk_texture_desc)));
    HK_HIP(c, hipMemcpy(c->tex_desc, desc.data(), count * sizeof(hk_texture_desc), hipMemcpyHostToDevice));
    HK_HIP(c, hipMalloc(&c->texels, total * 4));
    for (uint32_t i = 0; i < count; ++i)
        HK_HIP(c, hipMemcpy(c->texels + desc[i].offset, t[i].rgba8, (size_t)t[i].width * t[i].height * 4,
                            hipMemcpyHostToDevice));
    c->n_textures = count;
    return HK_OK;
}

int hk_set_noise(hk_ctx* c, const uint8_t* rgba, uint32_t count, uint32_t size)
{
    if (!c || !rgba) return HK_ERR_INVALID;
    if (count != 16 || size != 64) return fail(c, HK_ERR_INVALID, "blue noise must be 16 textures of 64x64 RGBA8");
    (void)hipSetDevice(c->device);
    HK_TRY(gb_serialize(c, true));
    if (!c->noise) HK_HIP(c, hipMalloc(&c->noise, 16 * 64 * 64 * 4));
    HK_HIP(c, hipMemcpy(c->noise, rgba, 16 * 64 * 64 * 4, hipMemcpyHostToDevice));
    c->has_noise = true;
    return HK_OK;
}

static int resize_impl(hk_ctx* c, uint32_t width, uint32_t height, float ratio, uint32_t band_y0, uint32_t band_rows,
                       uint32_t stripe_n, uint32_t stripe_k, uint32_t col0 = 0u, uint32_t cols = 0u);

int hk_resize(hk_ctx* c, uint32_t width, uint32_t height, float ratio, uint32_t band_y0, uint32_t band_rows)
{
    return resize_impl(c, width, height, ratio, band_y0, band_rows, 0u, 0u);
}

int hk_resize_tile(hk_ctx* c, uint32_t width, uint32_t height, uint32_t x0, uint32_t cols, uint32_t y0, uint32_t rows)
{
    if (!c || cols == 0 || rows == 0) return HK_ERR_INVALID;
    if (x0 + cols > width || y0 + rows > height) return fail(c, HK_ERR_INVALID, "tile outside the frame");
    return resize_impl(c, width, height, 1.0f, y0, rows, 0u, 0u, x0, cols);
}

int hk_tile_info(const hk_ctx* c, int32_t* col0, int32_t* cols)
{
    if (!c || !c->sized) return HK_ERR_STATE;
    if (col0) *col0 = c->core_col0;
    if (cols) *cols = c->core_cols;
    return HK_OK;
}

int hk_resize_striped(hk_ctx* c, uint32_t width, uint32_t height, uint32_t rank, uint32_t world)
{
    if (!c || world == 0 || rank >= world) return HK_ERR_INVALID;
    if (world == 1) return resize_impl(c, width, height, 1.0f, 0u, 0u, 0u, 0u);
    return resize_impl(c, width, height, 1.0f, 0u, 0u, world, rank);
}

static int resize_impl(hk_ctx* c, uint32_t width, uint32_t height, float ratio, uint32_t band_y0, uint32_t band_rows,
                       uint32_t stripe_n, uint32_t stripe_k, uint32_t col0, uint32_t cols)
{
    if (!c || width == 0 || height == 0) return HK_ERR_INVALID;
    if (cols == 0) {
        col0 = 0;
        cols = width;
    }
    (void)hipSetDevice(c->device);
    ratio = ratio < 1.0f ? 1.0f : (ratio > 2.0f ? 2.0f : ratio);  // Upscale::ratio (lib.rs:501-505)
    if (band_rows == 0) {
        band_y0 = 0;
        band_rows = height;
    }
    if (band_y0 + band_rows > height) return fail(c, HK_ERR_INVALID, "band outside the frame");
    bool whole = band_y0 == 0 && band_rows == height;
    if (!whole && ratio != 1.0f) return fail(c, HK_ERR_INVALID, "row bands require upscale ratio 1.0");
    const bool tile_cols = cols < width;
    if (tile_cols && (ratio != 1.0f || stripe_n >= 2)) return fail(c, HK_ERR_INVALID, "tiles require upscale ratio 1.0");
    uint32_t stripe_rows = 0;  // rows of stripes k, k + n, ... (STRIPE_H rows each, the last one may be short)
    if (stripe_n >= 2) {
        if (stripe_n > (height + STRIPE_H - 1) / STRIPE_H)
            return fail(c, HK_ERR_INVALID, "more stripe ranks than stripes in the frame");
        for (uint32_t t = stripe_k; t * STRIPE_H < height; t += stripe_n)
            stripe_rows += height - t * STRIPE_H < (uint32_t)STRIPE_H ? height - t * STRIPE_H : (uint32_t)STRIPE_H;
        whole = false;
    }
    HK_HIP(c, hipStreamSynchronize(c->stream));
    HK_HIP(c, hipStreamSynchronize(c->gb_stream));
    HK_HIP(c, hipStreamSynchronize(c->dn_stream));
    free_targets(c);
    c->gen++;
    c->albedo_fresh = false;
    c->S[0] = width;
    c->S[1] = height;
    c->ratio = ratio;
    float scale = 1.0f / ratio;  // light.rs:318-319: ceil(scale * size)
    c->s[0] = (uint32_t)std::ceil(scale * (float)width);
    c->s[1] = (uint32_t)std::ceil(scale * (float)height);
    c->stripe_n = (int32_t)stripe_n;
    c->stripe_k = (int32_t)stripe_k;
    c->core_col0 = (int32_t)col0;
    c->core_cols = (int32_t)cols;
    if (stripe_n >= 2) {
        c->S_row0 = c->s_row0 = 0;
        c->S_rows = c->s_rows = (int32_t)stripe_rows;
        c->core_row0 = 0;
        c->core_rows = (int32_t)stripe_rows;
    } else if (whole) {
        c->S_row0 = 0;
        c->S_rows = (int32_t)height;
        c->s_row0 = 0;
        c->s_rows = (int32_t)c->s[1];
        c->core_row0 = 0;
        c->core_rows = (int32_t)c->s[1];
    } else {
        int32_t r0 = (int32_t)band_y0 - c->halo;
        int32_t r1 = (int32_t)(band_y0 + band_rows) + c->halo;
        r0 = r0 < 0 ? 0 : r0;
        r1 = r1 > (int32_t)height ? (int32_t)height : r1;
        c->S_row0 = c->s_row0 = r0;
        c->S_rows = c->s_rows = r1 - r0;
        c->core_row0 = (int32_t)band_y0 - r0;
        c->core_rows = (int32_t)band_rows;
    }
    size_t SP = (size_t)width * c->S_rows, sp = (size_t)c->s[0] * c->s_rows;
    HK_HIP(c, hipMalloc(&c->g_position, SP * sizeof(float4)));
    HK_HIP(c, hipMalloc(&c->g_normal, SP * sizeof(uint32_t)));
    HK_HIP(c, hipMalloc(&c->g_depth_gradient, SP * sizeof(float2)));
    HK_HIP(c, hipMalloc(&c->g_instance_material, SP * sizeof(float2)));
    HK_HIP(c, hipMalloc(&c->g_velocity_uv, SP * sizeof(float4)));
    HK_HIP(c, hipMalloc(&c->g_prev_position, SP * sizeof(float4)));
    HK_HIP(c, hipMalloc(&c->g_prev_velocity_uv, SP * sizeof(float4)));
    HK_HIP(c, hipMemset(c->g_prev_position, 0, SP * sizeof(float4)));
    HK_HIP(c, hipMemset(c->g_prev_velocity_uv, 0, SP * sizeof(float4)));
    HK_HIP(c, hipMalloc(&c->g_prev_normal, SP * sizeof(uint32_t)));
    HK_HIP(c, hipMalloc(&c->g_prev_depth_gradient, SP * sizeof(float2)));
    HK_HIP(c, hipMalloc(&c->g_prev_instance_material, SP * sizeof(float2)));
    HK_HIP(c, hipMalloc(&c->albedo_prev, SP * sizeof(uint2)));
    HK_HIP(c, hipMemset(c->g_prev_normal, 0, SP * sizeof(uint32_t)));
    HK_HIP(c, hipMemset(c->g_prev_depth_gradient, 0, SP * sizeof(float2)));
    HK_HIP(c, hipMemset(c->g_prev_instance_material, 0, SP * sizeof(float2)));
    HK_HIP(c, hipMemset(c->albedo_prev, 0, SP * sizeof(uint2)));
    HK_HIP(c, hipMalloc(&c->albedo, SP * sizeof(uint2)));
    HK_HIP(c, hipMemset(c->g_position, 0, SP * sizeof(float4)));
    HK_HIP(c, hipMemset(c->g_normal, 0, SP * sizeof(uint32_t)));
    HK_HIP(c, hipMemset(c->g_depth_gradient, 0, SP * sizeof(float2)));
    HK_HIP(c, hipMemset(c->g_instance_material, 0, SP * sizeof(float2)));
    HK_HIP(c, hipMemset(c->g_velocity_uv, 0, SP * sizeof(float4)));
    HK_HIP(c, hipMemset(c->albedo, 0, SP * sizeof(uint2)));
    for (int i = 0; i < 3; ++i) {
        HK_HIP(c, hipMalloc(&c->variance[i], sp * sizeof(float)));
        HK_HIP(c, hipMalloc(&c->render[i], sp * sizeof(uint2)));
        HK_HIP(c, hipMalloc(&c->denoised[i], sp * sizeof(uint2)));
        HK_HIP(c, hipMemset(c->variance[i], 0, sp * sizeof(float)));
        HK_HIP(c, hipMemset(c->render[i], 0, sp * sizeof(uint2)));
        HK_HIP(c, hipMalloc(&c->variance_alt[i], sp * sizeof(float)));
        HK_HIP(c, hipMalloc(&c->render_alt[i], sp * sizeof(uint2)));
        HK_HIP(c, hipMemset(c->variance_alt[i], 0, sp * sizeof(float)));
        HK_HIP(c, hipMemset(c->render_alt[i], 0, sp * sizeof(uint2)));
        HK_HIP(c, hipMemset(c->denoised[i], 0, sp * sizeof(uint2)));
    }
    c->res_n = (uint32_t)sp;
    c->win_out = c->win_emi = c->win_ind = -1;
    for (int i = 0; i < HK_RESERVOIR_BUFFERS; ++i) {
        HK_HIP(c, hipMalloc(&c->reservoirs[i], 4 * sp * sizeof(uint4)));
        HK_HIP(c, hipMemset(c->reservoirs[i], 0, 4 * sp * sizeof(uint4)));  // light.rs:355-358 zero-fill
    }
    for (int k = 0; k < 2; ++k) {
        HK_HIP(c, hipMalloc(&c->bgmask[k], sp));
        c->bg_valid[k] = false;
    }
    HK_HIP(c, hipMalloc(&c->gbmask, SP));
    c->gb_valid = false;
    HK_HIP(c, hipMalloc(&c->sp_view, VIEW_PLANES * sp * sizeof(uint4)));
    HK_HIP(c, hipMemset(c->sp_view, 0, VIEW_PLANES * sp * sizeof(uint4)));
    for (int ch = 0; ch < 3; ++ch) {
        HK_HIP(c, hipMalloc(&c->internal_variance[ch], sp * sizeof(float)));
        HK_HIP(c, hipMemset(c->internal_variance[ch], 0, sp * sizeof(float)));
    }
    for (int i = 0; i < 4; ++i) {
        HK_HIP(c, hipMalloc(&c->dn_rgb[i], sp * sizeof(uint4)));
        HK_HIP(c, hipMemset(c->dn_rgb[i], 0, sp * sizeof(uint4)));
        HK_HIP(c, hipMalloc(&c->dn_bi[i], sp * sizeof(uint2)));
        HK_HIP(c, hipMemset(c->dn_bi[i], 0, sp * sizeof(uint2)));
    }
    HK_HIP(c, hipMalloc(&c->dn_nd, sp * sizeof(float4)));
    HK_HIP(c, hipMemset(c->dn_nd, 0, sp * sizeof(float4)));
    HK_HIP(c, hipMalloc(&c->dn_center, sp * sizeof(float4)));
    HK_HIP(c, hipMemset(c->dn_center, 0, sp * sizeof(float4)));
    HK_HIP(c, hipMalloc(&c->dn_den2, sp * sizeof(float)));
    HK_HIP(c, hipMemset(c->dn_den2, 0, sp * sizeof(float)));
    for (int k = 0; k < 2; ++k) {
        HK_HIP(c, hipMalloc(&c->tone_buf[k], sp * sizeof(uint2)));
        HK_HIP(c, hipMemset(c->tone_buf[k], 0, sp * sizeof(uint2)));
    }
    HK_HIP(c, hipDeviceSynchronize());
    c->sized = true;
    return HK_OK;
}

int hk_set_band_halo(hk_ctx* c, uint32_t rows)
{
    if (!c || rows > 4096) return HK_ERR_INVALID;
    c->halo = (int32_t)rows;
    c->bg_valid[0] = c->bg_valid[1] = false;
    c->gen++;
    return HK_OK;
}

int hk_band_info(const hk_ctx* c, int32_t* row0, int32_t* rows, int32_t* core_row0, int32_t* core_rows)
{
    if (!c || !c->sized) return HK_ERR_STATE;
    if (row0) *row0 = c->s_row0;
    if (rows) *rows = c->s_rows;
    if (core_row0) *core_row0 = c->core_row0;
    if (core_rows) *core_rows = c->core_rows;
    return HK_OK;
}

int hk_render_gbuffer(hk_ctx* c, const hk_frame_inputs* in, void* stream)
{
    int rc = check_ready(c, true);
    if (rc) return rc;
    if (!in) return fail(c, HK_ERR_INVALID, "null frame inputs");
    if (c->gb_stack_need > (uint32_t)GB_STACK)
        return fail(c, HK_ERR_INVALID, "scene BVH too deep for the G-buffer traversal stack (TLAS + BLAS depth > 64)");
    if (in->jitter > HK_JITTER_TAA_SMAA) return fail(c, HK_ERR_INVALID, "unknown jitter mode");
    (void)hipSetDevice(c->device);
    hipStream_t st = pick_frame(c, stream);
    // Pipelining: this frame's planes go to the slot frame f-2 used.  Its readers are the work
    // enqueued on the caller's stream before the previous hk_render_gbuffer call (frame f-2's
    // passes, denoise, tone-sum, readbacks) and a post-process of frame f-1 (it reads the previous
    // slot); k_gbuffer waits for exactly those on gb_stream and so overlaps frame f-1's light
    // passes.  A scene / size / plane change since the last call serialises it instead.
    const bool pipeline = c->on(OPT_GBUFFER_PIPELINE);
    // Event markers are recorded only on the pipelined path: each one between two kernels of a stream
    // costs it ~6 us (cornell 8-way stripe, where the serial frame is 3 kernels), and the serial path
    // has no other stream waiting on them.
    const uint32_t e = c->gb_calls & 1u;
    hipStream_t gs = st;
    // G-buffer reuse: the slot this frame's planes go to (the other one) already holds exactly them when the
    // k_gbuffer that wrote it saw the same view, jitter and band window, nothing it reads changed since
    // (generation) and nothing moved (no motion vectors: the velocity plane is zero in both).  The planes
    // then stay as they are, bit for bit what a new trace would store (the 16
    // sub-frames of a displayed frame share camera and scene).  Only the primary-ray counter differs: it
    // counts rays traced.
    hk_ctx::GbSig sig;
    std::memset(&sig, 0, sizeof(sig));
    {
        float* v = sig.view;
        for (int i = 0; i < 3; ++i) *v++ = in->view.world_position[i];
        for (int i = 0; i < 16; ++i) *v++ = in->view.view_proj[i];
        for (int i = 0; i < 16; ++i) *v++ = in->view.inverse_view_proj[i];
        for (int i = 0; i < 16; ++i) *v++ = in->has_previous_view ? in->previous_view_proj[i] : in->view.view_proj[i];
        *v++ = in->view.projection[15];
        *v++ = (float)in->jitter;
        sig.gen = c->gen;
        sig.valid = true;
    }
    const bool jitter_static = in->jitter == HK_JITTER_NONE;
    const bool still = !c->models_dirty &&
                       std::memcmp(sig.view + 3, sig.view + 3 + 32, 16 * sizeof(float)) == 0;  // previous view = view
    const bool pipe = pipeline && pipeline_size(c) && !c->gb_serial && c->gb_calls > 0;
    c->entry_other[e] = c->other_picks;
    c->entry_epoch[e] = c->frame_st_epoch;
    c->entry_rf[e] = c->rf_seq;
    c->entry_clean[e] = c->rf_seq > 0 && c->rf_rec_seq == c->rf_seq && c->other_picks == c->rf_other &&
                        c->frame_st_epoch == c->rf_epoch;
    c->gb_tail_seq = 0;
    c->gb_wait_valid = false;
    {
        const uint32_t next = c->gslot ^ 1u;  // the slot this frame's planes go to
        FrameArgs W = pass_window(c, frame_args(c, nullptr, in), GBUFFER_REACH);
        sig.win[0] = W.F.win_row0;
        sig.win[1] = W.F.win_rows;
        const hk_ctx::GbSig& have = c->gsig[next];
        if (c->on(OPT_GBUFFER_REUSE) && still && jitter_static && have.valid && c->velocity_zero &&
            c->albedo_fresh && have.gen == sig.gen && have.win[0] == sig.win[0] &&
            have.win[1] == sig.win[1] && std::memcmp(have.view, sig.view, sizeof(sig.view)) == 0 && !c->gb_serial && c->gb_calls > 0) {
            // (the previous frame's G-buffer came from k_gbuffer too — albedo_fresh, velocity_zero — so both
            // slots hold traced planes of a still camera)
            std::swap(c->g_position, c->g_prev_position);
            std::swap(c->g_velocity_uv, c->g_prev_velocity_uv);
            std::swap(c->g_normal, c->g_prev_normal);
            std::swap(c->g_depth_gradient, c->g_prev_depth_gradient);
            std::swap(c->g_instance_material, c->g_prev_instance_material);
            std::swap(c->albedo, c->albedo_prev);
            c->gslot = next;
            c->head = in->frame_number & 1u;
            c->timing_frame = in->frame_number % c->timing_every == 0u;
            // (post_pending stays: a post-process read both slots, and the next launch overwrites one)
            // no launch to reason about: the next hk_render_frame records its fork marker
            c->gb_call_rec = false;
            c->gb_on_gs = false;
            c->gb_calls++;
            c->primary_reused += gbuffer_primary_rays(W);
            return HK_OK;
        }
    }
    if (pipe) {
        HK_HIP(c, hipEventRecord(c->ev_gb_call[e], st));
        gs = c->gb_stream;
        // the caller stream at the previous call's entry; when that call was serial (its k_gbuffer ran
        // on st, no record), the caller stream now.  The previous pipelined k_gbuffer is earlier on gs.
        const uint32_t w = c->gb_call_rec ? e ^ 1u : e;
        // Frame f-2's tail (dn_stream) read this slot; it waited for ev_rf of a hk_render_frame (gslot_rf).
        // When that is the one whose ev_rf marked the caller stream where the previous call's entry
        // marker stands (nothing but the frame sequence ran in between: entry_clean) or a later one, the
        // tail's event implies the entry marker, and k_gbuffer waits for the tail alone: one packet fewer
        // ahead of it in the queue it shares with the indirect chain.
        const uint32_t g = c->gslot ^ 1u;
        const bool tail_covers = c->gb_call_rec && c->gslot_rec[g] && c->entry_clean[w] && c->entry_rf[w] > 0 &&
                                 c->gslot_rf[g] >= c->entry_rf[w];
        if (!tail_covers) HK_HIP(c, hipStreamWaitEvent(gs, c->ev_gb_call[w], 0));
        c->gb_wait_valid = true;
        c->gb_wait_other = c->entry_other[w];
        c->gb_wait_epoch = c->entry_epoch[w];
        if (c->post_pending) HK_HIP(c, hipStreamWaitEvent(gs, c->ev_post, 0));
        if (c->gslot_rec[g]) {
            HK_HIP(c, hipStreamWaitEvent(gs, c->ev_gslot[g], 0));
            c->gb_tail_seq = c->gslot_seq[g];
        }
    } else {
        HK_TRY(gb_join(c, st));
    }
    c->post_pending = false;
    // a new frame: this frame's planes replace the previous ones (prepass.rs:309-317)
    std::swap(c->g_position, c->g_prev_position);
    std::swap(c->g_velocity_uv, c->g_prev_velocity_uv);
    std::swap(c->g_normal, c->g_prev_normal);
    std::swap(c->g_depth_gradient, c->g_prev_depth_gradient);
    std::swap(c->g_instance_material, c->g_prev_instance_material);
    std::swap(c->albedo, c->albedo_prev);
    c->gslot ^= 1u;
    c->head = in->frame_number & 1u;
    c->timing_frame = in->frame_number % c->timing_every == 0u;
    FrameArgs A = frame_args(c, nullptr, in);
    ViewArgs V;
    for (int i = 0; i < 3; ++i) V.world_position[i] = in->view.world_position[i];
    std::memcpy(V.view_proj, in->view.view_proj, sizeof(V.view_proj));
    std::memcpy(V.inverse_view_proj, in->view.inverse_view_proj, sizeof(V.inverse_view_proj));
    // prepass.wgsl:30-38 frame_jitter (HALTON, view.rs:130-139), in pixels (jitter = 2 h / viewport
    // in NDC, added to clip.xy with y flipped: the surface point seen at a pixel centre c is the one
    // that projects to c - h without jitter)
    static const float HALTON[8][4] = {
        {0.000000f, 0.000000f, 0.500000f, 0.333333f}, {0.250000f, 0.666667f, 0.750000f, 0.111111f},
        {0.125000f, 0.444444f, 0.625000f, 0.777778f}, {0.375000f, 0.222222f, 0.875000f, 0.555556f},
        {0.062500f, 0.888889f, 0.562500f, 0.037037f}, {0.312500f, 0.370370f, 0.812500f, 0.703704f},
        {0.187500f, 0.148148f, 0.687500f, 0.481481f}, {0.437500f, 0.814815f, 0.937500f, 0.259259f}};
    V.jitter[0] = V.jitter[1] = 0.0f;
    if (in->jitter != HK_JITTER_NONE) {
        const uint32_t index = in->jitter == HK_JITTER_TAA_SMAA ? (in->frame_number >> 1) & 15u : in->frame_number & 15u;
        const float* h = HALTON[index >> 1];
        V.jitter[0] = (index & 1u) == 0u ? h[0] : h[2];
        V.jitter[1] = (index & 1u) == 0u ? h[1] : h[3];
    }
    // motion vectors: previous view (PreviousViewUniform) and previous models (GlobalTransformQueue)
    const float* pvp = in->has_previous_view ? in->previous_view_proj : in->view.view_proj;
    std::memcpy(V.previous_view_proj, pvp, sizeof(V.previous_view_proj));
    V.motion = (c->models_dirty || std::memcmp(pvp, in->view.view_proj, sizeof(V.previous_view_proj)) != 0) ? 1 : 0;
    V.previous_models = c->prev_models;
    c->velocity_zero = V.motion == 0;
    // full_screen_albedo is fused into the G-buffer kernel (it has every input in registers);
    // hk_render_frame runs it on its own only for host-supplied G-buffers
    A = pass_window(c, A, GBUFFER_REACH);
    V.bg = nullptr;
    V.bg_need = 0;
    if (bg_elision_off(c)) {
        c->gb_valid = false;  // the mask is rebuilt from zero when elision is switched back on
    } else {
        if (!c->gb_valid || c->gb_key[0] != A.F.win_row0 || c->gb_key[1] != A.F.win_rows) {
            HK_HIP(c, hipMemsetAsync(c->gbmask, 0, (size_t)c->S[0] * c->S_rows, gs));
            c->gb_valid = true;
            c->gb_key[0] = A.F.win_row0;
            c->gb_key[1] = A.F.win_rows;
        }
        V.bg = c->gbmask;
        V.bg_need = 1u << c->gslot;  // the planes' physical slot (swapped with gslot above)
    }
    for (const void* plane : {(const void*)c->g_position, (const void*)c->g_velocity_uv, (const void*)c->g_normal,
                              (const void*)c->g_depth_gradient, (const void*)c->g_instance_material, (const void*)c->albedo})
        HK_TRY(ext_wait(c, gs, plane));
    timed(c, "gbuffer", gs, [&] { launch_gbuffer(A, V, c->albedo, c->gb_stack_need, gs); });
    sig.win[0] = A.F.win_row0;
    sig.win[1] = A.F.win_rows;
    sig.valid = V.motion == 0;
    c->gsig[c->gslot] = sig;
    if (c->models_dirty) {  // this frame's models become the next frame's previous ones
        HK_HIP(c, hipMemcpy2DAsync(c->prev_models, 64, (const char*)c->buf[4] + offsetof(hk_instance, model),
                                   sizeof(hk_instance), 64, c->count[4], hipMemcpyDeviceToDevice, gs));
        c->models_dirty = false;
    }
    if (gs != st) {
        HK_HIP(c, hipEventRecord(c->ev_gb_done, gs));
        c->gb_pending = true;
    }
    c->gb_call_rec = pipe;
    c->gb_on_gs = gs != st;
    c->gb_serial = false;
    c->gb_calls++;
    c->albedo_fresh = true;
    HK_HIP(c, hipGetLastError());
    return HK_OK;
}

int hk_set_gbuffer_plane(hk_ctx* c, int plane, const void* data, size_t bytes, int device_ptr, void* stream)
{
    if (!c || !data) return HK_ERR_INVALID;
    if (!c->sized) return fail(c, HK_ERR_STATE, "hk_resize has not been called");
    c->albedo_fresh = false;
    size_t SP = (size_t)c->S[0] * c->S_rows;
    void* dst = nullptr;
    size_t need = 0;
    switch (plane) {
    case 0: dst = c->g_position; need = SP * 16; break;
    case 1: dst = c->g_normal; need = SP * 4; break;
    case 2: dst = c->g_depth_gradient; need = SP * 8; break;
    case 3: dst = c->g_instance_material; need = SP * 8; break;
    case 4: dst = c->g_velocity_uv; need = SP * 16; break;
    default: return fail(c, HK_ERR_INVALID, "unknown G-buffer plane");
    }
    if (bytes != need) return fail(c, HK_ERR_INVALID, "G-buffer plane size mismatch");
    c->gen++;
    c->gb_valid = false;  // host planes: the G-buffer elision mask no longer describes the slots
    // host planes may carry any velocity: the identity-reprojection paths (fused launch, band row windows,
    // the direct pair's elision) stay off until the next k_gbuffer of a static frame
    c->velocity_zero = false;
    // a new frame's position / velocity plane: the current one becomes the previous (prepass.rs:309-317)
    if (plane == 0) {
        std::swap(c->g_position, c->g_prev_position);
        dst = c->g_position;
    } else if (plane == 4) {
        std::swap(c->g_velocity_uv, c->g_prev_velocity_uv);
        dst = c->g_velocity_uv;
    }
    (void)hipSetDevice(c->device);
    hipStream_t st = pick(c, stream);
    HK_TRY(gb_join(c, st));
    HK_TRY(ext_wait(c, st, dst));
    c->gb_serial = true;
    HK_HIP(c, hipMemcpyAsync(dst, data, bytes, device_ptr ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
    if (!device_ptr) HK_HIP(c, hipStreamSynchronize(st));
    return HK_OK;
}

static ChannelArgs channel(hk_ctx* c, uint32_t number, int ch)
{
    // LightBindGroup reservoir pairs (light.rs:518-546); head = frame % 2 (light.rs:376)
    static const int pairs[3][2] = {{0, 4}, {2, 4}, {6, 8}};
    uint32_t current = number % 2u, previous = 1u - current;
    ChannelArgs C;
    C.bg = nullptr;
    C.bg_need = 0;
    C.view = nullptr;
    C.view_n = 0;
    C.prev = ResBuf{c->reservoirs[current + pairs[ch][0]], c->res_n};
    C.cur = ResBuf{c->reservoirs[previous + pairs[ch][0]], c->res_n};
    C.prev_spatial = ResBuf{c->reservoirs[current + pairs[ch][1]], c->res_n};
    C.spatial = ResBuf{c->reservoirs[previous + pairs[ch][1]], c->res_n};
    C.variance = c->variance[ch];
    C.render = c->render[ch];
    return C;
}

// The background elision mask k (0: direct/emissive pair, 1: indirect) for a launch over window A
// of this frame, or nullptr when the launch does not use it (use = false: another kernel writes the
// channel's targets this frame, so the mask is dropped and rebuilt from zero the next time).
static int bg_mask(hk_ctx* c, int k, const FrameArgs& A, bool use, bool pair, hipStream_t st, ChannelArgs& C)
{
    C.bg = nullptr;
    C.bg_need = 0;
    if (!use || bg_elision_off(c)) {
        c->bg_valid[k] = false;
        return HK_OK;
    }
    if (!c->bg_valid[k] || c->bg_key[k][0] != A.F.win_row0 || c->bg_key[k][1] != A.F.win_rows) {
        HK_HIP(c, hipMemsetAsync(c->bgmask[k], 0, c->res_n, st));
        c->bg_valid[k] = true;
        c->bg_key[k][0] = A.F.win_row0;
        c->bg_key[k][1] = A.F.win_rows;
    }
    C.bg = c->bgmask[k];
    // targets of this frame: reservoir parity (the temporal buffer), render / variance slot, and
    // (pair: no spatial reuse pass rewrites it) the spatial pair, both of whose buffers are stored
    C.bg_need = (1u << (A.F.number & 1u)) | (4u << c->rslot) | (pair ? 16u : 0u);
    return HK_OK;
}

int hk_render_frame(hk_ctx* c, const hk_settings* settings, const hk_frame_inputs* in, void* stream)
{
    int rc = check_ready(c, true);
    if (rc) return rc;
    if (!settings || !in) return fail(c, HK_ERR_INVALID, "null settings or frame inputs");
    float want = settings->upscale_ratio < 1.0f ? 1.0f : (settings->upscale_ratio > 2.0f ? 2.0f : settings->upscale_ratio);
    if (want != c->ratio) return fail(c, HK_ERR_STATE, "settings.upscale_ratio differs from the hk_resize ratio");
    // every argument / state check before any scheduling state changes: a rejected call leaves the
    // next frame's pipelining as it was
    if (c->stripe_n >= 2 && (settings->emissive_spatial_reuse || settings->indirect_spatial_reuse))
        return fail(c, HK_ERR_STATE, "interleaved stripes (hk_resize_striped) exclude spatial reuse: it reads neighbours");
    (void)hipSetDevice(c->device);
    hipStream_t st = pick_frame(c, stream);
    c->heavy = settings->indirect_spatial_reuse || settings->emissive_spatial_reuse || c->dn_calls > 0;  // pipeline_size
    c->dn_calls = 0;
    // Frame-tail pipelining: with all three channels rendered, this frame's render / variance
    // targets are the other slot, last read by frame f-2's denoise / tone-sum, so frame f-1's tail
    // (on dn_stream) can still be running while this frame's light passes start.
    const bool swap = dn_pipeline_enabled(c) && settings->indirect_bounces >= 1u;
    // This frame's G-buffer ran pipelined on gb_stream after the caller stream at the previous
    // hk_render_gbuffer's entry (W), and since W only the frame sequence ran, on this stream (no other
    // API call, no stream change): frame f-1's hk_render_frame, denoise, tone-sum and this frame's
    // hk_render_gbuffer.  See the fork below.
    const bool gb_fresh = c->gb_on_gs && c->gb_wait_valid && c->other_picks == c->gb_wait_other &&
                          c->frame_st_epoch == c->gb_wait_epoch && c->gb_pending;
    if (swap) {
        for (int ch = 0; ch < 3; ++ch) {
            std::swap(c->render[ch], c->render_alt[ch]);
            std::swap(c->variance[ch], c->variance_alt[ch]);
        }
        c->rslot ^= 1u;
    }
    // the render slot's last reader (frame f-2's tail) — also covered by ev_gb_done when k_gbuffer waited
    // for that tail or a later one (dn_stream is in order); each wait packet costs the stream latency
    const bool slot_wait = swap && c->rslot_rec[c->rslot];
    const bool slot_covered = gb_fresh && c->gb_pending && c->rslot_seq[c->rslot] <= c->gb_tail_seq;
    if (slot_wait && !slot_covered) HK_HIP(c, hipStreamWaitEvent(st, c->ev_rslot[c->rslot], 0));
    // (k_albedo rewrites the albedo plane a previous tail may still read: full join then)
    HK_TRY(gb_join(c, st, !swap || !c->albedo_fresh));
    // foreign-stream copies of the planes this call writes wait on st; when the indirect chain's own planes
    // are among them, its side stream must fork from st after those waits (no fork shortcut below)
    bool had_ext = false;
    for (const auto& r : c->ext_reads) had_ext |= r.first == c->render[2] || r.first == c->variance[2];
    if (!c->ext_reads.empty()) {
        HK_TRY(ext_wait(c, st, c->albedo));
        for (int ch = 0; ch < 3; ++ch) {
            HK_TRY(ext_wait(c, st, c->render[ch]));
            HK_TRY(ext_wait(c, st, c->variance[ch]));
        }
    }
    c->rf_swapped = swap;
    c->tail_open = false;
    c->head = in->frame_number & 1u;
    c->timing_frame = in->frame_number % c->timing_every == 0u;
    FrameArgs A = frame_args(c, settings, in);
    // The indirect channel owns reservoir buffers 6-9 (light.rs:518-546 pairs (6,8)); direct and
    // emissive share the spatial pair 4/5 and stay in reference order.  So the indirect chain can
    // run concurrently with albedo -> direct -> emissive: it goes to a side stream and joins
    // before returning.  The latency-bound traversal kernels leave issue slots and memory-level
    // parallelism idle, so the overlap pays even when one pass fills the GPU (cornell 1080p
    // 0.81 -> 0.77 ms/frame; 64x64 0.26 -> 0.18 ms).  Per-kernel event timings then include the
    // overlap.  Option channel_streams = 0 restores the serial order.
    const bool fork = c->on(OPT_CHANNEL_STREAMS);
    // fork_events: the indirect chain really runs on the side stream (not when k_light_merged takes it)
    bool fork_events = false;
    hipStream_t s1 = st, s2 = fork ? c->side[1] : st;
    const FrameArgs A_all = A;
    if (!c->albedo_fresh) {
        const FrameArgs AG = pass_window(c, A_all, GBUFFER_REACH);
        timed(c, "full_screen_albedo", st, [&] { launch_albedo(AG, c->albedo, st); });
    }
    // per-pass row windows of a band (pass_window): each channel's temporal pass on the rows its spatial
    // pass reads (core +-(OUT + that channel's range): direct_lit has no spatial pass, light.rs:656-676),
    // then spatial reuse.  A: the indirect channel; AE: direct + emissive.
    // (sticky margins: band_windows)
    HK_TRY(band_windows(c, settings, st));
    A = pass_window(c, A_all, c->win_ind);
    FrameArgs AE = pass_window(c, A_all, c->win_emi);
    const FrameArgs AS = pass_window(c, A_all, c->win_out);
    ChannelArgs C0 = channel(c, A.F.number, 0);
    ChannelArgs C1 = channel(c, A.F.number, 1);
    // direct_lit + emissive in one launch when every reprojection is the identity: see
    // k_direct_fused.  That needs a zero velocity plane (k_gbuffer of a frame without camera or
    // instance motion: velocity_zero; host planes may hold any velocity) at upscale ratio 1 (the
    // deferred jitter is the identity).  Only for frames of >= 1 Mpx: there it saves a launch and a
    // tail (cornell 1080p 0.652 -> 0.622 ms); on a small band (a 4- or 8-way split) the two passes
    // on their own overlap the indirect chain better (0.143 vs 0.151 ms).  Options fuse, fuse_min_px.
    const bool fuse = c->albedo_fresh && c->velocity_zero && c->ratio == 1.0f &&
                      ctx_px(c) >= c->opt[OPT_FUSE_MIN_PX] && c->on(OPT_FUSE);
    // background elision (bg_mask, hk_kernels.hip bg_elide); the separate launches share the pair's mask
    // (direct_pass).  A background pixel's own targets (temporal record, render, variance) are written by
    // that pixel alone, so they elide with or without motion.  Under motion the temporal passes also scatter
    // into the previous spatial buffer at reprojected pixels (light.wgsl:1092-1095, 1199-1202, 1453-1457),
    // and the record they scatter there is the zero reservoir (check_previous_reservoir zeroes it before the
    // store): the indirect channel's background constant, so its pair bit stays true; the direct pair's
    // background record is background_reservoir (count 1), so its pair elides only under the identity
    // reprojection — bg_elide rewrites a background byte without the pair bit whenever the frame's targets
    // do not include it, so a motion frame clears it.
    const bool identity = c->albedo_fresh && c->velocity_zero && c->ratio == 1.0f;
    const bool elide = c->albedo_fresh && c->ratio == 1.0f;
    ChannelArgs C2 = channel(c, A.F.number, 2);
    // spatial view planes (ChannelArgs::view): the indirect temporal pass writes them next to the records
    // it stores, this frame's spatial pass reads its neighbours from them.  Only when that temporal pass
    // stores its records (temporal_reuse; otherwise `cur` keeps older records the planes do not mirror).
    // Option spatial_view_planes = 0: off (the spatial pass gathers the records' own planes).
    if (settings->indirect_spatial_reuse && settings->temporal_reuse && c->on(OPT_SPATIAL_VIEW)) {
        C2.view = c->sp_view;
        C2.view_n = c->res_n;
    }
    bool multi = settings->indirect_bounces >= 2u;
    // the wavefront pipeline covers one bounce and scenes with up to WF_MAX_BINS - 1 materials
    const bool wf = c->wavefront && !multi && c->count[6] + 1u <= WF_MAX_BINS;
    // direct_lit + emissive (fused per pixel) and the one-bounce indirect pass in ONE launch
    // (k_light_merged), replacing the indirect side stream and its fork / join events.  It needs the
    // fused launch's conditions (identity reprojection) and a direct pass that does not stage the scene.
    // By default on the frames that are not pipelined (pipeline_size: < 1.2 Mpx, the 2- to 8-way
    // stripes of 1080p) and have no spatial reuse: there each kernel lasts a few wave lifetimes and
    // the fork / join events' latency is a large part of the frame (cornell stripes 2-way 0.270 ->
    // 0.263, 4-way 0.164 -> 0.160, 8-way 0.144 -> 0.112 ms/frame with the serial path's event
    // elision); on pipelined frames the streams overlap better (1080p 0.472 vs 0.486, city 4K 6.25
    // vs 7.21: spatial reuse would wait for the direct pass).  Not in the isolated-kernel measurement
    // mode (channel_streams = 0).  Option merge: 1 whenever possible, 0 never, -1 this default.
    const bool merge_possible = identity && fork && !multi && !wf && !light_lds_direct(A) && c->on(OPT_FUSE);
    const bool merge_default = !pipeline_size(c) && !settings->indirect_spatial_reuse && !settings->emissive_spatial_reuse;
    const bool merge = merge_possible && (c->opt[OPT_MERGE] < 0.0 ? merge_default : c->on(OPT_MERGE));
    // (one grid for all three channels: the wider window)
    if (merge) A = AE = pass_window(c, A_all, std::max(c->win_ind, c->win_emi));
    if (fork && !merge) {
        if (gb_fresh && c->rf_side_only && swap && c->albedo_fresh && !had_ext) {
            // The fork marker would make the side stream wait for the caller stream here.  What the
            // indirect chain reads of that stream's work: the work before W (k_gbuffer waited for it),
            // frame f-1's hk_render_frame (its indirect chain ran on the side stream itself; the rest of
            // it — k_albedo did not run, direct / emissive passes, their masks — writes buffers the chain
            // does not read), frame f-1's tail (on dn_stream; it reads the other render slot and no
            // reservoir), frame f-2's tail (the render slot this frame writes: covered when k_gbuffer
            // waited for that tail or a later one) and the G-buffer.  So the side stream waits for
            // ev_gb_done alone: every packet queued ahead of a kernel delays it, and the side stream
            // shares its hardware queue with gb_stream (cornell 1080p 0.472 -> 0.45 ms/frame).
            if (slot_wait && !slot_covered) HK_HIP(c, hipStreamWaitEvent(s2, c->ev_rslot[c->rslot], 0));
            HK_HIP(c, hipStreamWaitEvent(s2, c->ev_gb_done, 0));
        } else {
            HK_HIP(c, hipEventRecord(c->ev_fork, st));
            HK_HIP(c, hipStreamWaitEvent(s2, c->ev_fork, 0));
        }
        fork_events = true;
    }
    HK_TRY(bg_mask(c, 0, AE, elide, identity && !settings->emissive_spatial_reuse, st, C0));
    C1.bg = C0.bg;
    C1.bg_need = C0.bg_need;
    if (merge) {
        // (the elision mask of the indirect channel is prepared on the launch stream)
        HK_TRY(bg_mask(c, 1, A, elide, !settings->indirect_spatial_reuse, st, C2));
        timed(c, "light_merged", st, [&] { launch_light_merged(A, C0, C1, C2, st); });
        if (settings->emissive_spatial_reuse)
            timed(c, "emissive_spatial_reuse", st, [&] { launch_spatial(AS, C1, true, st); });
        if (settings->indirect_spatial_reuse)
            timed(c, "indirect_spatial_reuse", st, [&] { launch_spatial(AS, C2, false, st); });
    } else {
        if (fuse) {
            timed(c, "direct_lit_emissive", st, [&] { launch_direct_fused(AE, C0, C1, st); });
        } else {
            timed(c, "direct_lit", st, [&] { launch_direct(AE, C0, false, st); });
            timed(c, "direct_emissive", s1, [&] { launch_direct(AE, C1, true, s1); });
        }
        if (settings->emissive_spatial_reuse) timed(c, "emissive_spatial_reuse", s1, [&] { launch_spatial(AS, C1, true, s1); });
        // (the wavefront pass elides in its generation stage, which classifies every pixel)
        HK_TRY(bg_mask(c, 1, A, elide, !settings->indirect_spatial_reuse, s2, C2));
        if (wf) {
            HK_TRY(ensure_wavefront(c));
            WfArgs W{c->wf_queue1, c->wf_keys, c->wf_queue2, c->wf_hit, c->wf_hit_t, c->wf_ctl, c->count[6] + 1u,
                     c->wf_seg_cap};
            HK_HIP(c, hipMemsetAsync(W.ctl, 0, (size_t)wf_ctl_words(W.bins) * 4, s2));
            timed(c, "indirect_wavefront", s2, [&] { launch_indirect_wavefront(A, C2, W, s2); });
        } else {
            timed(c, multi ? "indirect_multiple_bounces" : "indirect_lit_ambient", s2, [&] { launch_indirect(A, C2, multi, s2); });
        }
        if (settings->indirect_spatial_reuse) timed(c, "indirect_spatial_reuse", s2, [&] { launch_spatial(AS, C2, false, s2); });
    }
    if (fork_events) {
        HK_HIP(c, hipEventRecord(c->ev_join[1], s2));
        HK_HIP(c, hipStreamWaitEvent(st, c->ev_join[1], 0));
    }
    c->rf_side_only = fork_events && c->albedo_fresh;  // (no k_albedo on the caller stream)
    c->rf_seq++;
    if (swap) {
        HK_HIP(c, hipEventRecord(c->ev_rf, st));
        c->rf_rec_seq = c->rf_seq;
        c->rf_other = c->other_picks;
        c->rf_epoch = c->frame_st_epoch;
    }
    HK_HIP(c, hipGetLastError());
    return HK_OK;
}

int hk_denoise(hk_ctx* c, const hk_settings* settings, const hk_frame_inputs* in, void* stream)
{
    int rc = check_ready(c, false);
    if (rc) return rc;
    if (!settings || !in) return fail(c, HK_ERR_INVALID, "null settings or frame inputs");
    if (!settings->denoise) return HK_OK;
    if (c->stripe_n >= 2) return fail(c, HK_ERR_STATE, "interleaved stripes (hk_resize_striped) exclude the denoiser: it reads neighbours");
    c->dn_calls++;
    (void)hipSetDevice(c->device);
    hipStream_t caller = pick_frame(c, stream);
    // after a slot-swapping hk_render_frame: on dn_stream, next to the following frame's passes
    const bool async = c->rf_swapped;
    hipStream_t st = async ? c->dn_stream : caller;
    if (async) HK_TRY(tail_begin(c));
    else HK_TRY(gb_join(c, st));
    for (int ch = 0; ch < 3; ++ch) {
        HK_TRY(ext_wait(c, st, c->denoised[ch]));
        HK_TRY(ext_wait(c, st, c->internal_variance[ch]));  // HK_OUT_DENOISE_INTERNAL_VARIANCE copies
    }
    FrameArgs A = frame_args(c, settings, in);
    int channels = settings->indirect_bounces == 0u ? 2 : 3;  // post_process.rs:949-954
    DenoiseArgs D;
    std::memset(&D, 0, sizeof(D));
    D.channels = channels;
    D.albedo = c->albedo;
    for (int ch = 0; ch < 3; ++ch) {
        D.render[ch] = c->render[ch];
        D.variance[ch] = c->variance[ch];
        D.internal_variance[ch] = c->internal_variance[ch];
        D.output[ch] = c->denoised[ch];
    }
    for (int i = 0; i < 4; ++i) {
        D.rgb[i] = c->dn_rgb[i];
        D.bi[i] = c->dn_bi[i];
    }
    D.nd = c->dn_nd;
    D.center = c->dn_center;
    D.den2 = c->dn_den2;
    c->last_denoised_channels = channels;
    // band windows (pass_window): demodulation on core +-15, the levels on +-7, 3, 1, 0
    const FrameArgs AD = pass_window(c, A, DENOISE_OUT_REACH - 1);
    timed(c, "demodulation", st, [&] { launch_demod(AD, D, st); });
    static constexpr int32_t LEVEL_REACH[4] = {7, 3, 1, 0};
    for (int level = 0; level < 4; ++level) {
        const FrameArgs AL = pass_window(c, A, LEVEL_REACH[level]);
        timed(c, "denoise", st, [&] { launch_denoise(AL, D, level, st); });
    }
    if (async) HK_TRY(tail_end(c));
    HK_HIP(c, hipGetLastError());
    return HK_OK;
}

int hk_tone_sum(hk_ctx* c, const hk_settings* settings, void* stream)
{
    int rc = check_ready(c, false);
    if (rc) return rc;
    if (!settings) return fail(c, HK_ERR_INVALID, "null settings");
    (void)hipSetDevice(c->device);
    // after a slot-swapping hk_render_frame: on dn_stream (after that frame's denoise, if any)
    const bool async = c->rf_swapped;
    hipStream_t st = async ? c->dn_stream : pick_frame(c, stream);
    if (async) HK_TRY(tail_begin(c));
    else HK_TRY(gb_join(c, st));
    hk_frame_inputs dummy;
    std::memset(&dummy, 0, sizeof(dummy));
    const FrameArgs A = pass_window(c, frame_args(c, settings, &dummy), 0);
    ToneArgs T;
    T.direct = settings->denoise ? c->denoised[0] : c->render[0];
    T.emissive = settings->denoise ? c->denoised[1] : c->render[1];
    T.indirect = settings->indirect_bounces == 0u ? nullptr : (settings->denoise ? c->denoised[2] : c->render[2]);
    T.output = c->tone_buf[c->head];
    HK_TRY(ext_wait(c, st, T.output));
    timed(c, "tone_mapping", st, [&] { launch_tone(A, T, st); });
    if (async) HK_TRY(tail_end(c));
    HK_HIP(c, hipGetLastError());
    return HK_OK;
}

int hk_post_process(hk_ctx* c, const hk_settings* st, const hk_frame_inputs* in, void* stream)
{
    int rc = check_ready(c, false);
    if (rc) return rc;
    if (!st || !in) return fail(c, HK_ERR_INVALID, "null settings or frame inputs");
    if (c->S_rows != (int32_t)c->S[1]) return fail(c, HK_ERR_STATE, "hk_post_process needs a whole-frame context");
    (void)hipSetDevice(c->device);
    hipStream_t s = pick(c, stream);
    HK_TRY(gb_join(c, s));
    c->head = in->frame_number & 1u;
    const uint32_t head = c->head;
    HK_TRY(ext_wait(c, s, c->upscale));
    HK_TRY(ext_wait(c, s, c->taa_buf[head]));
    // post_process.rs:663-731 sizes: ceil(S * scale), scale = 1 / ratio, x 2 after SMAA TU4x
    float scale = 1.0f / c->ratio;
    const bool smaa = st->upscale == 0u, taa = st->taa == 0u;
    PostArgs P;
    P.frame.number = in->frame_number;
    for (int k = 0; k < 4; ++k) P.frame.clear_color[k] = st->clear_color[k];
    P.frame.upscale_ratio = c->ratio;
    auto tex = [](const void* d, uint32_t w, uint32_t h, uint32_t f16, uint32_t comps) {
        hk_pp_tex t;
        t.data = d, t.w = w, t.h = h, t.f16 = f16, t.comps = comps;
        return t;
    };
    const uint32_t S0 = c->S[0], S1 = c->S[1];
    P.in.position = tex(c->g_position, S0, S1, 0, 4);
    P.in.previous_position = tex(c->g_prev_position, S0, S1, 0, 4);
    P.in.velocity_uv = tex(c->g_velocity_uv, S0, S1, 0, 4);
    P.in.previous_velocity_uv = tex(c->g_prev_velocity_uv, S0, S1, 0, 4);
    P.in.instance_material = tex(c->g_instance_material, S0, S1, 0, 2);
    hk_pp_tex taa_input = tex(c->tone_buf[head], c->s[0], c->s[1], 1, 4);
    if (smaa) {
        scale *= 2.0f;
        const uint32_t U0 = (uint32_t)std::ceil((float)S0 * scale), U1 = (uint32_t)std::ceil((float)S1 * scale);
        if (!c->upscale || c->upscale_wh[0] != U0 || c->upscale_wh[1] != U1) {
            release(c->upscale);
            HK_HIP(c, hipMalloc(&c->upscale, (size_t)U0 * U1 * sizeof(uint2)));
            HK_HIP(c, hipMemset(c->upscale, 0, (size_t)U0 * U1 * sizeof(uint2)));
            c->upscale_wh[0] = U0, c->upscale_wh[1] = U1;
        }
        P.in.render = tex(c->tone_buf[head], c->s[0], c->s[1], 1, 4);
        P.in.previous_render = tex(c->tone_buf[1u - head], c->s[0], c->s[1], 1, 4);
        P.in.output = hk_pp_out{(uint16_t*)c->upscale, U0, U1};
        timed(c, "smaa_tu4x", s, [&] { launch_smaa(P, s); });
        timed(c, "smaa_tu4x_extrapolate", s, [&] { launch_smaa_extrapolate(P, s); });
        taa_input = tex(c->upscale, U0, U1, 1, 4);
    }
    if (taa) {
        const uint32_t T0 = (uint32_t)std::ceil((float)S0 * scale), T1 = (uint32_t)std::ceil((float)S1 * scale);
        if (!c->taa_buf[0] || c->taa_wh[0] != T0 || c->taa_wh[1] != T1) {
            for (int k = 0; k < 2; ++k) {
                release(c->taa_buf[k]);
                HK_HIP(c, hipMalloc(&c->taa_buf[k], (size_t)T0 * T1 * sizeof(uint2)));
                HK_HIP(c, hipMemset(c->taa_buf[k], 0, (size_t)T0 * T1 * sizeof(uint2)));
            }
            c->taa_wh[0] = T0, c->taa_wh[1] = T1;
        }
        P.in.render = taa_input;
        P.in.previous_render = tex(c->taa_buf[1u - head], T0, T1, 1, 4);
        P.in.output = hk_pp_out{(uint16_t*)c->taa_buf[head], T0, T1};
        timed(c, "taa_jasmine", s, [&] { launch_taa(P, s); });
    }
    // the next k_gbuffer overwrites the previous-frame planes read here
    HK_HIP(c, hipEventRecord(c->ev_post, s));
    c->post_pending = true;
    HK_HIP(c, hipGetLastError());
    return HK_OK;
}

// Sub-frame accumulation is part of the frame sequence: after a slot-swapping hk_render_frame it runs in
// the frame's tail on dn_stream (after the tone-sum it reads), next to the following sub-frame's light
// passes; otherwise on the caller's stream.  Only these two calls touch the accumulator.
int hk_accumulate(hk_ctx* c, int reset, void* stream)
{
    int rc = check_ready(c, false);
    if (rc) return rc;
    (void)hipSetDevice(c->device);
    const bool async = c->rf_swapped && c->tail_open;  // this frame's tone-sum ran in the tail
    hipStream_t st = async ? c->dn_stream : pick_frame(c, stream);
    if (async) HK_TRY(tail_begin(c));
    else HK_TRY(gb_join(c, st));
    const size_t n = (size_t)c->s[0] * (size_t)c->s_rows;
    if (!c->accum) {
        HK_HIP(c, hipMalloc(&c->accum, n * sizeof(float4)));
        HK_HIP(c, hipMalloc(&c->accum_out, n * sizeof(uint2)));
        HK_HIP(c, hipMemset(c->accum_out, 0, n * sizeof(uint2)));
        reset = 1;
    }
    if (reset) c->accum_n = 0;
    timed(c, "accumulate", st, [&] { launch_accumulate(c->tone_buf[c->head], c->accum, (uint32_t)n, reset, st); });
    if (async) HK_TRY(tail_end(c));
    HK_HIP(c, hipGetLastError());
    c->accum_n += 1;
    return HK_OK;
}

int hk_resolve_accumulation(hk_ctx* c, void* stream)
{
    int rc = check_ready(c, false);
    if (rc) return rc;
    if (!c->accum || c->accum_n == 0) return fail(c, HK_ERR_STATE, "nothing accumulated (hk_accumulate)");
    (void)hipSetDevice(c->device);
    const bool async = c->rf_swapped && c->tail_open;
    hipStream_t st = async ? c->dn_stream : pick_frame(c, stream);
    if (async) HK_TRY(tail_begin(c));
    else HK_TRY(gb_join(c, st));
    HK_TRY(ext_wait(c, st, c->accum_out));
    const size_t n = (size_t)c->s[0] * (size_t)c->s_rows;
    timed(c, "resolve", st, [&] { launch_resolve(c->accum, (uint32_t)n, (float)c->accum_n, c->accum_out, st); });
    if (async) HK_TRY(tail_end(c));
    HK_HIP(c, hipGetLastError());
    return HK_OK;
}

static void* output_ptr(hk_ctx* c, int id, uint32_t* w, uint32_t* h, uint32_t* bpp)
{
    uint32_t W = c->s[0], H = (uint32_t)c->s_rows, B = 8;
    void* p = nullptr;
    switch (id) {
    case HK_OUT_ALBEDO: p = c->albedo; W = c->S[0]; H = (uint32_t)c->S_rows; break;
    case HK_OUT_VARIANCE_DIRECT: case HK_OUT_VARIANCE_EMISSIVE: case HK_OUT_VARIANCE_INDIRECT:
        p = c->variance[id - HK_OUT_VARIANCE_DIRECT]; B = 4; break;
    case HK_OUT_RENDER_DIRECT: case HK_OUT_RENDER_EMISSIVE: case HK_OUT_RENDER_INDIRECT:
        p = c->render[id - HK_OUT_RENDER_DIRECT]; break;
    case HK_OUT_DENOISED_DIRECT: case HK_OUT_DENOISED_EMISSIVE: case HK_OUT_DENOISED_INDIRECT:
        p = c->denoised[id - HK_OUT_DENOISED_DIRECT]; break;
    case HK_OUT_TONE_MAPPED: p = c->tone_buf[c->head]; break;
    case HK_OUT_TONE_MAPPED_PREVIOUS: p = c->tone_buf[c->head ^ 1u]; break;
    case HK_OUT_UPSCALED: p = c->upscale; W = c->upscale_wh[0]; H = c->upscale_wh[1]; break;
    case HK_OUT_TAA: p = c->taa_buf[c->head]; W = c->taa_wh[0]; H = c->taa_wh[1]; break;
    case HK_OUT_ACCUMULATED: p = c->accum_out; break;
    case HK_OUT_GBUF_POSITION: p = c->g_position; W = c->S[0]; H = (uint32_t)c->S_rows; B = 16; break;
    case HK_OUT_GBUF_NORMAL: p = c->g_normal; W = c->S[0]; H = (uint32_t)c->S_rows; B = 4; break;
    case HK_OUT_GBUF_DEPTH_GRADIENT: p = c->g_depth_gradient; W = c->S[0]; H = (uint32_t)c->S_rows; B = 8; break;
    case HK_OUT_GBUF_INSTANCE_MATERIAL: p = c->g_instance_material; W = c->S[0]; H = (uint32_t)c->S_rows; B = 8; break;
    case HK_OUT_GBUF_VELOCITY_UV: p = c->g_velocity_uv; W = c->S[0]; H = (uint32_t)c->S_rows; B = 16; break;
    case HK_OUT_DENOISE_INTERNAL_VARIANCE: p = c->internal_variance[c->last_denoised_channels - 1]; B = 4; break;
    default: return nullptr;
    }
    if (w) *w = W;
    if (h) *h = H;
    if (bpp) *bpp = B;
    return p;
}

int hk_output_info(const hk_ctx* c, int id, uint32_t* w, uint32_t* h, uint32_t* bpp)
{
    if (!c || !c->sized) return HK_ERR_STATE;
    return output_ptr(const_cast<hk_ctx*>(c), id, w, h, bpp) ? HK_OK : HK_ERR_INVALID;
}

const void* hk_output_device_ptr(hk_ctx* c, int id)
{
    if (!c || !c->sized) return nullptr;
    return output_ptr(c, id, nullptr, nullptr, nullptr);
}

int hk_lane_stats(hk_ctx* c, const char** names, unsigned long long* active, unsigned long long* iterations,
                  int capacity)
{
    if (!c) return HK_ERR_INVALID;
    const int n = (int)c->lane_names.size();
    for (int i = 0; i < n && i < capacity; ++i) {
        if (names) names[i] = c->lane_names[i].c_str();
        if (active) active[i] = c->lane_act[i];
        if (iterations) iterations[i] = c->lane_its[i];
    }
    return n;
}

int hk_set_wavefront(hk_ctx* c, int enable)
{
    if (!c) return HK_ERR_INVALID;
    c->wavefront = enable != 0;
    return HK_OK;
}

int hk_sync(hk_ctx* c, void* stream)
{
    if (!c) return HK_ERR_INVALID;
    (void)hipSetDevice(c->device);
    return gb_join(c, pick(c, stream));
}

int hk_get_output(hk_ctx* c, int id, void* dst, size_t bytes, int to_host, void* stream)
{
    if (!c || !dst) return HK_ERR_INVALID;
    if (!c->sized) return fail(c, HK_ERR_STATE, "hk_resize has not been called");
    uint32_t w, h, b;
    void* p = output_ptr(c, id, &w, &h, &b);
    if (!p) return fail(c, HK_ERR_INVALID, "unknown output id");
    size_t need = (size_t)w * h * b;
    if (bytes != need) return fail(c, HK_ERR_INVALID, "output size mismatch");
    (void)hipSetDevice(c->device);
    hipStream_t st = pick(c, stream);
    HK_TRY(gb_join(c, st));
    HK_HIP(c, hipMemcpyAsync(dst, p, bytes, to_host ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice, st));
    if (to_host) HK_HIP(c, hipStreamSynchronize(st));
    return HK_OK;
}

static int copy_output_rect(hk_ctx* c, int id, uint32_t row0, uint32_t rows, uint32_t col0, uint32_t cols, void* dst,
                            size_t dst_pitch, int to_host, void* stream);

int hk_copy_output_rows(hk_ctx* c, int id, uint32_t row0, uint32_t rows, void* dst, int to_host, void* stream)
{
    return copy_output_rect(c, id, row0, rows, 0u, 0u, dst, 0u, to_host, stream);
}

int hk_copy_output_rect(hk_ctx* c, int id, uint32_t row0, uint32_t rows, uint32_t col0, uint32_t cols, void* dst,
                        size_t dst_pitch, int to_host, void* stream)
{
    if (cols == 0) return HK_ERR_INVALID;
    return copy_output_rect(c, id, row0, rows, col0, cols, dst, dst_pitch, to_host, stream);
}

// cols 0: whole rows (hk_copy_output_rows); dst_pitch 0: the rectangle's own row bytes
static int copy_output_rect(hk_ctx* c, int id, uint32_t row0, uint32_t rows, uint32_t col0, uint32_t cols, void* dst,
                            size_t dst_pitch, int to_host, void* stream)
{
    if (!c || !dst) return HK_ERR_INVALID;
    if (!c->sized) return fail(c, HK_ERR_STATE, "hk_resize has not been called");
    uint32_t w, h, b;
    void* p = output_ptr(c, id, &w, &h, &b);
    if (!p) return fail(c, HK_ERR_INVALID, "unknown output id");
    if (row0 + rows > h) return fail(c, HK_ERR_INVALID, "row range outside the plane");
    if (cols == 0) {
        col0 = 0;
        cols = w;
    }
    if (col0 + cols > w) return fail(c, HK_ERR_INVALID, "column range outside the plane");
    if (dst_pitch == 0) dst_pitch = (size_t)cols * b;
    if (dst_pitch < (size_t)cols * b) return fail(c, HK_ERR_INVALID, "destination pitch below the rectangle's row bytes");
    (void)hipSetDevice(c->device);
    // A copy on a stream other than the frame sequence's (a communication stream) enqueues nothing on the
    // frame stream but, when the plane's producer may have run there, an event marker: the frame stream
    // never waits for the copy, and the plane's next writer waits for it (ext_reads).  The tone-mapped,
    // accumulated and denoised planes of a pipelined frame come from its tail (dn_stream, ev_dn_last).
    const hipStream_t given = stream ? (hipStream_t)stream : c->stream;
    const bool foreign = c->frame_st && given != c->frame_st && !to_host;
    hipStream_t st = foreign ? given : pick(c, stream);
    HK_TRY(gb_join(c, st));
    if (foreign) {
        const bool from_tail = c->rf_swapped && c->tail_open &&
                               (id == HK_OUT_TONE_MAPPED || id == HK_OUT_TONE_MAPPED_PREVIOUS || id == HK_OUT_ACCUMULATED ||
                                (id >= HK_OUT_DENOISED_DIRECT && id <= HK_OUT_DENOISED_INDIRECT));
        if (!from_tail) {
            HK_HIP(c, hipEventRecord(c->ev_frame_mark, c->frame_st));
            HK_HIP(c, hipStreamWaitEvent(st, c->ev_frame_mark, 0));
        }
    }
    size_t pitch = (size_t)w * b;
    const hipMemcpyKind kind = to_host ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    const char* src = (const char*)p + (size_t)row0 * pitch + (size_t)col0 * b;
    if (cols == w && dst_pitch == pitch)
        HK_HIP(c, hipMemcpyAsync(dst, src, (size_t)rows * pitch, kind, st));
    else
        HK_HIP(c, hipMemcpy2DAsync(dst, dst_pitch, src, pitch, (size_t)cols * b, rows, kind, st));
    if (to_host) HK_HIP(c, hipStreamSynchronize(st));
    if (foreign) {
        // entries whose copies have completed go back to the pool (a plane nobody rewrites would otherwise keep its
        // entries, and ext_reads would grow with every copy of it)
        for (size_t k = 0; k < c->ext_reads.size();) {
            if (hipEventQuery(c->ext_reads[k].second) == hipSuccess) {
                c->ext_pool.push_back(c->ext_reads[k].second);
                c->ext_reads[k] = c->ext_reads.back();
                c->ext_reads.pop_back();
            } else {
                ++k;
            }
        }
        hipEvent_t e = nullptr;
        if (!c->ext_pool.empty()) {
            e = c->ext_pool.back();
            c->ext_pool.pop_back();
        } else {
            HK_HIP(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        HK_HIP(c, hipEventRecord(e, st));
        c->ext_reads.emplace_back(p, e);
    }
    return HK_OK;
}

int hk_dump_reservoirs(hk_ctx* c, int id, hk_packed_reservoir* dst, size_t count, void* stream)
{
    if (!c || !dst || id < 0 || id >= HK_RESERVOIR_BUFFERS) return HK_ERR_INVALID;
    if (!c->sized) return fail(c, HK_ERR_STATE, "hk_resize has not been called");
    if (count != c->res_n) return fail(c, HK_ERR_INVALID, "reservoir count mismatch");
    (void)hipSetDevice(c->device);
    hipStream_t st = pick(c, stream);
    HK_TRY(gb_join(c, st));
    std::vector<uint4> planes((size_t)4 * c->res_n);
    HK_HIP(c, hipMemcpyAsync(planes.data(), c->reservoirs[id], planes.size() * sizeof(uint4), hipMemcpyDeviceToHost, st));
    HK_HIP(c, hipStreamSynchronize(st));
    const ResBuf layout{nullptr, c->res_n};
    for (size_t i = 0; i < count; ++i) {
        uint4* o = reinterpret_cast<uint4*>(dst + i);
        for (int k = 0; k < 4; ++k) o[k] = planes[res_chunk(layout, (uint32_t)k, (uint32_t)i)];
    }
    return HK_OK;
}

int hk_load_reservoirs(hk_ctx* c, int id, const hk_packed_reservoir* src, size_t count, void* stream)
{
    if (!c || !src || id < 0 || id >= HK_RESERVOIR_BUFFERS) return HK_ERR_INVALID;
    if (!c->sized) return fail(c, HK_ERR_STATE, "hk_resize has not been called");
    if (count != c->res_n) return fail(c, HK_ERR_INVALID, "reservoir count mismatch");
    (void)hipSetDevice(c->device);
    hipStream_t st = pick(c, stream);
    HK_TRY(gb_join(c, st));
    std::vector<uint4> planes((size_t)4 * c->res_n);
    const ResBuf layout{nullptr, c->res_n};
    for (size_t i = 0; i < count; ++i) {
        const uint4* s = reinterpret_cast<const uint4*>(src + i);
        for (int k = 0; k < 4; ++k) planes[res_chunk(layout, (uint32_t)k, (uint32_t)i)] = s[k];
    }
    HK_HIP(c, hipMemcpyAsync(c->reservoirs[id], planes.data(), planes.size() * sizeof(uint4), hipMemcpyHostToDevice, st));
    c->bg_valid[0] = c->bg_valid[1] = false;  // the elision masks no longer describe the buffers
    HK_HIP(c, hipStreamSynchronize(st));
    return HK_OK;
}

int hk_band_window_grow(hk_ctx* c, const hk_settings* settings, int32_t* ranges, int commit)
{
    if (!c || !settings || !ranges) return HK_ERR_INVALID;
    if (!c->sized) return fail(c, HK_ERR_STATE, "hk_resize has not been called");
    const WindowGrowth G = window_growth(c, settings);
    int n = 0;
    for (int b = 0; b < HK_RESERVOIR_BUFFERS; ++b) {
        bool any = false;
        for (int side = 0; side < 2; ++side) {
            const int32_t r0 = G.rows[b][side][0], r1 = G.rows[b][side][1];
            ranges[4 * b + 2 * side] = r1 > r0 ? c->s_row0 + r0 : 0;
            ranges[4 * b + 2 * side + 1] = r1 > r0 ? r1 - r0 : 0;
            any |= r1 > r0;
        }
        n += any;
    }
    if (commit && G.grows) commit_growth(c, G);
    return n;
}

int hk_reservoir_rows(hk_ctx* c, int id, int32_t frame_row0, int32_t rows, void* data, int store, void* stream)
{
    if (!c || !data || id < 0 || id >= HK_RESERVOIR_BUFFERS || rows < 0) return HK_ERR_INVALID;
    if (!c->sized) return fail(c, HK_ERR_STATE, "hk_resize has not been called");
    if (c->stripe_n >= 2) return fail(c, HK_ERR_STATE, "hk_reservoir_rows needs a contiguous band (not stripes)");
    const int32_t r0 = frame_row0 - c->s_row0;
    if (r0 < 0 || r0 + rows > c->s_rows) return fail(c, HK_ERR_INVALID, "rows outside the context's band");
    if (rows == 0) return HK_OK;
    (void)hipSetDevice(c->device);
    hipStream_t st = pick(c, stream);
    HK_TRY(gb_join(c, st));
    // after every pass the frame sequence enqueued (its side streams joined its stream before returning)
    if (c->frame_st && c->frame_st != st) {
        HK_HIP(c, hipEventRecord(c->ev_frame_mark, c->frame_st));
        HK_HIP(c, hipStreamWaitEvent(st, c->ev_frame_mark, 0));
    }
    const size_t w = c->s[0], n = (size_t)rows * w;
    for (size_t k = 0; k < 4; ++k) {
        uint4* dev = c->reservoirs[id] + k * c->res_n + (size_t)r0 * w;
        uint4* ext = reinterpret_cast<uint4*>(data) + k * n;
        HK_HIP(c, hipMemcpyAsync(store ? dev : ext, store ? ext : dev, n * sizeof(uint4), hipMemcpyDefault, st));
    }
    if (store) c->bg_valid[0] = c->bg_valid[1] = false;  // the elision masks no longer describe the buffers
    HK_HIP(c, hipStreamSynchronize(st));
    return HK_OK;
}

int hk_reset_counters(hk_ctx* c, void* stream)
{
    if (!c) return HK_ERR_INVALID;
    (void)hipSetDevice(c->device);
    HK_TRY(gb_join(c, pick(c, stream)));
    HK_HIP(c, hipMemsetAsync(c->counters, 0, COUNTER_BYTES, pick(c, stream)));
    c->primary_reused = 0;
    return HK_OK;
}

int hk_read_counters(hk_ctx* c, hk_counters* out, void* stream)
{
    if (!c || !out) return HK_ERR_INVALID;
    (void)hipSetDevice(c->device);
    hipStream_t st = pick(c, stream);
    HK_TRY(gb_join(c, st));
    std::vector<unsigned long long> v(3 * COUNTER_SPAN);
    HK_HIP(c, hipMemcpyAsync(v.data(), c->counters, COUNTER_BYTES, hipMemcpyDeviceToHost, st));
    HK_HIP(c, hipStreamSynchronize(st));
    unsigned long long sum[3] = {0, 0, 0};
    for (int k = 0; k < 3; ++k)
        for (size_t i = 0; i < COUNTER_SHARDS; ++i) sum[k] += v[k * COUNTER_SPAN + i * COUNTER_STRIDE];
    out->traverse_top = sum[0];
    out->traverse_emitter = sum[1];
    out->primary = sum[2] + c->primary_reused;
    out->primary_reused = c->primary_reused;
    return HK_OK;
}

int hk_enable_kernel_timing(hk_ctx* c, int enable)
{
    if (!c) return HK_ERR_INVALID;
    flush_timing(c);
    c->timing = enable != 0;
    c->timing_names.clear();
    c->timing_ms.clear();
    c->timing_n.clear();
    return HK_OK;
}

int hk_set_kernel_timing_interval(hk_ctx* c, uint32_t every)
{
    if (!c || every == 0) return HK_ERR_INVALID;
    c->timing_every = every;
    return HK_OK;
}

int hk_kernel_timing(hk_ctx* c, const char** names, float* ms, int capacity)
{
    if (!c) return HK_ERR_INVALID;
    flush_timing(c);
    int n = (int)c->timing_names.size();
    for (int i = 0; i < n && i < capacity; ++i) {
        if (names) names[i] = c->timing_names[i].c_str();
        if (ms) ms[i] = (float)(c->timing_ms[i] / (double)(c->timing_n[i] ? c->timing_n[i] : 1));
    }
    return n;
}

int hk_trace(hk_ctx* c, const float* rays, const float* max_d, const float* early_d, const uint32_t* excl, uint32_t n,
             void* hits, int device_ptrs, void* stream)
{
    if (!c || !rays || !hits) return HK_ERR_INVALID;
    if (!c->has_scene) return fail(c, HK_ERR_STATE, "no scene uploaded (hk_scene_upload)");
    if (n == 0) return HK_OK;
    (void)hipSetDevice(c->device);
    hipStream_t st = pick(c, stream);
    HK_TRY(gb_join(c, st));
    FrameArgs A = frame_args(c, nullptr, nullptr);
    if (device_ptrs) {
        launch_trace(A.sc, rays, max_d, early_d, excl, n, (uint32_t*)hits, c->counters, st);
        HK_HIP(c, hipGetLastError());
        return HK_OK;
    }
    float *d_rays = nullptr, *d_max = nullptr, *d_early = nullptr;
    uint32_t *d_excl = nullptr, *d_hits = nullptr;
    HK_HIP(c, hipMalloc(&d_rays, (size_t)n * 24));
    HK_HIP(c, hipMalloc(&d_hits, (size_t)n * 20));
    HK_HIP(c, hipMemcpy(d_rays, rays, (size_t)n * 24, hipMemcpyHostToDevice));
    if (max_d) {
        HK_HIP(c, hipMalloc(&d_max, (size_t)n * 4));
        HK_HIP(c, hipMemcpy(d_max, max_d, (size_t)n * 4, hipMemcpyHostToDevice));
    }
    if (early_d) {
        HK_HIP(c, hipMalloc(&d_early, (size_t)n * 4));
        HK_HIP(c, hipMemcpy(d_early, early_d, (size_t)n * 4, hipMemcpyHostToDevice));
    }
    if (excl) {
        HK_HIP(c, hipMalloc(&d_excl, (size_t)n * 4));
        HK_HIP(c, hipMemcpy(d_excl, excl, (size_t)n * 4, hipMemcpyHostToDevice));
    }
    launch_trace(A.sc, d_rays, d_max, d_early, d_excl, n, d_hits, c->counters, st);
    HK_HIP(c, hipGetLastError());
    HK_HIP(c, hipMemcpyAsync(hits, d_hits, (size_t)n * 20, hipMemcpyDeviceToHost, st));
    HK_HIP(c, hipStreamSynchronize(st));
    release(d_rays);
    release(d_hits);
    release(d_max);
    release(d_early);
    release(d_excl);
    return HK_OK;
}

int hk_selftest_f16(hk_ctx* c, const float* in, uint32_t n, uint16_t* out)
{
    if (!c || (n && (!in || !out))) return HK_ERR_INVALID;
    if (n == 0) return HK_OK;
    (void)hipSetDevice(c->device);
    hipStream_t st = pick(c, nullptr);
    float* d_in = nullptr;
    uint16_t* d_out = nullptr;
    HK_HIP(c, hipMalloc(&d_in, (size_t)n * 4));
    HK_HIP(c, hipMalloc(&d_out, (size_t)n * 2));
    HK_HIP(c, hipMemcpy(d_in, in, (size_t)n * 4, hipMemcpyHostToDevice));
    launch_f16(d_in, n, d_out, st);
    HK_HIP(c, hipGetLastError());
    HK_HIP(c, hipMemcpyAsync(out, d_out, (size_t)n * 2, hipMemcpyDeviceToHost, st));
    HK_HIP(c, hipStreamSynchronize(st));
    release(d_in);
    release(d_out);
    return HK_OK;
}

int hk_selftest_div(hk_ctx* c, float divisor, uint32_t lo, uint32_t hi, uint64_t* mismatches)
{
    if (!c || !mismatches || !(divisor > 0.0f)) return HK_ERR_INVALID;
    (void)hipSetDevice(c->device);
    hipStream_t st = pick(c, nullptr);
    unsigned long long* d_bad = nullptr;
    const size_t bytes = (size_t)COUNTER_SHARDS * COUNTER_STRIDE * 8;
    HK_HIP(c, hipMalloc(&d_bad, bytes));
    HK_HIP(c, hipMemsetAsync(d_bad, 0, bytes, st));
    launch_div_check(divisor, 1.0f / divisor, lo, hi, d_bad, st);
    HK_HIP(c, hipGetLastError());
    std::vector<unsigned long long> h(bytes / 8);
    HK_HIP(c, hipMemcpyAsync(h.data(), d_bad, bytes, hipMemcpyDeviceToHost, st));
    HK_HIP(c, hipStreamSynchronize(st));
    release(d_bad);
    uint64_t total = 0;
    for (size_t k = 0; k < h.size(); k += COUNTER_STRIDE) total += h[k];
    *mismatches = total;
    return HK_OK;
}

int hk_selftest_rcp(hk_ctx* c, uint32_t lo, uint32_t hi, uint64_t* mismatches)
{
    if (!c || !mismatches || lo > hi) return HK_ERR_INVALID;
    (void)hipSetDevice(c->device);
    hipStream_t st = pick(c, nullptr);
    unsigned long long* d_bad = nullptr;
    const size_t bytes = (size_t)COUNTER_SHARDS * COUNTER_STRIDE * 8;
    HK_HIP(c, hipMalloc(&d_bad, bytes));
    HK_HIP(c, hipMemsetAsync(d_bad, 0, bytes, st));
    launch_rcp_check(lo, hi, d_bad, st);
    HK_HIP(c, hipGetLastError());
    std::vector<unsigned long long> h(bytes / 8);
    HK_HIP(c, hipMemcpyAsync(h.data(), d_bad, bytes, hipMemcpyDeviceToHost, st));
    HK_HIP(c, hipStreamSynchronize(st));
    release(d_bad);
    uint64_t total = 0;
    for (size_t k = 0; k < h.size(); k += COUNTER_STRIDE) total += h[k];
    *mismatches = total;
    return HK_OK;
}

}  // extern "C"
