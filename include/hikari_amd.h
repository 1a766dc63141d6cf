/*
 * hikari_amd.h — C ABI of the MI355X-native bevy-hikari integrator (libhikari_amd.so).
 *
 * A Rust shim behind bevy-hikari's unchanged `HikariPlugin` / `HikariSettings` API binds
 * these symbols.  Each entry point replaces one piece of the
 * reference's render-world code:
 *
 *   hk_create / hk_destroy      one context per camera entity: owns what `ReservoirCache`
 *                               (light.rs:342-363), `LightTextures` (light.rs:297-383) and the
 *                               denoise part of `PostProcessTextures` (post_process.rs:622-747) own
 *   hk_scene_upload             the group-2 storage buffers written by
 *                               `MeshRenderAssets::set` (mesh.rs:43-58), `InstanceRenderAssets::set`
 *                               (instance.rs:82-99) and `MaterialRenderAssets` (material.rs:196-202)
 *   hk_texture_upload           the material textures of `MaterialTextures` (material.rs:54-127), bound
 *                               as group 3 `textures` / `samplers` (light.wgsl:15-19) when the
 *                               scene has textures (the reference's non-NO_TEXTURE pipeline)
 *   hk_set_noise                the 16 blue-noise textures of `NoiseTextures` (lib.rs:189-219)
 *   hk_resize                   `prepare_light_textures` reallocation (light.rs:307-383), which
 *                               zero-fills the 10 reservoir buffers (light.rs:353-360)
 *   hk_set_gbuffer              group-1 deferred textures produced by `PrepassNode` (prepass.rs:769-851)
 *   hk_render_gbuffer           primary-ray substitute for the raster prepass (prepass.wgsl:84-100)
 *   hk_render_frame             `LightNode::run` (light.rs:590-702): albedo, then per channel the
 *                               temporal pass and (if enabled) the spatial pass
 *   hk_denoise                  the denoise block of `PostProcessNode::run` (post_process.rs:1190-1224)
 *   hk_tone_sum                 the `tone_mapping` dispatch (post_process.rs:1226-1234)
 *   hk_get_output               reading `LightTextures` / `denoise_render` / tone-mapping output
 *   hk_trace                    stand-alone ray query over the TLAS/BLAS (light.wgsl:442-486)
 *
 * Conventions: every function returns 0 on success and a negative HK_ERR_* code on
 * failure; `hk_last_error` returns the message.  No exceptions cross the ABI.  A context
 * is externally synchronized (single-threaded, like one render-graph node).  `stream` is
 * a hipStream_t (NULL = the context's own stream); all GPU work is ordered on it and
 * the functions return without waiting, except hk_get_output(..., to_host=1) and
 * hk_read_counters.  Internally a frame's G-buffer and its tail (denoise, tone-sum) may run
 * on the context's own streams, overlapping the neighbouring frames' light passes; every
 * call that reads or changes their results first waits for them on `stream`
 * (hipStreamWaitEvent), so the observable order is the stream order.  A host-side
 * hipStreamSynchronize(stream) therefore does not cover them: use a readback call, or
 * hipDeviceSynchronize.
 */
#ifndef HIKARI_AMD_H
#define HIKARI_AMD_H

#include <stddef.h>
#include <stdint.h>
#include "hk_types.h"
#include "hk_texture.h"

#ifdef __cplusplus
extern "C" {
#endif

#define HK_ABI_VERSION 3

enum {
    HK_OK = 0,
    HK_ERR_INVALID = -1,   /* bad argument / shape */
    HK_ERR_HIP = -2,       /* HIP runtime failure */
    HK_ERR_STATE = -3,     /* called in the wrong order (e.g. render before upload) */
    HK_ERR_NO_DEVICE = -4, /* no gfx950 device */
};

typedef struct hk_ctx hk_ctx;

/* A {pointer, element count} array in a scene upload. */
typedef struct hk_array {
    const void* data;
    uint32_t count;
} hk_array;

/*
 * Scene buffers in group-2 binding order (mesh_material_bindings.wgsl:5-22).  The node
 * arrays carry their element count here (the WGSL `Nodes.count` header word).  The data is
 * COPIED: the caller keeps ownership.  A new upload replaces the whole scene.
 */
typedef struct hk_scene_desc {
    hk_array vertices;       /* hk_vertex,      binding 0 */
    hk_array primitives;     /* hk_primitive,   binding 1 */
    hk_array asset_nodes;    /* hk_node,        binding 2 */
    hk_array alias_table;    /* hk_alias_entry, binding 3 */
    hk_array instances;      /* hk_instance,    binding 4 */
    hk_array instance_nodes; /* hk_node,        binding 5 */
    hk_array materials;      /* hk_material,    binding 6 */
    hk_array emissive_nodes; /* hk_node,        binding 7 */
    hk_array emissives;      /* hk_emissive,    binding 8 */
} hk_scene_desc;

/*
 * Field-for-field mirror of `HikariSettings` (lib.rs:400-433); defaults in
 * hk_settings_default() follow lib.rs:435-455.
 */
typedef struct hk_settings {
    uint32_t direct_validate_interval;
    uint32_t emissive_validate_interval;
    uint32_t max_temporal_reuse_count;
    uint32_t max_spatial_reuse_count;
    float max_reservoir_lifetime;
    float solar_angle;
    uint32_t indirect_bounces;
    float max_indirect_luminance;
    float clear_color[4]; /* linear RGBA */
    uint32_t temporal_reuse;
    uint32_t emissive_spatial_reuse;
    uint32_t indirect_spatial_reuse;
    uint32_t denoise;
    uint32_t taa;           /* 0 = Jasmine, 1 = None (hk_post_process) */
    float upscale_ratio;    /* Upscale::ratio(), clamped to [1, 2] (lib.rs:501-505) */
    uint32_t upscale;       /* 0 = SmaaTu4x (default), 1 = Fsr1 (not provided: hk_post_process skips it) */
} hk_settings;

/* The parts of Bevy's `View` uniform the integrator reads (light.wgsl:714-727). */
typedef struct hk_view {
    float world_position[3];
    float _pad0;
    float view_proj[16];         /* column-major */
    float inverse_view_proj[16]; /* column-major, used by hk_render_gbuffer for ray generation */
    float projection[16];        /* column-major; projection[3].w == 1 => orthographic */
} hk_view;

/* The parts of Bevy's `Lights` uniform the integrator reads (light.wgsl:611,832,847,855). */
typedef struct hk_lights {
    float directional_color[4];     /* lights.directional_lights[0].color */
    float direction_to_light[3];    /* lights.directional_lights[0].direction_to_light */
    float _pad0;
    float ambient_color[4];         /* lights.ambient_color */
} hk_lights;

/* Prepass sub-pixel jitter (prepass.wgsl:30-38,52-54): the shader defs the prepass pipeline gets from
 * HikariSettings (prepass.rs:194-199) */
enum {
    HK_JITTER_NONE = 0, /* taa = None: no jitter */
    HK_JITTER_TAA = 1,  /* TEMPORAL_ANTI_ALIASING: halton index = frame_number & 15 */
    HK_JITTER_TAA_SMAA = 2, /* TEMPORAL_ANTI_ALIASING + SMAA_TU4X: index = (frame_number >> 1) & 15 */
};

/* Per-frame inputs: FrameUniform.number (view.rs:141-192) + view + lights, and the previous frame's
 * view (`PreviousViewUniform`, view.rs:31-73: projection * inverse(GlobalTransformQueue[1])) that the
 * prepass's motion vectors read (prepass.wgsl:96).  A zero-initialised tail (jitter 0,
 * has_previous_view 0) means no jitter and a static camera (previous view = this view). */
typedef struct hk_frame_inputs {
    uint32_t frame_number;
    uint32_t jitter;            /* HK_JITTER_*: hk_render_gbuffer's primary-ray jitter */
    uint32_t has_previous_view; /* 0: previous_view_proj is ignored and taken equal to view.view_proj */
    uint32_t _pad;
    hk_view view;
    hk_lights lights;
    float previous_view_proj[16]; /* column-major */
} hk_frame_inputs;

/* Output planes readable with hk_get_output. Sizes are per pixel of the plane's extent. */
typedef enum hk_output_id {
    HK_OUT_ALBEDO = 0,            /* RGBA16F, S (physical size)      */
    HK_OUT_VARIANCE_DIRECT = 1,   /* R32F, s                           */
    HK_OUT_VARIANCE_EMISSIVE = 2,
    HK_OUT_VARIANCE_INDIRECT = 3,
    HK_OUT_RENDER_DIRECT = 4,     /* RGBA16F, s                        */
    HK_OUT_RENDER_EMISSIVE = 5,
    HK_OUT_RENDER_INDIRECT = 6,
    HK_OUT_DENOISED_DIRECT = 7,   /* RGBA16F, s                        */
    HK_OUT_DENOISED_EMISSIVE = 8,
    HK_OUT_DENOISED_INDIRECT = 9,
    HK_OUT_TONE_MAPPED = 10,      /* RGBA16F, s                        */
    HK_OUT_GBUF_POSITION = 11,    /* float4, S */
    HK_OUT_GBUF_NORMAL = 12,      /* uint32 snorm8x4, S */
    HK_OUT_GBUF_DEPTH_GRADIENT = 13, /* float2, S */
    HK_OUT_GBUF_INSTANCE_MATERIAL = 14, /* float2, S */
    HK_OUT_GBUF_VELOCITY_UV = 15, /* float4, S */
    HK_OUT_DENOISE_INTERNAL_VARIANCE = 16, /* R32F, s (last channel denoised) */
    HK_OUT_ACCUMULATED = 17,      /* RGBA16F, s: hk_resolve_accumulation */
    HK_OUT_UPSCALED = 18,         /* RGBA16F, ceil(S * 2 / ratio): SMAA TU4x output (upscale_output[0]) */
    HK_OUT_TAA = 19,              /* RGBA16F: TAA Jasmine output of this frame (taa_output[head]) */
    HK_OUT_TONE_MAPPED_PREVIOUS = 20, /* RGBA16F, s: the previous frame's tone-mapped output (tone_mapping_output
                                       * [1 - head]), intact until this frame's successor's tone-sum */
    HK_OUT_COUNT = 21
} hk_output_id;

/* Reservoir buffer ids 0..9 as allocated by light.rs:350-361; the channel pairs
 * (temporal, spatial) are (0,4), (2,4), (6,8) + frame parity (light.rs:518-546). */
#define HK_RESERVOIR_BUFFERS 10

/* Per-frame device counters (ray queries issued; Mrays/s numerator). */
typedef struct hk_counters {
    uint64_t traverse_top;      /* traverse_top calls (light.wgsl:442) */
    uint64_t traverse_emitter;  /* emitter traverse_bottom calls in select_light_candidate (light.wgsl:687) */
    uint64_t primary;           /* primary rays of hk_render_gbuffer: one per pixel per frame */
    uint64_t primary_reused;    /* of those, the rays of frames whose planes were reused (option gbuffer_reuse), not traced */
} hk_counters;

/* ---- lifetime ---- */
int hk_abi_version(void);
/* Tuned configuration: the context creates its streams in a fixed order (caller
 * stream, two side streams — one carries no work, it only shifts the next ones — G-buffer stream,
 * tail stream), and HIP maps streams round-robin onto the process's hardware queues.  The defaults of
 * hk_set_option were measured with HIP's default GPU_MAX_HW_QUEUES=4; more queues let every stream
 * run concurrently and measured slower (cornell 1080p 0.58 -> 0.70 ms/frame). */
int hk_create(int device, hk_ctx** out_ctx);
void hk_destroy(hk_ctx* ctx);
const char* hk_last_error(const hk_ctx* ctx);
void hk_settings_default(hk_settings* out);

/* Runtime options of a context (no reference counterpart: the reference has one schedule).  Every
 * option chooses among schedules or kernel variants that produce the same bits, so results never
 * depend on them; the defaults are the measured-fastest configuration.  Nothing is read from the
 * environment.  Keys (default):
 *   pipeline_min_px (1.2e6)  frame pipelining from this many integrator pixels up
 *   pipeline_heavy_min_px (0)  ... and from this many up on frames with spatial reuse or the denoiser
 *   gbuffer_pipeline (1)     frame f's G-buffer on its own stream next to frame f-1's light passes
 *   tail_pipeline (1)        frame f's denoise / tone-sum / accumulation next to frame f+1's light passes
 *   channel_streams (1)      the indirect chain on a side stream next to direct -> emissive
 *   fuse (1), fuse_min_px (2^20)  direct_lit + emissive in one launch (identity reprojection only)
 *   merge (-1)               direct + indirect in one launch: -1 small unpipelined frames, 0 never, 1 always
 *   bg_elision (1)           skip background stores whose targets already hold their constant words
 *   spatial_view_planes (1)  the indirect temporal pass writes spatial reuse's neighbour view planes
 *   band_full_windows (0)    a band runs every pass on all its rows (no per-pass row windows)
 *   leaf_collapse (1)        leaf-collapsed node copies for the light walks (applied at the next upload)
 *   gbuffer_reuse (1)        skip the G-buffer trace when its slot already holds this frame's planes
 *                            (static camera, jitter and instances: the sub-frames of an accumulation)
 *   lds_scene (1)            0 no LDS scene staging, 1 where measured faster, 2 every traversal kernel
 *   gbuffer_stack_full (0), gbuffer_deep (0), gbuffer_lds_max_px (6e5: scene + stack in LDS on smaller
 *   frames), direct_w4_min_px (4e5), fused_w4 (1),
 *   persistent_indirect (0)  kernel-variant choices (tests force each variant with them)
 *   compact_emitter (0)      the fused direct/emissive launch runs a workgroup's emitter BLAS walks as one
 *                            compacted batch (long walks first) on frames without emissive validation
 *   compact_shadow (0)       shadow walks of a workgroup as one compacted batch (fused launch, indirect pass)
 *                            (both measured slower than the per-pixel walks: DESIGN §4)
 * hk_set_option returns HK_ERR_INVALID for an unknown key, a value outside the key's range, or a fractional value
 * for any key but the pixel-count thresholds (*_px). */
int hk_set_option(hk_ctx* ctx, const char* key, double value);
int hk_get_option(const hk_ctx* ctx, const char* key, double* value);
/* key of option `index` (0, 1, ...; NULL past the last one) */
const char* hk_option_name(int index);

/* ---- resources ---- */
int hk_scene_upload(hk_ctx* ctx, const hk_scene_desc* scene);
int hk_set_noise(hk_ctx* ctx, const uint8_t* rgba8, uint32_t count, uint32_t size);

/* Dynamic instances: `prepare_instances` (instance.rs:284-437) re-run ON THE GPU when
 * transforms change — instance records (world AABB from the 8 transformed corners of the local AABB,
 * inverse-transpose model), the TLAS (bvh 0.7.1 binned SAH, 6 buckets, rebuilt, not refitted),
 * emissive records with their alias tables, and the light BVH; bit-identical to a host rebuild
 * (hikari_scene.h hks_build) with the same transforms.  models: count x 16 floats
 * (GlobalTransform::compute_matrix, column-major); local_aabbs: count x 6 floats (the entity's
 * Bevy `Aabb`: center xyz, half_extents xyz).  count must equal the uploaded instance count
 * (same order, meshes and materials).  Waits for the stream once (singular-matrix check). */
int hk_update_instances(hk_ctx* ctx, const float* models, const float* local_aabbs, uint32_t count, void* stream);
/* copy group-2 scene array `array` (0..8, hk_scene_desc order) back from the device (test/debug) */
int hk_read_scene_array(hk_ctx* ctx, int array, void* dst, size_t bytes);

/* Post-process after tone mapping (post_process.rs:1236-1276): SMAA TU4x temporal 2x upsampling
 * (smaa.wgsl `smaa_tu4x` + `smaa_tu4x_extrapolate`, when settings->upscale == 0) then TAA Jasmine
 * (taa.wgsl, when settings->taa == 0).  Reads the previous frame's tone-mapped output and G-buffer
 * position / velocity planes (the reference's ping-pong textures, prepass.rs:309-317, head =
 * frame_number % 2).  Whole-frame contexts only. */
int hk_post_process(hk_ctx* ctx, const hk_settings* settings, const hk_frame_inputs* inputs, void* stream);

/* Sub-frame accumulation (N integrator sub-frames per displayed frame, each
 * exactly one reference frame): hk_accumulate adds the current tone-mapped output (HK_OUT_TONE_MAPPED)
 * to an f32 RGBA accumulator, restarting it when reset != 0; hk_resolve_accumulation writes
 * accumulator / count (RGBA16F) to HK_OUT_ACCUMULATED, the plane a displayed frame all-gathers. */
int hk_accumulate(hk_ctx* ctx, int reset, void* stream);
int hk_resolve_accumulation(hk_ctx* ctx, void* stream);

/* Material textures: hk_material.*_texture ids index this array (material.rs:78-86, U32_MAX =
 * none).  Each entry is a Bevy `GpuImage` level 0 (RGBA8, row-major, `width * height * 4`
 * bytes; base colour / emissive images are sRGB, metallic-roughness / occlusion linear) with its
 * `ImageSampler` (address mode per axis, magnification filter).  Sampling is defined in
 * include/hk_texture.h.  Copies the texels; re-upload replaces; count 0 removes all. */
typedef struct hk_texture {
    uint32_t width, height;
    uint32_t format;               /* HK_TEXTURE_RGBA8_SRGB / HK_TEXTURE_RGBA8_UNORM */
    uint32_t address_u, address_v; /* HK_ADDRESS_CLAMP_TO_EDGE / _REPEAT / _MIRROR_REPEAT */
    uint32_t filter;               /* HK_FILTER_NEAREST / HK_FILTER_LINEAR */
    const uint8_t* rgba8;
} hk_texture;
int hk_texture_upload(hk_ctx* ctx, const hk_texture* textures, uint32_t count);
/* physical size S = (width, height); integrator size s = ceil(S / ratio) (light.rs:318-319).
 * band_y0/band_rows select a horizontal band of the frame (multi-GPU); (0, height) = whole frame. */
int hk_resize(hk_ctx* ctx, uint32_t width, uint32_t height, float upscale_ratio,
              uint32_t band_y0, uint32_t band_rows);

/* Interleaved-stripe decomposition for N GPUs (no reference counterpart: the reference renders
 * on one device).  The context holds the 8-row stripes rank, rank + world, rank + 2 world, ... of a
 * width x height frame (upscale ratio 1.0), so every rank gets an equal share of every screen
 * region: balanced work where contiguous bands are not (cornell: the box fills the middle rows).
 * Only for frames without neighbour reads — spatial reuse and the denoiser return HK_ERR_STATE in
 * this mode; those use contiguous bands + halo (hk_resize with band rows).  Local row l holds
 * global row (l / 8 * world + rank) * 8 + l % 8; hk_band_info reports row0 = 0, rows = core_rows
 * = the local row count.  world == 1 is hk_resize of the whole frame. */
int hk_resize_striped(hk_ctx* ctx, uint32_t width, uint32_t height, uint32_t rank, uint32_t world);
/* rows of halo recomputed above and below a band by hk_resize (default 40, enough for spatial
 * reuse + 4 a-trous levels + the variance blur: 20 + 15 + 1); 0 is exact when spatial reuse and
 * denoise are both off.  Call before hk_resize. */
int hk_set_band_halo(hk_ctx* ctx, uint32_t rows);
/* 2-D tile decomposition for N GPUs (no reference counterpart; north_star: "frames tile-partition across the 8
 * GPUs"): the context renders the frame's columns [x0, x0 + cols) of rows [y0, y0 + rows) plus a halo of
 * hk_set_band_halo pixels on every side (upscale ratio 1.0).  The planes hold the band's rows (rows + halo) at full
 * width; every pass runs only on the columns and rows the later passes read (core +- its reach), so the core
 * rectangle is bit-identical to a whole-frame render for a static camera.  Each channel runs on its widest window
 * from the first frame, so settings changes need no refill (hk_band_window_grow lists nothing).  Ray counters count
 * the core rectangle only. */
int hk_resize_tile(hk_ctx* ctx, uint32_t width, uint32_t height, uint32_t x0, uint32_t cols, uint32_t y0,
                   uint32_t rows);
/* a tile's own columns (global); 0 and the frame width for row bands and whole frames */
int hk_tile_info(const hk_ctx* ctx, int32_t* col0, int32_t* cols);
/* band geometry after hk_resize: local rows [0, rows) hold global rows [row0, row0+rows);
 * the band's own (non-halo) rows are local [core_row0, core_row0+core_rows) */
int hk_band_info(const hk_ctx* ctx, int32_t* row0, int32_t* rows, int32_t* core_row0, int32_t* core_rows);
/* Band window refill (no reference counterpart: the reference renders one whole frame, whose temporal passes run
 * on every pixel whatever the spatial flags, light.rs:656-699).  A band runs each channel's light passes on its
 * core rows +- the margin `settings` needs (that channel's spatial range plus the denoiser's reach); a setting turned
 * on later widens the margin for good, and the rows it takes in hold records this band never computed.  Their
 * owner (the band whose core rows they are) holds them exactly.  For the next hk_render_frame with `settings`,
 * ranges[4 k + 0..3] = (frame row, rows) above the core and (frame row, rows) below it of reservoir buffer k's
 * records to take from the owners (rows 0 = none), k = 0..HK_RESERVOIR_BUFFERS-1; returns how many buffers need
 * any (< 0: error).  commit != 0 then widens the margins as hk_render_frame would, without zero-filling: call it
 * after loading the rows (hk_reservoir_rows).  Without a committed refill hk_render_frame zero-fills the new rows
 * (as hk_resize does, light.rs:355-358).  Call between frames: after the last frame's hk_render_frame (and this
 * frame's hk_render_gbuffer), on every band of the frame. */
int hk_band_window_grow(hk_ctx* ctx, const hk_settings* settings, int32_t* ranges, int commit);
/* The records of frame rows [frame_row0, frame_row0 + rows) of reservoir buffer `id`, which must lie in this
 * context's band: out of the context (store = 0) into `data`, or from `data` into it (store = 1).  `data` is host
 * memory or a device pointer of any device of the process, in the row-exchange layout: 4 x rows x width chunks of
 * 16 bytes (the context's four record chunks, each a plane of rows x width), the layout the same call of another
 * band's context reads and writes.  Ordered after the frame work queued so far; blocking. */
int hk_reservoir_rows(hk_ctx* ctx, int id, int32_t frame_row0, int32_t rows, void* data, int store, void* stream);

/* ---- per frame ---- */
/* Primary-ray G-buffer (prepass.wgsl:84-100).  Pixel (x, y) traces the ray through
 * (x + 0.5 - jx, y + 0.5 - jy), j = the frame's halton jitter in pixels (inputs->jitter), and writes
 * velocity = clip_to_uv(view_proj * model * p) - clip_to_uv(previous_view_proj * previous_model * p)
 * for the hit's object-space point p (prepass.wgsl:49-50,96).  previous_model is the instance's model
 * as of the previous hk_render_gbuffer call (GlobalTransformQueue, transform.rs:32-44; after
 * hk_scene_upload: the uploaded model), so instances moved by hk_update_instances get motion vectors
 * for one frame. */
int hk_render_gbuffer(hk_ctx* ctx, const hk_frame_inputs* inputs, void* stream);
/* plane: 0..4 = position, normal, depth_gradient, instance_material, velocity_uv
 * (full S-sized planes, or the band's rows); device_ptr != 0 => data is a device pointer */
int hk_set_gbuffer_plane(hk_ctx* ctx, int plane, const void* data, size_t bytes, int device_ptr,
                         void* stream);
int hk_render_frame(hk_ctx* ctx, const hk_settings* settings, const hk_frame_inputs* inputs,
                    void* stream);
int hk_denoise(hk_ctx* ctx, const hk_settings* settings, const hk_frame_inputs* inputs, void* stream);
int hk_tone_sum(hk_ctx* ctx, const hk_settings* settings, void* stream);

/* ---- readback / state ---- */
int hk_output_info(const hk_ctx* ctx, int output_id, uint32_t* width, uint32_t* height,
                   uint32_t* bytes_per_pixel);
/* rows [row0, row0+rows) of the plane (rows = 0 => all) */
int hk_get_output(hk_ctx* ctx, int output_id, void* dst, size_t bytes, int to_host, void* stream);
/* Device address of an output plane for zero-copy readers.  The planes of the G-buffer, render /
 * variance targets and albedo alternate between two slots from frame to frame, so the address is
 * valid for the current frame only; work on `stream` sees the plane's final contents after
 * hk_sync(ctx, stream) (the frame's G-buffer and tail may still run on the context's own streams).
 * The planes are read-only for the caller: the light passes skip background stores whose targets
 * already hold their constant words (background store elision), which a foreign write would break;
 * planes and reservoirs are written through hk_set_gbuffer_plane / hk_load_reservoirs only. */
const void* hk_output_device_ptr(hk_ctx* ctx, int output_id);
/* Make `stream` wait (device-side) for all work the context queued on its own streams. */
int hk_sync(hk_ctx* ctx, void* stream);
/* Integrator layout of the indirect pass (light.wgsl:1263-1498, one bounce): 0 = one thread per
 * pixel (default); 1 = wavefront with material-sorted shading (BASELINE configs[4]): live pixels
 * compacted into a queue, the bounce walk writes SoA hit records, the queue is grouped by the hit's
 * material and the shading / NEE / shadow / temporal tail runs in that order.  Same results. */
int hk_set_wavefront(hk_ctx* ctx, int enable);
/* copy band-local rows [row0, row0+rows) of an output plane (e.g. the band's core rows for the
 * multi-GPU all-gather); dst is host (to_host=1) or device memory.  On a stream other than the one
 * the frame sequence runs on (e.g. a communication stream), the copy waits only for the work that
 * produced the plane, device-side, and the context's next write of that plane waits for the copy: the
 * frame stream itself never waits for the copy or for what follows it on `stream`. */
int hk_copy_output_rows(hk_ctx* ctx, int output_id, uint32_t row0, uint32_t rows, void* dst, int to_host,
                        void* stream);
/* the same for the rectangle of band-local rows [row0, row0+rows) x columns [col0, col0+cols) (a tile's core rows and
 * columns), written with row pitch dst_pitch bytes (0: cols x bytes per pixel, packed) */
int hk_copy_output_rect(hk_ctx* ctx, int output_id, uint32_t row0, uint32_t rows, uint32_t col0, uint32_t cols,
                        void* dst, size_t dst_pitch, int to_host, void* stream);
/* copy reservoir buffer `id` (0..9) in the reference's AoS PackedReservoir layout */
int hk_dump_reservoirs(hk_ctx* ctx, int id, hk_packed_reservoir* dst, size_t count, void* stream);
int hk_load_reservoirs(hk_ctx* ctx, int id, const hk_packed_reservoir* src, size_t count, void* stream);
int hk_reset_counters(hk_ctx* ctx, void* stream);
int hk_read_counters(hk_ctx* ctx, hk_counters* out, void* stream);
/* mean duration (ms) of each kernel of the last hk_render_frame/hk_denoise call, if timing is enabled */
int hk_enable_kernel_timing(hk_ctx* ctx, int enable);
int hk_kernel_timing(hk_ctx* ctx, const char** names, float* ms, int capacity);
/* traverse_top lane statistics per kernel name since hk_create, in builds compiled with
 * -DHK_LANE_STATS (experiments; the product build returns 0 entries): per walk iteration the wave's
 * active lanes, so active / (64 x iterations) is the walk's SIMD lane efficiency */
int hk_lane_stats(hk_ctx* ctx, const char** names, unsigned long long* active, unsigned long long* iterations,
                  int capacity);
/* time only frames whose frame_number % every == 0 (default 1: every frame), so the timing
 * events of a long measured run do not perturb most of its frames */
int hk_set_kernel_timing_interval(hk_ctx* ctx, uint32_t every);

/* ---- stand-alone ray query (minimum slice: light.wgsl:442-486) ----
 * rays: n records of {origin xyz, direction xyz} (6 floats, host or device memory)
 * per ray: max_distance, early_distance, exclude_instance (arrays of n, may be NULL =>
 * closest-hit defaults F32_MAX, 0, 0xFFFFFFFF).
 * hits: n records of {u, v, distance (f32), instance_index, primitive_index (u32)}. */
int hk_trace(hk_ctx* ctx, const float* rays, const float* max_distance, const float* early_distance,
             const uint32_t* exclude_instance, uint32_t n, void* hits, int device_ptrs, void* stream);

/* ---- self-test of the device f16 conversion (pack2x16float, light.wgsl:173-216 pack_reservoir)
 * converts n host floats with the kernels' own conversion; out: n f16 bit patterns (host) */
int hk_selftest_f16(hk_ctx* ctx, const float* in, uint32_t n, uint16_t* out);
/* ---- self-test of the kernels' division by a frame dimension (div_by, hk_device.h): counts the
 * f32 bit patterns x in [lo, hi) (both signs) where div_by(x, divisor) != x / divisor */
int hk_selftest_div(hk_ctx* ctx, float divisor, uint32_t lo, uint32_t hi, uint64_t* mismatches);
/* ---- self-test of the kernels' reciprocal (rcp_exact, hk_device.h): counts the f32 bit patterns
 * x in [lo, hi) (both signs) where rcp_exact(x) != 1 / x (IEEE) */
int hk_selftest_rcp(hk_ctx* ctx, uint32_t lo, uint32_t hi, uint64_t* mismatches);

#ifdef __cplusplus
}
#endif

#endif /* HIKARI_AMD_H */
