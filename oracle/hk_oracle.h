/*
 * hk_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of bevy-hikari's per-pixel integrator and denoiser, used as the parity
 * checker for the HIP product path (libhikari_amd.so).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load liboracle.so; the product never links it.
 *
 * Parity status: the reference (WGSL under wgpu/Bevy 0.9.1) cannot be compiled or run in
 * this environment (no rustc/cargo, no WGSL compiler, no Vulkan ICD) and ships
 * no tests, golden vectors or fixtures.  The restatement is therefore pinned only by
 * independent known-answer tests of its building blocks (tests/test_oracle_kat.py: numpy
 * and pure-Python restatements of hash, f16/unorm/snorm packing, slab and triangle tests,
 * traversal, reservoir update, denoise weights) — full-frame parity with the reference
 * itself is UNPINNED.
 *
 * The oracle mirrors the WGSL structure: one function per entry point, stackless
 * skip-pointer traversal, AoS PackedReservoir buffers, textures as row-major planes.
 */
#ifndef HK_ORACLE_H
#define HK_ORACLE_H

#include <stdint.h>
#include "../include/hikari_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hko_ctx hko_ctx;

/* scene: as for hk_scene_upload; noise: 16 x 64 x 64 RGBA8; S = (width, height) */
hko_ctx* hko_create(const hk_scene_desc* scene, const uint8_t* noise, uint32_t width, uint32_t height,
                    float upscale_ratio, int threads);
void hko_destroy(hko_ctx* ctx);
/* SMAA TU4x + TAA Jasmine (hk_post_process) */
void hko_post_process(hko_ctx* ctx, const hk_settings* settings, const hk_frame_inputs* inputs);
/* material textures (hk_texture_upload) and a direct sampling entry for the KATs */
int hko_set_textures(hko_ctx* ctx, const hk_texture* textures, uint32_t count);
void hko_sample_texture(const hko_ctx* ctx, uint32_t id, const float* uv, uint32_t n, float* out);
/* restrict every pass to rows [y0 - halo, y0 + rows + halo) (multi-rank band tests; ratio 1) */
void hko_set_band(hko_ctx* ctx, int32_t y0, int32_t rows, int32_t halo);
void hko_set_tile(hko_ctx* ctx, int32_t x0, int32_t cols, int32_t y0, int32_t rows, int32_t halo);
/* compute only the rows of the 8-row stripes rank, rank + world, ... (hk_resize_striped; passes
 * without neighbour reads only) */
void hko_set_stripes(hko_ctx* ctx, int32_t rank, int32_t world);

/* replace the scene (e.g. after moving instances); the previous models of the motion vectors stay */
void hko_set_scene(hko_ctx* ctx, const hk_scene_desc* scene);
void hko_render_gbuffer(hko_ctx* ctx, const hk_frame_inputs* inputs);
void hko_render_frame(hko_ctx* ctx, const hk_settings* settings, const hk_frame_inputs* inputs);
void hko_denoise(hko_ctx* ctx, const hk_settings* settings, const hk_frame_inputs* inputs);
void hko_tone_sum(hko_ctx* ctx, const hk_settings* settings);

/* host pointer to an output plane (hk_output_id), NULL if unknown */
void* hko_output(hko_ctx* ctx, int output_id, uint32_t* width, uint32_t* height, uint32_t* bpp);
hk_packed_reservoir* hko_reservoirs(hko_ctx* ctx, int id, uint32_t* count);
void hko_counters(hko_ctx* ctx, hk_counters* out);
void hko_reset_counters(hko_ctx* ctx);
/* the closest-hit light walks: light.wgsl's order, the bounce walk with the ordered rule (as the HIP kernels), or
 * light.wgsl's order with every bounce and emitter walk also walked with the ordered rule and the differing rays
 * counted; stats = {bounce rays checked, differing, emitter walks checked, differing} */
enum { HKO_WALK_REFERENCE = 0, HKO_WALK_ORDERED = 1, HKO_WALK_CHECK = 2 };
void hko_set_light_walk(hko_ctx* ctx, int mode);
void hko_light_walk_stats(const hko_ctx* ctx, unsigned long long* stats);

/* light.wgsl:442-486 for n rays {origin, direction}; hits {u, v, t, instance, primitive} */
void hko_primary_hits(hko_ctx* ctx, const hk_frame_inputs* in, uint32_t* out);
void hko_trace(hko_ctx* ctx, const float* rays, const float* max_distance, const float* early_distance,
               const uint32_t* exclude_instance, uint32_t n, void* hits);
/* closest-hit rays with the ordered rule (closest_hit_ordered), hits as hko_trace */
void hko_trace_ordered(hko_ctx* ctx, const float* rays, uint32_t n, void* hits);

/* building blocks exposed for known-answer tests */
float hko_intersects_aabb(const float* origin, const float* inv_dir, const float* mn, const float* mx);
void hko_intersects_triangle(const float* origin, const float* dir, const float* v0, const float* v1,
                             const float* v2, float* out_uvt);
void hko_pack_reservoir_roundtrip(const float* fields, hk_packed_reservoir* packed, float* unpacked);
float hko_pow(float x, float y);
float hko_pow_int(float x, int n); /* n in {2, 5, 16} */
float hko_exp2(float x);
/* [exp2, log2, sincos]: inputs (every stride-th of the 2^32) where hk_math.h's branch-free forms differ from the
 * round-4 branchy ones */
void hko_math_form_mismatches(uint32_t stride, unsigned long long* out);
unsigned long long hko_exp_weight_mismatches(uint32_t stride);
float hko_log2(float x);
float hko_sin(float x);
float hko_cos(float x);
uint32_t hko_f32_to_f16(float x);
void hko_f32_to_f16_array(const float* in, size_t n, uint16_t* out);
uint32_t hko_hash(uint32_t x);

#ifdef __cplusplus
}
#endif

#endif
