// hk_post.hip — SMAA TU4x and TAA Jasmine kernels (smaa.wgsl, taa.wgsl; post_process.rs:1236-1276).
// The per-pixel bodies live in include/hk_post.h, shared verbatim with the CPU oracle.  These
// passes are HBM / L2 bound image filters: one thread per pixel, 16x16 tiles in the XCD-stripe
// order like the denoiser.
#include "hk_launch.h"

namespace hk {

HKD bool post_pixel(uint32_t w, uint32_t h, int32_t& x, int32_t& y)
{
    const uint32_t gx = gridDim.x, n = gridDim.x * gridDim.y;
    const uint32_t L = blockIdx.x + blockIdx.y * gx;
    const uint32_t xcd = L & 7u, i = L >> 3, q = n >> 3, r = n & 7u;
    const uint32_t tile = (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + i;
    x = (int32_t)((tile % gx) * 16u + (threadIdx.x & 15u));
    y = (int32_t)((tile / gx) * 16u + (threadIdx.x >> 4));
    return (uint32_t)x < w && (uint32_t)y < h;
}
static dim3 post_grid(uint32_t w, uint32_t h) { return dim3((w + 15u) / 16u, (h + 15u) / 16u); }

__global__ __launch_bounds__(256) void k_smaa_tu4x(PostArgs P)
{
    int32_t x, y;
    if (post_pixel(P.in.render.w, P.in.render.h, x, y)) hk_pp_smaa_tu4x(&P.frame, &P.in, x, y);
}
__global__ __launch_bounds__(256) void k_smaa_extrapolate(PostArgs P)
{
    int32_t x, y;
    if (post_pixel(P.in.render.w, P.in.render.h, x, y)) hk_pp_smaa_extrapolate(&P.in.output, x, y);
}
__global__ __launch_bounds__(256) void k_taa(PostArgs P)
{
    int32_t x, y;
    if (post_pixel(P.in.output.w, P.in.output.h, x, y)) hk_pp_taa(&P.frame, &P.in, x, y);
}

void launch_smaa(const PostArgs& P, hipStream_t st)
{
    hipLaunchKernelGGL(k_smaa_tu4x, post_grid(P.in.render.w, P.in.render.h), dim3(256), 0, st, P);
}
void launch_smaa_extrapolate(const PostArgs& P, hipStream_t st)
{
    hipLaunchKernelGGL(k_smaa_extrapolate, post_grid(P.in.render.w, P.in.render.h), dim3(256), 0, st, P);
}
void launch_taa(const PostArgs& P, hipStream_t st)
{
    hipLaunchKernelGGL(k_taa, post_grid(P.in.output.w, P.in.output.h), dim3(256), 0, st, P);
}

}  // namespace hk
