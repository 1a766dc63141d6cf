// hk_dynamic.hip — dynamic instances on the device.
//
// The reference re-runs `prepare_instances` on the CPU whenever a transform changes
// (instance.rs:284-437: instance records with world AABBs and inverse-transpose models, the
// TLAS built with bvh 0.7.1, emissive records with alias tables, the light BVH).  This file
// re-runs that whole derivation on the GPU from the new model matrices, with exactly the float
// (and, for the inverse, double) operations of the host builder (csrc/hk_scene.cpp), so the
// buffers are bit-identical to a host rebuild — the TLAS topology included, which the
// reference-order traversal depends on.
//
// BVH build (bvh 0.7.1 restatement, as hk_scene.cpp): every split is computed by one thread
// with the host's sequential algorithm; the segments of one tree level are split in parallel by
// the threads of one workgroup (one barrier per level).  A subtree of k shapes flattens to
// exactly 3k - 2 nodes, so each segment knows its output range without the rest of the tree.
#include "hk_device.h"
#include "hk_launch.h"

namespace hk {

struct BBox {
    float mn[3], mx[3];
};
HKD BBox bbox_empty()
{
    const float inf = __uint_as_float(0x7F800000u);
    return BBox{{inf, inf, inf}, {-inf, -inf, -inf}};
}
HKD void bbox_join(BBox& a, const BBox& b)
{
    for (int k = 0; k < 3; ++k) {
        a.mn[k] = fminf(a.mn[k], b.mn[k]);
        a.mx[k] = fmaxf(a.mx[k], b.mx[k]);
    }
}
HKD void bbox_grow(BBox& a, const float* p)
{
    for (int k = 0; k < 3; ++k) {
        a.mn[k] = fminf(a.mn[k], p[k]);
        a.mx[k] = fmaxf(a.mx[k], p[k]);
    }
}
HKD float bbox_center(const BBox& b, int k) { return (b.mn[k] + b.mx[k]) * 0.5f; }
HKD float bbox_area(const BBox& b)
{
    const float x = b.mx[0] - b.mn[0], y = b.mx[1] - b.mn[1], z = b.mx[2] - b.mn[2];
    return 2.0f * ((x * y + x * z) + y * z);
}
HKD int bbox_largest_axis(const BBox& b)
{
    const float x = b.mx[0] - b.mn[0], y = b.mx[1] - b.mn[1], z = b.mx[2] - b.mn[2];
    if (x > y && x > z) return 0;
    if (y > z) return 1;
    return 2;
}
HKD hk_node pack_node(const BBox& a, uint32_t entry, uint32_t exit)
{
    hk_node n;
    for (int k = 0; k < 3; ++k) {
        n.min[k] = a.mn[k];
        n.max[k] = a.mx[k];
    }
    n.entry_index = entry;
    n.exit_index = exit;
    return n;
}
HKD uint32_t flat_size(uint32_t k) { return 3u * k - 2u; }

struct Segment {
    uint32_t start, count, out;
};

constexpr int BVH_BUCKETS_MAX = 16;

// Split one segment (host BvhBuilder::build for one node) and write its two box nodes; returns
// the child segments (count 0 = none).  src/dst: the index buffers of this level / the next.
HKD void split_segment(const BBox* shapes, const uint32_t* src, uint32_t* dst, Segment s, int nb, hk_node* flat,
                       Segment& left, Segment& right)
{
    left.count = right.count = 0;
    if (s.count == 1) {
        flat[s.out] = pack_node(bbox_empty(), src[s.start] | HK_BVH_LEAF_FLAG, s.out + 1u);
        return;
    }
    BBox centroid = bbox_empty(), bounds = bbox_empty();
    for (uint32_t i = 0; i < s.count; ++i) {
        const BBox& b = shapes[src[s.start + i]];
        float c[3] = {bbox_center(b, 0), bbox_center(b, 1), bbox_center(b, 2)};
        bbox_grow(centroid, c);
        bbox_join(bounds, b);
    }
    const int axis = bbox_largest_axis(centroid);
    const float axis_size = centroid.mx[axis] - centroid.mn[axis];
    uint32_t nl = 0;
    bool halves = axis_size < HK_F32_EPSILON;
    if (!halves) {
        uint32_t bucket_n[BVH_BUCKETS_MAX];
        BBox bucket_box[BVH_BUCKETS_MAX];
        for (int b = 0; b < nb; ++b) {
            bucket_n[b] = 0;
            bucket_box[b] = bbox_empty();
        }
        auto bucket_of = [&](const BBox& b) {
            const float rel = (bbox_center(b, axis) - centroid.mn[axis]) / axis_size;
            int k = (int)(rel * ((float)nb - 0.01f));
            return k < 0 ? 0 : (k > nb - 1 ? nb - 1 : k);
        };
        for (uint32_t i = 0; i < s.count; ++i) {
            const BBox& b = shapes[src[s.start + i]];
            const int k = bucket_of(b);
            bucket_n[k]++;
            bbox_join(bucket_box[k], b);
        }
        int best = 0;
        float best_cost = __uint_as_float(0x7F800000u);
        for (int sp = 0; sp < nb - 1; ++sp) {
            BBox la = bbox_empty(), ra = bbox_empty();
            uint32_t ln = 0, rn = 0;
            for (int b = 0; b <= sp; ++b) {
                bbox_join(la, bucket_box[b]);
                ln += bucket_n[b];
            }
            for (int b = sp + 1; b < nb; ++b) {
                bbox_join(ra, bucket_box[b]);
                rn += bucket_n[b];
            }
            if (ln == 0 || rn == 0) continue;
            const float cost = ((float)ln * bbox_area(la) + (float)rn * bbox_area(ra)) / bbox_area(bounds);
            if (cost < best_cost) {
                best_cost = cost;
                best = sp;
            }
        }
        for (int b = 0; b <= best; ++b) nl += bucket_n[b];
        if (nl == 0 || nl == s.count) {
            halves = true;  // degenerate (NaN areas): halves, as the host
        } else {
            // children = buckets in bucket order, each in the parent's order (a stable sort by bucket)
            uint32_t at[BVH_BUCKETS_MAX];
            uint32_t run = 0;
            for (int b = 0; b < nb; ++b) {
                at[b] = run;
                run += bucket_n[b];
            }
            for (uint32_t i = 0; i < s.count; ++i) {
                const uint32_t id = src[s.start + i];
                dst[s.start + at[bucket_of(shapes[id])]++] = id;
            }
        }
    }
    if (halves) {
        nl = s.count / 2u;
        for (uint32_t i = 0; i < s.count; ++i) dst[s.start + i] = src[s.start + i];
    }
    const uint32_t nr = s.count - nl;
    BBox la = bbox_empty(), ra = bbox_empty();
    for (uint32_t i = 0; i < nl; ++i) bbox_join(la, shapes[dst[s.start + i]]);
    for (uint32_t i = nl; i < s.count; ++i) bbox_join(ra, shapes[dst[s.start + i]]);
    const uint32_t q = s.out + 1u + flat_size(nl);  // box node of the right child
    flat[s.out] = pack_node(la, s.out + 1u, q);
    flat[q] = pack_node(ra, q + 1u, q + 1u + flat_size(nr));
    left = Segment{s.start, nl, s.out + 1u};
    right = Segment{s.start + nl, nr, q + 1u};
}

// ---- cooperative split: the same decisions as split_segment, by all 256 threads of the block.
// min/max reductions are exact in any order; the children are a stable sort by bucket, ranked
// with wave ballots chunk by chunk.
constexpr uint32_t COOP_MIN = 128;  // segments larger than this are split cooperatively
constexpr int COOP_BUCKETS = 6;     // bvh 0.7.1 NUM_BUCKETS
struct CoopShared {
    float red[4][48];
    float f[48];
    uint32_t wave_n[4][COOP_BUCKETS];
    uint32_t cursor[COOP_BUCKETS];
    uint32_t u[4];
};
// reduce v[0..k) over the block: op 0 = min, 1 = max, 2 = sum (integer-valued floats)
template <int K>
HKD void block_reduce(float* v, const int* op, CoopShared& sh)
{
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k)
        for (int o = 32; o > 0; o >>= 1) {
            const float x = __shfl_xor(v[k], o, 64);
            v[k] = op[k] == 0 ? fminf(v[k], x) : (op[k] == 1 ? fmaxf(v[k], x) : v[k] + x);
        }
    if (lane == 0)
        for (int k = 0; k < K; ++k) sh.red[w][k] = v[k];
    __syncthreads();
    if (threadIdx.x < (uint32_t)K) {
        const int k = (int)threadIdx.x;
        float r = sh.red[0][k];
        for (int j = 1; j < 4; ++j) r = op[k] == 0 ? fminf(r, sh.red[j][k]) : (op[k] == 1 ? fmaxf(r, sh.red[j][k]) : r + sh.red[j][k]);
        sh.f[k] = r;
    }
    __syncthreads();
    for (int k = 0; k < K; ++k) v[k] = sh.f[k];
    __syncthreads();
}
HKD int coop_bucket(const BBox& b, int axis, float cmin, float axis_size)
{
    const float rel = (bbox_center(b, axis) - cmin) / axis_size;
    int k = (int)(rel * ((float)COOP_BUCKETS - 0.01f));
    return k < 0 ? 0 : (k > COOP_BUCKETS - 1 ? COOP_BUCKETS - 1 : k);
}
HKD void coop_split(const BBox* shapes, const uint32_t* src, uint32_t* dst, Segment s, hk_node* flat, CoopShared& sh,
                    Segment& left, Segment& right)
{
    const float inf = __uint_as_float(0x7F800000u);
    // centroid bounds + bounds
    {
        float v[12];
        int op[12];
        for (int k = 0; k < 3; ++k) {
            v[k] = inf, v[3 + k] = -inf, v[6 + k] = inf, v[9 + k] = -inf;
            op[k] = 0, op[3 + k] = 1, op[6 + k] = 0, op[9 + k] = 1;
        }
        for (uint32_t i = threadIdx.x; i < s.count; i += 256u) {
            const BBox& b = shapes[src[s.start + i]];
            for (int k = 0; k < 3; ++k) {
                const float c = bbox_center(b, k);
                v[k] = fminf(v[k], c), v[3 + k] = fmaxf(v[3 + k], c);
                v[6 + k] = fminf(v[6 + k], b.mn[k]), v[9 + k] = fmaxf(v[9 + k], b.mx[k]);
            }
        }
        block_reduce<12>(v, op, sh);
        BBox centroid{{v[0], v[1], v[2]}, {v[3], v[4], v[5]}};
        BBox bounds{{v[6], v[7], v[8]}, {v[9], v[10], v[11]}};
        const int axis = bbox_largest_axis(centroid);
        const float axis_size = centroid.mx[axis] - centroid.mn[axis];
        const float cmin = centroid.mn[axis];
        bool halves = axis_size < HK_F32_EPSILON;
        uint32_t nl = 0;
        if (!halves) {
            // per-bucket counts and boxes
            float bv[COOP_BUCKETS * 7];
            int bop[COOP_BUCKETS * 7];
            for (int b = 0; b < COOP_BUCKETS; ++b) {
                bv[7 * b] = 0.0f, bop[7 * b] = 2;
                for (int k = 0; k < 3; ++k) {
                    bv[7 * b + 1 + k] = inf, bop[7 * b + 1 + k] = 0;
                    bv[7 * b + 4 + k] = -inf, bop[7 * b + 4 + k] = 1;
                }
            }
            for (uint32_t i = threadIdx.x; i < s.count; i += 256u) {
                const BBox& bb = shapes[src[s.start + i]];
                const int b = coop_bucket(bb, axis, cmin, axis_size);
#pragma unroll
                for (int q = 0; q < COOP_BUCKETS; ++q)
                    if (q == b) {
                        bv[7 * q] += 1.0f;
                        for (int k = 0; k < 3; ++k) {
                            bv[7 * q + 1 + k] = fminf(bv[7 * q + 1 + k], bb.mn[k]);
                            bv[7 * q + 4 + k] = fmaxf(bv[7 * q + 4 + k], bb.mx[k]);
                        }
                    }
            }
            block_reduce<COOP_BUCKETS * 7>(bv, bop, sh);
            uint32_t bucket_n[COOP_BUCKETS];
            BBox bucket_box[COOP_BUCKETS];
            for (int b = 0; b < COOP_BUCKETS; ++b) {
                bucket_n[b] = (uint32_t)bv[7 * b];
                bucket_box[b] = BBox{{bv[7 * b + 1], bv[7 * b + 2], bv[7 * b + 3]}, {bv[7 * b + 4], bv[7 * b + 5], bv[7 * b + 6]}};
            }
            int best = 0;
            float best_cost = inf;
            for (int sp = 0; sp < COOP_BUCKETS - 1; ++sp) {
                BBox la = bbox_empty(), ra = bbox_empty();
                uint32_t ln = 0, rn = 0;
                for (int b = 0; b <= sp; ++b) {
                    bbox_join(la, bucket_box[b]);
                    ln += bucket_n[b];
                }
                for (int b = sp + 1; b < COOP_BUCKETS; ++b) {
                    bbox_join(ra, bucket_box[b]);
                    rn += bucket_n[b];
                }
                if (ln == 0 || rn == 0) continue;
                const float cost = ((float)ln * bbox_area(la) + (float)rn * bbox_area(ra)) / bbox_area(bounds);
                if (cost < best_cost) {
                    best_cost = cost;
                    best = sp;
                }
            }
            for (int b = 0; b <= best; ++b) nl += bucket_n[b];
            if (nl == 0 || nl == s.count) {
                halves = true;
            } else {
                // stable sort by bucket: cursor[b] = start of bucket b, ranks by wave ballots
                if (threadIdx.x == 0) {
                    uint32_t run = 0;
                    for (int b = 0; b < COOP_BUCKETS; ++b) {
                        sh.cursor[b] = run;
                        run += bucket_n[b];
                    }
                }
                __syncthreads();
                const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
                for (uint32_t base = 0; base < s.count; base += 256u) {
                    const uint32_t i = base + threadIdx.x;
                    const bool valid = i < s.count;
                    const uint32_t id = valid ? src[s.start + i] : 0u;
                    const int b = valid ? coop_bucket(shapes[id], axis, cmin, axis_size) : -1;
                    unsigned long long mine = 0;
#pragma unroll
                    for (int q = 0; q < COOP_BUCKETS; ++q) {
                        const unsigned long long m = __ballot(b == q);
                        if (b == q) mine = m;
                        if (lane == 0) sh.wave_n[w][q] = (uint32_t)__popcll(m);
                    }
                    __syncthreads();
                    if (valid) {
                        uint32_t off = sh.cursor[b];
                        for (uint32_t j = 0; j < w; ++j) off += sh.wave_n[j][b];
                        off += (uint32_t)__popcll(mine & ((1ull << lane) - 1ull));
                        dst[s.start + off] = id;
                    }
                    __syncthreads();
                    if (threadIdx.x < (uint32_t)COOP_BUCKETS)
                        sh.cursor[threadIdx.x] += sh.wave_n[0][threadIdx.x] + sh.wave_n[1][threadIdx.x] +
                                                  sh.wave_n[2][threadIdx.x] + sh.wave_n[3][threadIdx.x];
                    __syncthreads();
                }
            }
        }
        if (halves) {
            nl = s.count / 2u;
            for (uint32_t i = threadIdx.x; i < s.count; i += 256u) dst[s.start + i] = src[s.start + i];
            __syncthreads();
        }
        // children boxes
        float c[12];
        int cop[12];
        for (int k = 0; k < 3; ++k) {
            c[k] = inf, c[3 + k] = -inf, c[6 + k] = inf, c[9 + k] = -inf;
            cop[k] = 0, cop[3 + k] = 1, cop[6 + k] = 0, cop[9 + k] = 1;
        }
        for (uint32_t i = threadIdx.x; i < s.count; i += 256u) {
            const BBox& b = shapes[dst[s.start + i]];
            const int o = i < nl ? 0 : 6;
            for (int k = 0; k < 3; ++k) c[o + k] = fminf(c[o + k], b.mn[k]), c[o + 3 + k] = fmaxf(c[o + 3 + k], b.mx[k]);
        }
        block_reduce<12>(c, cop, sh);
        const uint32_t nr = s.count - nl;
        const uint32_t q = s.out + 1u + flat_size(nl);
        if (threadIdx.x == 0) {
            flat[s.out] = pack_node(BBox{{c[0], c[1], c[2]}, {c[3], c[4], c[5]}}, s.out + 1u, q);
            flat[q] = pack_node(BBox{{c[6], c[7], c[8]}, {c[9], c[10], c[11]}}, q + 1u, q + 1u + flat_size(nr));
        }
        left = Segment{s.start, nl, s.out + 1u};
        right = Segment{s.start + nl, nr, q + 1u};
    }
}

// One workgroup builds one flattened BVH over `n` shapes (n >= 1).  Segments of one tree level
// larger than COOP_MIN are split one after another by the whole block (coop_split), the others
// in parallel, one per thread (split_segment); one barrier per level.  idx: 2n scratch indices,
// seg: 2 x n scratch segments.  When the shapes and both index buffers fit BVH_LDS_SHAPES they
// are staged in LDS.  *levels: the number of tree levels that split (max inner nodes on a path).
constexpr uint32_t BVH_LDS_SHAPES = 1280;  // 1280 x (24 + 8) B = 40 KiB
constexpr uint32_t BIG_MAX = 64;           // big segments per level (<= n / COOP_MIN)
template <bool LDS>
__global__ __launch_bounds__(256) void k_build_bvh(const BBox* g_shapes, uint32_t n, int buckets, hk_node* flat,
                                                   uint32_t* g_idx, Segment* seg, uint32_t* levels)
{
    __shared__ uint32_t n_small, n_small_next, n_big, n_big_next;
    __shared__ Segment big[2][BIG_MAX];
    __shared__ CoopShared sh;
    __shared__ BBox s_shapes[LDS ? BVH_LDS_SHAPES : 1];
    __shared__ uint32_t s_idx[LDS ? 2 * BVH_LDS_SHAPES : 1];
    if (n == 0) return;
    const BBox* shapes = g_shapes;
    uint32_t* idx = g_idx;
    if (LDS) {
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) s_shapes[i] = g_shapes[i];
        shapes = s_shapes;
        idx = s_idx;
    }
    const bool coop = buckets == COOP_BUCKETS;
    uint32_t* buf[2] = {idx, idx + n};
    Segment* segs[2] = {seg, seg + n};
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) buf[0][i] = i;
    if (threadIdx.x == 0) {
        n_small = n_big = n_small_next = n_big_next = 0;
        const Segment root{0u, n, 0u};
        if (coop && n > COOP_MIN) big[0][n_big++] = root;
        else segs[0][n_small++] = root;
    }
    __syncthreads();
    uint32_t split_levels = 0;
    auto push = [&](int p, const Segment& l, const Segment& r) {  // children of a level-p split
        for (const Segment* c : {&l, &r}) {
            // only thread 0 pushes big segments (from coop_split), so the bound check is race-free
            if (coop && c->count > COOP_MIN && n_big_next < BIG_MAX) {
                uint32_t k = atomicAdd(&n_big_next, 1u);
                big[p ^ 1][k] = *c;
            } else {
                uint32_t k = atomicAdd(&n_small_next, 1u);
                segs[p ^ 1][k] = *c;
            }
        }
    };
    for (int level = 0;; ++level) {
        const int p = level & 1;
        const uint32_t nb_ = n_big, ns = n_small;
        if (nb_ + ns == 0) break;
        for (uint32_t i = 0; i < nb_; ++i) {
            Segment l, r;
            coop_split(shapes, buf[p], buf[p ^ 1], big[p][i], flat, sh, l, r);
            if (threadIdx.x == 0) push(p, l, r);
        }
        for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) {
            Segment l, r;
            split_segment(shapes, buf[p], buf[p ^ 1], segs[p][i], buckets, flat, l, r);
            if (l.count) push(p, l, r);
        }
        __syncthreads();
        if (n_small_next + n_big_next) split_levels = level + 1;
        __syncthreads();
        if (threadIdx.x == 0) {
            n_big = n_big_next;
            n_small = n_small_next;
            n_big_next = n_small_next = 0;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0 && levels) *levels = split_levels;
}

// ---- instance records (instance.rs:284-330; hk_scene.cpp hks_build "instances")
HKD void transform_point(const float* m, const float* p, float* o)
{
    for (int r = 0; r < 3; ++r) o[r] = ((m[r] * p[0] + m[4 + r] * p[1]) + m[8 + r] * p[2]) + m[12 + r];
}
HKD void transform_vector(const float* m, const float* p, float* o)
{
    for (int r = 0; r < 3; ++r) o[r] = (m[r] * p[0] + m[4 + r] * p[1]) + m[8 + r] * p[2];
}
HKD bool inverse_transpose_d(const float* m, float* out)
{
    double a[16], inv[16];
    for (int i = 0; i < 16; ++i) a[i] = m[i];
    inv[0] = a[5] * a[10] * a[15] - a[5] * a[11] * a[14] - a[9] * a[6] * a[15] + a[9] * a[7] * a[14] +
             a[13] * a[6] * a[11] - a[13] * a[7] * a[10];
    inv[4] = -a[4] * a[10] * a[15] + a[4] * a[11] * a[14] + a[8] * a[6] * a[15] - a[8] * a[7] * a[14] -
             a[12] * a[6] * a[11] + a[12] * a[7] * a[10];
    inv[8] = a[4] * a[9] * a[15] - a[4] * a[11] * a[13] - a[8] * a[5] * a[15] + a[8] * a[7] * a[13] +
             a[12] * a[5] * a[11] - a[12] * a[7] * a[9];
    inv[12] = -a[4] * a[9] * a[14] + a[4] * a[10] * a[13] + a[8] * a[5] * a[14] - a[8] * a[6] * a[13] -
              a[12] * a[5] * a[10] + a[12] * a[6] * a[9];
    inv[1] = -a[1] * a[10] * a[15] + a[1] * a[11] * a[14] + a[9] * a[2] * a[15] - a[9] * a[3] * a[14] -
             a[13] * a[2] * a[11] + a[13] * a[3] * a[10];
    inv[5] = a[0] * a[10] * a[15] - a[0] * a[11] * a[14] - a[8] * a[2] * a[15] + a[8] * a[3] * a[14] +
             a[12] * a[2] * a[11] - a[12] * a[3] * a[10];
    inv[9] = -a[0] * a[9] * a[15] + a[0] * a[11] * a[13] + a[8] * a[1] * a[15] - a[8] * a[3] * a[13] -
             a[12] * a[1] * a[11] + a[12] * a[3] * a[9];
    inv[13] = a[0] * a[9] * a[14] - a[0] * a[10] * a[13] - a[8] * a[1] * a[14] + a[8] * a[2] * a[13] +
              a[12] * a[1] * a[10] - a[12] * a[2] * a[9];
    inv[2] = a[1] * a[6] * a[15] - a[1] * a[7] * a[14] - a[5] * a[2] * a[15] + a[5] * a[3] * a[14] +
             a[13] * a[2] * a[7] - a[13] * a[3] * a[6];
    inv[6] = -a[0] * a[6] * a[15] + a[0] * a[7] * a[14] + a[4] * a[2] * a[15] - a[4] * a[3] * a[14] -
             a[12] * a[2] * a[7] + a[12] * a[3] * a[6];
    inv[10] = a[0] * a[5] * a[15] - a[0] * a[7] * a[13] - a[4] * a[1] * a[15] + a[4] * a[3] * a[13] +
              a[12] * a[1] * a[7] - a[12] * a[3] * a[5];
    inv[14] = -a[0] * a[5] * a[14] + a[0] * a[6] * a[13] + a[4] * a[1] * a[14] - a[4] * a[2] * a[13] -
              a[12] * a[1] * a[6] + a[12] * a[2] * a[5];
    inv[3] = -a[1] * a[6] * a[11] + a[1] * a[7] * a[10] + a[5] * a[2] * a[11] - a[5] * a[3] * a[10] -
             a[9] * a[2] * a[7] + a[9] * a[3] * a[6];
    inv[7] = a[0] * a[6] * a[11] - a[0] * a[7] * a[10] - a[4] * a[2] * a[11] + a[4] * a[3] * a[10] +
             a[8] * a[2] * a[7] - a[8] * a[3] * a[6];
    inv[11] = -a[0] * a[5] * a[11] + a[0] * a[7] * a[9] + a[4] * a[1] * a[11] - a[4] * a[3] * a[9] -
              a[8] * a[1] * a[7] + a[8] * a[3] * a[5];
    inv[15] = a[0] * a[5] * a[10] - a[0] * a[6] * a[9] - a[4] * a[1] * a[10] + a[4] * a[2] * a[9] +
              a[8] * a[1] * a[6] - a[8] * a[2] * a[5];
    const double det = a[0] * inv[0] + a[1] * inv[4] + a[2] * inv[8] + a[3] * inv[12];
    if (det == 0.0) return false;
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) out[c * 4 + r] = (float)(inv[r * 4 + c] / det);
    return true;
}

__global__ __launch_bounds__(256) void k_update_instances(hk_instance* inst, uint32_t n, const float* models,
                                                          const float* local_aabbs, BBox* boxes, uint32_t* singular)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    hk_instance& g = inst[i];
    const float* m = models + 16u * i;
    const float* center = local_aabbs + 6u * i;
    const float* half = center + 3;
    float c[3];
    transform_point(m, center, c);
    float mn[3] = {0.0f, 0.0f, 0.0f}, mx[3] = {0.0f, 0.0f, 0.0f};
    for (int k = 0; k < 8; ++k) {
        const float sx = (float)(2 * (k & 1) - 1), sy = (float)(2 * ((k >> 1) & 1) - 1), sz = (float)(2 * ((k >> 2) & 1) - 1);
        const float v[3] = {half[0] * sx, half[1] * sy, half[2] * sz};
        float corner[3];
        transform_vector(m, v, corner);
        for (int d = 0; d < 3; ++d) {
            mn[d] = fminf(mn[d], corner[d]);
            mx[d] = fmaxf(mx[d], corner[d]);
        }
    }
    BBox b;
    for (int d = 0; d < 3; ++d) {
        g.min[d] = b.mn[d] = mn[d] + c[d];
        g.max[d] = b.mx[d] = mx[d] + c[d];
    }
    for (int k = 0; k < 16; ++k) g.model[k] = m[k];
    if (!inverse_transpose_d(m, g.inverse_transpose_model)) atomicOr(singular, 1u);
    boxes[i] = b;
}

// ---- emissive records + alias tables (instance.rs:377-420, mod.rs:318-376)
struct AliasWork {
    uint32_t index;
    float prob;
};
// transformed_primitive_areas (mod.rs:318-328): one thread per (emitter, primitive) = alias entry
__global__ __launch_bounds__(256) void k_emissive_areas(const hk_emissive* em, uint32_t n_em, const hk_instance* inst,
                                                        const hk_primitive* prims, uint32_t n_alias, float* areas)
{
    const uint32_t a = blockIdx.x * 256u + threadIdx.x;
    if (a >= n_alias) return;
    uint32_t lo = 0, hi = n_em;  // the emitter whose alias range holds a (offsets ascend)
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (em[mid].alias_table[0] <= a) lo = mid;
        else hi = mid;
    }
    const hk_emissive& r = em[lo];
    if (a < r.alias_table[0] || a >= r.alias_table[0] + r.alias_table[1]) return;
    const hk_instance& in = inst[r.instance];
    const hk_primitive& pr = prims[in.mesh.primitive + (a - r.alias_table[0])];
    float w[3][3];
    for (int k = 0; k < 3; ++k) transform_point(in.model, pr.vertices[k].position, w[k]);
    const float ux = w[1][0] - w[0][0], uy = w[1][1] - w[0][1], uz = w[1][2] - w[0][2];
    const float vx = w[2][0] - w[0][0], vy = w[2][1] - w[0][1], vz = w[2][2] - w[0][2];
    // hk_scene.cpp cross(): (a.y b.z - b.y a.z, a.z b.x - b.z a.x, a.x b.y - b.x a.y)
    const float cx = uy * vz - vy * uz, cy = uz * vx - vz * ux, cz = ux * vy - vx * uy;
    areas[a] = 0.5f * fabsf(sqrtf((cx * cx + cy * cy) + cz * cz));
}

// One wave per emitter: the host's sequential surface-area sum (lane 0), the over / under lists
// by wave-ballot compaction (index order, as the host's two passes), then the alias while-loop
// on lane 0 with the stacks in LDS (global scratch beyond ALIAS_LDS entries).
constexpr uint32_t ALIAS_LDS = 3072;
__global__ __launch_bounds__(64) void k_update_emissives(hk_emissive* em, uint32_t n_em, const hk_instance* inst,
                                                         const hk_material* mats, hk_alias_entry* alias,
                                                         const float* areas, AliasWork* work, BBox* boxes)
{
    __shared__ AliasWork s_over[ALIAS_LDS], s_under[ALIAS_LDS];
    __shared__ float s_sum;
    const uint32_t e = blockIdx.x;
    if (e >= n_em) return;
    const uint32_t lane = threadIdx.x;
    hk_emissive& r = em[e];
    const hk_instance& in = inst[r.instance];
    const hk_material& mat = mats[in.material];
    const uint32_t off = r.alias_table[0], count = r.alias_table[1];
    const float* a = areas + off;  // k_emissive_areas
    if (lane == 0) {
        float sum = 0.0f;
        for (uint32_t p = 0; p < count; ++p) sum += a[p];  // the host's summation order
        s_sum = sum;
    }
    hk_alias_entry* t = alias + off;
    for (uint32_t i = lane; i < count; i += 64u) t[i] = hk_alias_entry{0.0f, i};
    __syncthreads();
    const float surface_area = s_sum;
    const float mean_area = surface_area / (float)count;
    const bool in_lds = count <= ALIAS_LDS;
    AliasWork* over = in_lds ? s_over : work + 2u * off;
    AliasWork* under = in_lds ? s_under : work + 2u * off + count;
    uint32_t n_over = 0, n_under = 0;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (uint32_t base = 0; base < count; base += 64u) {
        const uint32_t i = base + lane;
        const float prob = i < count ? a[i] / mean_area : 1.0f;
        const bool o = prob > 1.0f, u = prob < 1.0f;
        const unsigned long long mo = __ballot(o), mu = __ballot(u);
        if (o) over[n_over + (uint32_t)__popcll(mo & lt)] = AliasWork{i, prob};
        if (u) under[n_under + (uint32_t)__popcll(mu & lt)] = AliasWork{i, prob};
        n_over += (uint32_t)__popcll(mo);
        n_under += (uint32_t)__popcll(mu);
    }
    __syncthreads();
    if (lane == 0) {
        while (n_under && n_over) {
            AliasWork ob = over[--n_over];
            AliasWork ub = under[--n_under];
            const float delta = 1.0f - ub.prob;
            ob.prob -= delta;
            if (ob.prob > 1.0f) over[n_over++] = ob;
            else if (ob.prob < 1.0f) under[n_under++] = ob;
            t[ub.index] = hk_alias_entry{delta, ob.index};
        }
        const float el = sqrtf((mat.emissive[0] * mat.emissive[0] + mat.emissive[1] * mat.emissive[1]) +
                               mat.emissive[2] * mat.emissive[2]);
        const float intensity = (255.0f * mat.emissive[3]) * el;
        const float dx = in.max[0] - in.min[0], dy = in.max[1] - in.min[1], dz = in.max[2] - in.min[2];
        const float d2 = (dx * dx + dy * dy) + dz * dz;
        float pos[3];
        for (int k = 0; k < 3; ++k) pos[k] = (in.max[k] + in.min[k]) * 0.5f;
        const float radius = 0.5f * sqrtf(d2) + sqrtf(intensity);
        for (int k = 0; k < 4; ++k) r.emissive[k] = mat.emissive[k];
        for (int k = 0; k < 3; ++k) r.position[k] = pos[k];
        r.radius = radius;
        r.surface_area = surface_area;
        BBox b;
        for (int k = 0; k < 3; ++k) {
            b.mn[k] = pos[k] - radius;
            b.mx[k] = pos[k] + radius;
        }
        boxes[e] = b;
    }
}

// BHShape::set_bh_node_index: leaf node index back into the shape record
__global__ __launch_bounds__(256) void k_backfill_nodes(const hk_node* tlas, uint32_t n_tlas, hk_instance* inst,
                                                        const hk_node* lbvh, uint32_t n_lbvh, hk_emissive* em)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n_tlas && tlas[i].entry_index >= HK_BVH_LEAF_FLAG) inst[tlas[i].entry_index - HK_BVH_LEAF_FLAG].node_index = i;
    if (i < n_lbvh && lbvh[i].entry_index >= HK_BVH_LEAF_FLAG) em[lbvh[i].entry_index - HK_BVH_LEAF_FLAG].node_index = i;
}

void launch_dynamic_update(const DynamicArgs& D, hipStream_t st)
{
    const uint32_t n = D.n_instances;
    hipLaunchKernelGGL(k_update_instances, dim3((n + 255u) / 256u), dim3(256), 0, st, D.instances, n, D.models,
                       D.local_aabbs, (BBox*)D.boxes, D.flags);
    auto build = [&](uint32_t count, hk_node* out, uint32_t* levels) {
        if (count <= BVH_LDS_SHAPES)
            hipLaunchKernelGGL(k_build_bvh<true>, dim3(1), dim3(256), 0, st, (const BBox*)D.boxes, count, D.buckets, out,
                               D.idx, (Segment*)D.segments, levels);
        else
            hipLaunchKernelGGL(k_build_bvh<false>, dim3(1), dim3(256), 0, st, (const BBox*)D.boxes, count, D.buckets,
                               out, D.idx, (Segment*)D.segments, levels);
    };
    build(n, D.tlas, D.flags + 1);
    if (D.n_emissives) {
        hipLaunchKernelGGL(k_emissive_areas, dim3((D.n_alias + 255u) / 256u), dim3(256), 0, st, D.emissives,
                           D.n_emissives, D.instances, D.primitives, D.n_alias, D.areas);
        hipLaunchKernelGGL(k_update_emissives, dim3(D.n_emissives), dim3(64), 0, st, D.emissives, D.n_emissives,
                           D.instances, D.materials, D.alias, D.areas, (AliasWork*)D.alias_work, (BBox*)D.boxes);
        build(D.n_emissives, D.lbvh, nullptr);
    }
    const uint32_t m = 3u * n - 2u > 3u * D.n_emissives ? 3u * n - 2u : 3u * D.n_emissives;
    hipLaunchKernelGGL(k_backfill_nodes, dim3((m + 255u) / 256u), dim3(256), 0, st, D.tlas, 3u * n - 2u, D.instances,
                       D.lbvh, D.n_emissives ? 3u * D.n_emissives - 2u : 0u, D.emissives);
}

}  // namespace hk
