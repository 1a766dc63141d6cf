// hk_scene.cpp — host scene builder: bevy-hikari's mesh_material upload path in C++.
//
// Reference call sites restated here:
//   GpuMesh::try_from            mod.rs:379-467   (attributes, topology -> primitives, BLAS)
//   GpuMesh::build_alias_table   mod.rs:330-376
//   transformed_primitive_areas  mod.rs:318-328
//   GpuNode::pack                mod.rs:185-201
//   prepare_mesh_assets          mesh.rs:106-166  (concatenation, GpuMeshIndex)
//   prepare_instances            instance.rs:245-444 (AABB, TLAS, emissives, light BVH)
//   bvh 0.7.1 BVH::build + flatten_custom (third-party, restated from its published algorithm)
#include "../../include/hikari_scene.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

namespace {

struct V3 {
    float x, y, z;
};
static inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
static inline V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline V3 vmin(V3 a, V3 b) { return v3(std::fmin(a.x, b.x), std::fmin(a.y, b.y), std::fmin(a.z, b.z)); }
static inline V3 vmax(V3 a, V3 b) { return v3(std::fmax(a.x, b.x), std::fmax(a.y, b.y), std::fmax(a.z, b.z)); }
static inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline V3 cross(V3 a, V3 b)
{
    return v3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
static inline float length(V3 a) { return std::sqrt(dot(a, a)); }
static inline float comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

struct Aabb {
    V3 min, max;
    static Aabb empty()
    {
        const float inf = std::numeric_limits<float>::infinity();
        return Aabb{v3(inf, inf, inf), v3(-inf, -inf, -inf)};
    }
    void grow(V3 p)
    {
        min = vmin(min, p);
        max = vmax(max, p);
    }
    void join(const Aabb& o)
    {
        min = vmin(min, o.min);
        max = vmax(max, o.max);
    }
    V3 center() const { return (min + max) * 0.5f; }
    float surface_area() const
    {
        V3 s = max - min;
        return 2.0f * (s.x * s.y + s.x * s.z + s.y * s.z);
    }
    int largest_axis() const
    {
        V3 s = max - min;
        if (s.x > s.y && s.x > s.z) return 0;
        if (s.y > s.z) return 1;
        return 2;
    }
};

// ---- bvh 0.7.1 restatement ---------------------------------------------------------
// Build: recursive; a single shape makes a leaf; otherwise split on the largest axis of
// the centroid bounds (halves if the centroids coincide), choosing among NUM_BUCKETS-1
// bucket boundaries by SAH cost.  Flatten: DFS, left first; every child subtree gets an
// "entry" node carrying the child's AABB (entry = next index, exit = index after the
// subtree), every leaf gets an empty-AABB node (entry = shape | LEAF_FLAG, exit = next).
struct BuildNode {
    bool leaf;
    uint32_t shape;
    int left, right;
    Aabb left_aabb, right_aabb;
};

class BvhBuilder {
  public:
    BvhBuilder(const std::vector<Aabb>& shapes, int buckets) : shapes_(shapes), buckets_(buckets) {}

    std::vector<hk_node> build_flat()
    {
        std::vector<hk_node> flat;
        if (shapes_.empty()) return flat;
        std::vector<uint32_t> idx(shapes_.size());
        for (size_t i = 0; i < idx.size(); ++i) idx[i] = (uint32_t)i;
        nodes_.clear();
        nodes_.reserve(2 * shapes_.size());
        int root = build(idx);
        flatten(root, flat);
        return flat;
    }

  private:
    const std::vector<Aabb>& shapes_;
    int buckets_;
    std::vector<BuildNode> nodes_;

    Aabb bounds_of(const std::vector<uint32_t>& idx) const
    {
        Aabb b = Aabb::empty();
        for (uint32_t i : idx) b.join(shapes_[i]);
        return b;
    }

    int build(std::vector<uint32_t>& idx)
    {
        if (idx.size() == 1) {
            nodes_.push_back(BuildNode{true, idx[0], -1, -1, Aabb::empty(), Aabb::empty()});
            return (int)nodes_.size() - 1;
        }
        Aabb centroid = Aabb::empty();
        for (uint32_t i : idx) centroid.grow(shapes_[i].center());
        Aabb aabb_bounds = bounds_of(idx);
        int axis = centroid.largest_axis();
        float axis_size = comp(centroid.max, axis) - comp(centroid.min, axis);

        std::vector<uint32_t> left, right;
        if (axis_size < std::numeric_limits<float>::epsilon()) {
            size_t half = idx.size() / 2;
            left.assign(idx.begin(), idx.begin() + half);
            right.assign(idx.begin() + half, idx.end());
        } else {
            const int nb = buckets_;
            std::vector<std::vector<uint32_t>> bucket_idx(nb);
            std::vector<Aabb> bucket_aabb(nb, Aabb::empty());
            for (uint32_t i : idx) {
                float rel = (comp(shapes_[i].center(), axis) - comp(centroid.min, axis)) / axis_size;
                int b = (int)(rel * ((float)nb - 0.01f));
                b = std::min(std::max(b, 0), nb - 1);
                bucket_idx[b].push_back(i);
                bucket_aabb[b].join(shapes_[i]);
            }
            int best = 0;
            float best_cost = std::numeric_limits<float>::infinity();
            for (int s = 0; s < nb - 1; ++s) {
                Aabb la = Aabb::empty(), ra = Aabb::empty();
                size_t ln = 0, rn = 0;
                for (int b = 0; b <= s; ++b) {
                    la.join(bucket_aabb[b]);
                    ln += bucket_idx[b].size();
                }
                for (int b = s + 1; b < nb; ++b) {
                    ra.join(bucket_aabb[b]);
                    rn += bucket_idx[b].size();
                }
                if (ln == 0 || rn == 0) continue;
                float cost = ((float)ln * la.surface_area() + (float)rn * ra.surface_area()) /
                             aabb_bounds.surface_area();
                if (cost < best_cost) {
                    best_cost = cost;
                    best = s;
                }
            }
            for (int b = 0; b < nb; ++b) {
                auto& dst = b <= best ? left : right;
                dst.insert(dst.end(), bucket_idx[b].begin(), bucket_idx[b].end());
            }
            if (left.empty() || right.empty()) {  // degenerate (NaN areas): fall back to halves
                left.assign(idx.begin(), idx.begin() + idx.size() / 2);
                right.assign(idx.begin() + idx.size() / 2, idx.end());
            }
        }
        Aabb la = bounds_of(left), ra = bounds_of(right);
        int l = build(left);
        int r = build(right);
        nodes_.push_back(BuildNode{false, 0, l, r, la, ra});
        return (int)nodes_.size() - 1;
    }

    static hk_node pack(const Aabb& a, uint32_t entry, uint32_t exit, uint32_t shape)
    {
        // GpuNode::pack (mod.rs:186-200)
        hk_node n;
        n.min[0] = a.min.x; n.min[1] = a.min.y; n.min[2] = a.min.z;
        n.max[0] = a.max.x; n.max[1] = a.max.y; n.max[2] = a.max.z;
        n.entry_index = entry == HK_U32_MAX ? (shape | HK_BVH_LEAF_FLAG) : entry;
        n.exit_index = exit;
        return n;
    }

    uint32_t flatten(int node, std::vector<hk_node>& flat)
    {
        const BuildNode& n = nodes_[node];
        uint32_t next_free = (uint32_t)flat.size();
        if (n.leaf) {
            flat.push_back(pack(Aabb::empty(), HK_U32_MAX, next_free + 1, n.shape));
            return next_free + 1;
        }
        flat.push_back(pack(n.left_aabb, next_free + 1, 0, HK_U32_MAX));
        uint32_t after_l = flatten(n.left, flat);
        flat[next_free].exit_index = after_l;
        flat.push_back(pack(n.right_aabb, after_l + 1, 0, HK_U32_MAX));
        uint32_t after_r = flatten(nodes_[node].right, flat);
        flat[after_l].exit_index = after_r;
        return after_r;
    }
};

// ---- column-major 4x4 helpers ----
static V3 transform_point(const float* m, V3 p)
{
    float x = m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12];
    float y = m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13];
    float z = m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14];
    return v3(x, y, z);
}
static V3 transform_vector(const float* m, V3 p)
{
    float x = m[0] * p.x + m[4] * p.y + m[8] * p.z;
    float y = m[1] * p.x + m[5] * p.y + m[9] * p.z;
    float z = m[2] * p.x + m[6] * p.y + m[10] * p.z;
    return v3(x, y, z);
}

static bool inverse_transpose(const float* m, float* out)
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
    double det = a[0] * inv[0] + a[1] * inv[4] + a[2] * inv[8] + a[3] * inv[12];
    if (det == 0.0) return false;
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) out[c * 4 + r] = (float)(inv[r * 4 + c] / det);  // transpose
    return true;
}

struct Mesh {
    std::vector<hk_vertex> vertices;
    std::vector<hk_primitive> primitives;
    std::vector<hk_node> nodes;
    Aabb aabb;  // Bevy's mesh Aabb from vertex positions
};

struct Instance {
    uint32_t mesh, material;
    float model[16];
};

}  // namespace

struct hks_scene {
    std::string error;
    std::vector<Mesh> meshes;
    std::vector<hk_material> materials;
    std::vector<Instance> instances;
    // built buffers
    std::vector<hk_vertex> vertices;
    std::vector<hk_primitive> primitives;
    std::vector<hk_node> asset_nodes;
    std::vector<hk_alias_entry> alias_table;
    std::vector<hk_instance> gpu_instances;
    std::vector<hk_node> instance_nodes;
    std::vector<hk_emissive> emissives;
    std::vector<hk_node> emissive_nodes;
    int buckets = 6;
};

extern "C" {

hks_scene* hks_create(void) { return new hks_scene(); }
void hks_destroy(hks_scene* s) { delete s; }
const char* hks_last_error(const hks_scene* s) { return s ? s->error.c_str() : "null scene"; }

int hks_add_mesh(hks_scene* s, const float* pos, const float* nrm, const float* uv, uint32_t n,
                 const uint32_t* indices, uint32_t index_count, int topology)
{
    if (!s) return HK_ERR_INVALID;
    // PrepareMeshError::{MissingAttributePosition, MissingAttributeNormal, MissingAttributeUV}
    if (!pos) { s->error = "MissingAttributePosition"; return -10; }
    if (!nrm) { s->error = "MissingAttributeNormal"; return -11; }
    if (!uv) { s->error = "MissingAttributeUV"; return -12; }
    Mesh m;
    m.aabb = Aabb::empty();
    m.vertices.resize(n);
    for (uint32_t i = 0; i < n; ++i) {
        hk_vertex& v = m.vertices[i];
        for (int c = 0; c < 3; ++c) {
            v.position[c] = pos[3 * i + c];
            v.normal[c] = nrm[3 * i + c];
        }
        v.u = uv[2 * i];
        v.v = uv[2 * i + 1];
        m.aabb.grow(v3(v.position[0], v.position[1], v.position[2]));
    }
    std::vector<uint32_t> idx;
    if (indices) idx.assign(indices, indices + index_count);
    else {
        idx.resize(n);
        for (uint32_t i = 0; i < n; ++i) idx[i] = i;
    }
    for (uint32_t i : idx)
        if (i >= n) { s->error = "index out of range"; return HK_ERR_INVALID; }
    auto push = [&](uint32_t a, uint32_t b, uint32_t c) {
        hk_primitive p;
        uint32_t ids[3] = {a, b, c};
        for (int k = 0; k < 3; ++k) {
            for (int d = 0; d < 3; ++d) p.vertices[k].position[d] = m.vertices[ids[k]].position[d];
            p.vertices[k].index = ids[k];
        }
        m.primitives.push_back(p);
    };
    if (topology == HKS_TRIANGLE_LIST) {
        if (idx.size() % 3 != 0) { s->error = "IncompatiblePrimitiveTopology"; return -13; }
        for (size_t i = 0; i + 2 < idx.size(); i += 3) push(idx[i], idx[i + 1], idx[i + 2]);
    } else if (topology == HKS_TRIANGLE_STRIP) {
        for (size_t i = 0; i + 2 < idx.size(); ++i) {
            if ((i & 1) == 0) push(idx[i], idx[i + 1], idx[i + 2]);
            else push(idx[i + 1], idx[i], idx[i + 2]);
        }
    } else {
        s->error = "IncompatiblePrimitiveTopology";
        return -13;
    }
    if (m.primitives.empty()) { s->error = "NoPrimitive"; return -14; }
    s->meshes.push_back(std::move(m));
    return (int)s->meshes.size() - 1;
}

int hks_add_material(hks_scene* s, const hk_material* mat)
{
    if (!s || !mat) return HK_ERR_INVALID;
    s->materials.push_back(*mat);
    return (int)s->materials.size() - 1;
}

int hks_add_instance(hks_scene* s, uint32_t mesh, uint32_t material, const float* model)
{
    if (!s || !model) return HK_ERR_INVALID;
    if (mesh >= s->meshes.size() || material >= s->materials.size()) {
        s->error = "instance references unknown mesh/material";
        return HK_ERR_INVALID;
    }
    Instance in;
    in.mesh = mesh;
    in.material = material;
    std::memcpy(in.model, model, sizeof(in.model));
    s->instances.push_back(in);
    return (int)s->instances.size() - 1;
}

int hks_build(hks_scene* s, int buckets)
{
    if (!s) return HK_ERR_INVALID;
    if (buckets < 2) buckets = 6;
    s->buckets = buckets;
    // BLAS per mesh (mod.rs:458-459)
    for (Mesh& m : s->meshes) {
        std::vector<Aabb> shapes(m.primitives.size());
        for (size_t i = 0; i < m.primitives.size(); ++i) {
            Aabb a = Aabb::empty();
            for (int k = 0; k < 3; ++k)
                a.grow(v3(m.primitives[i].vertices[k].position[0], m.primitives[i].vertices[k].position[1],
                          m.primitives[i].vertices[k].position[2]));
            shapes[i] = a;
        }
        m.nodes = BvhBuilder(shapes, buckets).build_flat();
    }
    // concatenate (mesh.rs:140-163)
    s->vertices.clear();
    s->primitives.clear();
    s->asset_nodes.clear();
    std::vector<hk_mesh_index> mesh_index(s->meshes.size());
    for (size_t i = 0; i < s->meshes.size(); ++i) {
        const Mesh& m = s->meshes[i];
        mesh_index[i].vertex = (uint32_t)s->vertices.size();
        mesh_index[i].primitive = (uint32_t)s->primitives.size();
        mesh_index[i].node[0] = (uint32_t)s->asset_nodes.size();
        mesh_index[i].node[1] = (uint32_t)m.nodes.size();
        s->vertices.insert(s->vertices.end(), m.vertices.begin(), m.vertices.end());
        s->primitives.insert(s->primitives.end(), m.primitives.begin(), m.primitives.end());
        s->asset_nodes.insert(s->asset_nodes.end(), m.nodes.begin(), m.nodes.end());
    }
    // instances (instance.rs:284-330): world AABB from the 8 transformed corners
    s->gpu_instances.clear();
    std::vector<Aabb> inst_aabb;
    for (const Instance& in : s->instances) {
        const Mesh& m = s->meshes[in.mesh];
        V3 center = m.aabb.center();
        V3 half = (m.aabb.max - m.aabb.min) * 0.5f;
        V3 c = transform_point(in.model, center);
        V3 mn = v3(0, 0, 0), mx = v3(0, 0, 0);
        for (int k = 0; k < 8; ++k) {
            float x = (float)(2 * (k & 1) - 1), y = (float)(2 * ((k >> 1) & 1) - 1), z = (float)(2 * ((k >> 2) & 1) - 1);
            V3 corner = transform_vector(in.model, v3(half.x * x, half.y * y, half.z * z));
            mn = vmin(mn, corner);
            mx = vmax(mx, corner);
        }
        mn = mn + c;
        mx = mx + c;
        hk_instance g;
        std::memset(&g, 0, sizeof(g));
        g.min[0] = mn.x; g.min[1] = mn.y; g.min[2] = mn.z;
        g.max[0] = mx.x; g.max[1] = mx.y; g.max[2] = mx.z;
        g.material = in.material;
        std::memcpy(g.model, in.model, sizeof(g.model));
        if (!inverse_transpose(in.model, g.inverse_transpose_model)) {
            s->error = "singular instance transform";
            return HK_ERR_INVALID;
        }
        g.mesh = mesh_index[in.mesh];
        s->gpu_instances.push_back(g);
        inst_aabb.push_back(Aabb{mn, mx});
    }
    // TLAS (instance.rs:365-371)
    s->instance_nodes = BvhBuilder(inst_aabb, buckets).build_flat();
    // BHShape::set_bh_node_index: the leaf node index of each shape
    for (uint32_t n = 0; n < s->instance_nodes.size(); ++n) {
        const hk_node& nd = s->instance_nodes[n];
        if (nd.entry_index >= HK_BVH_LEAF_FLAG) s->gpu_instances[nd.entry_index - HK_BVH_LEAF_FLAG].node_index = n;
    }
    // emissives (instance.rs:377-420)
    s->emissives.clear();
    s->alias_table.clear();
    std::vector<Aabb> emissive_aabb;
    for (size_t id = 0; id < s->instances.size(); ++id) {
        const Instance& in = s->instances[id];
        const hk_material& mat = s->materials[in.material];
        V3 e = v3(mat.emissive[0], mat.emissive[1], mat.emissive[2]);
        float intensity = 255.0f * mat.emissive[3] * length(e);
        if (!(intensity > 0.0f)) continue;
        const Mesh& m = s->meshes[in.mesh];
        // transformed_primitive_areas (mod.rs:318-328)
        std::vector<float> areas(m.primitives.size());
        float surface_area = 0.0f;
        for (size_t p = 0; p < m.primitives.size(); ++p) {
            V3 w[3];
            for (int k = 0; k < 3; ++k) {
                const hk_vertex& vx = m.vertices[m.primitives[p].vertices[k].index];
                w[k] = transform_point(in.model, v3(vx.position[0], vx.position[1], vx.position[2]));
            }
            areas[p] = 0.5f * std::fabs(length(cross(w[1] - w[0], w[2] - w[0])));
            surface_area += areas[p];
        }
        // build_alias_table (mod.rs:330-376)
        size_t count = m.primitives.size();
        std::vector<hk_alias_entry> table(count);
        for (size_t i = 0; i < count; ++i) table[i] = hk_alias_entry{0.0f, (uint32_t)i};
        float mean_area = surface_area / (float)count;
        std::vector<std::pair<size_t, float>> over, under;
        for (size_t i = 0; i < count; ++i) {
            float prob = areas[i] / mean_area;
            if (prob > 1.0f) over.emplace_back(i, prob);
        }
        for (size_t i = 0; i < count; ++i) {
            float prob = areas[i] / mean_area;
            if (prob < 1.0f) under.emplace_back(i, prob);
        }
        while (!under.empty() && !over.empty()) {
            auto ob = over.back();
            over.pop_back();
            auto ub = under.back();
            under.pop_back();
            float delta = 1.0f - ub.second;
            ob.second -= delta;
            if (ob.second > 1.0f) over.push_back(ob);
            else if (ob.second < 1.0f) under.push_back(ob);
            table[ub.first] = hk_alias_entry{delta, (uint32_t)ob.first};
        }
        hk_emissive em;
        std::memset(&em, 0, sizeof(em));
        for (int c = 0; c < 4; ++c) em.emissive[c] = mat.emissive[c];
        const hk_instance& g = s->gpu_instances[id];
        V3 mn = v3(g.min[0], g.min[1], g.min[2]), mx = v3(g.max[0], g.max[1], g.max[2]);
        V3 position = (mx + mn) * 0.5f;
        float radius = 0.5f * length(mx - mn) + std::sqrt(intensity);
        em.position[0] = position.x; em.position[1] = position.y; em.position[2] = position.z;
        em.radius = radius;
        em.instance = (uint32_t)id;
        em.alias_table[0] = (uint32_t)s->alias_table.size();
        em.alias_table[1] = (uint32_t)table.size();
        em.surface_area = surface_area;
        s->alias_table.insert(s->alias_table.end(), table.begin(), table.end());
        s->emissives.push_back(em);
        V3 r = v3(radius, radius, radius);
        emissive_aabb.push_back(Aabb{position - r, position + r});
    }
    // light BVH (instance.rs:422-428)
    s->emissive_nodes = BvhBuilder(emissive_aabb, buckets).build_flat();
    for (uint32_t n = 0; n < s->emissive_nodes.size(); ++n) {
        const hk_node& nd = s->emissive_nodes[n];
        if (nd.entry_index >= HK_BVH_LEAF_FLAG) s->emissives[nd.entry_index - HK_BVH_LEAF_FLAG].node_index = n;
    }
    return HK_OK;
}

int hks_get_desc(const hks_scene* s, hk_scene_desc* out)
{
    if (!s || !out) return HK_ERR_INVALID;
    out->vertices = hk_array{s->vertices.data(), (uint32_t)s->vertices.size()};
    out->primitives = hk_array{s->primitives.data(), (uint32_t)s->primitives.size()};
    out->asset_nodes = hk_array{s->asset_nodes.data(), (uint32_t)s->asset_nodes.size()};
    out->alias_table = hk_array{s->alias_table.data(), (uint32_t)s->alias_table.size()};
    out->instances = hk_array{s->gpu_instances.data(), (uint32_t)s->gpu_instances.size()};
    out->instance_nodes = hk_array{s->instance_nodes.data(), (uint32_t)s->instance_nodes.size()};
    out->materials = hk_array{s->materials.data(), (uint32_t)s->materials.size()};
    out->emissive_nodes = hk_array{s->emissive_nodes.data(), (uint32_t)s->emissive_nodes.size()};
    out->emissives = hk_array{s->emissives.data(), (uint32_t)s->emissives.size()};
    return HK_OK;
}

}  // extern "C"
