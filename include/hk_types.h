/*
 * hk_types.h — byte-exact std430 mirrors of bevy-hikari's scene, reservoir and G-buffer
 * records: the data contract at the drop-in boundary.
 *
 * Every struct here has the size and field offsets that the reference's WGSL bindings
 * read (checked by static asserts below), so a Rust shim can hand the exact buffers that
 * `MeshRenderAssets::set` / `InstanceRenderAssets::set` build to `hk_scene_upload`.
 *
 *   Vertex            mesh_material_types.wgsl:3-8      host mod.rs:67-73       32 B
 *   PrimitiveVertex   mesh_material_types.wgsl:10-13    host mod.rs:115-119     16 B
 *   Primitive         mesh_material_types.wgsl:15-17    host mod.rs:121-124     48 B
 *   MeshIndex         mesh_material_types.wgsl:19-23    host mod.rs:471-476     16 B
 *   Instance          mesh_material_types.wgsl:25-33    host mod.rs:147-156    176 B
 *   Node              mesh_material_types.wgsl:35-40    host mod.rs:177-183     32 B
 *   Material          mesh_material_types.wgsl:42-56    host mod.rs:203-218     80 B
 *   AliasEntry        mesh_material_types.wgsl:58-61    host mod.rs:220-226      8 B
 *   Emissive          mesh_material_types.wgsl:63-71    host mod.rs:228-237     64 B
 *   PackedReservoir   light.wgsl:35-43                  host light.rs:51-60     64 B
 *
 * Plain C (C99) so the gcc-built oracle and the hipcc-built library share it.
 */
#ifndef HK_TYPES_H
#define HK_TYPES_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
#define HK_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define HK_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif

/* Leaf flag of a flattened skip-pointer node (light.wgsl:232, mod.rs:186-200). */
#define HK_BVH_LEAF_FLAG 0x80000000u
/* "no texture" id in Material (material.rs:78-86) and "none" instance/material ids. */
#define HK_U32_MAX 0xFFFFFFFFu

typedef struct hk_vertex {
    float position[3];
    float u;
    float normal[3];
    float v;
} hk_vertex;

typedef struct hk_primitive_vertex {
    float position[3];
    uint32_t index; /* mesh-local vertex index */
} hk_primitive_vertex;

typedef struct hk_primitive {
    hk_primitive_vertex vertices[3];
} hk_primitive;

typedef struct hk_mesh_index {
    uint32_t vertex;    /* offset into the vertex buffer */
    uint32_t primitive; /* offset into the primitive buffer */
    uint32_t node[2];   /* (offset, length) into the asset node buffer */
} hk_mesh_index;

typedef struct hk_instance {
    float min[3];
    uint32_t material;
    float max[3];
    uint32_t node_index;
    float model[16];                   /* column-major mat4x4 */
    float inverse_transpose_model[16]; /* column-major mat4x4 */
    hk_mesh_index mesh;
} hk_instance;

typedef struct hk_node {
    float min[3];
    uint32_t entry_index; /* inner: next node; leaf: payload | HK_BVH_LEAF_FLAG */
    float max[3];
    uint32_t exit_index; /* skip pointer */
} hk_node;

typedef struct hk_material {
    float base_color[4];
    uint32_t base_color_texture;
    uint32_t _pad0[3];
    float emissive[4];
    uint32_t emissive_texture;
    float perceptual_roughness;
    float metallic;
    uint32_t metallic_roughness_texture;
    float reflectance;
    uint32_t normal_map_texture;
    uint32_t occlusion_texture;
    uint32_t _pad1;
} hk_material;

typedef struct hk_alias_entry {
    float prob;
    uint32_t index;
} hk_alias_entry;

typedef struct hk_emissive {
    float emissive[4];
    float position[3];
    float radius;
    uint32_t instance;
    uint32_t _pad0;
    uint32_t alias_table[2]; /* (offset, length) */
    float surface_area;
    uint32_t node_index;
    uint32_t _pad1[2];
} hk_emissive;

/* light.wgsl:35-43 — 64-byte packed ReSTIR reservoir. */
typedef struct hk_packed_reservoir {
    uint32_t radiance[2];         /* RGBA16F */
    uint32_t random[2];           /* RGBA unorm16 */
    float visible_position[4];    /* xyz + depth in w */
    float sample_position[4];     /* xyz + f32(visible_instance) in w */
    uint32_t visible_normal;      /* snorm8 xyz + lifetime code in w */
    uint32_t sample_normal;       /* snorm8 xyz + sample_position.w */
    uint32_t reservoir[2];        /* f16 (count, w), (w_sum, w2_sum) */
} hk_packed_reservoir;

HK_STATIC_ASSERT(sizeof(hk_vertex) == 32, "Vertex must be 32 B");
HK_STATIC_ASSERT(sizeof(hk_primitive) == 48, "Primitive must be 48 B");
HK_STATIC_ASSERT(sizeof(hk_mesh_index) == 16, "MeshIndex must be 16 B");
HK_STATIC_ASSERT(sizeof(hk_instance) == 176, "Instance must be 176 B");
HK_STATIC_ASSERT(offsetof(hk_instance, model) == 32, "Instance.model at 32");
HK_STATIC_ASSERT(offsetof(hk_instance, inverse_transpose_model) == 96, "Instance.itm at 96");
HK_STATIC_ASSERT(offsetof(hk_instance, mesh) == 160, "Instance.mesh at 160");
HK_STATIC_ASSERT(sizeof(hk_node) == 32, "Node must be 32 B");
HK_STATIC_ASSERT(sizeof(hk_material) == 80, "Material must be 80 B");
HK_STATIC_ASSERT(offsetof(hk_material, emissive) == 32, "Material.emissive at 32");
HK_STATIC_ASSERT(offsetof(hk_material, perceptual_roughness) == 52, "Material.pr at 52");
HK_STATIC_ASSERT(offsetof(hk_material, reflectance) == 64, "Material.reflectance at 64");
HK_STATIC_ASSERT(offsetof(hk_material, occlusion_texture) == 72, "Material.occlusion at 72");
HK_STATIC_ASSERT(sizeof(hk_alias_entry) == 8, "AliasEntry must be 8 B");
HK_STATIC_ASSERT(sizeof(hk_emissive) == 64, "Emissive must be 64 B");
HK_STATIC_ASSERT(offsetof(hk_emissive, instance) == 32, "Emissive.instance at 32");
HK_STATIC_ASSERT(offsetof(hk_emissive, alias_table) == 40, "Emissive.alias_table at 40");
HK_STATIC_ASSERT(offsetof(hk_emissive, surface_area) == 48, "Emissive.surface_area at 48");
HK_STATIC_ASSERT(offsetof(hk_emissive, node_index) == 52, "Emissive.node_index at 52");
HK_STATIC_ASSERT(sizeof(hk_packed_reservoir) == 64, "PackedReservoir must be 64 B");
HK_STATIC_ASSERT(offsetof(hk_packed_reservoir, visible_normal) == 48, "visible_normal at 48");

/*
 * G-buffer planes (prepass.rs:43-47 formats, prepass.wgsl:84-100 contents), one plane
 * per texture, row-major, width = S.x:
 *   position       float4  (world xyz, NDC reverse-Z depth; 0 = background)
 *   normal         uint32  (RGBA8 snorm: world normal xyz, w = 1.0)
 *   depth_gradient float2  (dpdx, dpdy of NDC depth)
 *   instance_mat   float2  (instance + 0.5, material + 0.5)
 *   velocity_uv    float4  (screen-space velocity xy, mesh uv zw)
 */
#define HK_GBUFFER_BYTES_PER_PIXEL (16 + 4 + 8 + 8 + 16)

#endif /* HK_TYPES_H */
