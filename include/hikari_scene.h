/*
 * hikari_scene.h — C ABI of the host-side scene builder (part of libhikari_amd.so).
 *
 * Restates bevy-hikari's `mesh_material` upload path, which the north star keeps on the
 * host: Mesh -> GpuMesh conversion with one BLAS per mesh (mod.rs:379-467), concatenation
 * into the universal vertex/primitive/node buffers (mesh.rs:106-166), material table
 * (material.rs:139-203), and `prepare_instances` (instance.rs:245-444): world AABBs, TLAS,
 * per-emitter alias tables, emissive list and light BVH.  The result is an hk_scene_desc
 * ready for hk_scene_upload.
 *
 * The BVH builder restates the third-party crate `bvh = "=0.7.1"` (Cargo.toml:21), which
 * is not in the reference checkout: SAH over 6 centroid buckets on the largest centroid
 * axis, one shape per leaf, `flatten_custom` DFS order with entry/exit skip pointers
 * (3n-2 nodes for n shapes).  Structural parity with that crate is unpinned.
 */
#ifndef HIKARI_SCENE_H
#define HIKARI_SCENE_H

#include <stdint.h>
#include "hikari_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hks_scene hks_scene;

enum { HKS_TRIANGLE_LIST = 0, HKS_TRIANGLE_STRIP = 1 };

hks_scene* hks_create(void);
void hks_destroy(hks_scene* scene);
const char* hks_last_error(const hks_scene* scene);

/* Mesh asset (Bevy `Mesh`): positions/normals xyz, uvs (u, v); indices may be NULL (=> 0..n-1).
 * Returns the mesh id (>= 0) or a negative error like `PrepareMeshError` (mod.rs:302-309). */
int hks_add_mesh(hks_scene* scene, const float* positions, const float* normals, const float* uvs,
                 uint32_t vertex_count, const uint32_t* indices, uint32_t index_count, int topology);
/* StandardMaterial as the GpuStandardMaterial record (material.rs:162-199). Returns id. */
int hks_add_material(hks_scene* scene, const hk_material* material);
/* Visible entity with (mesh, material) and its GlobalTransform (column-major 4x4). Returns id. */
int hks_add_instance(hks_scene* scene, uint32_t mesh, uint32_t material, const float* model);

/* Build BLAS/TLAS/light BVH and the flat buffers; `buckets` = SAH buckets (6 = bvh 0.7.1). */
int hks_build(hks_scene* scene, int buckets);
/* Pointers stay valid until the next hks_build / hks_destroy. */
int hks_get_desc(const hks_scene* scene, hk_scene_desc* out);

#ifdef __cplusplus
}
#endif

#endif /* HIKARI_SCENE_H */
