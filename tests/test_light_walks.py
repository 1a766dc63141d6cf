"""Ordered closest-hit light walks against light.wgsl's order: the record behind DESIGN §4's measured negative (CPU).

light.wgsl walks the indirect bounce ray (`traverse_top(ray, F32_MAX, 0.0, DONT_EXCLUDE)`, light.wgsl:1319,1401) and
the emitter BLAS walk of select_light_candidate (`traverse_bottom(..., 0.0)`, light.wgsl:687) with its stackless
skip-pointer order.  Neither has an early exit, so either returns the closest hit in any visit order — except for
exact-distance ties and box tests that round across the hit distance.  Round 5 tried walking them with the
G-buffer's ordered rule (nearer child first, the oracle's closest_hit_ordered):
  * bounce rays: no ray of the bench workloads' scenes differs in any bit (checked here, and by the whole GPU
    suite with the oracle in CHECK mode, profiles/r05/c1/tests_ordered.log) — but the kernel was slower (cornell
    1080p k_indirect 0.184 -> 0.240 ms; the stack's registers cost a wave per SIMD), so the kernels keep
    light.wgsl's order;
  * emitter walks aim at sampled points of emitter triangles, shared edges included whenever a quantised
    blue-noise coordinate is 0 or 1, and there the two orders break ties differently (scene.rs at 1080p: one walk
    in 2.2 M), so the ordered rule is not an option for them at all.
"""
import pytest

CASES = [
    # (config, width, height, frames, spatial): configs[1] at full size; scene.rs and city.rs at 960x540
    ("cornell", 1920, 1080, 2, False),
    ("scene", 960, 540, 2, True),
    ("city", 960, 540, 2, True),
]


@pytest.mark.parametrize("scene_fn,w,h,frames,spatial", CASES)
def test_ordered_bounce_walk_matches_reference_order(scene_fn, w, h, frames, spatial):
    from hikari_amd import HikariSettings, Upscale, examples, frame_inputs, load_noise
    from oracle import Oracle
    scene, cam, lights = examples.SCENES[scene_fn]()
    o = Oracle(scene.build(), load_noise(), w, h, 1.0, light_walk=Oracle.WALK_CHECK)
    s = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=spatial, denoise=False).to_c()
    for f in range(frames):
        fi = frame_inputs(f, cam, lights, w, h)
        o.render_gbuffer(fi)
        o.render_frame(s, fi)  # raises on the first frame with a differing ray
    st = o.light_walk_stats()
    assert st["bounce_checked"] > 0.2 * w * h * frames, st
    assert st["emitter_checked"] > 0, st
    assert st["bounce_differ"] == 0, st


def test_orders_differ_only_on_ties():
    """The two orders are NOT equivalent in general: rays aimed exactly at the shared edge of two triangles hit both
    at (nearly) the same distance, and the first one found wins.  Such rays do occur and are caught by the bitwise
    comparison above; every difference found here is a near-tie (distances within 1e-4 relative: the ordered walk pruned by a box
    test that rounded across the other triangle's distance, or found the other triangle of an exact tie first), which is why the
    equivalence is checked on the workloads' own rays rather than assumed."""
    import ctypes as C
    import numpy as np
    from hikari_amd import examples, load_noise
    from oracle import Oracle
    scene, _, _ = examples.SCENES["cornell"]()
    d = scene.build()
    o = Oracle(d, load_noise(), 16, 16, 1.0)
    prims = np.frombuffer((C.c_char * (d.primitives.count * 48)).from_address(d.primitives.data),
                          np.float32).reshape(-1, 3, 4)[:, :, :3]
    inst = np.frombuffer((C.c_char * (d.instances.count * 176)).from_address(d.instances.data), np.uint32).reshape(-1, 44)
    pts = []
    for k in range(len(inst)):
        model = inst[k, 8:24].view(np.float32).reshape(4, 4).T  # column-major (mod.rs:147-156)
        p0, n_nodes = int(inst[k, 41]), int(inst[k, 43])
        tris = prims[p0:p0 + (n_nodes + 2) // 3]  # one primitive per leaf: 2n - 1 nodes (+ leaf boxes) for n
        for i in range(len(tris)):
            for j in range(i + 1, len(tris)):
                shared = set(map(tuple, tris[i])) & set(map(tuple, tris[j]))
                if len(shared) == 2:
                    a, b = (np.array(v, np.float64) for v in shared)
                    for t in np.linspace(0.05, 0.95, 20):
                        w = model @ np.append(a + (b - a) * t, 1.0)
                        pts.append(w[:3] / w[3])
    assert len(pts) > 100
    rng = np.random.default_rng(3)
    org = rng.uniform(-0.9, 0.9, (len(pts) * 100, 3)) + [0.0, 1.0, 0.0]
    dirs = np.repeat(np.array(pts), 100, axis=0) - org
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    rays = np.concatenate([org, dirs], 1).astype(np.float32)
    a, b = o.trace(rays), o.trace_ordered(rays)
    differ = (a != b).any(1)
    assert differ.sum() > 0  # ties exist and the comparison sees them
    da, db = a[differ, 2].view(np.float32).astype(np.float64), b[differ, 2].view(np.float32).astype(np.float64)
    assert np.all(np.abs(da - db) <= 1e-4 * np.maximum(da, db)), np.sort(np.abs(da - db) / np.maximum(da, db))[-5:]
