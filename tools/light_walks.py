"""The closest-hit light walks in light.wgsl's order against the ordered rule (analysis tool, CPU).

Two questions about the bounce ray (light.wgsl:1319,1401) and the emitter BLAS walk (light.wgsl:687):
  1. equivalence: the oracle walks every such ray both ways (hko_set_light_walk CHECK) and counts the rays whose
     two results differ in any bit (instance, primitive, distance, uv);
  2. cost: the oracle's statistics build (-DHKO_STATS) counts each walk's steps per pixel — node visits + leaf
     tests in light.wgsl's order, wide-entry iterations + leaf tests in the ordered rule — and the SIMD cost model
     of tools/walk_lanes.py (a wave runs until its longest lane ends: 64 x max over its 8x8 lanes) prices both.
     (The oracle's ORDERED mode orders the bounce walk only, as the kernels do; the emitter walk's ordered cost
     was measured before that restriction: 0.49-0.83x of its steps)
usage: python tools/light_walks.py [config] [width height] [--frames N]
"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "bevy-hikari_amd"))
sys.path.insert(0, str(ROOT / "oracle"))

PASSES = ["direct_lit", "emissive", "indirect"]
CLASSES = ["closest", "directional_any_hit", "emissive_any_hit", "emitter_blas"]


def wave_cost(a, h, w):
    th, tw = h // 16, w // 16
    g = a[:th * 16, :tw * 16].reshape(th, 2, 8, tw, 2, 8).transpose(0, 3, 1, 4, 2, 5).reshape(-1, 64)
    return int(g.sum()), int(64 * g.max(axis=1).sum())


def run(O, desc, cfg, w, h, frames, mode, steps_lib):
    from hikari_amd import HikariSettings, Upscale, frame_inputs, load_noise
    import bench
    from hikari_amd import examples
    _, cam, lights = examples.SCENES[cfg["scene"]]()
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=cfg["spatial"], denoise=False)
    s = st.to_c()
    o = O.Oracle(desc, load_noise(), w, h, 1.0)
    o.set_light_walk(mode)
    n = w * h
    steps = np.zeros(3 * 4 * n, np.uint32) if steps_lib else None
    ptr = C.c_void_p.in_dll(O.lib(), "hko_pixel_steps_out") if steps_lib else None
    tot = {}
    for f in range(frames):
        if steps is not None:
            steps[:] = 0
            ptr.value = steps.ctypes.data
        fi = frame_inputs(f, cam, lights, w, h)
        o.render_gbuffer(fi)
        o.render_frame(s, fi)
        if steps is not None:
            ptr.value = None
            a = steps.reshape(3, 4, h, w).astype(np.int64)
            for p, k in ((2, 0), (0, 3), (1, 3), (2, 3)):
                u, c = wave_cost(a[p, k], h, w)
                t = tot.setdefault((p, k), [0, 0])
                t[0] += u
                t[1] += c
    stats = o.light_walk_stats()
    o.close()
    return tot, stats


def main():
    import bench
    import oracle as O
    from hikari_amd import examples
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "cornell-1080p-nee"
    cfg = bench.CONFIGS[cfg_name]
    nums = [a for a in sys.argv[2:] if a.isdigit()]
    w, h = (int(nums[0]), int(nums[1])) if len(nums) >= 2 else (cfg["width"], cfg["height"])
    frames = int(sys.argv[sys.argv.index("--frames") + 1]) if "--frames" in sys.argv else 3
    scene, _, _ = examples.SCENES[cfg["scene"]]()
    desc = scene.build()
    _, stats = run(O, desc, cfg, w, h, frames, O.Oracle.WALK_CHECK, False)
    print(f"{cfg_name} {w}x{h} frames 0..{frames - 1}: {stats}")
    lib = ROOT / "oracle" / "_build" / "liboracle_stats.so"
    subprocess.run(["gcc", "-O3", "-std=gnu11", "-fPIC", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", "-DHKO_STATS",
                    "-shared", "-o", str(lib), str(ROOT / "oracle" / "hk_oracle.c"), "-lm"], check=True)
    O._L = None
    O.LIB = lib
    ref, _ = run(O, desc, cfg, w, h, frames, O.Oracle.WALK_REFERENCE, True)
    ordd, _ = run(O, desc, cfg, w, h, frames, O.Oracle.WALK_ORDERED, True)
    for key in sorted(ref):
        (ur, cr), (uo, co) = ref[key], ordd.get(key, (0, 0))
        if ur == 0:
            continue
        print(f"  {PASSES[key[0]]:10s} {CLASSES[key[1]]:13s} steps ref {ur:12d} ordered {uo:12d} ({uo / ur:.3f})  "
              f"wave-steps ref {cr:12d} ordered {co:12d} ({co / max(cr, 1):.3f})")


if __name__ == "__main__":
    main()
