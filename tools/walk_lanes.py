"""SIMD lane model of the light passes' walks from the oracle's per-pixel walk steps (analysis tool).

The oracle's statistics build (-DHKO_STATS) counts, per pixel, the node visits + leaf tests of every walk of
each light pass (direct_lit, emissive, indirect) by walk class (closest hit, directional any-hit, emissive
any-hit, emitter BLAS walk of select_light_candidate).  A wave runs a walk until its longest lane ends, so
with the kernels' layout (256-thread workgroups over 16x16 tiles, each wave an 8x8 sub-tile):
  wave cost     = 64 x max(steps of its lanes)       useful = sum(steps)      efficiency = useful / cost
and if a workgroup first compacted the pixels that take a walk into dense waves (ballot + LDS queue, in pixel
order), the cost is sum over its dense waves of 64 x max(steps).  Prints both per (pass, class).
usage: python tools/walk_lanes.py [config] [width height] [--frames N]
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


def main():
    import bench
    import oracle as O
    from hikari_amd import HikariSettings, Upscale, examples, frame_inputs, load_noise
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "city-4k"
    cfg = bench.CONFIGS[cfg_name]
    nums = [a for a in sys.argv[2:] if a.isdigit()]
    w, h = (int(nums[0]), int(nums[1])) if len(nums) >= 2 else (cfg["width"], cfg["height"])
    frames = int(sys.argv[sys.argv.index("--frames") + 1]) if "--frames" in sys.argv else 4
    lib = ROOT / "oracle" / "_build" / "liboracle_stats.so"
    subprocess.run(["gcc", "-O3", "-std=gnu11", "-fPIC", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", "-DHKO_STATS",
                    "-shared", "-o", str(lib), str(ROOT / "oracle" / "hk_oracle.c"), "-lm"], check=True)
    O.LIB = lib
    L = O.lib()
    scene, cam, lights = examples.SCENES[cfg["scene"]]()
    desc = scene.build()
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=cfg["spatial"], denoise=False)
    s = st.to_c()
    o = O.Oracle(desc, load_noise(), w, h, 1.0)
    n = w * h
    steps = np.zeros(3 * 4 * n, np.uint32)
    ptr = C.c_void_p.in_dll(L, "hko_pixel_steps_out")
    tot = {}
    for f in range(frames):
        steps[:] = 0
        ptr.value = steps.ctypes.data
        fi = frame_inputs(f, cam, lights, w, h)
        o.render_gbuffer(fi)
        o.render_frame(s, fi)
        ptr.value = None
        a = steps.reshape(3, 4, h, w).astype(np.int64)
        th, tw = h // 16, w // 16
        for p in range(3):
            for k in range(4):
                g = a[p, k, :th * 16, :tw * 16].reshape(th, 2, 8, tw, 2, 8).transpose(0, 3, 1, 4, 2, 5)
                g = g.reshape(th * tw, 4, 64)  # workgroup, wave, lane (wave = 8x8 sub-tile)
                useful = int(g.sum())
                if useful == 0:
                    continue
                cost = int(64 * g.max(axis=2).sum())
                flat = g.reshape(th * tw, 256)
                comp = 0
                for wg in flat[flat.max(axis=1) > 0]:
                    v = wg[wg > 0]
                    for c0 in range(0, len(v), 64):
                        comp += 64 * int(v[c0:c0 + 64].max())
                walking = int((flat > 0).sum())
                t = tot.setdefault((p, k), [0, 0, 0, 0])
                t[0] += useful
                t[1] += cost
                t[2] += comp
                t[3] += walking
    print(f"{cfg_name} {w}x{h}, frames 0..{frames - 1}")
    for (p, k), (useful, cost, comp, walking) in sorted(tot.items()):
        print(f"  {PASSES[p]:10s} {CLASSES[k]:20s} walking px/frame {walking / frames:10.0f}  steps/walk "
              f"{useful / max(walking, 1):7.1f}  lane eff {useful / cost:.3f}  compacted {useful / comp:.3f}  "
              f"wave-steps saved {1 - comp / cost:.1%}")


if __name__ == "__main__":
    main()
