"""Traversal bytes per frame of the bench workloads (SURVEY §8d "Algorithmic bytes, traversal").

Counts, with the oracle's statistics build (oracle/hk_oracle.c compiled with -DHKO_STATS), every
node visited, triangle fetched, instance entered and hit_info evaluated by the light passes
(direct_lit, emissive, indirect: every traverse_top and every emitter traverse_bottom) of frames
0..F-1 of a bench config, and prices them as §8d does:
  32 B per node visited + 48 B per triangle fetched (leaf box passed) + 176 B per instance leaf
  entered + (176 + 48 + 3*32 + 80) B per hit_info.
The primary-ray G-buffer walk is not counted (its hit_info calls are reported separately).
These bytes are cache traffic (the scenes are L2/MALL resident), reported next to the HBM
roofline, never inside it.  Analysis tool: runs on the CPU here; writes profiles/traversal_bytes.json.

usage: python tools/traversal_bytes.py [--frames 15] [configs...]
"""
import argparse
import ctypes as C
import json
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "bevy-hikari_amd"))
sys.path.insert(0, str(ROOT / "oracle"))

NODE_B, TRI_B, INST_B, HIT_INFO_B = 32, 48, 176, 176 + 48 + 3 * 32 + 80
CLASSES = ["closest", "directional_any_hit", "emissive_any_hit", "emitter_blas"]


def build_stats_lib() -> Path:
    out = ROOT / "oracle" / "_build" / "liboracle_stats.so"
    out.parent.mkdir(exist_ok=True)
    subprocess.run(["gcc", "-O3", "-std=gnu11", "-fPIC", "-fopenmp", "-ffp-contract=off", "-fno-fast-math",
                    "-DHKO_STATS", "-shared", "-o", str(out), str(ROOT / "oracle" / "hk_oracle.c"), "-lm"], check=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=15, help="frames 0..F-1 (15 = one cycle of the 3/5 validation intervals)")
    ap.add_argument("configs", nargs="*", default=["cornell-1080p-nee", "scene-1080p-full", "city-4k"])
    args = ap.parse_args()

    import oracle as O
    O.LIB = build_stats_lib()
    L = O.lib()
    stats = (C.c_ulonglong * 20).in_dll(L, "hko_stats")
    hit_infos = C.c_ulonglong.in_dll(L, "hko_hit_infos")

    import bench
    import hikari_amd
    from hikari_amd import HikariSettings, Upscale, examples, frame_inputs

    path = ROOT / "profiles" / "traversal_bytes.json"
    result = json.loads(path.read_text()) if path.exists() else {"configs": {}}
    result["doc"] = __doc__.split("\n\n")[1].replace("\n", " ")
    for name in args.configs:
        cfg = bench.CONFIGS[name]
        W, H = cfg["width"], cfg["height"]
        scene, cam, lights = examples.SCENES[cfg["scene"]]()
        st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=cfg["spatial"], denoise=cfg["denoise"])
        s = st.to_c()
        o = O.Oracle(scene.build(), hikari_amd.load_noise(), W, H, 1.0)
        tot = [[0] * 5 for _ in range(4)]
        gb_infos = light_infos = rays = 0
        t0 = time.time()
        for f in range(args.frames):
            fi = frame_inputs(f, cam, lights, W, H)
            o.reset_counters()
            hit_infos.value = 0
            o.render_gbuffer(fi)
            gb_infos += hit_infos.value
            for i in range(20):
                stats[i] = 0
            hit_infos.value = 0
            o.render_frame(s, fi)  # light passes only (spatial reuse traces no rays)
            light_infos += hit_infos.value
            for k in range(4):
                for j in range(5):
                    tot[k][j] += stats[5 * k + j]
            c = o.counters()
            rays += c["traverse_top"] + c["traverse_emitter"]
        o.close()
        F = args.frames
        per = {CLASSES[k]: {"calls": tot[k][0] / F, "tlas_nodes": tot[k][1] / F, "instances_entered": tot[k][2] / F,
                            "blas_nodes": tot[k][3] / F, "triangles": tot[k][4] / F} for k in range(4)}
        nodes = sum(tot[k][1] + tot[k][3] for k in range(4)) / F
        tris = sum(tot[k][4] for k in range(4)) / F
        inst = sum(tot[k][2] for k in range(4)) / F
        infos = light_infos / F
        b = nodes * NODE_B + tris * TRI_B + inst * INST_B + infos * HIT_INFO_B
        result["configs"][name] = {
            "frames": F, "resolution": [W, H], "light_pass_queries_per_frame": rays / F,
            "nodes_per_frame": nodes, "triangles_per_frame": tris, "instances_entered_per_frame": inst,
            "hit_infos_per_frame": infos, "gbuffer_hit_infos_per_frame": gb_infos / F,
            "traversal_bytes_per_frame": int(b), "bytes_per_query": b / max(1, rays / F), "per_class": per}
        print(f"{name}: {rays / F / 1e6:.2f} M queries/frame, {nodes / 1e6:.1f} M nodes, {tris / 1e6:.2f} M tris, "
              f"{inst / 1e6:.2f} M instances, {b / 1e9:.2f} GB/frame ({time.time() - t0:.0f} s)", flush=True)
        path.write_text(json.dumps(result, indent=1) + "\n")


if __name__ == "__main__":
    main()
