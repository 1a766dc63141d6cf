"""SIMD lane efficiency of the traverse_top walks per kernel (GPU; instrumented library).

Runs a few frames of each bench config with the library built with -DHK_LANE_STATS
(make -C bevy-hikari_amd OUT=../exp_lanestats/lanestats.so BUILD=../exp_lanestats/obj
EXTRA=-DHK_LANE_STATS), once with the megakernel indirect pass and once with the wavefront one,
and writes {config: {layout: {kernel: {active, iterations, efficiency}}}} where efficiency =
active lanes / (64 x walk iterations) — the fraction of a wave's lanes doing walk work per
iteration (lanes whose walk ended or that trace no ray count as idle).  bench.py reports it next
to the roofline.  usage: HK_LIB=exp_lanestats/lanestats.so python tools/lane_stats.py out.json
"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "bevy-hikari_amd"))
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from hikari_amd import HikariRenderer, HikariSettings, Taa, Upscale, examples, frame_inputs  # noqa: E402

CONFIGS = ["cornell-1080p-nee", "scene-1080p-full", "city-4k"]
if len(sys.argv) > 2:
    CONFIGS = sys.argv[2].split(",")


def measure(config: str, wavefront: bool, warmup: int = 3, frames: int = 3) -> dict:
    cfg = bench.CONFIGS[config]
    W, H = cfg["width"], cfg["height"]
    scene, cam, lights = examples.SCENES[cfg["scene"]]()
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, taa=Taa.None_, indirect_spatial_reuse=cfg["spatial"],
                        denoise=cfg["denoise"])
    s = st.to_c()
    r = HikariRenderer(0)
    r.set_noise()
    r.upload_scene(scene)
    r.resize(W, H, 1.0)
    r.set_wavefront(wavefront)
    base = {}
    for f in range(warmup + frames):
        if f == warmup:
            base = r.lane_stats()
        fi = frame_inputs(f, cam, lights, W, H)
        r.render_gbuffer(fi)
        r.render_frame(s, fi)
        if st.denoise:
            r.denoise(s, fi)
        r.tone_sum(s)
    r.counters()  # joins the context's streams
    out = {}
    for k, (a, i) in r.lane_stats().items():
        a0, i0 = base.get(k, (0, 0))
        a, i = a - a0, i - i0
        if i:
            out[k] = {"active": a, "iterations": i, "efficiency": round(a / (64.0 * i), 4)}
    r.close()
    return out


def main():
    dst = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "gpurun_out" / "lane_stats.json"
    if "HK_LIB" not in os.environ:
        sys.exit("set HK_LIB to the -DHK_LANE_STATS build")
    res = {"note": "traverse_top SIMD lane efficiency = active lanes / (64 x walk iterations), per kernel, "
                   "frames 3..5 of each config (instrumented build; the product build has no counters)",
           "configs": {}}
    for c in CONFIGS:
        res["configs"][c] = {"megakernel": measure(c, False), "wavefront": measure(c, True)}
        print(c, json.dumps(res["configs"][c]), flush=True)
    dst.parent.mkdir(parents=True, exist_ok=True)
    dst.write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
