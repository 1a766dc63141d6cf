"""Benchmark: bevy-hikari's headline path (per-pixel integrator [+ SVGF denoiser]) on MI355X.

BASELINE.json metric: Mrays/sec + ms/frame @1080p 1spp.  Workload at N=1 = configs[1]:
examples/cornell.rs at 1920x1080, 1 spp, traversal + NEE only (full-screen albedo, direct,
emissive and indirect temporal passes; spatial reuse and denoise off).  One "step" = one
frame: primary-ray G-buffer + hk_render_frame + tone-sum (+ denoise when enabled).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): the frame is
split over the N ranks — interleaved 8-row stripes when no pass reads neighbours (config 2:
balanced work), otherwise N contiguous row bands plus a recomputed halo (spatial reuse and the
denoiser read up to 36 rows away); each rank renders its rows, the tone-mapped RGBA16F rows are
all-gathered over RCCL (stripes are then put back in frame order on a side stream), so every
rank ends each step with the whole frame.  Total work is fixed => "strong" scaling.

Mrays/s = traversal queries of the light passes issued for the frame's own pixels
(every traverse_top + every emitter traverse_bottom of select_light_candidate; device counters,
halo rows excluded) / wall time.  This build's primary rays (the reference rasterises its G-buffer)
are reported separately (`primary_mrays`), as is the primary-equivalent rate W*H*spp / t.
`ms_per_step` is pipelined throughput (frame f's G-buffer overlaps frame f-1's light passes, its
tail frame f+1's); `latency_ms` is one frame alone with frame pipelining off (median of 10).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "bevy-hikari_amd"))

# torch first: libhikari_amd.so then binds to the HIP runtime torch already loaded (same soname,
# libamdhip64.so.7), so device pointers, streams and RCCL share one runtime in this process.
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import hikari_amd  # noqa: E402
from hikari_amd import HikariRenderer, HikariSettings, Taa, Upscale, examples, frame_inputs  # noqa: E402
from hikari_amd.bands import (aligned_bounds, band_gather_rows, band_of, equal_bounds, halo_rows,  # noqa: E402
                              peer_exchange, peer_gather, reassembly_copies, rebalance, rebalance_tiles,
                              stripe_gather_rows, tile_gather_shape, tile_grid, tile_of, tile_reassembly_copies,
                              use_stripes)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec

# Compulsory HBM bytes per pixel per launch (reference texel formats; DESIGN.md "Roofline"):
# Algorithmic HBM bytes per pixel of each kernel, (covered pixel, background pixel): the reference's
# texel / record formats each kernel must read and write once.  A background pixel
# (G-buffer depth 0) takes the passes' early exits: the temporal passes then store a zero reservoir
# into three buffers (light.wgsl:1063-1071), spatial reuse copies the temporal record.
BYTES_PER_PIXEL = {
    "gbuffer": (60, 60),             # writes position 16 + normal 4 + gradient 8 + ids 8 + velocity/uv 16
                                     # + the fused full_screen_albedo's RGBA16F 8
    "full_screen_albedo": (52, 52),  # reads 44 B of G-buffer, writes RGBA16F
    # G 44 + reservoir read 64 + write 64 + variance 4 + render 8 | position 16 + 3 x 64 + 4 + 8; direct_lit's
    # background pixels store only their temporal record (the emissive pass rewrites the shared spatial pair)
    "direct_lit": (184, 92),
    "direct_emissive": (184, 220),
    "direct_lit_emissive": (324, 296),  # both passes in one launch (k_direct_fused): the G-buffer read once
    "light_merged": (508, 516),          # k_light_merged: direct_lit_emissive + indirect_lit_ambient
    "indirect_lit_ambient": (184, 220),
    "indirect_multiple_bounces": (184, 220),
    "indirect_wavefront": (184, 220),    # the same compulsory streams (queues / hit records are extra traffic)
    # G 40 + temporal 64 + previous spatial 64 + spatial 64 + var 4 + render 8 | position 16 + spatial 64 +
    # render 8 (the background record is repacked from registers: the temporal pass just stored it)
    "indirect_spatial_reuse": (244, 88),
    "emissive_spatial_reuse": (244, 88),
    "demodulation": (148, 148),      # reads G-buffer normal 4 + position 16 (RGBA32F texel, .w used) + ids 8 +
                                     # depth gradient 8 + albedo 8 + 3 x (render 8 + variance 4); writes geom 32
                                     # (the levels' per-pixel geometry) + 3 x (internal 8 + ivar 4)
    "denoise": (120, 56),            # geom 32 + 3 x (ivar 4 + input 8 + output 8) (+ albedo 8 at L3) | geom 32 + 3 x 8
    "tone_mapping": (32, 32),
}


# Background store elision (hk_kernels.hip bg_elide): in steady state a background pixel of the
# fused direct/emissive launch and of the indirect pass reads its position texel (16) and its mask
# byte (1) and stores nothing — its targets already hold the constant zero words — except, when the
# channel's spatial reuse runs (it rewrites the pair with other bits), both spatial-pair records
# (2 x 64); a G-buffer miss reads its mask byte only.  Not with option bg_elision = 0.
BG_ELIDED_BYTES = {"gbuffer": (None, 1, 1),  # a miss: its mask byte (the slot already holds the zero texels)
                   "direct_lit_emissive": ("emissive_spatial_reuse", 17, 145),
                   "indirect_lit_ambient": ("indirect_spatial_reuse", 17, 145),
                   "indirect_multiple_bounces": ("indirect_spatial_reuse", 17, 145),
                   "indirect_wavefront": ("indirect_spatial_reuse", 17, 145)}


def kernel_bytes(name: str, covered_px: float, background_px: float, settings=None) -> float:
    """Bytes of one launch over covered_px + background_px pixels: the reference kernel's algorithmic
    bytes (settings None), or what this build's launch must move with background store elision on
    (settings given: the elided background stores depend on the spatial reuse flags)."""
    if name == "light_merged":  # k_light_merged: the fused direct/emissive pass and the indirect pass in one launch
        return (kernel_bytes("direct_lit_emissive", covered_px, background_px, settings) +
                kernel_bytes("indirect_lit_ambient", covered_px, background_px, settings))
    c, b = BYTES_PER_PIXEL.get(name, (0, 0))
    if settings is not None and name in BG_ELIDED_BYTES:
        flag, alone, with_pair = BG_ELIDED_BYTES[name]
        b = with_pair if flag and getattr(settings, flag) else alone
    return c * covered_px + b * background_px

CONFIGS = {
    # BASELINE.json configs[1]
    "cornell-1080p-nee": dict(scene="cornell", width=1920, height=1080, spatial=False, denoise=False,
                              workload="examples/cornell.rs 1920x1080 1spp, traversal + NEE only "
                                       "(albedo + direct + emissive + indirect temporal; denoise off)"),
    # configs[2]
    "scene-1080p-full": dict(scene="scene", width=1920, height=1080, spatial=True, denoise=True,
                             workload="examples/scene.rs layout (City proxy geometry) 1920x1080 1spp + ReSTIR "
                                      "temporal/spatial + SVGF denoise"),
    # configs[3]
    "city-4k": dict(scene="city", width=3840, height=2160, spatial=True, denoise=True,
                    workload="examples/city.rs layout (City proxy houses) 3840x2160 1spp, row bands + RCCL all-gather"),
    # city.rs with its emissive sphere rotating every frame (sphere_rotate_system, city.rs:290-294:
    # rotate_local_z(0.2 rad/s x 1/60 s)): instances, TLAS, emissives and light BVH rebuilt on
    # the GPU each frame (hk_update_instances) before rendering
    "city-4k-dynamic": dict(scene="city", width=3840, height=2160, spatial=True, denoise=True, dynamic=True,
                            workload="examples/city.rs layout (City proxy houses) 3840x2160 1spp, rotating "
                                     "emissive sphere: GPU instance/TLAS/light-BVH rebuild every frame"),
    # configs[1] / configs[3] under camera motion: the examples' orbit camera (OrbitCameraBundle,
    # cornell.rs:56-60, city.rs:134-138) yawing 0.5 deg per frame (examples.orbit).  Reprojection is no
    # longer the identity, so the fused direct/emissive launch is off and the direct pair's background stores
    # stay; background store elision of each pass's own targets (and of the indirect pair) stays on
    "cornell-1080p-nee-orbit": dict(scene="cornell", width=1920, height=1080, spatial=False, denoise=False, orbit=True,
                                    workload="examples/cornell.rs 1920x1080 1spp, traversal + NEE only, orbit "
                                             "camera (0.5 deg/frame)"),
    "city-4k-orbit": dict(scene="city", width=3840, height=2160, spatial=True, denoise=True, orbit=True,
                          workload="examples/city.rs layout (City proxy houses) 3840x2160 1spp, orbit camera "
                                   "(0.5 deg/frame)"),
    # configs[0]: the reference's CPU-runnable case (a parity case; bench line for completeness)
    "cornell-256-all": dict(scene="cornell", width=256, height=256, spatial=True, denoise=True,
                            workload="examples/cornell.rs 256x256 1spp, all passes (ReSTIR temporal/spatial "
                                     "+ SVGF denoise)"),
    # per-frame fixed cost probe (launch / host overhead floor); not a BASELINE config
    "cornell-tiny-overhead": dict(scene="cornell", width=64, height=64, spatial=False, denoise=False,
                                  workload="examples/cornell.rs 64x64 (host/launch overhead probe)"),
    # configs[4]: 16 integrator sub-frames (each one reference frame) accumulated per displayed frame,
    # one all-gather per displayed frame
    "city-4k-16spp": dict(scene="city", width=3840, height=2160, spatial=True, denoise=True, spp=16, wavefront=True,
                          workload="examples/city.rs layout (City proxy houses) 3840x2160 16spp accumulation "
                                   "(16 sub-frames per displayed frame; static camera: the G-buffer traced once per "
                                   "displayed frame, gbuffer_reuse), wavefront material-sorted indirect "
                                   "shading, row bands + RCCL all-gather"),
}


def cpu_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 16))  # the GPU box grants 16 host cores to one GPU


def cpu_baseline(scene_desc, camera_at, lights, st, w, h, budget_s: float) -> dict:
    """The oracle (C restatement, OpenMP) on the same workload, bounded to ~budget_s seconds."""
    sys.path.insert(0, str(ROOT / "oracle"))
    from oracle import Oracle  # test-infrastructure checker, used here only as the CPU baseline
    threads = cpu_threads()
    o = Oracle(scene_desc, hikari_amd.load_noise(), w, h, st.upscale.ratio(), threads=threads)
    s = st.to_c()
    rays = primary = 0
    frames = 0
    t0 = time.perf_counter()
    while frames < 64:
        cam, prev = camera_at(frames)
        fi = frame_inputs(frames, cam, lights, w, h, previous_camera=prev)
        o.reset_counters()
        o.render_gbuffer(fi)
        o.render_frame(s, fi)
        if st.denoise:
            o.denoise(s, fi)
        o.tone_sum(s)
        c = o.counters()
        rays += c["traverse_top"] + c["traverse_emitter"]
        primary += c["primary"]
        frames += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    o.close()
    return {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "ms_per_frame": round(dt / frames * 1e3, 1), "primary_mrays": round(primary / dt / 1e6, 3),
            "sample": f"same workload, frames 0..{frames - 1} ({frames} frames, {dt:.1f} s) on the CPU oracle "
                      f"(C restatement of light.wgsl/denoise.wgsl, {threads} OpenMP threads)"}


def load_pmc_traffic(config: str, kernel: str):
    """HBM bytes per launch of `kernel` under `config` from the committed rocprofv3 --pmc summary
    (profiles/pmc_traffic.json, written by tools/pmc_summary.py), if present."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        return d["configs"][config]["kernels"][kernel].get("hbm_bytes_per_launch")
    except (KeyError, ValueError):
        return None


def load_valu_issue(config: str, kernel: str):
    """VALU instructions per launch of `kernel` under `config` (rocprofv3 --pmc SQ_INSTS_VALU, every kernel alone) from
    the committed profiles/valu_issue.json (tools/valu_summary.py), if present."""
    p = ROOT / "profiles" / "valu_issue.json"
    if not p.exists():
        return None
    try:
        return json.loads(p.read_text())["configs"][config]["kernels"][kernel]["valu_per_launch"]
    except (KeyError, ValueError):
        return None


def load_traversal_bytes(config: str):
    """Traversal bytes per frame of `config` (nodes, triangles, instances, hit_info of the
    light passes, priced in reference record sizes) from the committed profiles/traversal_bytes.json
    (written offline by tools/traversal_bytes.py), if present.  Cache traffic, not HBM bytes."""
    p = ROOT / "profiles" / "traversal_bytes.json"
    if not p.exists():
        return None
    try:
        return json.loads(p.read_text())["configs"][config]["traversal_bytes_per_frame"]
    except (KeyError, ValueError):
        return None


def load_lane_efficiency(config: str, wavefront: bool):
    """traverse_top SIMD lane efficiency per kernel (active lanes / (64 x walk iterations)) of `config`
    from the committed instrumented-build measurement (profiles/r02/lane_stats.json, tools/lane_stats.py);
    the 16-spp config's sub-frames are city-4k frames."""
    p = ROOT / "profiles" / "r02" / "lane_stats.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())["configs"][{"city-4k-16spp": "city-4k"}.get(config, config)]
        return {k: v["efficiency"] for k, v in d["wavefront" if wavefront else "megakernel"].items()}
    except (KeyError, ValueError):
        return None


def valu_issue(config: str, kernel: str, dur_ms: float):
    valu = load_valu_issue(config, kernel)
    if valu is None or not dur_ms:
        return None
    floor = valu * 2 / (1024 * 2.4e9) * 1e3
    return {"valu_per_launch": valu, "alu_floor_ms": round(floor, 4), "valu_frac": round(floor / dur_ms, 4),
            "clock_ghz": 2.4, "simds": 1024}


def json_stdout():
    """The bench's stdout carries its one JSON line only: file descriptor 1 is pointed at stderr for the
    rest of the run (RCCL prints its version banner on descriptor 1 when the communicator is created), and the
    JSON line goes to the original stdout through the returned file."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(fd, "w")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--config", default="cornell-1080p-nee", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU-baseline work (0 = skip)")
    args = ap.parse_args()
    out = json_stdout()

    cfg = CONFIGS[args.config]
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus and world == 1 and args.gpus != 1:
        print(f"warning: --gpus {args.gpus} without a distributed launcher; running 1 rank", file=sys.stderr)
    # HK_BENCH_REHEARSAL=1: rehearse the multi-rank path on ONE GPU (every rank on cuda:0, gloo
    # collectives through host memory) — a correctness check of the band / gather / reduction
    # logic, never a measurement.  The real N-GPU run uses RCCL over xGMI.
    rehearsal = os.environ.get("HK_BENCH_REHEARSAL") == "1"
    # HK_BENCH_DIST=1: the collective path at world size 1 too (RCCL init, the per-frame all-gather and the
    # reductions on one GPU) — a check of the RCCL calls on the hardware; its line is not the N=1 result
    dist_on = world > 1 or os.environ.get("HK_BENCH_DIST") == "1"
    device = 0 if rehearsal else local
    torch.cuda.set_device(device)
    # the context first: HIP maps streams onto the process's hardware queues in creation order, and the
    # context's streams are tuned for the mapping they get when nothing else created streams before them
    # (DESIGN §4); RCCL's communicator (created eagerly below) and torch's stream pool come after
    r = HikariRenderer(device)
    if dist_on:
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    W, H = cfg["width"], cfg["height"]
    scene, cam, lights = examples.SCENES[cfg["scene"]]()
    desc = scene.build()
    # SURVEY §8d common settings: SMAA TU4x at ratio 1.0 (s = S), taa None (no prepass jitter)
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, taa=Taa.None_, indirect_spatial_reuse=cfg["spatial"],
                        denoise=cfg["denoise"])
    s = st.to_c()

    # rows of this rank (hikari_amd/bands.py): interleaved stripes, or a contiguous band + halo
    stripes = dist_on and use_stripes(cfg["spatial"], cfg["denoise"])
    # HK_BENCH_OPTS="key=value,..." (or "+"-separated): runtime options (hk_set_option) for A/B runs (tools/ab.sh); the
    # defaults are the tuned configuration
    bench_opts = {kv.split("=")[0]: float(kv.split("=")[1])
                  for kv in os.environ.get("HK_BENCH_OPTS", "").replace("+", ",").split(",") if kv}
    # G-buffer reuse (skipping the primary-ray trace when the slot already holds the frame's planes) only
    # for the sub-frames of an accumulated frame (configs[4]); a 1-spp frame traces its G-buffer every time,
    # as the reference rasterises its prepass every frame, even with the static camera of the bench
    r.set_options({"gbuffer_reuse": 1 if cfg.get("spp", 1) > 1 else 0, **bench_opts})
    r.set_noise()
    r.upload_scene(scene)
    r.set_band_halo(halo_rows(cfg["spatial"], cfg["denoise"]))
    # the indirect pass as a wavefront with material-sorted shading (hk_set_wavefront); HK_BENCH_WAVEFRONT
    # overrides the config (0 = megakernel, 1 = wavefront) for comparisons
    wavefront = os.environ.get("HK_BENCH_WAVEFRONT", "1" if cfg.get("wavefront") else "0") == "1"
    r.set_wavefront(wavefront)
    bounds, balance = None, []
    # 2-D tiles (north_star: "frames tile-partition across the 8 GPUs"; bands.tile_grid: 2x2 at N = 4, 4x2 at N = 8)
    # for the frames with neighbour reads with HK_BENCH_DECOMP=tiles.  Default: cost-balanced row bands, which measured
    # faster on the bench scenes (their cost sits in the middle rows, and N balanced bands follow it more closely than
    # N / 2 balanced row bands of 2 tiles: scene N = 4 0.609 vs 0.661 ms, N = 8 0.448 vs 0.498; city N = 8 0.795 vs
    # 0.804; profiles/r06/c7, c8)
    tiles = dist_on and not stripes and tile_grid(world)[1] > 1 and os.environ.get("HK_BENCH_DECOMP", "bands") == "tiles"
    col_bounds, my_tile, all_tiles = None, None, None
    if stripes:
        r.resize_striped(W, H, rank, world)
        band, gather_index = stripe_gather_rows(world, H)  # padded rows per rank
    elif tiles:
        # cost-balanced tiles (bands.rebalance_tiles): the same calibration as the bands, each rank timing its tile
        ny, nx = tile_grid(world)
        bounds, col_bounds = aligned_bounds(ny, H), [aligned_bounds(nx, W)] * ny
        for _ in range(int(os.environ.get("HK_BENCH_BALANCE", "5"))):
            t = tile_of(rank, world, W, H, bounds, col_bounds)
            r.resize_tile(W, H, t.x0, t.cols, t.y0, t.rows)
            for f in range(6):
                if f == 3:
                    torch.cuda.synchronize()
                    t_cal = time.perf_counter()
                fi = frame_inputs(f, cam, lights, W, H)
                r.render_gbuffer(fi)
                r.render_frame(s, fi)
                if st.denoise:
                    r.denoise(s, fi)
                r.tone_sum(s)
            r.sync()
            torch.cuda.synchronize()
            t_cal = torch.tensor([(time.perf_counter() - t_cal) / 3.0], dtype=torch.float64,
                                 device="cpu" if rehearsal else "cuda")
            times = torch.zeros(world, dtype=torch.float64, device=t_cal.device)
            dist.all_gather_into_tensor(times, t_cal)
            times = times.cpu().numpy()
            balance.append({"rows": list(bounds), "cols": [list(c) for c in col_bounds],
                            "ms": [round(float(v) * 1e3, 4) for v in times]})
            bounds, col_bounds = rebalance_tiles(bounds, col_bounds, times)
        all_tiles = [tile_of(k, world, W, H, bounds, col_bounds) for k in range(world)]
        my_tile = all_tiles[rank]
        r.resize_tile(W, H, my_tile.x0, my_tile.cols, my_tile.y0, my_tile.rows)
        tile_rows, tile_cols = tile_gather_shape(bounds, col_bounds)
        band = tile_rows
    elif dist_on:
        # cost-balanced row bands (bands.rebalance): HK_BENCH_BALANCE rounds (default 5) of a short
        # calibration on the current bands — frames 0..5 rendered, 3..5 timed per rank, the times all-gathered
        # — each moving the boundaries to equal measured cost.  Then every rank starts the run from frame 0
        # on its final band (hk_resize zero-fills the reservoirs, as at the start of any run).
        bounds = equal_bounds(world, H)
        for _ in range(int(os.environ.get("HK_BENCH_BALANCE", "5")) if world > 1 else 0):
            b = band_of(rank, world, H, bounds)
            r.resize(W, H, 1.0, b.y0, b.rows)
            for f in range(6):
                if f == 3:
                    torch.cuda.synchronize()
                    t_cal = time.perf_counter()
                fi = frame_inputs(f, cam, lights, W, H)
                r.render_gbuffer(fi)
                r.render_frame(s, fi)
                if st.denoise:
                    r.denoise(s, fi)
                r.tone_sum(s)
            r.sync()
            torch.cuda.synchronize()
            t_cal = torch.tensor([(time.perf_counter() - t_cal) / 3.0], dtype=torch.float64,
                                 device="cpu" if rehearsal else "cuda")
            times = torch.zeros(world, dtype=torch.float64, device=t_cal.device)
            dist.all_gather_into_tensor(times, t_cal)
            times = times.cpu().numpy()
            balance.append({"bounds": list(bounds), "ms": [round(float(t) * 1e3, 4) for t in times]})
            bounds = rebalance(bounds, times)
        b = band_of(rank, world, H, bounds)
        r.resize(W, H, 1.0, b.y0, b.rows)
        band, gather_index = band_gather_rows(bounds)
    else:
        band = H
        r.resize(W, H, 1.0)
    row0, rows, core0, core_rows = r.band_info()
    # How the ranks' rows reach every rank (HK_BENCH_GATHER): "peer" (the default) sends each rank's rows straight
    # to every peer while receiving every peer's rows on that peer's own xGMI link (batch_isend_irecv: N-1
    # transfers of one band each at once, instead of a ring moving (N-1)/N of the frame through one link).  Row
    # bands are exchanged in place in a whole-frame buffer (bands.peer_exchange: each band lands in its rows, no
    # reassembly); the interleaved stripes' padded rows go into the all-gather's layout (bands.peer_gather) and are
    # put back in frame order as before.  "ring": one all-gather of the padded rows (RCCL's ring), reassembled on a
    # side stream when not already in frame order (stripes, uneven bands).
    # Tiles: each rank's core rectangle goes into a padded (rows, cols) part of the largest tile's size, the parts are
    # gathered per peer (bands.peer_gather, as the stripes') or by the ring all-gather, and put back in frame order by
    # one strided copy per tile (bands.tile_reassembly_copies) on the side stream.
    gather_mode = os.environ.get("HK_BENCH_GATHER", "peer")
    peer = dist_on and not stripes and not tiles and gather_mode == "peer"
    peer_stripes = dist_on and (stripes or tiles) and gather_mode == "peer"
    my_y0 = band_of(rank, world, H, bounds).y0 if peer else 0
    reorder = True if tiles else ((dist_on and not peer and not np.array_equal(gather_index, np.arange(H))
                                   if (stripes or bounds is not None) else False))
    part_w = tile_cols if tiles else W

    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    # The band copy and the all-gather run on a communication stream: hk_copy_output_rows on a stream other
    # than the frame stream waits (device-side) only for the work that produced the plane, and the frame
    # stream never waits for the copy or the gather, so frame pipelining is kept on every frame.
    comm = torch.cuda.Stream() if dist_on else None
    # double-buffered band / gathered frame: the all-gather of frame f runs on RCCL's stream
    # while frame f+1 renders; a buffer is reused only after its previous gather completed
    band_t = [torch.zeros((band, part_w, 4), dtype=torch.float16, device="cuda") for _ in range(2)] if not peer else None
    full_t = [torch.empty((world * band, part_w, 4), dtype=torch.float16, device="cuda") for _ in range(2)] \
        if dist_on and not peer else None
    peer_t = [torch.zeros((H, W, 4), dtype=torch.float16, device="cuda") for _ in range(2)] if peer else None
    # world size 1: the per-peer exchange sends the band to this rank itself (bands.peer_exchange self_buf), so the
    # line carries the RCCL point-to-point group's launch, transfer and device-side wait of every frame
    self_t = [torch.empty((core_rows, W, 4), dtype=torch.float16, device="cuda") for _ in range(2)] \
        if peer and world == 1 and not rehearsal else None
    pending = [None, None]
    if reorder:  # stripes / uneven bands back in frame order, on a side stream after each gather
        frame_t = [torch.empty((H, W, 4), dtype=torch.float16, device="cuda") for _ in range(2)]
        index_t = None if tiles else torch.from_numpy(gather_index).to("cuda")

        # one strided row copy per rank (bands.reassembly_copies); torch.index_select over the frame's row
        # indices took ~0.1 ms per 1080p frame (per-element index arithmetic), the row copies a few microseconds
        if tiles:
            row_copies = [tile_reassembly_copies(frame_t[k], full_t[k].view(world, band, part_w, 4), all_tiles)
                          for k in range(2)]
        else:
            row_copies = [reassembly_copies(frame_t[k], full_t[k], world, H, band, None if stripes else bounds)
                          for k in range(2)] if H % 8 == 0 else None
        side = torch.cuda.Stream()
        reorder_done = [None, None]

    spp = cfg.get("spp", 1)
    shown = hikari_amd._abi.OUT_TONE_MAPPED if spp == 1 else hikari_amd._abi.OUT_ACCUMULATED
    # 1-spp frames gather frame f's rows after frame f + 1 has been queued (HK_OUT_TONE_MAPPED_PREVIOUS): the
    # copy and the all-gather wait for frame f's tail, and their wait packets sit in hardware queues that the
    # context's streams share (4 queues per process); queued behind frame f + 1's passes they hold back only
    # frame f + 2's work, by which time frame f's tail has long ended.  Queued right after frame f, they held
    # frame f + 1's G-buffer and light passes until frame f's tail ended (cornell world-1 0.58 vs 0.43 ms).
    delay = spp == 1

    # camera of frame f and of frame f - 1 (None: static, PreviousViewUniform = the current view)
    if cfg.get("orbit"):
        target = examples.ORBIT_TARGETS[cfg["scene"]]

        def camera_at(f):
            return examples.orbit(cam, target, f), (examples.orbit(cam, target, f - 1) if f > 0 else None)
    else:
        def camera_at(f):
            return cam, None

    dynamic = cfg.get("dynamic", False)
    if dynamic:
        models0, aabbs = scene.instance_models(), scene.instance_local_aabbs()
        sphere = [i for i, (m, _, _) in enumerate(scene.instances)
                  if len(scene.meshes[m].positions) == 37 * 19][-1]  # the UV sphere (36 x 18 sectors)

    def step(f):
        if dynamic:  # rotate_local_z(0.2 * dt): model = model0 * Rz(angle)
            a = 0.2 * (f / 60.0)
            rz = np.array([[np.cos(a), -np.sin(a), 0, 0], [np.sin(a), np.cos(a), 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]])
            models = models0.copy()
            m0 = models0[sphere].reshape(4, 4).T  # column-major storage -> matrix
            models[sphere] = (m0 @ rz).T.reshape(16).astype(np.float32)
            r.update_instances(models, aabbs, sp)
        # one displayed frame = spp integrator sub-frames, each exactly one reference frame
        for k in range(spp):
            c, prev = camera_at(f * spp + k)
            fi = frame_inputs(f * spp + k, c, lights, W, H, previous_camera=prev)
            r.render_gbuffer(fi, sp)
            r.render_frame(s, fi, sp)
            if st.denoise:
                r.denoise(s, fi, sp)
            r.tone_sum(s, sp)
            if spp > 1:
                r.accumulate(k == 0, sp)
        if spp > 1:
            r.resolve_accumulation(sp)
        if dist_on:
            if not delay:
                gather(f, shown)
            elif f - 1 > gathered[0]:
                gather(f - 1, hikari_amd._abi.OUT_TONE_MAPPED_PREVIOUS)

    gathered = [-1]  # the latest frame whose rows were gathered
    # HK_BENCH_COMM (diagnostic of the collective path's cost, never a result): "copy" = the band copy only,
    # "noreorder" = copy + all-gather without the frame-order reorder, "none" = nothing
    comm_mode = os.environ.get("HK_BENCH_COMM", "full")

    def wait_all(p):
        for q in (p if isinstance(p, list) else [p]):
            q.wait()

    def gather(f, plane):
        gathered[0] = f
        if comm_mode == "none":
            return
        k = f & 1
        if peer:
            with torch.cuda.stream(comm):
                if pending[k] is not None:
                    wait_all(pending[k])  # device-side: the comm stream waits for that exchange
                r.copy_output_rows(plane, core0, core_rows, peer_t[k][my_y0].data_ptr(), False, comm.cuda_stream)
                if comm_mode == "copy":
                    return
                if rehearsal:  # gloo on one GPU: the exchange through host copies
                    host = peer_t[k].cpu()
                    wait_all(peer_exchange(host, bounds, rank, world))
                    peer_t[k].copy_(host)
                else:
                    pending[k] = peer_exchange(peer_t[k], bounds, rank, world, None if self_t is None else self_t[k])
            return
        with torch.cuda.stream(comm):
            if pending[k] is not None:
                wait_all(pending[k])  # device-side: the comm stream waits for that gather
            if reorder and reorder_done[k] is not None:
                comm.wait_event(reorder_done[k])  # full_t[k] was read by the reorder of frame f - 2
            if tiles:  # the core rectangle into the padded part (pitch: the part's row)
                r.copy_output_rect(plane, core0, core_rows, my_tile.x0, my_tile.cols, band_t[k].data_ptr(),
                                   part_w * 8, False, comm.cuda_stream)
            else:
                r.copy_output_rows(plane, core0, core_rows, band_t[k].data_ptr(), False, comm.cuda_stream)
            if comm_mode == "copy":
                return
            if rehearsal:
                if peer_stripes:
                    host = torch.empty((world * band, part_w, 4), dtype=torch.float16)
                    wait_all(peer_gather(host, band_t[k].cpu(), rank, world))
                    full_t[k].copy_(host)
                else:
                    parts = [torch.empty((band, part_w, 4), dtype=torch.float16) for _ in range(world)]
                    dist.all_gather(parts, band_t[k].cpu())
                    full_t[k].copy_(torch.cat(parts))
            elif peer_stripes:
                pending[k] = peer_gather(full_t[k], band_t[k], rank, world, self_transfer=world == 1)
            else:
                pending[k] = dist.all_gather_into_tensor(full_t[k], band_t[k], async_op=True)
        if reorder and comm_mode != "noreorder":
            with torch.cuda.stream(side):
                if pending[k] is not None:
                    wait_all(pending[k])
                else:
                    side.wait_stream(comm)
                if row_copies is not None:
                    for dst, src in row_copies[k]:
                        dst.copy_(src)
                else:
                    torch.index_select(full_t[k], 0, index_t, out=frame_t[k])
                reorder_done[k] = side.record_event()

    def drain(last):
        if delay and last > gathered[0]:  # the last queued frame's rows (no frame follows it)
            gather(last, shown)
        for k in range(2):
            if pending[k] is not None:
                wait_all(pending[k])
                pending[k] = None
        torch.cuda.current_stream().wait_stream(comm)
        if reorder:
            torch.cuda.current_stream().wait_stream(side)

    for f in range(args.warmup):
        step(f)
    if dist_on:
        drain(args.warmup - 1)
        dist.barrier()
    torch.cuda.synchronize()
    r.reset_counters()
    # per-kernel HIP events on every 4th frame of the timed region (frame_number % 4 == 0): the
    # averages the roofline needs, without event records perturbing the other frames
    r.set_kernel_timing_interval(max(1, min(args.steps, int(os.environ.get("HK_BENCH_TIMING_EVERY", "4")))))
    r.enable_kernel_timing(True)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for f in range(args.warmup, args.warmup + args.steps):
        step(f)
    if dist_on:
        drain(args.warmup + args.steps - 1)  # every timed frame's gather is complete inside the timed region
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timing = r.kernel_timing()
    # fraction of the rank's pixels with geometry (G-buffer depth > 0): background pixels take the
    # passes' early exits and move different bytes (BYTES_PER_PIXEL); read after the timed region
    depth = r.output(11).view(np.float32)
    if tiles:  # the tile's columns + halo (the planes are full width; other columns are never computed)
        hx = halo_rows(cfg["spatial"], cfg["denoise"])
        depth = depth.reshape(rows, W, 4)[:, max(0, my_tile.x0 - hx): my_tile.x0 + my_tile.cols + hx]
    depth = depth.reshape(-1, 4)[:, 3]
    coverage = float((depth >= np.finfo(np.float32).eps).mean())
    c = r.counters()
    rays = c["traverse_top"] + c["traverse_emitter"]
    primary = c["primary"] - r.primary_reused()  # rays traced (G-buffer reuse skips static sub-frames)
    if dist_on:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearsal else "cuda")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
        n = torch.tensor([rays, primary], dtype=torch.float64, device="cpu" if rehearsal else "cuda")
        dist.all_reduce(n, op=dist.ReduceOp.SUM)
        rays, primary = int(n[0].item()), int(n[1].item())

    # per-frame latency: frames alone (frame pipelining off), each bracketed by a device sync
    latency = None
    if world == 1 and not dynamic:
        saved = r.set_options({"gbuffer_pipeline": 0, "tail_pipeline": 0})
        r.enable_kernel_timing(False)
        f0 = args.warmup + args.steps
        times = []
        for f in range(f0, f0 + 10):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            step(f)
            r.sync(sp)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t1)
        latency = float(np.median(times)) * 1e3
        r.set_options(saved)

    # after the timed region: a few frames with every kernel alone on the GPU (no channel fork, no
    # frame pipelining), so the roofline can also quote the dominant kernel's isolated duration
    isolated = None
    if world == 1 and spp == 1 and not dynamic:
        saved = r.set_options({"channel_streams": 0, "gbuffer_pipeline": 0, "tail_pipeline": 0})
        r.set_kernel_timing_interval(1)
        r.enable_kernel_timing(True)
        f0 = args.warmup + args.steps + 10
        for f in range(f0, f0 + 8):
            step(f)
        torch.cuda.synchronize()
        isolated = r.kernel_timing()
        r.enable_kernel_timing(False)
        r.set_options(saved)

    if rank == 0:
        ms = elapsed / args.steps * 1e3
        mrays = rays / elapsed / 1e6
        # Roofline of the dominant kernel, one definition: the kernel with the largest GPU
        # time per frame when it runs alone (isolated frames; the timed region's overlapped durations
        # when no isolated frames exist: bands, accumulation, dynamic scenes).
        #   bytes_per_launch = SURVEY §8(d)'s reference-format bytes per pixel x the launch's pixels
        #   achieved = bytes_per_launch / duration_ms, frac = achieved / 8 TB/s
        #   traffic  = PMC-measured HBM bytes per launch (steady-state dispatches, profiles/pmc_traffic.json),
        #              hbm_frac = traffic / duration_ms / 8 TB/s: the bandwidth the launch really draws
        launches_per_frame = {"denoise": 4}
        source = isolated if isolated else timing
        per_frame = {k: v * launches_per_frame.get(k, 1) for k, v in source.items()}
        dom = max(per_frame, key=per_frame.get)
        pix = (depth.size // rows) * rows if tiles else W * rows
        cov_px, bg_px = pix * coverage, pix * (1.0 - coverage)
        # the reference kernel's algorithmic bytes for this frame: its covered pixels' streams plus its
        # background pixels' constant stores (BYTES_PER_PIXEL (covered, background); e.g. indirect_lit_ambient
        # 184 / 220 B).  Round 3 priced every pixel at the covered rate; that figure is kept in diagnostics.
        ref_bytes = int(kernel_bytes(dom, cov_px, bg_px))
        r03_bytes = int(BYTES_PER_PIXEL.get(dom, (0, 0))[0] * pix)
        dur = source[dom]
        achieved = ref_bytes / (dur * 1e-3) / 1e9
        elide = r.get_option("bg_elision") != 0
        # the committed PMC numbers are per launch of a whole 1-GPU frame; a band launch differs
        traffic = load_pmc_traffic(args.config, dom) if world == 1 else None
        result = {
            "metric": "Mrays/sec + ms/frame @1080p 1spp; cornell & city scenes, 1/2/4/8 GPU",
            "value": round(mrays, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic ({} camera; reference assets: cornell.glb, blue noise)".format(
                "orbiting" if cfg.get("orbit") else "static"),
            "latency_ms": None if latency is None else round(latency, 4),
            "primary_mrays": round(primary / elapsed / 1e6, 2),
            "primary_equivalent_mrays": round(W * H * spp * args.steps / elapsed / 1e6, 2),
            "config": {"workload": cfg["workload"], "resolution": [W, H], "spp": spp,
                       "indirect": "wavefront material-sorted" if wavefront else "megakernel",
                       # background pixels' constant stores skipped where their targets already hold
                       # them (every buffer keeps the reference's bits; option bg_elision = 0: off)
                       "background_store_elision": elide,
                       "options": {k: v for k, v in r.options().items()},
                       "rays_per_frame": int(rays // (args.steps * spp)),
                       "primary_rays_per_frame": int(primary // (args.steps * spp)),
                       "parallelism": (f"interleaved 8-row stripes x{world}" if stripes else
                                       "cost-balanced {}x{} tiles".format(*tile_grid(world)) if tiles else
                                       f"cost-balanced row-bands x{world}") +
                                      ((" + gloo rehearsal on one GPU" if rehearsal else
                                        " + RCCL per-peer exchange" if gather_mode == "peer" else " + RCCL all-gather"))
                                      if world > 1 else
                                      (f"single GPU through the RCCL path (world size 1, " +
                                       ("per-peer exchange as an RCCL self send/recv of the frame)"
                                        if peer or peer_stripes else
                                        f"{gather_mode} gather)")
                                       if dist_on else "single GPU"),
                       "band_bounds": None if bounds is None else [int(v) for v in bounds],
                       "tile_col_bounds": None if col_bounds is None else [[int(v) for v in c] for c in col_bounds],
                       "band_calibration": balance or None},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "hbm_frac": None if traffic is None else
                         round(traffic / (dur * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "bytes_per_launch": ref_bytes, "bytes_per_pixel": list(BYTES_PER_PIXEL.get(dom, (0, 0))),
                         "pixels_per_launch": pix, "covered_pixels": int(cov_px), "duration_ms": round(dur, 4),
                         "duration": "isolated" if isolated else "in frame (overlapped)",
                         # the traversal kernels' other bound: vector issue.  A wave64 VALU instruction holds its SIMD's
                         # 32-lane ALU for 2 cycles (one wave alone issues one per 4), so the launch needs at least
                         # valu x 2 / (1024 SIMDs x 2.4 GHz) of ALU time; valu_frac = that floor / the measured duration
                         # (profiles/valu_issue.json: PMC SQ_INSTS_VALU per launch of the kernel alone)
                         "valu_issue": valu_issue(args.config, dom, dur) if world == 1 else None},
            "kernel_ms": {k: round(v, 4) for k, v in timing.items()},
            # each kernel alone on the GPU (the untimed isolated frames after the timed region)
            "isolated_kernel_ms": None if not isolated else {k: round(v, 4) for k, v in isolated.items()},
            # context for the roofline (not fractions of it): the bytes the build's launch must move
            # (background store elision skips constant stores), the share of covered pixels, and all
            # of a frame's compulsory bytes over the frame time
            "diagnostics": {"coverage": round(coverage, 4),
                            "moved_bytes_per_launch": int(kernel_bytes(dom, cov_px, bg_px, st if elide else None)),
                            # round 3's roofline bytes (every pixel at the covered rate) and its fraction
                            "r03_bytes_per_launch": r03_bytes,
                            "r03_frac": round(r03_bytes / (dur * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                            "frame_compulsory_bytes": int(sum(kernel_bytes(k, cov_px, bg_px) *
                                                              launches_per_frame.get(k, 1) for k in timing) * spp)},
        }
        tb = load_traversal_bytes(args.config) if world == 1 and spp == 1 else None
        if tb is not None:
            # SURVEY §8d's second component: node / triangle / instance / hit_info bytes of the light
            # passes, priced in reference record sizes (L1/L2/MALL traffic: the scene is cache resident)
            result["diagnostics"]["frame_traversal_bytes"] = tb
        lanes = load_lane_efficiency(args.config, wavefront)
        if lanes is not None:
            result["diagnostics"]["lane_efficiency"] = lanes
        if world == 1 and args.cpu_budget > 0:
            result["cpu_baseline"] = cpu_baseline(desc, camera_at, lights, st, W, H, args.cpu_budget)
        else:
            result["cpu_baseline"] = None
        print(json.dumps(result), file=out, flush=True)
    if dist_on:
        drain(-1)
        torch.cuda.synchronize()
    r.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
