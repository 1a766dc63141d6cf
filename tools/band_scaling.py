"""Per-rank compute time of the row-band decomposition, measured on ONE GPU (development aid).

For N in 1, 2, 4, 8 a renderer holds the band a rank of an N-GPU run renders (band rows + halo)
and runs the bench workload on it; the slowest band's ms/frame is the per-GPU compute floor of
the N-GPU frame (the RCCL all-gather of frame f overlaps frame f+1 in bench.py).  This projects
the strong-scaling curve when no multi-GPU box is at hand; it is not a multi-GPU measurement.
Frames without neighbour reads use bench.py's interleaved stripes (--bands: contiguous bands).

The projection adds the collective: one gather of the tone-mapped RGBA16F frame (8 B/px) per
displayed frame.  bench.py's default per-peer gather (HK_BENCH_GATHER=peer, bands.peer_exchange / peer_gather)
sends each rank's rows straight to every peer over that pair's own xGMI link, so it is bound by one band per link
at ~153 GB/s (MI355X: 7 links x ~153 GB/s per GPU); --gather ring models the all-gather ring instead, which moves
(N-1)/N of the frame through each GPU's busiest link.  bench.py double-buffers it, so the gather of frame f runs
next to frame f+1: frame time = max(compute, gather) when it overlaps, compute + gather when it does not; both
are printed.
Row bands are cost-balanced as bench.py balances them (bands.rebalance, --balance R rounds, default 5:
every rank's band timed, the boundaries moved to equal measured cost, timed again); the equal-row split is
printed beside it.  --overhead-ms X adds the measured per-frame cost of the collective path itself (the
band copy, the all-gather's stream waits and the reorder at world size 1: HK_BENCH_DIST=1 minus the
single-GPU line) to every N > 1 frame.
--tiles: 2-D tiles instead of row bands (hk_resize_tile; bands.tile_grid: 2x1 at N = 2, 2x2 at 4, 4x2 at 8), balanced
with bands.rebalance_tiles (row bands on their slowest tile, the column split inside each row band on its two tiles);
the per-peer gather then moves the largest tile per link.
usage: python tools/band_scaling.py [config] [steps] [--bands] [--tiles] [--kernels] [--only N] [--balance R]
                                   [--overhead-ms X] [--gather peer|ring] [--opts key=value,...]
--opts: runtime options (hk_set_option) of every band's renderer, for A/B runs."""
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "bevy-hikari_amd"))
import bench  # noqa: E402
from hikari_amd import HikariRenderer, HikariSettings, Upscale, examples, frame_inputs  # noqa: E402
from hikari_amd.bands import (aligned_bounds, band_of, equal_bounds, halo_rows, rebalance, rebalance_tiles,  # noqa: E402
                              stripe_gather_rows, tile_gather_shape, tile_grid, tile_of, use_stripes)

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "cornell-1080p-nee"
steps = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 50
cfg = bench.CONFIGS[cfg_name]
W, H = cfg["width"], cfg["height"]
scene, cam, lights = examples.SCENES[cfg["scene"]]()
scene.build()
st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=cfg["spatial"], denoise=cfg["denoise"])
s = st.to_c()
torch.cuda.set_device(0)
sp = torch.cuda.current_stream().cuda_stream
XGMI_LINK_GBS = 153.0  # one xGMI link, GB/s per direction


def allgather_ms(n: int) -> float:
    """Ring all-gather of the W x H RGBA16F frame over N GPUs, bound by one link: (N-1)/N x 8 B/px."""
    return 0.0 if n == 1 else (n - 1) / n * W * H * 8 / (XGMI_LINK_GBS * 1e9) * 1e3


def peer_gather_ms(n: int, part_rows: int) -> float:
    """Per-peer gather: every pair of GPUs exchanges one part (the largest band, or a rank's padded stripe rows) on
    its own link, all links at once."""
    return 0.0 if n == 1 else part_rows * W * 8 / (XGMI_LINK_GBS * 1e9) * 1e3


def arg(name, default):
    return type(default)(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


gather = sys.argv[sys.argv.index("--gather") + 1] if "--gather" in sys.argv else "peer"
out = {"config": cfg_name, "resolution": [W, H], "gather": gather, "bands": {}, "allgather_ms": {}, "projected_ms": {},
       "equal_bands": {}, "bounds": {}, "overhead_ms": arg("--overhead-ms", 0.0)}
only = arg("--only", 0) or None
rounds = arg("--balance", 5)
# bench.py's options: the G-buffer is rendered every frame at 1 spp (gbuffer_reuse would skip it on a static camera)
opts = {"gbuffer_reuse": 1 if cfg.get("spp", 1) > 1 else 0,
        **{k: float(v) for k, v in (kv.split("=") for kv in arg("--opts", "").split(",") if kv)}}


def rank_ms(n, rank, stripes, bounds, col_bounds=None):
    """ms/frame of rank `rank`'s rows (or tile: col_bounds given) of an N-way split, alone on the GPU."""
    if True:
        r = HikariRenderer(0, opts)
        r.set_noise()
        r.upload_scene(scene)
        r.set_band_halo(halo_rows(cfg["spatial"], cfg["denoise"]))
        if n == 1:
            r.resize(W, H, 1.0)
        elif stripes:
            r.resize_striped(W, H, rank, n)
        elif col_bounds is not None:
            t = tile_of(rank, n, W, H, bounds, col_bounds)
            r.resize_tile(W, H, t.x0, t.cols, t.y0, t.rows)
        else:
            b = band_of(rank, n, H, bounds)
            r.resize(W, H, 1.0, b.y0, b.rows)

        def step(f):
            fi = frame_inputs(f, cam, lights, W, H)
            r.render_gbuffer(fi, sp)
            r.render_frame(s, fi, sp)
            if st.denoise:
                r.denoise(s, fi, sp)
            r.tone_sum(s, sp)

        for f in range(10):
            step(f)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for f in range(10, 10 + steps):
            step(f)
        t_host = time.perf_counter() - t0  # enqueue time (the queue may throttle it)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        if "--kernels" in sys.argv and rank == n // 2:
            print(f"  N={n} host enqueue {t_host / steps * 1e3:.4f} ms/frame", flush=True)
            r.enable_kernel_timing(True)
            for f in range(10 + steps, 20 + steps):
                step(f)
            torch.cuda.synchronize()
            print(f"  N={n} rank {rank} kernel ms:", {k: round(v, 4) for k, v in r.kernel_timing().items()}, flush=True)
            r.enable_kernel_timing(False)
        r.close()
        return ms


for n in (1, 2, 4, 8):
    if only is not None and n != only:
        continue
    stripes = use_stripes(cfg["spatial"], cfg["denoise"]) and "--bands" not in sys.argv
    tiles = "--tiles" in sys.argv and not stripes and tile_grid(n)[1] > 1
    if n == 1 or stripes:
        worst = max(rank_ms(n, rank, stripes, None) for rank in sorted({0, n // 2, n - 1}))  # edge and middle
    elif tiles:
        ny, nx = tile_grid(n)
        bounds, cols = aligned_bounds(ny, H), [aligned_bounds(nx, W)] * ny
        times = [rank_ms(n, k, False, bounds, cols) for k in range(n)]
        out["equal_bands"][n] = round(max(times), 4)
        print(f"N={n}: equal {ny}x{nx} tiles {[round(t, 3) for t in times]}", flush=True)
        for _ in range(rounds):
            bounds, cols = rebalance_tiles(bounds, cols, times)
            times = [rank_ms(n, k, False, bounds, cols) for k in range(n)]
            print(f"N={n}: tiles rows {bounds} cols {cols} -> {[round(t, 3) for t in times]}", flush=True)
        out["bounds"][n] = {"rows": [int(v) for v in bounds], "cols": [[int(v) for v in c] for c in cols]}
        worst = max(times)
    else:
        bounds = equal_bounds(n, H)
        times = [rank_ms(n, k, False, bounds) for k in range(n)]
        out["equal_bands"][n] = round(max(times), 4)
        print(f"N={n}: equal bands {[round(t, 3) for t in times]}", flush=True)
        for _ in range(rounds):
            bounds = rebalance(bounds, times)
            times = [rank_ms(n, k, False, bounds) for k in range(n)]
            print(f"N={n}: bands {bounds} -> {[round(t, 3) for t in times]}", flush=True)
        out["bounds"][n] = [int(v) for v in bounds]
        worst = max(times)
    out["bands"][n] = round(worst, 4)
    if gather == "ring":
        g = allgather_ms(n)
    elif n == 1 or stripes:
        g = peer_gather_ms(n, stripe_gather_rows(n, H)[0] if n > 1 else H)
    elif tiles:
        tr, tc = tile_gather_shape(bounds, cols)
        g = peer_gather_ms(n, tr) * tc / W  # the largest (padded) tile per link
    else:
        g = peer_gather_ms(n, max(b - a for a, b in zip(bounds[:-1], bounds[1:])))
    ov = out["overhead_ms"] if n > 1 else 0.0
    out["allgather_ms"][n] = round(g, 4)
    out["projected_ms"][n] = {"overlapped": round(max(worst, g) + ov, 4), "serial": round(worst + g + ov, 4)}
    base = out["bands"].get(1)
    speedup = (f"  speedup {base / (max(worst, g) + ov):.2f}x overlapped, {base / (worst + g + ov):.2f}x serial"
               if base else "")
    print(f"N={n}: slowest band {worst:.4f} ms/frame, {gather} gather {g:.4f} ms, collective-path overhead {ov:.4f} ms"
          f"{speedup}", flush=True)
print(json.dumps(out))
