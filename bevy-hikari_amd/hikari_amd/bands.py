"""Screen-space row-band sharding across GPUs.

The reference runs on one wgpu device; the MI355X build splits a frame into N horizontal bands,
one per rank (one process per GPU).  Each rank recomputes a halo of `halo_rows(...)` rows above
and below its band so that spatial reuse (<= 20 px), the 4-level à-trous filter (<= 15 px) and
the 3x3 variance blur (1 px) see exactly the inputs a whole-frame render sees: for a static
camera the band's own rows are bit-identical to the single-GPU frame.  The tone-mapped RGBA16F
bands are then all-gathered (RCCL over xGMI on GPUs, gloo on CPU) so every rank holds the frame.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

SPATIAL_REACH = 20  # light.wgsl:251 SPATIAL_REUSE_RANGE (indirect); emissive uses 10
ATROUS_REACH = 8 + 4 + 2 + 1  # denoise.wgsl:101-114 step sizes of levels 0..3
VARIANCE_REACH = 1  # denoise.wgsl:151-159 3x3 variance blur
DEFAULT_HALO = 40  # >= SPATIAL_REACH + ATROUS_REACH + VARIANCE_REACH = 36, rounded to a multiple of 8


def halo_rows(spatial_reuse: bool, denoise: bool) -> int:
    """Rows of halo a band needs so its own rows are exact."""
    need = (SPATIAL_REACH if spatial_reuse else 0) + ((ATROUS_REACH + VARIANCE_REACH) if denoise else 0)
    return 0 if need == 0 else DEFAULT_HALO


@dataclass(frozen=True)
class Band:
    rank: int
    world: int
    y0: int    # first global row of the band
    rows: int  # band rows (without halo)


def band_of(rank: int, world: int, height: int, bounds=None) -> Band:
    """Rank's band: equal rows, or rows [bounds[rank], bounds[rank + 1]) of a partition (rebalance)."""
    if bounds is not None:
        if len(bounds) != world + 1 or bounds[0] != 0 or bounds[-1] != height:
            raise ValueError(f"bounds {list(bounds)} are not a partition of {height} rows into {world} bands")
        return Band(rank, world, int(bounds[rank]), int(bounds[rank + 1] - bounds[rank]))
    if height % world != 0:
        raise ValueError(f"frame height {height} does not split into {world} equal bands")
    rows = height // world
    return Band(rank, world, rank * rows, rows)


def equal_bounds(world: int, height: int) -> list:
    return [k * height // world for k in range(world + 1)]


# ---------------------------------------------------------------- cost-balanced bands
# The frame's cost is far from uniform over its rows (city: the houses and the emissive sphere fill the
# lower half), so equal-row bands leave the slowest rank with most of the work: city 4K measured 1.51x at
# N = 2.  rebalance() moves the boundaries so that every band gets the same share of the
# measured cost: the per-row cost is taken piecewise constant over the current bands (each band's measured
# frame time spread evenly over its rows, its halo and fixed costs included), and the new boundaries cut
# the cumulative cost into `world` equal parts.  Iterated (a second measurement on the new bands refines
# the density where it changed).  With a static camera the frame's cost is deterministic, so every rank
# computes the same boundaries from the same all-gathered times.
BAND_ALIGN = 8  # band boundaries on 8-row multiples (the kernels' 8x8 wave tiles)


def rebalance(bounds, times, align: int = BAND_ALIGN) -> list:
    """New boundaries [0, y1, ..., H] from the per-band times measured on `bounds`."""
    b = np.asarray(bounds, np.float64)
    n = len(b) - 1
    height = int(b[-1])
    rows = np.diff(b)
    t = np.maximum(np.asarray(times, np.float64), 1e-12)
    if len(t) != n or (rows <= 0).any():
        raise ValueError("one time per non-empty band")
    dens = t / rows
    cum = np.concatenate([[0.0], np.cumsum(t)])
    new = [0]
    for k in range(1, n):
        target = cum[-1] * k / n
        j = min(int(np.searchsorted(cum, target, side="right")) - 1, n - 1)
        y = b[j] + (target - cum[j]) / dens[j]
        new.append(int(round(y / align)) * align)
    new.append(height)
    for k in range(1, n):  # strictly increasing, every band at least `align` rows
        new[k] = min(max(new[k], new[k - 1] + align), height - (n - k) * align)
    return new


def band_gather_rows(bounds) -> tuple:
    """(padded rows per rank, index) for reassembling an all-gather of uneven bands: every rank
    contributes `pad` rows (its band, zero-padded), and frame row y = gathered row index[y]."""
    rows = np.diff(np.asarray(bounds))
    pad = int(rows.max())
    index = np.concatenate([k * pad + np.arange(r) for k, r in enumerate(rows)])
    return pad, index


# ---------------------------------------------------------------- 2-D tiles
# north_star: "frames tile-partition across the 8 GPUs".  A rank renders a tile — columns [x0, x0 + cols) of rows
# [y0, y0 + rows) — plus a halo on every side (hk_resize_tile): its planes hold the band's rows at full width and every
# pass runs only on the rows and columns later passes read, so the tile's own pixels equal a whole-frame render.  At
# N = 8 the frame is 4 row bands x 2 column bands: a 4K tile of 1920 x 540 recomputes (540 + 2 x 36) rows x (1920 + 36)
# columns for its G-buffer and indirect temporal pass (1.15x) where a 270-row band recomputes 342 x 3840 (1.27x); for
# scene 1080p's narrow balanced bands the saving is larger.
@dataclass(frozen=True)
class Tile:
    rank: int
    world: int
    x0: int    # first global column of the tile
    cols: int
    y0: int    # first global row
    rows: int


def tile_grid(world: int) -> tuple:
    """(row bands, column bands) of a world-rank tiling: two columns once there are 4 or more (even) ranks."""
    nx = 2 if world >= 4 and world % 2 == 0 else 1
    return world // nx, nx


def tile_of(rank: int, world: int, width: int, height: int, row_bounds=None, col_bounds=None) -> Tile:
    """Rank's tile: row band rank // nx of `row_bounds` (equal 8-aligned bands by default), column band rank % nx of
    col_bounds[row band] (equal halves by default; cost-balanced per row band by rebalance_tiles)."""
    ny, nx = tile_grid(world)
    ty, tx = divmod(rank, nx)
    rb = list(row_bounds) if row_bounds is not None else aligned_bounds(ny, height)
    cb = list(col_bounds[ty]) if col_bounds is not None else aligned_bounds(nx, width)
    if len(rb) != ny + 1 or len(cb) != nx + 1:
        raise ValueError("bounds do not match the tile grid")
    return Tile(rank, world, int(cb[tx]), int(cb[tx + 1] - cb[tx]), int(rb[ty]), int(rb[ty + 1] - rb[ty]))


def aligned_bounds(n: int, size: int, align: int = BAND_ALIGN) -> list:
    """n near-equal parts of `size` with inner boundaries on multiples of `align`."""
    return [0] + [int(round(k * size / n / align)) * align for k in range(1, n)] + [size]


def rebalance_tiles(row_bounds, col_bounds, times, align: int = BAND_ALIGN):
    """New (row_bounds, col_bounds) from per-tile times (rank order): the row bands get equal shares of their
    slowest tile's time x tiles (rebalance over rows), and inside every row band the column boundary moves to equal
    tile times (rebalance over that band's columns)."""
    ny, nx = len(row_bounds) - 1, len(col_bounds[0]) - 1
    t = np.asarray(times, np.float64).reshape(ny, nx)
    new_rows = rebalance(row_bounds, t.max(axis=1) * nx, align)
    new_cols = [rebalance(col_bounds[j], t[j], align) if nx > 1 else list(col_bounds[j]) for j in range(ny)]
    return new_rows, new_cols


def tile_gather_shape(row_bounds, col_bounds) -> tuple:
    """(rows, cols) every rank contributes to the gather of tiles: the largest tile (smaller ones zero-padded)."""
    rows = int(np.diff(np.asarray(row_bounds)).max())
    cols = int(max(np.diff(np.asarray(c)).max() for c in col_bounds))
    return rows, cols


def tile_reassembly_copies(frame, gathered, tiles) -> list:
    """(destination, source) views putting a gather of padded tiles back in frame order: frame (H, W, C), gathered
    (world, rows_max, cols_max, C); tiles: the Tile of every rank."""
    return [(frame[t.y0: t.y0 + t.rows, t.x0: t.x0 + t.cols], gathered[t.rank, : t.rows, : t.cols]) for t in tiles]


# ---------------------------------------------------------------- interleaved stripes
# Frames without neighbour reads (spatial reuse and denoise off, halo 0) are split into 8-row
# stripes dealt round-robin to the ranks (hk_resize_striped): every rank gets an equal share of
# every screen region, so the ranks' work is balanced where contiguous bands are not (cornell:
# the box fills the middle rows, the top and bottom bands are mostly background).
STRIPE_H = 8  # hk_device.h STRIPE_H


def stripe_rows(rank: int, world: int, height: int) -> np.ndarray:
    """Global rows held by `rank`, in local-row order."""
    rows = [np.arange(t * STRIPE_H, min(height, (t + 1) * STRIPE_H))
            for t in range(rank, (height + STRIPE_H - 1) // STRIPE_H, world)]
    return np.concatenate(rows) if rows else np.zeros(0, np.int64)


def stripe_gather_rows(world: int, height: int) -> tuple:
    """(padded rows per rank, index) for reassembling an all-gather of stripe planes: every rank
    contributes `pad` rows (its stripes, zero-padded), and frame row y = gathered row index[y]."""
    per = [stripe_rows(k, world, height) for k in range(world)]
    pad = max(len(p) for p in per)
    index = np.empty(height, np.int64)
    for k, p in enumerate(per):
        index[p] = k * pad + np.arange(len(p))
    return pad, index


def use_stripes(spatial_reuse: bool, denoise: bool) -> bool:
    """Stripes where no pass reads neighbours; contiguous bands + halo otherwise."""
    return halo_rows(spatial_reuse, denoise) == 0


def reassembly_copies(frame, gathered, world: int, height: int, pad: int, bounds=None) -> list:
    """(destination, source) views that put an all-gather of `world` ranks x `pad` rows back in frame order:
    one strided copy per rank moving whole rows — its interleaved 8-row stripes (bounds None) or its band of
    `bounds`.  frame: (height, W, C), gathered: (world * pad, W, C) tensors (torch or numpy, with .view /
    .reshape on contiguous buffers); height must be a multiple of STRIPE_H for stripes."""
    out = []
    for q in range(world):
        if bounds is None:
            if height % STRIPE_H:
                raise ValueError("stripe reassembly needs a height that is a multiple of 8")
            n = len(stripe_rows(q, world, height)) // STRIPE_H
            dst = frame.view(height // STRIPE_H, STRIPE_H, *frame.shape[1:])[q::world][:n]
            src = gathered[q * pad: q * pad + n * STRIPE_H].view(n, STRIPE_H, *frame.shape[1:])
        else:
            b = band_of(q, world, height, bounds)
            dst, src = frame[b.y0: b.y0 + b.rows], gathered[q * pad: q * pad + b.rows]
        out.append((dst, src))
    return out


# ---------------------------------------------------------------- per-peer gather (row bands)
# A ring all-gather moves (N-1)/N of the frame through each GPU's busiest xGMI link, one band per step; an MI355X
# node connects every GPU to every other one (7 links of ~153 GB/s per GPU), so each rank can instead send its band
# straight to every peer and receive every peer's band on that peer's own link: N-1 transfers at once, each the size
# of one band (cornell 1080p at N = 8: 0.518 MB per link instead of 3.6 MB through one).
# The bands are contiguous rows, so each peer's band lands directly in its place in the frame: no reassembly pass
# for uneven (cost-balanced) bands either.
def peer_exchange_ops(frame, bounds, rank: int, world: int) -> list:
    """The point-to-point operations of the per-peer gather over `frame` (rows x ... tensor holding the whole frame,
    this rank's rows [bounds[rank], bounds[rank + 1]) already in place): this rank's rows sent to every peer, every
    peer's rows received into their place.  For torch.distributed.batch_isend_irecv (RCCL runs the group's
    transfers together).  Peers are visited in a staggered order (rank + k, rank - k) so that no rank is every
    rank's first partner."""
    import torch.distributed as dist
    mine = frame[bounds[rank]: bounds[rank + 1]]
    ops = []
    for k in range(1, world):
        dst, src = (rank + k) % world, (rank - k) % world
        ops.append(dist.P2POp(dist.isend, mine, dst))
        ops.append(dist.P2POp(dist.irecv, frame[bounds[src]: bounds[src + 1]], src))
    return ops


def peer_exchange(frame, bounds, rank: int, world: int, self_buf=None) -> list:
    """Start the per-peer gather; returns the requests (wait() each).  self_buf (world size 1 only): the band is also
    sent to this rank itself and received into self_buf (a tensor of the band's shape), so that a one-rank run
    issues the per-peer path's RCCL point-to-point group — one send and one receive of a band, the transfer every
    link carries at N > 1 — instead of no collective work at all."""
    import torch.distributed as dist
    ops = peer_exchange_ops(frame, bounds, rank, world)
    if world == 1 and self_buf is not None:
        mine = frame[bounds[rank]: bounds[rank + 1]]
        ops = [dist.P2POp(dist.isend, mine, rank), dist.P2POp(dist.irecv, self_buf, rank)]
    return dist.batch_isend_irecv(ops) if ops else []


def peer_gather(full, mine, rank: int, world: int, self_transfer: bool = False) -> list:
    """The per-peer form of all_gather_into_tensor(full, mine) for the interleaved stripes' padded rows (or any
    equal-size parts): `mine` sent to every peer, peer j's part received into full[j * n : (j + 1) * n] (n =
    len(mine)), this rank's own part copied into its slot; returns the requests (wait() each).  The slots keep the
    all-gather's layout, so bench.py's reassembly (reassembly_copies / stripe_gather_rows) applies unchanged.
    self_transfer (world size 1 only): this rank's own part reaches its slot by an RCCL send to itself instead of a
    copy, so a one-rank run issues the per-peer path's point-to-point group."""
    import torch.distributed as dist
    n = mine.shape[0]
    if world == 1 and self_transfer:
        return dist.batch_isend_irecv([dist.P2POp(dist.isend, mine, rank),
                                       dist.P2POp(dist.irecv, full[rank * n: (rank + 1) * n], rank)])
    full[rank * n: (rank + 1) * n].copy_(mine)
    ops = []
    for k in range(1, world):
        dst, src = (rank + k) % world, (rank - k) % world
        ops.append(dist.P2POp(dist.isend, mine, dst))
        ops.append(dist.P2POp(dist.irecv, full[src * n: (src + 1) * n], src))
    return dist.batch_isend_irecv(ops) if ops else []


# ---------------------------------------------------------------- band window refill (settings changes)
# A band runs each channel's light passes on its core rows +- the margin the settings need; turning a setting on
# (denoise, emissive / indirect spatial reuse) widens a margin for good, and the rows it takes in hold records the
# band never computed, where a whole-frame render holds their history (its temporal passes run on every pixel,
# light.rs:656-699).  The band owning those rows as core rows holds them exactly, so before the first frame with the
# new settings every band takes them from their owners (hk_band_window_grow lists them, hk_reservoir_rows moves
# them) and commits the wider windows: the frame stays bit-identical to the whole-frame render.  Call it on frames
# whose settings differ from the previous frame's (a no-op otherwise), after hk_render_gbuffer, before
# hk_render_frame.
def _overlap(y0: int, n: int, lo: int, hi: int):
    a, b = max(y0, lo), min(y0 + n, hi)
    return (a, b - a) if b > a else None


def refill_windows_local(bands, settings) -> int:
    """In-process refill over the bands of one frame (one context per band, e.g. on one GPU): `bands` is a list of
    (Band, renderer).  Returns the number of row blocks copied."""
    needs = [r.band_window_grow(settings) for _, r in bands]
    moved = 0
    for (_, r), ranges in zip(bands, needs):
        for buf in range(len(ranges)):
            for side in range(2):
                y0, n = int(ranges[buf, 2 * side]), int(ranges[buf, 2 * side + 1])
                for ob, owner in bands:
                    if owner is r:
                        continue
                    o = _overlap(y0, n, ob.y0, ob.y0 + ob.rows)
                    if o:
                        r.reservoir_rows(buf, o[0], o[1], owner.reservoir_rows(buf, o[0], o[1]), store=True)
                        moved += 1
    for _, r in bands:
        r.band_window_grow(settings, commit=True)
    return moved


def refill_windows(renderer, settings, bounds, rank: int, world: int, device="cuda") -> int:
    """The refill across ranks (one band per rank, bands = `bounds`): every rank's needs all-gathered, each block
    sent by its owner straight to the rank that needs it (batch_isend_irecv: RCCL over xGMI on GPUs, gloo with
    device "cpu").  Collective: every rank calls it.  Returns the number of row blocks this rank received."""
    import torch
    import torch.distributed as dist
    mine = renderer.band_window_grow(settings)
    t = torch.from_numpy(np.ascontiguousarray(mine.reshape(-1))).to(device)
    everyone = torch.zeros(world * t.numel(), dtype=t.dtype, device=device)
    dist.all_gather_into_tensor(everyone, t)
    need = everyone.cpu().numpy().reshape(world, *mine.shape)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    ops, stores = [], []
    # one pass per (sender, receiver) pair in the same (buffer, side) order on both ends, so point-to-point
    # messages between two ranks match in posting order
    for q in range(world):
        for buf in range(need.shape[1]):
            for side in range(2):
                y0, n = int(need[q, buf, 2 * side]), int(need[q, buf, 2 * side + 1])
                if q == rank:
                    for p in range(world):
                        o = _overlap(y0, n, int(bounds[p]), int(bounds[p + 1])) if p != rank else None
                        if o:
                            block = torch.empty(renderer.reservoir_rows_bytes(o[1]), dtype=torch.uint8, device=device)
                            ops.append(dist.P2POp(dist.irecv, block, p))
                            stores.append((buf, o, block))
                else:
                    o = _overlap(y0, n, lo, hi)
                    if o:
                        block = torch.empty(renderer.reservoir_rows_bytes(o[1]), dtype=torch.uint8, device=device)
                        renderer.reservoir_rows(buf, o[0], o[1], block.data_ptr() if block.is_cuda else block.numpy())
                        ops.append(dist.P2POp(dist.isend, block, q))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
        if str(device).startswith("cuda"):
            torch.cuda.synchronize()
    for buf, o, block in stores:
        renderer.reservoir_rows(buf, o[0], o[1], block.data_ptr() if block.is_cuda else block.numpy(), store=True)
    renderer.band_window_grow(settings, commit=True)
    return len(stores)
