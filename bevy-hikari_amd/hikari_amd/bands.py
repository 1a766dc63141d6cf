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


def band_of(rank: int, world: int, height: int) -> Band:
    if height % world != 0:
        raise ValueError(f"frame height {height} does not split into {world} equal bands")
    rows = height // world
    return Band(rank, world, rank * rows, rows)


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
