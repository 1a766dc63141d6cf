"""N>1 path on CPU: world_size-2 and -4 gloo ranks each render only their own rows with the oracle —
a row band + halo (hko_set_band) or their interleaved 8-row stripes (hko_set_stripes) — all-gather
the tone-mapped rows, and must reproduce the whole-frame render bit-exactly (bands.py halo
sufficiency + the gather wiring that bench.py uses with RCCL on GPUs).  The frame is 192 rows, so a
band plus its 40-row halo on both sides is a strict part of it (96 + 80 and 48 + 80 rows)."""
import os
import socket

import numpy as np
import pytest

W, H, FRAMES = 48, 192, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _render(band=None, halo=40, spatial=True, denoise=True, stripes=None, counters=False):
    from oracle import Oracle

    from hikari_amd import HikariSettings, Upscale, examples, frame_inputs, load_noise
    scene, cam, lights = examples.cornell()
    desc = scene.build()
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=spatial, denoise=denoise)
    s = st.to_c()
    o = Oracle(desc, load_noise(), W, H, 1.0, threads=2)
    if band is not None:
        o.set_band(band.y0, band.rows, halo)
    if stripes is not None:
        o.set_stripes(*stripes)
    for f in range(FRAMES):
        fi = frame_inputs(f, cam, lights, W, H)
        o.render_gbuffer(fi)
        o.render_frame(s, fi)
        o.denoise(s, fi)
        o.tone_sum(s)
    return (o.output(10), o.counters()) if counters else o.output(10)


def _stripe_worker(rank, world, port, q):
    """bench.py's stripe wiring: each rank renders only its stripes (an oracle context restricted to
    them, as hk_resize_striped restricts a GPU context), contributes its (zero-padded) stripe rows,
    and the gather is reassembled with stripe_gather_rows' index."""
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    for p in (root / "bevy-hikari_amd", root / "oracle", root / "tests"):
        sys.path.insert(0, str(p))
    import torch
    import torch.distributed as dist

    from hikari_amd.bands import stripe_gather_rows, stripe_rows
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    img, cnt = _render(None, 0, False, False, stripes=(rank, world), counters=True)
    pad, index = stripe_gather_rows(world, H)
    mine = np.zeros((pad, W, 8), np.uint8)
    rows = stripe_rows(rank, world, H)
    mine[:len(rows)] = img[rows]
    full = torch.empty((world * pad, W, 8), dtype=torch.uint8)
    dist.all_gather_into_tensor(full, torch.from_numpy(mine))
    n = torch.tensor([cnt["traverse_top"], cnt["traverse_emitter"], cnt["primary"]], dtype=torch.int64)
    dist.all_reduce(n)
    if rank == 0:
        q.put((full.numpy()[index].copy(), n.tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_rank_stripes_reassemble_whole_frame(world):
    """Each rank computes only its stripes; the gathered frame equals the whole-frame render and the
    ranks' ray counts add up to the whole frame's (every pixel traced exactly once)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stripe_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, counts = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    whole, c = _render(None, 0, False, False, counters=True)
    assert np.array_equal(gathered, whole)
    assert counts == [c["traverse_top"], c["traverse_emitter"], c["primary"]]


@pytest.mark.parametrize("world,height", [(1, 48), (2, 48), (3, 100), (8, 1080), (8, 2160), (5, 7)])
def test_stripe_rows_partition_the_frame(world, height):
    from hikari_amd.bands import STRIPE_H, stripe_gather_rows, stripe_rows
    rows = [stripe_rows(k, world, height) for k in range(world)]
    allr = np.sort(np.concatenate(rows))
    assert np.array_equal(allr, np.arange(height))  # every row exactly once
    for k, r in enumerate(rows):  # local order: stripe k, k + world, ...; 8-row stripes
        assert np.all((r // STRIPE_H) % world == k) and np.all(np.diff(r) > 0)
    pad, index = stripe_gather_rows(world, height)
    assert pad == max(len(r) for r in rows)
    assert max(len(r) for r in rows) - min(len(r) for r in rows) <= STRIPE_H  # balanced
    for k, r in enumerate(rows):
        assert np.array_equal(index[r], k * pad + np.arange(len(r)))


def _worker(rank, world, port, spatial, denoise, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    for p in (root / "bevy-hikari_amd", root / "oracle", root / "tests"):
        sys.path.insert(0, str(p))
    import torch
    import torch.distributed as dist

    from hikari_amd.bands import band_of, halo_rows
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    band = band_of(rank, world, H)
    img = _render(band, halo_rows(spatial, denoise), spatial, denoise)
    mine = torch.from_numpy(np.ascontiguousarray(img[band.y0: band.y0 + band.rows]))
    full = torch.empty((world * band.rows, W, 8), dtype=torch.uint8)
    dist.all_gather_into_tensor(full, mine)
    if rank == 0:
        q.put(full.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("spatial,denoise", [(True, True), (False, False)])
def test_rank_bands_reassemble_whole_frame(world, spatial, denoise):
    import torch.multiprocessing as mp
    from hikari_amd.bands import band_of, halo_rows
    b = band_of(0, world, H)
    assert b.rows + 2 * halo_rows(True, True) < H  # a band + halo is a strict part of the frame
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, spatial, denoise, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    whole = _render(None, 0, spatial, denoise)
    assert np.array_equal(gathered, whole)


def test_insufficient_halo_is_detectable():
    """Sanity: without the halo the seam rows differ (so the test above is meaningful)."""
    from hikari_amd.bands import band_of
    whole = _render(None, 0, True, True)
    b = band_of(0, 2, H)
    part = _render(b, 0, True, True)
    assert not np.array_equal(part[b.y0: b.y0 + b.rows], whole[b.y0: b.y0 + b.rows])


def _balanced_worker(rank, world, port, q):
    """bench.py's cost-balanced band wiring: every rank times its equal band, the times are all-gathered,
    every rank computes the same new boundaries (bands.rebalance), renders its uneven band + halo from
    frame 0, contributes it zero-padded to the largest band, and the gather is put back in frame order
    with band_gather_rows' index."""
    import sys
    import time
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    for p in (root / "bevy-hikari_amd", root / "oracle", root / "tests"):
        sys.path.insert(0, str(p))
    import torch
    import torch.distributed as dist

    from hikari_amd.bands import band_gather_rows, band_of, equal_bounds, halo_rows, rebalance
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bounds = equal_bounds(world, H)
    t0 = time.perf_counter()
    _render(band_of(rank, world, H, bounds), halo_rows(True, True))
    # a skewed cost on top of the measured one, so that the boundaries really move
    t = torch.tensor([(time.perf_counter() - t0) * (1.0 + 3.0 * rank)], dtype=torch.float64)
    times = torch.zeros(world, dtype=torch.float64)
    dist.all_gather_into_tensor(times, t)
    bounds = rebalance(bounds, times.numpy())
    mine_b = torch.tensor(bounds, dtype=torch.int64)
    all_b = torch.zeros(world * len(bounds), dtype=torch.int64)
    dist.all_gather_into_tensor(all_b, mine_b)
    band = band_of(rank, world, H, bounds)
    img = _render(band, halo_rows(True, True))
    pad, index = band_gather_rows(bounds)
    mine = np.zeros((pad, W, 8), np.uint8)
    mine[:band.rows] = img[band.y0: band.y0 + band.rows]
    full = torch.empty((world * pad, W, 8), dtype=torch.uint8)
    dist.all_gather_into_tensor(full, torch.from_numpy(mine))
    if rank == 0:
        q.put((full.numpy()[index].copy(), all_b.numpy().reshape(world, -1).tolist(), bounds))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_balanced_uneven_bands_reassemble_whole_frame(world):
    """Uneven (cost-balanced) bands: all ranks agree on the boundaries, the boundaries moved away from
    the equal split, and the reassembled gather equals the whole-frame render."""
    import torch.multiprocessing as mp
    from hikari_amd.bands import equal_bounds
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_balanced_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, per_rank_bounds, bounds = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert all(b == list(bounds) for b in per_rank_bounds)
    assert list(bounds) != equal_bounds(world, H)
    whole = _render(None, 0, True, True)
    assert np.array_equal(gathered, whole)


def _peer_worker(rank, world, port, balanced, q):
    """bench.py's per-peer gather (HK_BENCH_GATHER=peer, bands.peer_exchange): each rank renders its band + halo,
    places its own rows in a whole-frame buffer and exchanges bands point to point with every peer
    (batch_isend_irecv); every rank must end with the whole frame."""
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    for p in (root / "bevy-hikari_amd", root / "oracle", root / "tests"):
        sys.path.insert(0, str(p))
    import torch
    import torch.distributed as dist

    from hikari_amd.bands import band_of, equal_bounds, halo_rows, peer_exchange
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bounds = equal_bounds(world, H)
    if balanced:  # uneven bands on 8-row multiples
        bounds = [0] + [int(round(H * (k / world) ** 1.5 / 8)) * 8 for k in range(1, world)] + [H]
    band = band_of(rank, world, H, bounds)
    img = _render(band, halo_rows(True, True))
    frame = torch.full((H, W, 8), 0xAB, dtype=torch.uint8)
    frame[band.y0: band.y0 + band.rows] = torch.from_numpy(np.ascontiguousarray(img[band.y0: band.y0 + band.rows]))
    for req in peer_exchange(frame, bounds, rank, world):
        req.wait()
    q.put((rank, frame.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,balanced", [(2, False), (4, False), (3, True)])
def test_peer_exchange_gathers_whole_frame(world, balanced):
    """The per-peer gather (direct band transfers instead of the ring all-gather) leaves every rank with the
    whole-frame render, for equal and uneven bands."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_peer_worker, args=(r, world, port, balanced, q)) for r in range(world)]
    for p in procs:
        p.start()
    frames = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    whole = _render(None, 0, True, True)
    for rank in range(world):
        assert np.array_equal(frames[rank], whole), rank


def _stripe_peer_worker(rank, world, port, q):
    """bench.py's interleaved stripes with the per-peer gather (bands.peer_gather into the all-gather's padded
    layout, then stripe_gather_rows' reassembly)."""
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    for p in (root / "bevy-hikari_amd", root / "oracle", root / "tests"):
        sys.path.insert(0, str(p))
    import torch
    import torch.distributed as dist

    from hikari_amd.bands import peer_gather, stripe_gather_rows, stripe_rows
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    img = _render(None, 0, False, False, stripes=(rank, world))
    pad, index = stripe_gather_rows(world, H)
    rows = stripe_rows(rank, world, H)
    mine = np.zeros((pad, W, 8), np.uint8)
    mine[:len(rows)] = img[rows]
    full = torch.empty((world * pad, W, 8), dtype=torch.uint8)
    for req in peer_gather(full, torch.from_numpy(mine), rank, world):
        req.wait()
    q.put((rank, full.numpy()[index].copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_stripes_peer_gather_reassemble_whole_frame(world):
    """The interleaved stripes gathered per peer (bench.py's default for frames without neighbour reads) and put
    back in frame order equal the whole-frame render on every rank."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stripe_peer_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    frames = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    whole = _render(None, 0, False, False)
    for rank in range(world):
        assert np.array_equal(frames[rank], whole), rank


def test_rebalance_converges_on_a_skewed_cost():
    """bands.rebalance on a known per-row cost (city-like: the lower rows 6x as costly), each band's
    time = its rows' cost + a fixed per-band cost: three rounds bring the slowest band within 6 % of the
    mean, from 1.7x with equal bands; boundaries stay an increasing 8-row-aligned partition."""
    from hikari_amd.bands import BAND_ALIGN, equal_bounds, rebalance
    height = 2160
    y = np.arange(height)
    cost = 1.0 + 5.0 / (1.0 + np.exp(-(y - 1300) / 120.0))

    def times(b):
        return np.array([cost[b[k]:b[k + 1]].sum() + 40.0 for k in range(len(b) - 1)])

    for world in (2, 4, 8):
        b = equal_bounds(world, height)
        t = times(b)
        first = t.max() / t.mean()
        for _ in range(3):
            b = rebalance(b, t)
            t = times(b)
            assert b[0] == 0 and b[-1] == height and all(np.diff(b) >= BAND_ALIGN)
            assert all(v % BAND_ALIGN == 0 for v in b)
        assert first > 1.3 and t.max() / t.mean() < 1.06, (world, first, t.max() / t.mean())


@pytest.mark.parametrize("world,height", [(2, 192), (8, 1080), (8, 2160), (3, 256)])
def test_reassembly_row_copies_equal_the_gather_index(world, height):
    """bench.py puts the all-gathered stripes / uneven bands back in frame order with one strided row copy
    per rank (bands.reassembly_copies); the result equals the gather index's reordering for both layouts."""
    import torch

    from hikari_amd.bands import (band_gather_rows, band_of, equal_bounds, reassembly_copies, rebalance,
                                  stripe_gather_rows, stripe_rows)
    w = 5
    frame = torch.arange(height * w * 4, dtype=torch.float32).view(height, w, 4)
    for bounds in (None, rebalance(equal_bounds(world, height), np.arange(1, world + 1, dtype=float))):
        pad, index = stripe_gather_rows(world, height) if bounds is None else band_gather_rows(bounds)
        gathered = torch.zeros(world * pad, w, 4)
        for q in range(world):
            rows = stripe_rows(q, world, height) if bounds is None else \
                np.arange(band_of(q, world, height, bounds).y0, band_of(q, world, height, bounds).y0 +
                          band_of(q, world, height, bounds).rows)
            gathered[q * pad: q * pad + len(rows)] = frame[torch.from_numpy(np.asarray(rows))]
        out = torch.full_like(frame, -1.0)
        for dst, src in reassembly_copies(out, gathered, world, height, pad, bounds):
            dst.copy_(src)
        assert torch.equal(out, frame)
        assert torch.equal(gathered[torch.from_numpy(index)], frame)


class _FakeBand:
    """Stands in for a band context in the window refill's exchange logic (bands.refill_windows): reservoir buffers
    as (4, rows, W, 16) byte planes in the row-exchange layout of hk_reservoir_rows; the core rows hold the
    whole frame's records (a pattern of buffer, frame row and column), the halo rows garbage until refilled.  Its
    needs are what hk_band_window_grow lists for windows widening from 0 to `margins[buffer]` rows."""
    HALO = 40  # bands.DEFAULT_HALO

    def __init__(self, band, height, width, margins):
        self.band, self.width = band, width
        self.row0 = max(0, band.y0 - self.HALO)
        self.rows = min(height, band.y0 + band.rows + self.HALO) - self.row0
        rng = np.random.default_rng(band.y0)
        self.store = rng.integers(0, 256, (len(margins), 4, self.rows, width, 16), dtype=np.uint8)
        for b in range(len(margins)):
            for y in range(band.y0, band.y0 + band.rows):
                self.store[b, :, y - self.row0] = self.truth(b, y, width)
        self.ranges = np.zeros((len(margins), 4), np.int32)
        for b, m in enumerate(margins):
            lo, hi = band.y0, band.y0 + band.rows
            a0, a1 = max(0, lo - m), lo
            b0, b1 = hi, min(height, hi + m)
            self.ranges[b] = [a0 if a1 > a0 else 0, a1 - a0, b0 if b1 > b0 else 0, max(0, b1 - b0)]
        self.committed = False

    @staticmethod
    def truth(buf, y, width):
        x = np.arange(width)
        v = (buf * 131 + y * 7 + x[:, None] * 3 + np.arange(16)[None, :]) % 251
        return np.broadcast_to(v.astype(np.uint8), (4, width, 16))

    def band_window_grow(self, settings, commit=False):
        if commit:
            self.committed = True
        return self.ranges.copy()

    def reservoir_rows_bytes(self, rows):
        return 4 * rows * self.width * 16

    def reservoir_rows(self, buf, frame_row0, rows, data=None, store=False, stream=None):
        r0 = frame_row0 - self.row0
        assert 0 <= r0 and r0 + rows <= self.rows
        if data is None:
            data = np.empty(self.reservoir_rows_bytes(rows), np.uint8)
        view = data.reshape(4, rows, self.width, 16)
        if store:
            self.store[buf, :, r0: r0 + rows] = view
        else:
            view[...] = self.store[buf, :, r0: r0 + rows]
        return data

    def check(self):
        for b in range(len(self.ranges)):
            for side in range(2):
                y0, n = self.ranges[b, 2 * side], self.ranges[b, 2 * side + 1]
                for y in range(y0, y0 + n):
                    assert np.array_equal(self.store[b, :, y - self.row0], self.truth(b, y, self.width)), (b, y)
        assert self.committed


MARGINS = [0, 10, 10, 10, 16, 16, 20, 20, 36, 36]


def _refill_worker(rank, world, port, bounds, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root / "bevy-hikari_amd"))
    import torch.distributed as dist

    from hikari_amd.bands import band_of, refill_windows
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = -1
    try:
        fake = _FakeBand(band_of(rank, world, bounds[-1], bounds), bounds[-1], 8, MARGINS)
        got = refill_windows(fake, None, bounds, rank, world, device="cpu")
        fake.check()
        q.put((rank, got, None))
    except Exception as e:  # reported through the queue, so the test fails instead of waiting
        q.put((rank, got, repr(e)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("bounds", [[0, 48, 96], [0, 40, 56, 120, 160], [0, 24, 48, 72, 96, 120, 144]],
                         ids=["world2", "world4-uneven", "world6-narrow"])
def test_band_window_refill_exchange(bounds):
    """bands.refill_windows (a settings change widening the bands' light-pass windows): every rank's needs are
    all-gathered and each row block comes point-to-point from the band whose core holds it — across two bands when
    a band is narrower than the margin (world6-narrow: 24-row bands, 36-row margins); the in-process form
    (refill_windows_local) moves the same blocks."""
    import torch.multiprocessing as mp

    from hikari_amd.bands import band_of, refill_windows_local
    world = len(bounds) - 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_refill_worker, args=(r, world, port, bounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert all(err is None for _, _, err in res), res
    local = [(band_of(k, world, bounds[-1], bounds), _FakeBand(band_of(k, world, bounds[-1], bounds), bounds[-1], 8,
                                                               MARGINS)) for k in range(world)]
    moved = refill_windows_local(local, None)
    for _, fake in local:
        fake.check()
    assert moved == sum(got for _, got, _ in res) > 0



TW, TH = 128, 128


def _tile_render(tile=None, counters=False):
    from oracle import Oracle

    from hikari_amd import HikariSettings, Upscale, examples, frame_inputs, load_noise
    scene, cam, lights = examples.cornell()
    desc = scene.build()
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=True, denoise=True)
    s = st.to_c()
    o = Oracle(desc, load_noise(), TW, TH, 1.0, threads=2)
    if tile is not None:
        o.set_tile(tile.x0, tile.cols, tile.y0, tile.rows, 40)
    for f in range(3):
        fi = frame_inputs(f, cam, lights, TW, TH)
        o.render_gbuffer(fi)
        o.render_frame(s, fi)
        o.denoise(s, fi)
        o.tone_sum(s)
    img = o.output(10)
    c = o.counters()
    o.close()
    return (img, c) if counters else img


def _tile_worker(rank, world, port, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    for p in (root / "bevy-hikari_amd", root / "oracle", root / "tests"):
        sys.path.insert(0, str(p))
    import torch
    import torch.distributed as dist

    from hikari_amd.bands import aligned_bounds, tile_gather_shape, tile_grid, tile_of
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ny, nx = tile_grid(world)
        rb, cb = aligned_bounds(ny, TH), [aligned_bounds(nx, TW)] * ny
        t = tile_of(rank, world, TW, TH, rb, cb)
        img, cnt = _tile_render(t, counters=True)
        rows, cols = tile_gather_shape(rb, cb)
        mine = np.zeros((rows, cols, 8), np.uint8)
        mine[: t.rows, : t.cols] = img[t.y0: t.y0 + t.rows, t.x0: t.x0 + t.cols]
        full = torch.empty((world * rows, cols, 8), dtype=torch.uint8)
        dist.all_gather_into_tensor(full, torch.from_numpy(mine))
        n = torch.tensor([cnt["traverse_top"], cnt["traverse_emitter"], cnt["primary"]], dtype=torch.int64)
        dist.all_reduce(n)
        if rank == 0:
            q.put((full.numpy().reshape(world, rows, cols, 8).copy(), n.tolist(), None))
    except Exception as e:  # reported through the queue
        q.put((None, None, repr(e)))
    dist.barrier()
    dist.destroy_process_group()


def test_rank_tiles_reassemble_whole_frame():
    """2-D tiles (hk_resize_tile's decomposition, north_star "frames tile-partition across the GPUs"): 4 gloo ranks
    each render a 64x64 tile of a 128x128 frame plus a 40-pixel halo on every side with their own oracle context
    (hko_set_tile: only those rows and columns computed), all-gather the padded tiles and reassemble them
    (bands.tile_reassembly_copies): the frame equals the whole-frame render (spatial reuse and the denoiser on).  (The
    oracle counts the halo's rays too; the GPU tile test checks that the contexts count only their own pixels.)"""
    import torch
    import torch.multiprocessing as mp

    from hikari_amd.bands import aligned_bounds, tile_grid, tile_of, tile_reassembly_copies
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tile_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, counts, err = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert err is None, err
    ny, nx = tile_grid(world)
    assert (ny, nx) == (2, 2)
    tiles = [tile_of(k, world, TW, TH, aligned_bounds(ny, TH), [aligned_bounds(nx, TW)] * ny) for k in range(world)]
    frame = torch.zeros((TH, TW, 8), dtype=torch.uint8)
    for dst, src in tile_reassembly_copies(frame, torch.from_numpy(gathered), tiles):
        dst.copy_(src)
    whole = _tile_render(None)
    assert np.array_equal(frame.numpy(), whole)
    assert all(v > 0 for v in counts)


@pytest.mark.parametrize("world", [2, 4, 6, 8])
def test_tiles_partition_and_rebalance(world):
    """Tile geometry: the tiles of every world size partition the frame, and rebalance_tiles keeps a partition while
    moving the boundaries towards equal per-tile times."""
    from hikari_amd.bands import aligned_bounds, rebalance_tiles, tile_grid, tile_of
    W, H = 3840, 2160
    ny, nx = tile_grid(world)
    rb, cb = aligned_bounds(ny, H), [aligned_bounds(nx, W)] * ny
    for _ in range(2):
        cover = np.zeros((H, W), np.int32)
        tiles = [tile_of(k, world, W, H, rb, cb) for k in range(world)]
        for t in tiles:
            cover[t.y0: t.y0 + t.rows, t.x0: t.x0 + t.cols] += 1
        assert (cover == 1).all()
        times = [1.0 + (t.y0 + t.rows / 2) / H + 0.5 * (t.x0 > 0) for t in tiles]  # costlier lower / right tiles
        rb, cb = rebalance_tiles(rb, cb, times)
        assert rb[0] == 0 and rb[-1] == H and all(c[0] == 0 and c[-1] == W for c in cb)
