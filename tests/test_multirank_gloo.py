"""N>1 path on CPU: world_size-2 gloo ranks each render their row band (+ halo) with the oracle,
all-gather the tone-mapped bands, and must reproduce the whole-frame render bit-exactly
(bands.py halo sufficiency + the gather wiring that bench.py uses with RCCL on GPUs)."""
import os
import socket

import numpy as np
import pytest

W, H, FRAMES = 40, 48, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _render(band=None, halo=40, spatial=True, denoise=True):
    from oracle import Oracle

    from hikari_amd import HikariSettings, Upscale, examples, frame_inputs, load_noise
    scene, cam, lights = examples.cornell()
    desc = scene.build()
    st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=spatial, denoise=denoise)
    s = st.to_c()
    o = Oracle(desc, load_noise(), W, H, 1.0, threads=2)
    if band is not None:
        o.set_band(band.y0, band.rows, halo)
    for f in range(FRAMES):
        fi = frame_inputs(f, cam, lights, W, H)
        o.render_gbuffer(fi)
        o.render_frame(s, fi)
        o.denoise(s, fi)
        o.tone_sum(s)
    return o.output(10)


def _stripe_worker(rank, world, port, q):
    """bench.py's stripe wiring: each rank contributes its (zero-padded) stripe rows, the gather
    is reassembled with stripe_gather_rows' index.  No pass reads neighbours in this mode, so a
    rank's stripe rows are the whole-frame render's rows (the GPU test checks the striped
    contexts themselves)."""
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
    img = _render(None, 0, False, False)
    pad, index = stripe_gather_rows(world, H)
    mine = np.zeros((pad, W, 8), np.uint8)
    rows = stripe_rows(rank, world, H)
    mine[:len(rows)] = img[rows]
    full = torch.empty((world * pad, W, 8), dtype=torch.uint8)
    dist.all_gather_into_tensor(full, torch.from_numpy(mine))
    if rank == 0:
        q.put(full.numpy()[index].copy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_stripes_reassemble_whole_frame():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stripe_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.array_equal(gathered, _render(None, 0, False, False))


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


@pytest.mark.parametrize("spatial,denoise", [(True, True), (False, False)])
def test_two_rank_bands_reassemble_whole_frame(spatial, denoise):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, spatial, denoise, q)) for r in range(2)]
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
