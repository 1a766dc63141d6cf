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
