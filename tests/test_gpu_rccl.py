"""The per-peer exchange paths at world size 1 over RCCL (bench.py's world-1 line): gloo has no
point-to-point to self (its pair to rank 0 is never connected), so this runs on the GPU with the nccl (RCCL) backend in
a child process: the row band sent by the rank to itself arrives in self_buf, and the stripes' own part reaches its
slot of the gathered frame through the self send instead of a copy."""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _self_worker(port, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root / "bevy-hikari_amd"))
    try:
        import torch
        import torch.distributed as dist

        from hikari_amd.bands import peer_exchange, peer_gather
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        frame = torch.arange(1080 * 64 * 4, dtype=torch.float32, device="cuda").reshape(1080, 64, 4).half()
        got = torch.zeros_like(frame)
        for req in peer_exchange(frame, [0, 1080], 0, 1, self_buf=got):
            req.wait()
        full = torch.zeros_like(frame)
        for req in peer_gather(full, frame, 0, 1, self_transfer=True):
            req.wait()
        torch.cuda.synchronize()
        q.put((bool(torch.equal(got, frame)), bool(torch.equal(full, frame)), None))
        dist.destroy_process_group()
    except Exception as e:  # reported through the queue
        q.put((False, False, repr(e)))


def test_world1_peer_paths_send_to_self():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_self_worker, args=(_free_port(), q))
    p.start()
    band_ok, stripe_ok, err = q.get(timeout=100)
    p.join(timeout=60)
    assert err is None and band_ok and stripe_ok, err
    assert p.exitcode == 0
