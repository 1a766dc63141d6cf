"""Traversal micro-benchmark (development aid): the stand-alone reference-order ray query (hk_trace,
k_trace) over rays shaped like the integrator's — shadow rays and cosine bounce rays from the
cornell G-buffer's surfaces, in 8x8 tile order — on device-resident buffers.
usage: python tools/trace_bench.py [W H [shadow|bounce|all]]"""
import sys, time
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'bevy-hikari_amd'))
import numpy as np
import torch
from hikari_amd import HikariRenderer, examples, frame_inputs, _abi

W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (1920, 1080)
ONLY = sys.argv[3] if len(sys.argv) > 3 else None  # shadow | bounce | all
scene, cam, lights = examples.cornell()
scene.build()
r = HikariRenderer(0); r.set_noise(); r.upload_scene(scene); r.resize(W, H, 1.0)
r.render_gbuffer(frame_inputs(0, cam, lights, W, H))
pos = r.output(_abi.OUT_GBUF_POSITION).view(np.float32).reshape(H, W, 4)
nrm = r.output(_abi.OUT_GBUF_NORMAL).view(np.int8).reshape(H, W, 4)[..., :3].astype(np.float32) / 127.0
# 8x8 tile order
ty, tx = np.meshgrid(np.arange(H), np.arange(W), indexing='ij')
key = ((ty // 8) * ((W + 7) // 8) + tx // 8) * 64 + (ty % 8) * 8 + tx % 8
order = np.argsort(key.ravel(), kind='stable')
P = pos.reshape(-1, 4)[order]; N = nrm.reshape(-1, 3)[order]
N = N / np.maximum(np.linalg.norm(N, axis=1, keepdims=True), 1e-6)
cov = P[:, 3] > 1e-7
rng = np.random.default_rng(1)
origin = P[:, :3] + N * 0.02

def run(name, dirs, mask, early, maxd=np.float32(3.4e38)):
    if ONLY and not name.startswith(ONLY):
        return
    o = origin[mask]; d = dirs[mask].astype(np.float32)
    rays = torch.tensor(np.concatenate([o, d], 1).astype(np.float32), device='cuda')
    n = len(rays)
    md = torch.full((n,), float(maxd), device='cuda'); ed = torch.full((n,), float(early), device='cuda')
    ex = torch.full((n,), 0xFFFFFFFF, dtype=torch.int64, device='cuda').to(torch.int32)
    hits = torch.empty((n, 5), dtype=torch.int32, device='cuda')
    def go():
        _abi.lib().hk_trace(r.ctx, C.c_void_p(rays.data_ptr()), C.c_void_p(md.data_ptr()), C.c_void_p(ed.data_ptr()),
                            C.c_void_p(ex.data_ptr()), n, C.c_void_p(hits.data_ptr()), 1, None)
    for _ in range(3): go()
    torch.cuda.synchronize(); t = time.time(); K = 20
    for _ in range(K): go()
    torch.cuda.synchronize(); dt = (time.time() - t) / K
    print(f"{name:28s} rays {n/1e6:.3f}M  {dt*1e6:8.1f} us  {n/dt/1e9:6.2f} Grays/s")

import ctypes as C
phi = rng.random(len(P)) * 2 * np.pi
xy = np.stack([np.cos(phi), np.sin(phi), np.zeros_like(phi)], 1)
run("shadow XY any-hit (direct)", xy, cov & ((xy * N).sum(1) > 0), 65535.0)
u1, u2 = rng.random(len(P)), rng.random(len(P))
rr = np.sqrt(u1); th = 2 * np.pi * u2
loc = np.stack([rr * np.cos(th), rr * np.sin(th), np.sqrt(1 - u1)], 1)
a = np.where(np.abs(N[:, :1]) > 0.9, np.array([[0, 1, 0]]), np.array([[1, 0, 0]]))
t1 = np.cross(N, a); t1 /= np.linalg.norm(t1, axis=1, keepdims=True); t2 = np.cross(N, t1)
hemi = t1 * loc[:, :1] + t2 * loc[:, 1:2] + N * loc[:, 2:]
run("bounce closest (indirect)", hemi, cov, 0.0)
run("all pixels closest", hemi, np.ones(len(P), bool), 0.0)
