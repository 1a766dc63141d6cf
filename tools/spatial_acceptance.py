"""Which of spatial reuse's rejection tests reject how many neighbours (light.wgsl:1566-1628), on an
oracle city frame: a numpy pass over every covered pixel x 16 neighbours with approximate float64
arithmetic — statistics for design decisions, not a parity check.  CPU only.
usage: python tools/spatial_acceptance.py <width> <height>   (results: profiles/r03/spatial_acceptance.txt)"""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "bevy-hikari_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
from hikari_amd import HikariSettings, Taa, Upscale, examples, frame_inputs, load_noise
from oracle import Oracle
W, H = int(sys.argv[1]), int(sys.argv[2])
scene, cam, lights = examples.city()
st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, taa=Taa.None_, indirect_spatial_reuse=True, denoise=False)
s = st.to_c()
o = Oracle(scene.build(), load_noise(), W, H, 1.0, threads=8)
t = time.time()
F = 4
for f in range(F):
    fi = frame_inputs(f, cam, lights, W, H); o.render_gbuffer(fi); o.render_frame(s, fi)
print("oracle", time.time() - t)
f = F - 1; previous = 1 - f % 2
rec = o.reservoirs(previous + 6).view(np.uint32).reshape(-1, 16)[: W * H]
pos = o.output(11).view(np.float32).reshape(H, W, 4); depth = pos[..., 3]
def snorm(u, k): return np.maximum(((u >> (8 * k)) & 0xFF).astype(np.uint8).view(np.int8).astype(np.float32) / 127.0, -1.0)
def nrm(u):
    v = np.stack([snorm(u, k) for k in range(3)], -1); return v / np.linalg.norm(v, axis=-1, keepdims=True).clip(1e-30)
vn = nrm(rec[:, 12]).reshape(H, W, 3)
cnt = rec[:, 14].astype(np.uint16).view(np.float16).astype(np.float32).reshape(H, W)
sp = rec[:, 8:11].view(np.float32).reshape(H, W, 3); vp = rec[:, 4:7].view(np.float32).reshape(H, W, 3)
rnd = np.stack([(rec[:, 2] & 0xFFFF), rec[:, 2] >> 16, rec[:, 3] & 0xFFFF, rec[:, 3] >> 16], -1).astype(np.float32) / 65535
srand = rnd.sum(-1).reshape(H, W)
import indirect_python as ip
rf = float(ip.random_float(f))
yy, xx = np.mgrid[0:H, 0:W]
cov = depth >= 1.1920929e-7
stats = {k: 0 for k in ("tried", "inside", "depth", "gate", "dir", "march")}
for i in range(1, 17):
    px = 6.283185307 * np.modf(i * 1.618033989 + srand + rf)[0]
    py = np.sqrt(i / 16) * 20
    ox, oy = py * np.cos(px), py * np.sin(px)
    sx, sy = np.trunc(ox + xx).astype(int), np.trunc(oy + yy).astype(int)
    m = cov.copy(); stats["tried"] += m.sum()
    m &= (sx >= 0) & (sy >= 0) & (sx < W) & (sy < H); stats["inside"] += m.sum()
    sxc, syc = sx.clip(0, W - 1), sy.clip(0, H - 1)
    with np.errstate(all="ignore"):
        r = depth / depth[syc, sxc]
    m &= (r >= 0.9) & (r <= 1.1); stats["depth"] += m.sum()
    m &= (cnt[syc, sxc] >= 1.1920929e-7) & ((vn * vn[syc, sxc]).sum(-1) >= 0.866); stats["gate"] += m.sum()
    d = sp[syc, sxc] - vp; d /= np.linalg.norm(d, axis=-1, keepdims=True).clip(1e-30)
    m &= (d * vn).sum(-1) >= 0; stats["dir"] += m.sum()
    interval = max(1.0, py / 5); tc = int(py / interval)
    occ = np.zeros_like(m)
    ln = np.sqrt(ox * ox + oy * oy)
    for j in range(1, tc + 1):
        tx = np.trunc(xx + 0.5 + j * interval * ox / ln).astype(int); ty = np.trunc(yy + 0.5 + j * interval * oy / ln).astype(int)
        inb = (tx >= 0) & (ty >= 0) & (tx < W) & (ty < H)
        td = np.where(inb, depth[ty.clip(0, H - 1), tx.clip(0, W - 1)], 0)
        t = j / (tc + 1); ref = depth * (1 - t) + depth[syc, sxc] * t
        occ |= td > ref + 1e-5
    m &= ~occ; stats["march"] += m.sum()
print(W, H, "coverage", cov.mean(), {k: round(v / stats["tried"], 3) for k, v in stats.items()})
