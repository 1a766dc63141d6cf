"""Diagnose a GPU-vs-oracle mismatch: render cornell to a frame, print differing words per output."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, "bevy-hikari_amd")
sys.path.insert(0, "oracle")
from parity import canon_plane
from hikari_amd import HikariRenderer, HikariSettings, Upscale, examples, frame_inputs, load_noise
from oracle import Oracle

w, h = 64, 64
st = HikariSettings(upscale=Upscale.SMAA_TU_1_0)
scene, cam, lights = examples.cornell()
desc = scene.build()
r = HikariRenderer(0); r.set_noise(); r.upload_scene(scene); r.resize(w, h, 1.0)
o = Oracle(desc, load_noise(), w, h, 1.0)
s = st.to_c()
for f in range(2):
    fi = frame_inputs(f, cam, lights, w, h)
    for x in (r, o):
        x.render_gbuffer(fi); x.render_frame(s, fi); x.denoise(s, fi); x.tone_sum(s)
    for oid in range(17):
        a, b = r.output(oid), o.output(oid)
        ca, cb = canon_plane(oid, a), canon_plane(oid, b)
        d = np.argwhere(ca != cb)
        if len(d):
            print("frame", f, "output", oid, "n", len(d))
            for idx in d[:4]:
                pa, pb = a[tuple(idx[:2])], b[tuple(idx[:2])]; print("   ", idx, pa.view(np.float16) if len(pa) == 8 else pa, pb.view(np.float16) if len(pb) == 8 else pb)
import oracle as orc
L = orc.lib()
vals = np.arange(0, 1 << 32, 256, dtype=np.uint64).astype(np.uint32).view(np.float32)
g = r.selftest_f16(vals)
want = np.empty(len(vals), np.uint16)
L.hko_f32_to_f16_array(vals.ctypes.data, len(vals), want.ctypes.data)
bad = np.flatnonzero((g != want) & ~np.isnan(vals))
print("f16 mismatches", len(bad), [(hex(vals.view(np.uint32)[i]), hex(g[i]), hex(want[i])) for i in bad[:8]])
