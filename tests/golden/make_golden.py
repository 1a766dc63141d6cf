"""Generate tests/golden/cornell_golden.json: SHA-256 digests of every output plane and
reservoir buffer of the CPU oracle for small Cornell renders (frames 0..5) under several
HikariSettings variants, plus the raw tone-mapped bytes of the last frame.

These are regression pins of the oracle (the reference itself cannot run here: SURVEY §8c);
tests/test_golden.py re-renders with the oracle and tests/test_gpu_parity.py with the GPU.
Run:  python tests/golden/make_golden.py
"""
import base64
import hashlib
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
for p in (ROOT / "bevy-hikari_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

from parity import canon_plane, canon_reservoirs  # noqa: E402

W, H, FRAMES = 32, 24, 6
VARIANTS = {
    "default_ratio1": dict(),
    "emissive_spatial_multibounce": dict(emissive_spatial_reuse=True, indirect_bounces=3),
    "no_temporal_no_spatial": dict(temporal_reuse=False, indirect_spatial_reuse=False),
    "no_indirect": dict(indirect_bounces=0),
    "validate_every_frame": dict(direct_validate_interval=1, emissive_validate_interval=2, max_temporal_reuse_count=8,
                                 max_spatial_reuse_count=30, max_reservoir_lifetime=3.0),
}


def settings(v):
    from hikari_amd import HikariSettings, Upscale
    return HikariSettings(upscale=Upscale.SMAA_TU_1_0, **VARIANTS[v])


def digest_frame(src):
    d = {}
    for oid in range(17):
        d[f"out{oid}"] = hashlib.sha256(canon_plane(oid, src.output(oid)).tobytes()).hexdigest()
    for rid in range(10):
        d[f"res{rid}"] = hashlib.sha256(canon_reservoirs(src.reservoirs(rid)).tobytes()).hexdigest()
    return d


def render(src_factory, variant):
    from hikari_amd import examples, frame_inputs
    scene, cam, lights = examples.cornell()
    desc = scene.build()
    src = src_factory(scene, desc)
    s = settings(variant).to_c()
    frames = []
    for f in range(FRAMES):
        fi = frame_inputs(f, cam, lights, W, H)
        src.render_gbuffer(fi)
        src.render_frame(s, fi)
        src.denoise(s, fi)
        src.tone_sum(s)
        frames.append(digest_frame(src))
    return frames, src.output(10)


def oracle_factory(scene, desc):
    from oracle import Oracle

    from hikari_amd import load_noise
    return Oracle(desc, load_noise(), W, H, 1.0, threads=4)


def main():
    out = {"size": [W, H], "frames": FRAMES, "scene": "cornell", "variants": {}}
    for v in VARIANTS:
        frames, tone = render(oracle_factory, v)
        out["variants"][v] = {"settings": VARIANTS[v], "digests": frames,
                              "tone_mapped_last_frame_b64": base64.b64encode(tone.tobytes()).decode()}
    (Path(__file__).parent / "cornell_golden.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
