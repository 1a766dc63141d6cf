"""The reference-held inputs this build commits as assets, pinned to the reference checkout.

The reference ships no golden vectors for the path; its input assets are the only reference-held
pins: the blue-noise textures (src/noise/LDR_RGBA_{0..15}.png, loaded as linear Rgba8Unorm, lib.rs:189-219), the
Cornell box (assets/models/cornell.glb, examples/cornell.rs) and the City scene's layout (assets/models/City/
scene.gltf, the proxy geometry of configs 3-5).  The committed files must equal what bevy-hikari_amd/tools/
extract_assets.py derives from the checkout.  Skipped where /root/reference is absent (the GPU box)."""
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
REF = Path("/root/reference")
ASSETS = ROOT / "bevy-hikari_amd" / "hikari_amd" / "assets"

pytestmark = pytest.mark.skipif(not REF.is_dir(), reason="reference checkout absent")


def _tools():
    p = str(ROOT / "bevy-hikari_amd" / "tools")
    if p not in sys.path:
        sys.path.insert(0, p)
    import extract_assets
    return extract_assets


def test_blue_noise_equals_reference_pngs():
    pytest.importorskip("PIL")
    want = _tools().blue_noise(REF)
    got = np.fromfile(ASSETS / "blue_noise_16x64x64_rgba8.bin", np.uint8).reshape(16, 64, 64, 4)
    assert np.array_equal(got, want)
    # and the package's loader hands exactly these bytes to hk_set_noise
    sys.path.insert(0, str(ROOT / "bevy-hikari_amd"))
    from hikari_amd import load_noise
    assert np.array_equal(np.asarray(load_noise(), np.uint8).reshape(16, 64, 64, 4), want)


def test_cornell_glb_is_the_reference_file():
    assert (ASSETS / "cornell.glb").read_bytes() == (REF / "assets" / "models" / "cornell.glb").read_bytes()


def test_city_layout_rederived_without_diff():
    t = _tools()
    assert (ASSETS / "city_layout.json").read_text() == t.city_layout_text(t.city_layout(REF))
