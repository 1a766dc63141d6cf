"""Per-pass row windows of a band (hk_runtime.hip pass_window), checked on the CPU.

A band context runs each pass only on the halo rows the later passes read.  The windows are
constants in hk_runtime.hip; this test reads them from the source and checks the coverage rule the
bit-exactness of the band's core rows rests on: for every pass P that reads the output of pass Q
at up to R rows away, window(Q) >= window(P) + R, down to the tone-sum on the core rows.  The
reaches are the reference's: spatial reuse RANGE 20 (indirect) / 10 (emissive) for the temporal
reservoirs and the depth it marches through (light.wgsl:1568-1600), the 3x3 variance blur of
demodulation (denoise.wgsl:151-159), the a-trous steps 8, 4, 2, 1 of levels 0..3
(denoise.wgsl:101-114).  The GPU side of the claim is test_gpu_parity.py::
test_gpu_row_bands_match_whole_frame (3 and 4 bands of 192 rows, windows strictly inside the frame).
"""
import itertools
import re
from pathlib import Path

import pytest

SRC = Path(__file__).resolve().parents[1] / "bevy-hikari_amd" / "csrc" / "hk_runtime.hip"


def _constants():
    text = SRC.read_text()
    c = dict((k, int(v)) for k, v in re.findall(r"(DENOISE_OUT_REACH|SPATIAL_RANGE|EMISSIVE_SPATIAL_RANGE) = (\d+)", text))
    c["GBUFFER_REACH"] = c["DENOISE_OUT_REACH"] + c["SPATIAL_RANGE"]
    assert "GBUFFER_REACH = DENOISE_OUT_REACH + SPATIAL_RANGE" in text
    levels = re.search(r"LEVEL_REACH\[4\] = \{(\d+), (\d+), (\d+), (\d+)\}", text)
    c["LEVEL_REACH"] = tuple(int(v) for v in levels.groups())
    assert "pass_window(c, A, DENOISE_OUT_REACH - 1)" in text  # demodulation
    halo = int(re.search(r"constexpr int32_t BAND_HALO = (\d+);", text).group(1))
    c["BAND_HALO"] = halo
    return c


def _windows(c, indirect_spatial, emissive_spatial, denoise):
    """The margins hk_render_gbuffer / hk_render_frame / hk_denoise / hk_tone_sum pass to pass_window."""
    out = c["DENOISE_OUT_REACH"] if denoise else 0
    rng = c["SPATIAL_RANGE"] if indirect_spatial else (c["EMISSIVE_SPATIAL_RANGE"] if emissive_spatial else 0)
    w = {"gbuffer": c["GBUFFER_REACH"], "temporal": out + rng, "spatial": out, "tone": 0}
    if denoise:
        w["demod"] = c["DENOISE_OUT_REACH"] - 1
        for k in range(4):
            w[f"L{k}"] = c["LEVEL_REACH"][k]
    return w


def _reads(indirect_spatial, emissive_spatial, denoise):
    """(consumer, producer, reach in rows) of every neighbour or own-pixel read between passes."""
    light = "spatial" if (indirect_spatial or emissive_spatial) else "temporal"
    r = [("temporal", "gbuffer", 0)]
    if indirect_spatial or emissive_spatial:
        rng = 20 if indirect_spatial else 10
        r += [("spatial", "temporal", rng), ("spatial", "gbuffer", rng)]
        # a channel without spatial reuse feeds demodulation / tone from its temporal pass
        r += [(("demod" if denoise else "tone"), "temporal", 1 if denoise else 0)]
    if denoise:
        r += [("demod", light, 1), ("demod", "gbuffer", 0), ("L0", "demod", 8), ("L1", "L0", 4),
              ("L2", "L1", 2), ("L3", "L2", 1), ("L3", "gbuffer", 0), ("tone", "L3", 0)]
    else:
        r += [("tone", light, 0)]
    return r


@pytest.mark.parametrize("indirect_spatial,emissive_spatial,denoise", list(itertools.product([False, True], repeat=3)))
def test_pass_windows_cover_every_read(indirect_spatial, emissive_spatial, denoise):
    c = _constants()
    w = _windows(c, indirect_spatial, emissive_spatial, denoise)
    for consumer, producer, reach in _reads(indirect_spatial, emissive_spatial, denoise):
        assert w[producer] >= w[consumer] + reach, (consumer, producer, reach, w)
    assert max(w.values()) <= c["BAND_HALO"]  # every window fits the allocated halo


def test_windows_shrink_the_redundant_work():
    """City 4K, 8 bands of 270 rows: per-pass windows do 1.15x the core rows' work (uniform 40-row
    halos: 1.30x), weighted by the round-2 serial kernel times (profiles/r02/serial_city-4k.json)."""
    c = _constants()
    w = _windows(c, True, False, True)
    ms = {"gbuffer": 0.362, "temporal": 1.629 + 0.584, "spatial": 2.052, "demod": 0.462,
          "L0": 0.426, "L1": 0.426, "L2": 0.426, "L3": 0.426, "tone": 0.057}
    core = 270
    windowed = sum(t * (core + 2 * w[p]) for p, t in ms.items()) / (core * sum(ms.values()))
    uniform = (core + 2 * 40) / core
    assert windowed < 1.16 and uniform > 1.29
