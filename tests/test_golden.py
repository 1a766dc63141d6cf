"""The oracle still reproduces the committed golden digests (tests/golden/make_golden.py)."""
import json
from pathlib import Path

import pytest

import make_golden_path  # noqa: F401  (adds tests/golden to sys.path)
from make_golden import FRAMES, VARIANTS, oracle_factory, render

GOLD = json.loads((Path(__file__).parent / "golden" / "cornell_golden.json").read_text())


@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_oracle_matches_golden(variant):
    frames, _ = render(oracle_factory, variant)
    want = GOLD["variants"][variant]["digests"]
    assert len(frames) == FRAMES
    for f, (a, b) in enumerate(zip(frames, want)):
        bad = [k for k in b if a[k] != b[k]]
        assert not bad, f"frame {f}: {bad}"
