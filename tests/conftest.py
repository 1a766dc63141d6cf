import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "bevy-hikari_amd", ROOT / "oracle", ROOT / "tests"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    return oracle.lib()


@pytest.fixture
def hk_options(monkeypatch):
    """Runtime options (hk_set_option) for every HikariRenderer the test creates: a dict the test fills
    before creating its contexts (kernel variants and schedules; results must not depend on them)."""
    from hikari_amd import HikariRenderer
    opts = {}
    monkeypatch.setattr(HikariRenderer, "defaults", opts)
    return opts
