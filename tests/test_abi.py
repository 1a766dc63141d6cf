"""The C-ABI library loads without a GPU and exports every symbol include/*.h declares."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def declared_symbols():
    names = set()
    for h in ("hikari_amd.h", "hikari_scene.h"):
        text = (ROOT / "include" / h).read_text()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \t\*]*?\b(hks?_\w+)\s*\(", text, flags=re.M):
            names.add(m.group(1))
    return names


def test_headers_declare_expected_entry_points():
    names = declared_symbols()
    for required in ("hk_create", "hk_destroy", "hk_scene_upload", "hk_resize", "hk_render_frame", "hk_denoise",
                     "hk_tone_sum", "hk_get_output", "hk_trace", "hk_last_error", "hks_build"):
        assert required in names


def test_library_exports_all_declared_symbols():
    import hikari_amd
    L = hikari_amd._abi.lib()
    missing = [n for n in sorted(declared_symbols()) if not hasattr(L, n)]
    assert not missing, f"declared but not exported: {missing}"
    assert set(hikari_amd._abi.EXPORTED_SYMBOLS) == declared_symbols()


def test_abi_version_and_defaults():
    import ctypes as C

    import hikari_amd
    L = hikari_amd._abi.lib()
    assert L.hk_abi_version() == 3
    s = hikari_amd._abi.hk_settings()
    L.hk_settings_default(C.byref(s))
    # HikariSettings::default() (lib.rs:435-455)
    assert (s.direct_validate_interval, s.emissive_validate_interval) == (3, 5)
    assert (s.max_temporal_reuse_count, s.max_spatial_reuse_count) == (50, 800)
    assert s.max_reservoir_lifetime == 100.0 and abs(s.solar_angle - 0.046) < 1e-7
    assert s.indirect_bounces == 1 and s.max_indirect_luminance == 10.0
    assert (s.temporal_reuse, s.emissive_spatial_reuse, s.indirect_spatial_reuse, s.denoise) == (1, 0, 1, 1)
    assert s.upscale_ratio == 2.0
    py = hikari_amd.HikariSettings().to_c()
    for f, _ in hikari_amd._abi.hk_settings._fields_:
        a, b = getattr(s, f), getattr(py, f)
        if hasattr(a, "__len__"):
            assert list(a) == pytest.approx(list(b), abs=1e-6), f
        else:
            assert a == pytest.approx(b, abs=1e-6), f


def test_upscale_ratio_clamps():
    from hikari_amd import Upscale
    assert Upscale.smaa_tu4x(0.5).ratio() == 1.0
    assert Upscale.smaa_tu4x(3.0).ratio() == 2.0
    assert Upscale.fsr1(1.5, 0.2).ratio() == 1.5 and Upscale.fsr1(1.5, 0.2).sharpness() == 0.2
    assert Upscale.SMAA_TU_2_0.sharpness() == 0.0


def test_create_without_gpu_fails_cleanly():
    """No gfx950 device in this container: hk_create must report it, not crash or fall back."""
    import ctypes as C

    import hikari_amd
    if Path("/dev/kfd").exists():
        pytest.skip("a GPU is visible")
    L = hikari_amd._abi.lib()
    h = C.c_void_p()
    rc = L.hk_create(0, C.byref(h))
    assert rc in (hikari_amd._abi.HK_ERR_NO_DEVICE, hikari_amd._abi.HK_ERR_HIP) and not h.value
    with pytest.raises(hikari_amd.HikariError):
        hikari_amd.HikariRenderer(0)


def test_struct_sizes_match_header(tmp_path):
    """ctypes mirrors == the C compiler's view of include/hikari_amd.h (sizes and offsets)."""
    import ctypes as C
    import subprocess

    import hikari_amd
    A = hikari_amd._abi
    checks = {"hk_settings": A.hk_settings, "hk_view": A.hk_view, "hk_lights": A.hk_lights,
              "hk_frame_inputs": A.hk_frame_inputs, "hk_scene_desc": A.hk_scene_desc, "hk_counters": A.hk_counters,
              "hk_array": A.hk_array}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "hikari_amd.h"', "int main(void){"]
    for name, cls in checks.items():
        lines.append(f'printf("{name} %zu\\n", sizeof({name}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{name}.{f} %zu\\n", offsetof({name}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "sizes.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "sizes"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    out = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                        check=True).stdout.split("\n") if l)
    for name, cls in checks.items():
        assert int(out[name]) == C.sizeof(cls), name
        for f, _ in cls._fields_:
            assert int(out[f"{name}.{f}"]) == getattr(cls, f).offset, f"{name}.{f}"
    assert hikari_amd.RESERVOIR_DTYPE.itemsize == 64


def test_runtime_options_documented():
    """Every runtime option key (hk_option_name) is documented in include/hikari_amd.h's hk_set_option
    comment, and nothing on the frame path reads the environment (options through the ABI)."""
    import hikari_amd
    L = hikari_amd._abi.lib()
    keys, i = [], 0
    while L.hk_option_name(i) is not None:
        keys.append(L.hk_option_name(i).decode())
        i += 1
    assert len(keys) >= 15 and L.hk_option_name(-1) is None
    root = Path(__file__).resolve().parents[1]
    header = (root / "include" / "hikari_amd.h").read_text()
    doc = header[header.index("Runtime options"):header.index("int hk_set_option")]
    for k in keys:
        assert re.search(r"\b" + k + r"\b", doc), f"option {k} not documented"
    for src in (root / "bevy-hikari_amd" / "csrc").glob("*"):
        assert "getenv" not in src.read_text(), f"{src.name} reads the environment"
