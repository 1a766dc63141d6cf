"""Mirror of bevy-hikari's public settings API (src/lib.rs).

`HikariSettings` (lib.rs:400-455), `HikariUniversalSettings` (lib.rs:372-389), `Taa`
(lib.rs:470-476) and `Upscale` (lib.rs:478-513) keep the reference's field names, defaults
and semantics; `to_c()` produces the `hk_settings` record the C ABI consumes.
"""
from __future__ import annotations

import enum
from dataclasses import dataclass, field

from . import _abi


class Taa(enum.Enum):
    Jasmine = 0
    None_ = 1


@dataclass(frozen=True)
class Upscale:
    """`Upscale::Fsr1 { ratio, sharpness }` or `Upscale::SmaaTu4x { ratio }`."""

    kind: str = "SmaaTu4x"
    ratio_: float = 2.0
    sharpness_: float = 0.0

    @staticmethod
    def smaa_tu4x(ratio: float) -> "Upscale":
        return Upscale("SmaaTu4x", ratio, 0.0)

    @staticmethod
    def fsr1(ratio: float, sharpness: float) -> "Upscale":
        return Upscale("Fsr1", ratio, sharpness)

    def ratio(self) -> float:
        """lib.rs:501-505: clamped to [1, 2]."""
        return min(max(self.ratio_, 1.0), 2.0)

    def sharpness(self) -> float:
        return self.sharpness_ if self.kind == "Fsr1" else 0.0


Upscale.SMAA_TU_1_0 = Upscale.smaa_tu4x(1.0)
Upscale.SMAA_TU_2_0 = Upscale.smaa_tu4x(2.0)


def srgb_to_linear(c: float) -> float:
    """Bevy `Color::rgb` is sRGB; conversion used by `as_linear_rgba_f32`."""
    return c / 12.92 if c <= 0.04045 else ((c + 0.055) / 1.055) ** 2.4


@dataclass
class HikariSettings:
    """Camera component; defaults = `HikariSettings::default()` (lib.rs:435-455)."""

    direct_validate_interval: int = 3
    emissive_validate_interval: int = 5
    max_temporal_reuse_count: int = 50
    max_spatial_reuse_count: int = 800
    max_reservoir_lifetime: float = 100.0
    solar_angle: float = 0.046
    indirect_bounces: int = 1
    max_indirect_luminance: float = 10.0
    clear_color: tuple = (0.4, 0.4, 0.4, 1.0)  # sRGB `Color::rgb(0.4, 0.4, 0.4)`
    temporal_reuse: bool = True
    emissive_spatial_reuse: bool = False
    indirect_spatial_reuse: bool = True
    denoise: bool = True
    taa: Taa = Taa.Jasmine
    upscale: Upscale = field(default_factory=lambda: Upscale.SMAA_TU_2_0)

    def to_c(self) -> _abi.hk_settings:
        s = _abi.hk_settings()
        s.direct_validate_interval = int(self.direct_validate_interval)
        s.emissive_validate_interval = int(self.emissive_validate_interval)
        s.max_temporal_reuse_count = int(self.max_temporal_reuse_count)
        s.max_spatial_reuse_count = int(self.max_spatial_reuse_count)
        s.max_reservoir_lifetime = float(self.max_reservoir_lifetime)
        s.solar_angle = float(self.solar_angle)
        s.indirect_bounces = int(self.indirect_bounces)
        s.max_indirect_luminance = float(self.max_indirect_luminance)
        cc = [srgb_to_linear(c) for c in self.clear_color[:3]] + [self.clear_color[3]]
        for i in range(4):
            s.clear_color[i] = float(cc[i])
        s.temporal_reuse = int(bool(self.temporal_reuse))
        s.emissive_spatial_reuse = int(bool(self.emissive_spatial_reuse))
        s.indirect_spatial_reuse = int(bool(self.indirect_spatial_reuse))
        s.denoise = int(bool(self.denoise))
        s.taa = self.taa.value
        s.upscale_ratio = float(self.upscale.ratio())
        s.upscale = 0 if self.upscale.kind == "SmaaTu4x" else 1
        return s


@dataclass
class HikariUniversalSettings:
    """Resource; gates the acceleration-structure builds (mesh.rs:115-117, instance.rs:257-259)."""

    build_mesh_acceleration_structure: bool = True
    build_instance_acceleration_structure: bool = True
