"""Shared helpers for the parity tests (bit-exact comparison with NaN canonicalisation)."""
from __future__ import annotations

import numpy as np

F16_IDS = {0, 4, 5, 6, 7, 8, 9, 10}   # RGBA16F planes
F32_IDS = {1, 2, 3, 11, 13, 14, 15, 16}  # f32 planes


def canon_f16(u16: np.ndarray) -> np.ndarray:
    u = u16.astype(np.uint16).copy()
    nan = ((u & 0x7C00) == 0x7C00) & ((u & 0x03FF) != 0)
    u[nan] = 0x7E00
    return u


def canon_f32(u32: np.ndarray) -> np.ndarray:
    u = u32.astype(np.uint32).copy()
    nan = ((u & 0x7F800000) == 0x7F800000) & ((u & 0x007FFFFF) != 0)
    u[nan] = 0x7FC00000
    return u


def canon_plane(output_id: int, raw: np.ndarray) -> np.ndarray:
    b = np.ascontiguousarray(raw)
    if output_id in F16_IDS:
        return canon_f16(b.view(np.uint16))
    if output_id in F32_IDS:
        return canon_f32(b.view(np.uint32))
    return b


def canon_reservoirs(r: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(r).view(np.uint32).reshape(-1, 16).copy()
    f16_words = [0, 1, 14, 15]  # radiance, reservoir (random is unorm16: compared raw)
    halves = canon_f16(np.ascontiguousarray(u[:, f16_words]).view(np.uint16))
    u[:, f16_words] = halves.view(np.uint32).reshape(len(u), len(f16_words))
    u[:, 4:12] = canon_f32(u[:, 4:12])
    return u


def mismatch_report(a: np.ndarray, b: np.ndarray, label: str) -> str:
    if a.shape != b.shape:
        return f"{label}: shape {a.shape} != {b.shape}"
    diff = a != b
    n = int(diff.sum())
    if n == 0:
        return ""
    where = np.argwhere(diff)[:5]
    return f"{label}: {n}/{a.size} words differ, first at {where.tolist()}"
