"""Deterministic synthetic packet bytes shared by the fixture generator, the tests and bench.py.

splitmix64 (Steele/Lea/Flood), little-endian byte order: byte j of a stream
seeded with `seed` is byte (j % 8) of output (j // 8) of
    z_i = mix(seed + (i + 1) * 0x9E3779B97F4A7C15).
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

ENET_SEED = 0x454E4554  # "ENET", BASELINE.md C1


def splitmix64_bytes(seed: int, n: int) -> np.ndarray:
    words = (n + 7) // 8
    with np.errstate(over="ignore"):
        i = np.arange(1, words + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + i * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:n].copy()


def ragged_lengths(seed: int, count: int, lo: int = 64, hi: int = 1392) -> np.ndarray:
    """Lengths ~ U{lo..hi} (BASELINE config 3), from the same generator."""
    raw = splitmix64_bytes(seed, 8 * count).view("<u8")
    return (lo + (raw % np.uint64(hi - lo + 1))).astype(np.uint32)


def packed_offsets(lengths: np.ndarray) -> np.ndarray:
    off = np.zeros(lengths.size, dtype=np.uint64)
    if lengths.size > 1:
        np.cumsum(lengths[:-1], dtype=np.uint64, out=off[1:])
    return off


def enet_like_bytes(seed: int, n: int) -> np.ndarray:
    """Compressible game-traffic-like bytes for the range-coder workloads: per byte,
    ~50 % a small value (0..15), ~25 % zero, ~25 % uniform, from the splitmix64 stream."""
    r = splitmix64_bytes(seed, 2 * n).reshape(-1, 2) if n else np.zeros((0, 2), np.uint8)
    sel, v = r[:, 0], r[:, 1]
    out = np.where(sel < 128, v & np.uint8(15), np.where(sel < 192, np.uint8(0), v))
    return out.astype(np.uint8)
