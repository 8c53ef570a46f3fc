"""Deterministic synthetic byte streams shared by tests, golden fixtures and bench.py.

Byte i of stream(seed) is byte (i & 7), little-endian, of
splitmix64_mix(seed + ((i >> 3) + 1) * 0x9E3779B97F4A7C15) -- the same
generator as oracle_fill_splitmix (oracle/crc32_ref.c) and the device fill
kernel (ambrycrc_fill_random_dev).
"""
from __future__ import annotations

import numpy as np

_G = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def stream_bytes(seed: int, stream_off: int, n: int) -> np.ndarray:
    if n == 0:
        return np.zeros(0, dtype=np.uint8)
    w0 = stream_off >> 3
    w1 = (stream_off + n + 7) >> 3
    with np.errstate(over="ignore"):
        k = np.arange(w0, w1, dtype=np.uint64)
        words = _mix(np.uint64(seed) + (k + np.uint64(1)) * _G)
    b = words.astype("<u8").view(np.uint8)
    s = stream_off - (w0 << 3)
    return b[s:s + n].copy()


def zipf_sizes(n: int, seed: int = 20261015, alpha: float = 1.2, unit: int = 4096, rmax: int = 1024):
    """C4's size distribution: unit * r, r ~ Zipf(alpha) truncated to [1, rmax]
    by inverse CDF from numpy.random.default_rng(seed)."""
    rng = np.random.default_rng(seed)
    r = np.arange(1, rmax + 1, dtype=np.float64)
    pmf = r ** (-alpha)
    cdf = np.cumsum(pmf) / pmf.sum()
    u = rng.random(n)
    idx = np.searchsorted(cdf, u, side="left")
    return (idx + 1).astype(np.int64) * unit
