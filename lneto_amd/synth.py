"""Synthetic frame batches for tests and the benchmark (BASELINE.md "Inputs").

Bytes: word k (8 bytes, little-endian) of the packed buffer is the k-th output
of splitmix64 seeded with SEED (0x6C6E65746F, "lneto"): a counter hash, so any
slice can be regenerated independently on host (numpy) or device (torch).
Frames are packed back to back and described by N+1 uint64 offsets.

Lengths:
  fixed(L)   every frame L bytes (60, 1500, 9000, ...)
  zipf       L in [64, 1500], P(L) proportional to 1/(L-63), drawn by inverse CDF from
             numpy default_rng(20261015) — mean ~246.1 bytes, arbitrary alignment.
"""
from __future__ import annotations

import numpy as np

SEED = 0x6C6E65746F
ZIPF_SEED = 20261015
GOLDEN = 0x9E3779B97F4A7C15
M1 = 0xBF58476D1CE4E5B9
M2 = 0x94D049BB133111EB
MASK64 = (1 << 64) - 1


def _s64(c: int) -> int:
    return c - (1 << 64) if c >= (1 << 63) else c


# ------------------------------------------------------------------ lengths
def zipf_lengths(n: int, lo: int = 64, hi: int = 1500, seed: int = ZIPF_SEED) -> np.ndarray:
    L = np.arange(lo, hi + 1, dtype=np.int64)
    p = 1.0 / (L - (lo - 1)).astype(np.float64)
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    u = np.random.default_rng(seed).random(n)
    idx = np.searchsorted(cdf, u, side="right")
    idx = np.minimum(idx, len(L) - 1)
    return L[idx]


def offsets_from_lengths(lengths: np.ndarray) -> np.ndarray:
    off = np.zeros(len(lengths) + 1, dtype=np.uint64)
    np.cumsum(np.asarray(lengths, dtype=np.uint64), out=off[1:])
    return off


def fixed_offsets(n: int, length: int) -> np.ndarray:
    return np.arange(n + 1, dtype=np.uint64) * np.uint64(length)


# ------------------------------------------------------------------ bytes
def splitmix_words_np(k0: int, count: int, seed: int = SEED) -> np.ndarray:
    """uint64 words k0 .. k0+count-1 (numpy, wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        k = np.arange(k0, k0 + count, dtype=np.uint64)
        z = np.uint64(seed) + (k + np.uint64(1)) * np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(M1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(M2)
        z = z ^ (z >> np.uint64(31))
    return z


def bytes_np(nbytes: int, seed: int = SEED) -> np.ndarray:
    words = splitmix_words_np(0, (nbytes + 7) // 8, seed)
    return words.view(np.uint8)[:nbytes].copy()


def _srl(x, s: int):
    """Logical right shift of an int64 torch tensor."""
    return (x >> s) & ((1 << (64 - s)) - 1)


def bytes_torch(nbytes: int, device, seed: int = SEED, chunk_words: int = 1 << 25):
    """Same bytes as bytes_np, generated on `device` in chunks (no host staging)."""
    import torch
    nwords = (nbytes + 7) // 8
    out = torch.empty(nwords * 8, dtype=torch.uint8, device=device)
    o64 = out.view(torch.int64)
    for k0 in range(0, nwords, chunk_words):
        cnt = min(chunk_words, nwords - k0)
        k = torch.arange(k0 + 1, k0 + 1 + cnt, dtype=torch.int64, device=device)
        z = k * _s64(GOLDEN) + _s64(seed)
        z = (z ^ _srl(z, 30)) * _s64(M1)
        z = (z ^ _srl(z, 27)) * _s64(M2)
        z = z ^ _srl(z, 31)
        o64[k0:k0 + cnt] = z
        del k, z
    return out[:nbytes]


# ------------------------------------------------------------- workloads
WORKLOADS = {
    "min64_host": dict(kind="fixed", length=60, n=1 << 16),
    "mtu1500": dict(kind="fixed", length=1500, n=1 << 20),
    "jumbo9000": dict(kind="fixed", length=9000, n=1 << 20),
    "zipf64_1500": dict(kind="zipf", n=1 << 24),
    "mtu1500_x8": dict(kind="fixed", length=1500, n=1 << 27),
    # dispatch-tuning workloads (not bench configs): row-width thresholds
    "fixed1024": dict(kind="fixed", length=1024, n=1 << 20),
    "fixed2048": dict(kind="fixed", length=2048, n=1 << 20),
    "fixed3072": dict(kind="fixed", length=3072, n=1 << 19),
    "uni640_1536": dict(kind="uniform", lo=640, hi=1536, n=1 << 21),
}


def workload_offsets(name: str, n: int | None = None) -> np.ndarray:
    w = WORKLOADS[name]
    n = w["n"] if n is None else n
    if w["kind"] == "fixed":
        return fixed_offsets(n, w["length"])
    if w["kind"] == "uniform":
        rng = np.random.default_rng(ZIPF_SEED)
        return offsets_from_lengths(rng.integers(w["lo"], w["hi"] + 1, size=n))
    return offsets_from_lengths(zipf_lengths(n))
