"""Deterministic synthetic payloads for BASELINE.json config 4 (1,048,576 x 8 KiB parts, buffer i on
GPU i mod N), generated where they are scanned.

Every byte is a function of its global position only, so any rank can build exactly its shard of the
set on its own GPU (no payload crosses GPUs or the host) and every world size scans the same bytes:

    word j (8 bytes, little-endian) of global buffer i, with w = L / 8 words per buffer:
        splitmix64(state = SEED + (i * w + j + 1) * GOLDEN  mod 2^64)

splitmix64 is Steele, Lea & Flood's finaliser (the generator SURVEY.md 8(c) names for the fixtures).
`words_np` (numpy, uint64) and `words_torch` (torch int64 bit patterns, any device) are the same
function; tests/test_synth.py checks them against each other, and tests/golden/gen_c4_digest.py uses
the numpy one to commit the set's digest.  Benchmarks and tests only: not a checksum path.
"""
from __future__ import annotations

import numpy as np

C4_COUNT = 1 << 20
C4_LEN = 8192
C4_SEED = 0xC4C4_5EED_0000_0004
GOLDEN = 0x9E3779B97F4A7C15
MIX1 = 0xBF58476D1CE4E5B9
MIX2 = 0x94D049BB133111EB
M64 = (1 << 64) - 1


def _s64(c: int) -> int:
    """an unsigned 64-bit constant as the int64 with the same bits"""
    c &= M64
    return c - (1 << 64) if c >> 63 else c


def words_np(idx: np.ndarray, seed: int = C4_SEED) -> np.ndarray:
    """splitmix64 outputs for global word indexes idx (uint64 array)"""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx.astype(np.uint64) + np.uint64(1)) * np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(MIX1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(MIX2)
        return z ^ (z >> np.uint64(31))


def words_torch(idx, seed: int = C4_SEED):
    """the same as words_np on a torch int64 tensor of word indexes (any device): int64 bit patterns.
    torch's >> on int64 is arithmetic, so each shift is masked to the logical result."""
    import torch

    z = (idx + 1) * _s64(GOLDEN) + _s64(seed)
    for sh, mul in ((30, MIX1), (27, MIX2), (31, None)):
        z = torch.bitwise_xor(z, torch.bitwise_and(torch.bitwise_right_shift(z, sh), (1 << (64 - sh)) - 1))
        if mul is not None:
            z = z * _s64(mul)
    return z


def buffers_np(first: int, count: int, length: int = C4_LEN, step: int = 1, seed: int = C4_SEED) -> np.ndarray:
    """the bytes of global buffers first, first + step, ... (count of them), back to back (uint8)"""
    w = length // 8
    gi = first + step * np.arange(count, dtype=np.uint64)
    idx = gi[:, None] * np.uint64(w) + np.arange(w, dtype=np.uint64)[None, :]
    return words_np(idx, seed).astype("<u8").view(np.uint8).reshape(-1)


def fill_shard(dst, rank: int, world: int, count: int = C4_COUNT, length: int = C4_LEN, seed: int = C4_SEED,
               chunk: int = 1 << 16) -> int:
    """Write this rank's shard (global buffers rank, rank + world, ...) into the uint8 device tensor dst,
    back to back at stride `length`, generated on dst's device in chunks of `chunk` buffers.  Returns
    the shard's buffer count."""
    import torch

    if length % 8:
        raise ValueError("length must be a multiple of 8")
    n = len(range(rank, count, world))
    if dst.numel() < n * length:
        raise ValueError("destination too small for the shard")
    w = length // 8
    dev = dst.device
    cols = torch.arange(w, dtype=torch.int64, device=dev)
    for k0 in range(0, n, chunk):
        k1 = min(n, k0 + chunk)
        gi = torch.arange(k0, k1, dtype=torch.int64, device=dev) * world + rank
        words = words_torch(gi[:, None] * w + cols[None, :], seed)
        dst[k0 * length:k1 * length].copy_(words.reshape(-1).view(torch.uint8))
    return n
