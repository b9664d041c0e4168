"""Deterministic input patterns shared by the golden-vector generator and the tests."""
import numpy as np

MASK64 = (1 << 64) - 1


def splitmix64_bytes(n: int, seed: int) -> bytes:
    """n bytes of the splitmix64 stream (little-endian 64-bit words) started at `seed`."""
    words = (n + 7) // 8
    out = np.empty(words, dtype=np.uint64)
    x = np.uint64(seed & MASK64)
    with np.errstate(over="ignore"):
        idx = np.arange(1, words + 1, dtype=np.uint64)
        z = x + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
        out[:] = z
    return out.tobytes()[:n]


def pattern(name: str, n: int) -> bytes:
    if name == "zeros":
        return bytes(n)
    if name == "ff":
        return b"\xff" * n
    if name == "ramp":
        return bytes(i & 0xFF for i in range(n))
    if name.startswith("splitmix:"):
        return splitmix64_bytes(n, int(name.split(":", 1)[1], 0))
    raise ValueError(name)
