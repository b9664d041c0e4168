"""CPU: a Python model of the kernel's work decomposition (crc_kernels.hip / engine.h), checked
against the oracle.  It uses exactly the kernel's algebra -- head bytes folded into ~seed, the main
region front-padded with virtual zeros to T tiles of 64 lanes x seg bytes, per-lane shift
K_l = x^(8*seg*(63-l)), per-tile shift x^(8*TILE*(T-1-k)), head state injected at virtual offset
`pad`, tail bytes after -- so a failure here is a design bug, not a kernel bug.
"""
import random

import pytest

from oracle import oracle

MASK = {"crc32": (1 << 32) - 1, "crc32c": (1 << 32) - 1, "crc64nvme": (1 << 64) - 1}


def advance(alg, state, data):
    """register state after `data` starting from register `state` (no final complement)."""
    m = MASK[alg]
    return ~oracle.crc(alg, data, ~state & m, "sw") & m


def kernel_model(alg, data: bytes, addr: int, seed: int, seg: int) -> int:
    m = MASK[alg]
    n = len(data)
    ptr, end = addr, addr + n
    H, Ea = (ptr + 15) & ~15, end & ~15
    if Ea > H:
        mainlen, headend, tail = Ea - H, H, Ea
    else:
        mainlen, headend, tail = 0, end, end
    tile = 64 * seg
    T = -(-mainlen // tile) if mainlen else 1
    pad = T * tile - mainlen
    s_h = advance(alg, ~seed & m, data[: headend - ptr])
    acc = 0
    fin = None
    for k in range(T):
        R = 0
        if mainlen:
            vbase = (H - ptr) - pad + k * tile  # data offset of the tile's virtual byte 0
            for lane in range(64):
                s = s_h if (k == 0 and pad == 0 and lane == 0) else 0
                for v in range(seg // 16):
                    vo = lane * seg + 16 * v
                    if k == 0 and pad:
                        vec = bytes(16) if vo < pad else data[vbase + vo: vbase + vo + 16]
                        if vo == pad:
                            s ^= s_h
                    else:
                        vec = data[vbase + vo: vbase + vo + 16]
                    assert len(vec) == 16
                    s = advance(alg, s, vec)
                R ^= oracle.mulmod(alg, s, oracle.xpow8n(alg, seg * (63 - lane)))
        if T == 1:
            fin = R if mainlen else s_h
        else:
            acc ^= oracle.mulmod(alg, R, oracle.xpow8n(alg, tile * (T - 1 - k)))
    if T > 1:
        fin = acc
    fin = advance(alg, fin, data[tail - ptr:])
    return ~fin & m


@pytest.mark.parametrize("alg", ["crc32", "crc32c", "crc64nvme"])
def test_model_matches_oracle(alg):
    rng = random.Random(hash(alg) & 0xFFFF)
    cases = [(0, 0), (1, 0), (15, 3), (16, 0), (31, 1), (32, 15), (100, 7), (8192, 0), (8192, 5), (8191, 9),
             (16384 + 48, 0), (20000, 13), (3 * 8192 + 17, 2)]
    for n, misalign in cases:
        data = rng.randbytes(n)
        seed = rng.getrandbits(64 if alg == "crc64nvme" else 32)
        addr = 0x10000 + misalign
        for seg in (128, 256):
            got = kernel_model(alg, data, addr, seed, seg)
            assert got == oracle.crc(alg, data, seed), (n, misalign, seg)
