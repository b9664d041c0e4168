"""CPU model of the event-stream framing kernel's lane pair (crc_kernels.hip eventstream_kernel, round 4).

A message's CRC span is n = total - 4 bytes.  The second lane folds the last h = 64 floor(n / 128)
bytes from state 0 (h < 1 KiB; otherwise h = 0), the first lane the first n - h bytes from ~0 and
then multiplies its register by x^(8h) with eight nibble lookups in tables built as the kernel builds
them (entry (k, v) of table m = (v << 4k) * x^(512 m), each m the previous times x^512 through the 32
columns of x^512).  The message CRC is ~(first ^ second).  Checked against zlib's CRC32 for every
length class around the split points, and the prelude CRC for the first eight bytes.
"""
import random
import zlib

import pytest

POLY = 0xEDB88320
M32 = 0xFFFFFFFF
SPLIT_MAX = 16


def reg(s, data):
    """raw reflected CRC32 register s advanced over data (no complements)"""
    for b in data:
        s ^= b
        for _ in range(8):
            s = (s >> 1) ^ (POLY if s & 1 else 0)
    return s


def mulx(v):
    return (v >> 1) ^ (POLY if v & 1 else 0)


def mulmod(a, b):
    """a * b mod P, reflected: bit 31 is x^0"""
    p, m = 0, 1 << 31
    while m:
        if a & m:
            p ^= b
        m >>= 1
        b = mulx(b)
    return p


def xpow8n(n):
    r = 1 << 31
    for _ in range(8 * n):
        r = mulx(r)
    return r


def shift_tables():
    k512 = xpow8n(64)
    cols = [mulmod(1 << b, k512) for b in range(32)]
    t = [[0] * 128 for _ in range(SPLIT_MAX)]
    for i in range(128):
        val = (i & 15) << (4 * (i >> 4))
        t[0][i] = val
        for m in range(1, SPLIT_MAX):
            nv = 0
            for b in range(32):
                if (val >> b) & 1:
                    nv ^= cols[b]
            val = nv
            t[m][i] = val
    return t


TABLES = shift_tables()


def es_shift(r, m):
    acc = 0
    for k in range(8):
        acc ^= TABLES[m][16 * k + ((r >> (4 * k)) & 15)]
    return acc


def pair_crcs(msg):
    n = len(msg) - 4
    h = 64 * (n // 128)
    if h >= 64 * SPLIT_MAX:
        h = 0
    s_pre = reg(M32, msg[:8])
    first = reg(s_pre, msg[8:n - h])
    second = reg(0, msg[n - h:n])
    return (~s_pre) & M32, (~(es_shift(first, h // 64) ^ second)) & M32


def test_shift_tables_are_powers_of_x512():
    rnd = random.Random(5)
    for m in range(SPLIT_MAX):
        k = xpow8n(64 * m)
        for _ in range(20):
            r = rnd.getrandbits(32)
            assert es_shift(r, m) == mulmod(r, k)


@pytest.mark.parametrize("total", [16, 17, 23, 100, 131, 132, 133, 200, 259, 260, 261, 517, 1028, 1031, 1032,
                                   1033, 1100, 2051, 2052, 2053, 2100, 4000])
def test_pair_matches_zlib(total):
    rnd = random.Random(total)
    msg = bytes(rnd.getrandbits(8) for _ in range(total))
    pre, crc = pair_crcs(msg)
    assert pre == zlib.crc32(msg[:8])
    assert crc == zlib.crc32(msg[:total - 4])
