"""CPU model of the block-parallel event-stream kernel (crc_kernels.hip eventstream_block_kernel):
a wave's 64 messages cut into the aligned 64-byte blocks holding them, each block folded from a zero
register with the bytes outside its message masked to zero, and the message register assembled as

    U(~0, m) = x^(-8 pad) * ( sum_i c_i X^(n-1-i)  ^  I[lo] X^(n-1) ),   X = x^512,

round by round: the lanes of a round form one segment per message, each lane's c times X^(segment end
- lane), an XOR prefix over the 64 lanes, and a message running on from the previous round entering as
a carry times X^(segment length).  The constants are built as engine.cpp get_es_consts builds them
(nibble tables of X^e for e <= 64, x^(-8 p) for p < 64, I[l] = ~0 x^(8 (64 - l))).

Checked against zlib.crc32 for streams of back-to-back messages (16..1100 bytes, at every start
alignment), for messages longer than a round (a carry across rounds), and for the stored CRC / prelude
CRC fields as the kernel reads them.
"""
import random
import struct
import zlib

M32 = 0xFFFFFFFF
POLY = 0xEDB88320


def mulx(v):
    return (v >> 1) ^ (POLY if v & 1 else 0)


def inv_mulx(t):
    return (((t ^ POLY) << 1) | 1) & M32 if t & 0x80000000 else (t << 1) & M32


def mulmod(a, b):
    m, p = 0x80000000, 0
    while m:
        if a & m:
            p ^= b
        m >>= 1
        b = mulx(b)
    return p


def xpow8n(n):
    r, sq = 0x80000000, 0x80000000 >> 8
    while n:
        if n & 1:
            r = mulmod(r, sq)
        sq = mulmod(sq, sq)
        n >>= 1
    return r


def nibble_table(k):
    return [[mulmod(u << (4 * i), k) for u in range(16)] for i in range(8)]


def mul_nib(tab, v):
    x = 0
    for i in range(8):
        x ^= tab[i][(v >> (4 * i)) & 15]
    return x


def consts():
    xe = [nibble_table(xpow8n(64 * e)) for e in range(65)]
    xi, k = [], 0x80000000
    for _ in range(64):
        xi.append(nibble_table(k))
        for _ in range(8):
            k = inv_mulx(k)
    init = [mulmod(M32, xpow8n(64 - lo)) for lo in range(64)]
    return xe, xi, init


T0 = [0] * 256
for _e in range(256):
    _c = _e
    for _ in range(8):
        _c = mulx(_c)
    T0[_e] = _c


def fold(reg, data):
    for b in data:
        reg = (reg >> 8) ^ T0[(reg ^ b) & 0xFF]
    return reg


def wave(mem, starts, totals, C):
    """the kernel's rounds over one wave's messages; returns {message: (message CRC, prelude CRC)}"""
    xe, xi, init = C
    fb = [a >> 6 for a in starts]
    ep = [a + t - 4 for a, t in zip(starts, totals)]
    n = [((e + 63) >> 6) - f for e, f in zip(ep, fb)]
    pref = [0]
    for k in n:
        pref.append(pref[-1] + k)
    B = pref[-1]
    out, carry = {}, 0
    for r in range((B + 63) // 64):
        lanes = []
        for lane in range(64):
            b = 64 * r + lane
            if b >= B:
                lanes.append(None)
                continue
            mi = max(i for i in range(len(n)) if pref[i] <= b)
            k = b - pref[mi]
            bs = (fb[mi] + k) << 6
            lo = max(starts[mi] - bs, 0)
            hi = min(ep[mi] - bs, 64)
            blk = bytes(mem[bs + j] if lo <= j < hi else 0 for j in range(64))
            c = fold(0, blk)
            if k == 0:
                c ^= init[lo]
            lanes.append((mi, k, c, bs))
        heads = [ln is None or ln[1] == 0 for ln in lanes]
        heads[0] = True
        v = []
        for lane, ln in enumerate(lanes):
            send = next((j - 1 for j in range(lane + 1, 64) if heads[j]), 63)
            v.append(mul_nib(xe[send - lane], ln[2]) if ln else 0)
        P, acc = [], 0
        for x in v:
            acc ^= x
            P.append(acc)
        T = [0] * 64
        for lane in range(64):
            sst = max(j for j in range(lane + 1) if heads[j])
            send = next((j - 1 for j in range(lane + 1, 64) if heads[j]), 63)
            T[lane] = P[lane] ^ (P[sst - 1] if sst else 0)
            if sst == 0 and carry:
                T[lane] ^= mul_nib(xe[send + 1], carry)
        last = lanes[63]
        carry = T[63] if last and last[1] != n[last[0]] - 1 else 0
        for lane, ln in enumerate(lanes):
            if ln and ln[1] == n[ln[0]] - 1:
                pad = ln[3] + 64 - ep[ln[0]]
                out[ln[0]] = (~mul_nib(xi[pad], T[lane])) & M32
    return out


def stream(rng, sizes, lead):
    mem, starts = bytearray(rng.randbytes(lead)), []
    for t in sizes:
        body = bytearray(rng.randbytes(t))
        body[0:4] = struct.pack(">I", t)
        starts.append(len(mem))
        mem += body
    mem += rng.randbytes(80)
    return mem, starts


def test_block_assembly_matches_zlib():
    C = consts()
    rng = random.Random(5)
    for lead in range(64):
        sizes = [rng.randrange(16, 1100) for _ in range(64)]
        mem, starts = stream(rng, sizes, lead)
        got = wave(mem, starts, sizes, C)
        for i, (a, t) in enumerate(zip(starts, sizes)):
            assert got[i] == zlib.crc32(bytes(mem[a:a + t - 4])), (lead, i)


def test_messages_longer_than_a_round_carry():
    """messages of 5..20 KiB: every one spans rounds (64 blocks = 4 KiB per round)"""
    C = consts()
    rng = random.Random(9)
    sizes = [16, 17] + [rng.randrange(5000, 20000) for _ in range(6)] + [16, 4100, 4096 + 4, 63, 64, 65]
    mem, starts = stream(rng, sizes, 13)
    got = wave(mem, starts, sizes, C)
    for i, (a, t) in enumerate(zip(starts, sizes)):
        assert got[i] == zlib.crc32(bytes(mem[a:a + t - 4])), i


def test_prelude_word_step():
    """the prelude CRC is one word step from ~0 over the first 8 bytes (LaneW8::word(~0, ...))"""
    rng = random.Random(3)
    for _ in range(200):
        b = rng.randbytes(8)
        assert (~fold(M32, b)) & M32 == zlib.crc32(b)
