"""CPU: Python models of the W=32 braided scans (crc_kernels.hip crc32_braid_kernel /
crc32_stream_kernel), checked against the oracle.  The first model is the 4-byte-word form
(AMDCRC_STREAM_W8=0 builds); BraidW8 below models the default 8-byte-word form, whole tiles and
front-padded ones.  They restate the kernels' algebra independently of the C++ host code:

  * rows of 256 bytes; lane l owns the 4-byte word at 4l of every row;
  * braid step u <- T'(u ^ w) with T'_k[e] = e * x^(8(k+1)) * x^(8*252) (slice-by-4 plus the skip
    over the other 63 lanes' words);
  * lane share u * K_l, K_l = x^(-32 l) (x^-1 by inverting the reflected multiply-by-x);
  * head state injected at virtual offset `pad` of the front-padded first tile;
  * tiles in groups of 32: a tile moves to its group end (x^(8*TILE*m), m < 32), a group to the
    buffer end (x^(8*TILE*(T - group_end))).

Rows per tile R is a free parameter here (the kernel uses multiples of 16), so small buffers
already exercise multi-group buffers.  A failure here is a design bug, not a kernel bug.
"""
import random

import pytest

from oracle import oracle

POLY = {"crc32": 0xEDB88320, "crc32c": 0x82F63B78}
M32 = 0xFFFFFFFF
ROW = 256


def mulx(v, P):
    return (v >> 1) ^ (P if v & 1 else 0)


def inv_mulx(t, P):
    return ((((t ^ P) << 1) | 1) & M32) if t & 0x80000000 else (t << 1) & M32


def mulmod(a, b, P):
    m, p = 0x80000000, 0
    while m:
        if a & m:
            p ^= b
        m >>= 1
        b = mulx(b, P)
    return p


def xpow8n(n, P):
    r, sq = 0x80000000, 0x00800000  # x^0, x^8
    while n:
        if n & 1:
            r = mulmod(r, sq, P)
        sq = mulmod(sq, sq, P)
        n >>= 1
    return r


def table_entry(e, k, P):
    c = e
    for _ in range(8 * (k + 1)):
        c = mulx(c, P)
    return c


class Braid:
    def __init__(self, alg):
        P = self.P = POLY[alg]
        skip = xpow8n(ROW - 4, P)
        self.Tp = [[mulmod(table_entry(e, k, P), skip, P) for e in range(256)] for k in range(4)]
        self.T0 = [table_entry(e, 0, P) for e in range(256)]
        self.K = []
        kl = 0x80000000
        for _ in range(64):
            self.K.append(kl)
            for _ in range(32):
                kl = inv_mulx(kl, P)

    def step(self, a):
        T = self.Tp
        return T[3][a & 255] ^ T[2][(a >> 8) & 255] ^ T[1][(a >> 16) & 255] ^ T[0][a >> 24]

    def byte(self, s, b):
        return (s >> 8) ^ self.T0[(s ^ b) & 255]

    def bytes_(self, s, data):
        for b in data:
            s = self.byte(s, b)
        return s


def braid_model(br: Braid, data: bytes, addr: int, seed: int, rows: int) -> int:
    P = br.P
    n = len(data)
    ptr, end = addr, addr + n
    H, Ea = (ptr + 15) & ~15, end & ~15
    if Ea > H:
        mainlen, headend, tail = Ea - H, H, Ea
    else:
        mainlen, headend, tail = 0, end, end
    tile = ROW * rows
    T = -(-mainlen // tile) if mainlen else 1
    pad = T * tile - mainlen
    s_h = br.bytes_(~seed & M32, data[: headend - ptr])
    groups = {}
    fin = None
    for k in range(T):
        r = 0
        if mainlen:
            vbase = (H - ptr) - pad + k * tile  # data offset of the tile's virtual byte 0
            for lane in range(64):
                u = s_h if (k == 0 and pad == 0 and lane == 0) else 0
                for c in range(rows):
                    vo = ROW * c + 4 * lane
                    if k == 0 and pad and vo < pad:
                        w = 0
                    else:
                        w = int.from_bytes(data[vbase + vo: vbase + vo + 4], "little")
                    if k == 0 and pad and vo == pad:
                        w ^= s_h
                    u = br.step(u ^ w)
                r ^= mulmod(u, br.K[lane], P)
        if T == 1:
            fin = r if mainlen else s_h
        else:
            g0 = k & ~31
            gend = min(g0 + 32, T)
            groups[g0] = groups.get(g0, 0) ^ mulmod(r, xpow8n(tile * (gend - 1 - k), P), P)
    if T > 1:
        fin = 0
        for g0, v in groups.items():
            gend = min(g0 + 32, T)
            fin ^= mulmod(v, xpow8n(tile * (T - gend), P), P)
    fin = br.bytes_(fin, data[tail - ptr:])
    return ~fin & M32


@pytest.fixture(scope="module", params=["crc32", "crc32c"])
def braid(request):
    return request.param, Braid(request.param)


def test_inverse_x(braid):
    alg, br = braid
    for l in range(64):
        # K_l * x^(32 l) == 1
        assert mulmod(br.K[l], xpow8n(4 * l, br.P), br.P) == 0x80000000


def test_column_multiply_matches_mulmod(braid):
    """mul_pcols / the LDS column select: bit (31-j) of r picks column j = X * x^j."""
    alg, br = braid
    rnd = random.Random(5)
    for _ in range(20):
        X, r = rnd.getrandbits(32), rnd.getrandbits(32)
        cols, c = [], X
        for _ in range(32):
            cols.append(c)
            c = mulx(c, br.P)
        acc = 0
        for j in range(32):
            if (r >> (31 - j)) & 1:
                acc ^= cols[j]
        assert acc == mulmod(r, X, br.P)


@pytest.mark.parametrize("rows", [1, 2, 16])
def test_braid_model_vs_oracle(braid, rows):
    alg, br = braid
    rnd = random.Random(hash((alg, rows)) & 0xFFFF)
    tile = ROW * rows
    sizes = [0, 1, 15, 16, 17, 255, 256, 4096, tile - 16, tile, tile + 16, 3 * tile + 7, 33 * tile + 48,
             70 * tile - 32]
    for n in sizes:
        for misalign in (0, 3, 9):
            if n > 20000 and misalign:
                continue
            data = bytes(rnd.getrandbits(8) for _ in range(n))
            seed = rnd.choice([0, rnd.getrandbits(32)])
            want = oracle.crc(alg, data, seed)
            got = braid_model(br, data, 0x1000 + misalign, seed, rows)
            assert got == want, (alg, rows, n, misalign, hex(seed))


# ---- the streaming scan on 8-byte words (crc32_stream_kernel<POLY, true>)
ROW8 = 512


class BraidW8:
    """512-byte rows, lane l owning the 8-byte word at 8l; the row step is slice-by-8 on
    a = (u ^ lo(w), hi(w)) with T'_t[e] = e * x^(8(t+1)) * x^(8*504); K_l = x^(-64 l)."""

    def __init__(self, alg):
        P = self.P = POLY[alg]
        skip = xpow8n(ROW8 - 8, P)
        self.Tp = [[mulmod(table_entry(e, t, P), skip, P) for e in range(256)] for t in range(8)]
        self.K = []
        kl = 0x80000000
        for _ in range(64):
            self.K.append(kl)
            for _ in range(64):
                kl = inv_mulx(kl, P)

    def step(self, lo, hi):
        v = 0
        for i in range(4):
            v ^= self.Tp[7 - i][(lo >> (8 * i)) & 255] ^ self.Tp[3 - i][(hi >> (8 * i)) & 255]
        return v


def lds_w8_schedule(lane):
    """(slot -> (which dword, byte q, table t, column)) of the kernel's Braid32W8::init"""
    j, c = (lane >> 3) & 3, lane & 7
    out = []
    for k in range(8):
        q = ((k & 3) + j) & 3
        hi = k >= 4
        t = (3 - q) if hi else (7 - q)
        out.append((hi, q, t, t * 8 + c))
    return out


def test_w8_lds_schedule_conflict_free_and_complete():
    for half in (range(32), range(32, 64)):
        for k in range(8):
            cols = [lds_w8_schedule(l)[k][3] for l in half]
            assert len(set(cols)) == 32, k  # one dword column (bank) per lane: conflict-free
    for lane in range(64):
        seen = {(hi, q) for hi, q, _, _ in lds_w8_schedule(lane)}
        assert seen == {(h, q) for h in (False, True) for q in range(4)}  # all 8 bytes, once each
        for hi, q, t, _ in lds_w8_schedule(lane):
            assert t == 7 - (4 * hi + q)  # byte i of the 8-byte a indexes T'_(7-i)


@pytest.mark.parametrize("alg", ["crc32", "crc32c"])
@pytest.mark.parametrize("rows", [1, 8, 24])
def test_braid_w8_model_vs_oracle(alg, rows):
    """whole-tile buffers (the streaming scan's case): lanes run the fused chain of the kernel's
    stream_rows (x = u ^ lo(w_r); hi(w_r) enters its own step), shares combine with K_l, tiles
    with x^(8*TILE*(T-1-k))"""
    br = BraidW8(alg)
    P = br.P
    rnd = random.Random(hash((alg, rows, "w8")) & 0xFFFF)
    tile = ROW8 * rows
    for ntiles in (1, 2, 3):
        data = bytes(rnd.getrandbits(8) for _ in range(tile * ntiles))
        seed = rnd.choice([0, rnd.getrandbits(32)])
        fin = 0
        for k in range(ntiles):
            r = 0
            for lane in range(64):
                u = (~seed & M32) if (k == 0 and lane == 0) else 0
                words = [int.from_bytes(data[k * tile + ROW8 * c + 8 * lane: k * tile + ROW8 * c + 8 * lane + 8], "little")
                         for c in range(rows)]
                x = u ^ (words[0] & M32)
                for c in range(1, rows):
                    x = br.step(x, words[c - 1] >> 32) ^ (words[c] & M32)
                u = br.step(x, words[-1] >> 32)
                r ^= mulmod(u, br.K[lane], P)
            fin ^= mulmod(r, xpow8n(tile * (ntiles - 1 - k), P), P)
        assert (~fin & M32) == oracle.crc(alg, data, seed), (alg, rows, ntiles)


def braid_w8_model(br: BraidW8, data: bytes, addr: int, seed: int, rows: int) -> int:
    """crc32_braid_kernel<POLY, LIST, NT, true> on one buffer: head bytes folded bytewise, the
    16-aligned main region front-padded to tiles of `rows` 512-byte rows, words in the pad zero, the
    head state XORed into the low half of the word at the pad's end, groups of 8 rows before the
    pad's end skipped (the braids are zero there), tiles combined as the W=32 model does."""
    P = br.P
    T0 = [table_entry(e, 0, P) for e in range(256)]

    def bytes_(s, bs):
        for b in bs:
            s = (s >> 8) ^ T0[(s ^ b) & 255]
        return s

    n = len(data)
    ptr, end = addr, addr + n
    H, Ea = (ptr + 15) & ~15, end & ~15
    if Ea > H:
        mainlen, headend, tail = Ea - H, H, Ea
    else:
        mainlen, headend, tail = 0, end, end
    tile = ROW8 * rows
    T = -(-mainlen // tile) if mainlen else 1
    pad = T * tile - mainlen
    s_h = bytes_(~seed & M32, data[: headend - ptr])
    groups = {}
    fin = None
    for k in range(T):
        r = 0
        if mainlen:
            vbase = (H - ptr) - pad + k * tile
            first_row = (pad // 4096) * 8 if k == 0 else 0  # the kernel's first_group, in rows
            for lane in range(64):
                u = s_h if (k == 0 and pad == 0 and lane == 0) else 0
                for c in range(first_row, rows):
                    vo = ROW8 * c + 8 * lane
                    if k == 0 and pad and vo < pad:
                        w = 0
                    else:
                        w = int.from_bytes(data[vbase + vo: vbase + vo + 8], "little")
                    if k == 0 and pad and vo == pad:
                        w ^= s_h
                    u = br.step(u ^ (w & M32), w >> 32)
                r ^= mulmod(u, br.K[lane], P)
        if T == 1:
            fin = r if mainlen else s_h
        else:
            g0 = k & ~31
            gend = min(g0 + 32, T)
            groups[g0] = groups.get(g0, 0) ^ mulmod(r, xpow8n(tile * (gend - 1 - k), P), P)
    if T > 1:
        fin = 0
        for g0, v in groups.items():
            gend = min(g0 + 32, T)
            fin ^= mulmod(v, xpow8n(tile * (T - gend), P), P)
    fin = bytes_(fin, data[tail - ptr:])
    return ~fin & M32


@pytest.mark.parametrize("alg", ["crc32", "crc32c"])
@pytest.mark.parametrize("rows", [8, 16])
def test_braid_w8_padded_model_vs_oracle(alg, rows):
    """front pads ending before, on and after 4 KiB group boundaries (rows = 16: two groups per tile),
    unaligned heads and tails, seeds, multi-tile buffers"""
    br = BraidW8(alg)
    rnd = random.Random(hash((alg, rows, "w8pad")) & 0xFFFF)
    tile = ROW8 * rows
    sizes = [0, 5, 16, 17, 512, tile - 16, tile, tile + 16, tile - 4096, tile - 4096 - 16, tile - 4096 + 16,
             2 * tile - 4096, 3 * tile + 7]
    for n in sizes:
        if n < 0:
            continue
        for misalign in (0, 3, 9):
            data = bytes(rnd.getrandbits(8) for _ in range(n))
            seed = rnd.choice([0, rnd.getrandbits(32)])
            assert braid_w8_model(br, data, 0x1000 + misalign, seed, rows) == oracle.crc(alg, data, seed), \
                (alg, rows, n, misalign)


# ---- the streaming scan on 16-byte words (crc32_stream_kernel<POLY, 16>)
ROW16 = 1024


class BraidW16:
    """1024-byte rows, lane l owning the 16-byte word at 16l; the row step is slice-by-16 on
    a = (u ^ d0, d1, d2, d3) with T'_t[e] = e * x^(8(t+1)) * x^(8*1008), byte i indexing T'_(15-i);
    K_l = x^(-128 l)."""

    def __init__(self, alg):
        P = self.P = POLY[alg]
        skip = xpow8n(ROW16 - 16, P)
        self.Tp = [[mulmod(table_entry(e, t, P), skip, P) for e in range(256)] for t in range(16)]
        self.K = []
        kl = 0x80000000
        for _ in range(64):
            self.K.append(kl)
            for _ in range(128):
                kl = inv_mulx(kl, P)

    def hi(self, d1, d2, d3):
        """the twelve lookups of d1..d3 (independent of the braid state)"""
        v = 0
        for d, w in ((1, d1), (2, d2), (3, d3)):
            for q in range(4):
                v ^= self.Tp[15 - (4 * d + q)][(w >> (8 * q)) & 255]
        return v

    def lo(self, x):
        v = 0
        for q in range(4):
            v ^= self.Tp[15 - q][(x >> (8 * q)) & 255]
        return v


def lds_w16_schedule(lane):
    """(dword d, slot k) -> (byte i, table t, LDS byte address without the entry row) of the kernel's
    Braid32W16::init: region B (tables 7..0) at 64 KiB, table t at (t & 7) * 32, copy at 4 * copy"""
    j, c = (lane >> 3) & 3, lane & 7
    out = {}
    for d in range(4):
        for k in range(4):
            q = (k + j) & 3
            t = 15 - (4 * d + q)
            addr = (65536 if t < 8 else 0) + (t & 7) * 32 + 4 * c
            out[(d, k)] = (4 * d + q, t, addr)
    return out


def test_w16_lds_schedule_conflict_free_and_complete():
    for half in (range(32), range(32, 64)):
        for d in range(4):
            for k in range(4):
                # ds_read_b32: bank = (address / 4) mod 32; the entry row (e * 256) adds 0 mod 32 banks
                banks = [(lds_w16_schedule(l)[(d, k)][2] // 4) % 32 for l in half]
                assert len(set(banks)) == 32, (d, k)
    for lane in range(64):
        sch = lds_w16_schedule(lane)
        assert sorted(i for i, _, _ in sch.values()) == list(range(16))  # all 16 bytes, once each
        for (d, k), (i, t, addr) in sch.items():
            assert t == 15 - i and i // 4 == d
            assert addr + 255 * 256 + 4 <= 131072  # inside the 128 KiB of tables


@pytest.mark.parametrize("alg", ["crc32", "crc32c"])
@pytest.mark.parametrize("rows", [1, 4, 12])
def test_braid_w16_model_vs_oracle(alg, rows):
    """whole-tile buffers: the kernel's stream_rows_w16 chain (x = u ^ d0(w_r); d1..d3 of row r enter
    with row r's chain step), shares with K_l = x^(-128 l), tiles with x^(8*TILE*(T-1-k))"""
    br = BraidW16(alg)
    P = br.P
    rnd = random.Random(hash((alg, rows, "w16")) & 0xFFFF)
    tile = ROW16 * rows
    for ntiles in (1, 2, 3):
        data = bytes(rnd.getrandbits(8) for _ in range(tile * ntiles))
        seed = rnd.choice([0, rnd.getrandbits(32)])
        fin = 0
        for k in range(ntiles):
            r = 0
            for lane in range(64):
                u = (~seed & M32) if (k == 0 and lane == 0) else 0
                words = []
                for c in range(rows):
                    o = k * tile + ROW16 * c + 16 * lane
                    words.append([int.from_bytes(data[o + 4 * d: o + 4 * d + 4], "little") for d in range(4)])
                x = u ^ words[0][0]
                for c in range(1, rows):
                    x = br.lo(x) ^ br.hi(*words[c - 1][1:]) ^ words[c][0]
                u = br.lo(x) ^ br.hi(*words[-1][1:])
                r ^= mulmod(u, br.K[lane], P)
            fin ^= mulmod(r, xpow8n(tile * (ntiles - 1 - k), P), P)
        assert (~fin & M32) == oracle.crc(alg, data, seed), (alg, rows, ntiles)
