"""CPU: a Python model of the W=64 braided scan (crc_kernels.hip crc64_braid_kernel, CRC64NVME),
checked against the oracle.  It restates the kernel's algebra independently of the C++ host code:

  * rows of 512 bytes; lane l owns the 8-byte word at 8l of every row;
  * braid step u <- T'(u ^ w) with T'_t[e] = e * x^(8(t+1)) * x^(8*504): slice-by-8 plus the skip
    over the other 63 lanes' words; byte i of the 64-bit a indexes T'_(7-i);
  * the kernel's LDS layout: region r = dword r of a, quarter q = byte q of that dword, copy c;
    lane quarter j reads quarter (k + j) & 3 in table slot k (conflict-free bank pairs);
  * lane share u * K_l, K_l = x^(-64 l);
  * head state injected at virtual offset `pad` of the front-padded first tile;
  * tiles in groups of 32: a tile moves to its group end (x^(8*TILE*m), m < 32), a group to the
    buffer end (x^(8*TILE*(T - group_end))), arrivals counted per group and per buffer.

Rows per tile R is a free parameter here (the kernel uses multiples of 8), so small buffers already
exercise multi-group buffers.  A failure here is a design bug, not a kernel bug.
"""
import random

import pytest

from oracle import oracle

P64 = 0x9A6C9329AC4BC9B5
M64 = (1 << 64) - 1
ROW = 512


def mulx(v):
    return (v >> 1) ^ (P64 if v & 1 else 0)


def inv_mulx(t):
    return ((((t ^ P64) << 1) | 1) & M64) if t >> 63 else (t << 1) & M64


def mulmod(a, b):
    m, p = 1 << 63, 0
    while m:
        if a & m:
            p ^= b
        m >>= 1
        b = mulx(b)
    return p


def xpow8n(n):
    r, sq = 1 << 63, 1 << 55  # x^0, x^8
    while n:
        if n & 1:
            r = mulmod(r, sq)
        sq = mulmod(sq, sq)
        n >>= 1
    return r


def table_entry(e, t):
    c = e
    for _ in range(8 * (t + 1)):
        c = mulx(c)
    return c


class Braid64:
    def __init__(self):
        skip = xpow8n(ROW - 8)
        self.Tp = [[mulmod(table_entry(e, t), skip) for e in range(256)] for t in range(8)]
        self.T0 = [table_entry(e, 0) for e in range(256)]
        # the kernel's LDS image: byte address -> value (only the written entries)
        self.lds = {}
        for r in range(2):
            for q in range(4):
                t = 7 - q if r == 0 else 3 - q
                for e in range(256):
                    for c in range(8):
                        self.lds[(r << 16) | (e << 8) | (q << 6) | (c << 3)] = self.Tp[t][e]
        self.K = []
        kl = 1 << 63
        for _ in range(64):
            self.K.append(kl)
            for _ in range(64):
                kl = inv_mulx(kl)

    def step(self, a):
        v = 0
        for i in range(8):
            v ^= self.Tp[7 - i][(a >> (8 * i)) & 255]
        return v

    def step_lds(self, a, lane):
        """the kernel's lookup schedule: slot k, lane quarter j -> byte (k+j)&3 of each dword"""
        j, c = (lane >> 3) & 3, lane & 7
        v = 0
        for k in range(4):
            q = (k + j) & 3
            for r in range(2):
                e = (a >> (32 * r + 8 * q)) & 255
                v ^= self.lds[(r << 16) | (e << 8) | (q << 6) | (c << 3)]
        return v

    def bytes_(self, s, data):
        for b in data:
            s = (s >> 8) ^ self.T0[(s ^ b) & 255]
        return s

    def mulK(self, r, lane):
        """the kernel's Braid64::mulK: Horner over the bytes of r, columns K_l x^i (i < 8), a * x^8
        as one plain byte step through T0"""
        c, b = [], self.K[lane]
        for _ in range(8):
            c.append(b)
            b = mulx(b)

        def bm(m):
            word = r >> 32 if m < 4 else r & 0xFFFFFFFF
            sh = 8 * ((7 - m) & 3)
            a = 0
            for i in range(8):
                if (word >> (sh + 7 - i)) & 1:
                    a ^= c[i]
            return a

        acc = bm(7)
        for m in range(6, -1, -1):
            acc = (acc >> 8) ^ self.T0[acc & 0xFF] ^ bm(m)
        return acc


@pytest.fixture(scope="module")
def br():
    return Braid64()


def braid64_model(br, data, addr, seed, rows):
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
    s_h = br.bytes_(~seed & M64, data[: headend - ptr])
    group_val, group_cnt, buf_val, buf_cnt = {}, {}, 0, 0
    G = -(-T // 32)
    fin = None
    for k in range(T):
        r = 0
        if mainlen:
            vbase = (H - ptr) - pad + k * tile
            for lane in range(64):
                u = s_h if (k == 0 and pad == 0 and lane == 0) else 0
                for c in range(rows):
                    vo = ROW * c + 8 * lane
                    w = 0 if (k == 0 and pad and vo < pad) else int.from_bytes(data[vbase + vo: vbase + vo + 8], "little")
                    if k == 0 and pad and vo == pad:
                        w ^= s_h
                    u = br.step(u ^ w)
                r ^= br.mulK(u, lane)
        if T == 1:
            fin = r if mainlen else s_h
            break
        g0 = k & ~31
        gend = min(g0 + 32, T)
        group_val[g0] = group_val.get(g0, 0) ^ mulmod(r, xpow8n(tile * (gend - 1 - k)))
        group_cnt[g0] = group_cnt.get(g0, 0) + 1
        if group_cnt[g0] == gend - g0:  # the group's last arrival
            gv = group_val.pop(g0)
            if G == 1:
                fin = gv
            else:
                buf_val ^= mulmod(gv, xpow8n(tile * (T - gend)))
                buf_cnt += 1
                if buf_cnt == G:
                    fin = buf_val
    fin = br.bytes_(fin, data[tail - ptr:])
    return ~fin & M64


def test_mulk_nibble_tables(br):
    """Braid64<POLY, 4>::mulK_nib: per-lane nibble multiples NT_l[v] = sum_(i<4) bit(3-i) of v *
    K_l x^i, B_m = NT_l[hi nibble] ^ NT_l[lo nibble] * x^4 with a * x^4 = (a >> 4) ^ R4[a & 15],
    then the byte-Horner chain through T0"""
    R4 = []
    for u in range(16):
        a = u
        for _ in range(4):
            a = mulx(a)
        R4.append(a)
    rng = random.Random(11)
    for lane in range(64):
        c = [br.K[lane]]
        for _ in range(3):
            c.append(mulx(c[-1]))
        NT = [0] * 16
        for v in range(16):
            for i in range(4):
                if (v >> (3 - i)) & 1:
                    NT[v] ^= c[i]
        for r in (0, 1, 1 << 63, M64, rng.getrandbits(64), rng.getrandbits(64)):
            acc = None
            for m in range(7, -1, -1):
                byte = (r >> (8 * (7 - m))) & 0xFF
                nl = NT[byte & 15]
                b = NT[byte >> 4] ^ (nl >> 4) ^ R4[nl & 15]
                acc = b if acc is None else (acc >> 8) ^ br.T0[acc & 0xFF] ^ b
            assert acc == mulmod(r, br.K[lane]), (lane, hex(r))


def test_mulk_byte_horner(br):
    rng = random.Random(7)
    for lane in range(64):
        for r in (0, 1, 1 << 63, M64, rng.getrandbits(64), rng.getrandbits(64)):
            assert br.mulK(r, lane) == mulmod(r, br.K[lane])


def test_inverse_x(br):
    for l in range(64):
        assert mulmod(br.K[l], xpow8n(8 * l)) == 1 << 63


def test_lds_schedule_is_conflict_free_and_complete(br):
    """in every slot the 32 lanes of a ds_read_b64 group hit 32 distinct bank pairs, and over the
    four slots each lane reads each byte of both dwords once"""
    for k in range(4):
        for r in range(2):
            pairs = set()
            for lane in range(32):
                j, c = (lane >> 3) & 3, lane & 7
                q = (k + j) & 3
                addr = (r << 16) | (0xA5 << 8) | (q << 6) | (c << 3)
                pairs.add((addr >> 3) & 31)
            assert len(pairs) == 32
    rnd = random.Random(3)
    for _ in range(200):
        a = rnd.getrandbits(64)
        assert br.step_lds(a, rnd.randrange(64)) == br.step(a)


def test_four_copy_layout(br):
    """crc64_stream4_kernel's 64 KiB layout (Braid64<POLY, 4>, b64x4_build_tables): row e holds the
    table of byte t of a (T'_(7-t)) at bytes [32 t, 32 t + 32), 4 copies x 8 B.  The table build
    (thread i: byte t = i >> 6, entries (i & 63) + 64 n, both 16-byte halves) fills every address the
    lookups form with the right entry; the lookups (lane group jp = (lane >> 2) & 7 reads byte
    (k + jp) & 3 of the low dword in slots 0..3 when jp < 4, of the high dword otherwise, and the
    other dword in slots 4..7) reproduce the slice-by-8 step; and every ds_read_b64 half-wave meets
    32 distinct bank pairs (conflict-free), whatever the entries."""
    lds = {}
    for i in range(512):
        t = i >> 6
        for n in range(4):
            e = (i & 63) + 64 * n
            row = (e << 8) + (t << 5)
            for half in range(2):
                for c in range(2):
                    lds[row + (half << 4) + 8 * c] = br.Tp[7 - t][e]
    assert len(lds) == 256 * 8 * 4  # 64 KiB of 8-byte entries, all distinct addresses

    def slots(lane):
        """(column offset, source dword, byte q) of the 8 table slots of a lane"""
        jp, cp = (lane >> 2) & 7, lane & 3
        low = jp < 4
        out = []
        for second in (False, True):
            for k in range(4):
                q = (k + jp) & 3
                hi_src = (not low) != second  # first set: low dword iff jp < 4; second set: the other
                t = (4 if hi_src else 0) + q
                out.append(((t << 5) | (cp << 3), hi_src, q))
        return out

    def step_lds4(a, lane):
        v = 0
        for col, hi_src, q in slots(lane):
            e = (a >> ((32 if hi_src else 0) + 8 * q)) & 255
            v ^= lds[col | (e << 8)]
        return v

    rnd = random.Random(5)
    for _ in range(300):
        a = rnd.getrandbits(64)
        assert step_lds4(a, rnd.randrange(64)) == br.step(a)
    for lane in range(64):  # each lane reads each byte of a exactly once
        assert sorted((4 if h else 0) + q for _, h, q in slots(lane)) == list(range(8))
    for s_ in range(8):
        for g in (0, 32):
            pairs = set()
            for lane in range(g, g + 32):
                addr = slots(lane)[s_][0] + (rnd.randrange(256) << 8)
                pairs.add((addr >> 3) & 31)
            assert len(pairs) == 32


def test_step_is_multiply_by_x4096(br):
    rnd = random.Random(4)
    for _ in range(20):
        a = rnd.getrandbits(64)
        assert br.step(a) == mulmod(a, xpow8n(ROW))


@pytest.mark.parametrize("rows", [1, 2, 8])
def test_braid64_model_vs_oracle(br, rows):
    rnd = random.Random(rows * 7 + 1)
    tile = ROW * rows
    sizes = [0, 1, 15, 16, 17, 511, 512, 4096, tile - 16, tile, tile + 16, 3 * tile + 7, 33 * tile + 48,
             70 * tile - 32]
    for n in sizes:
        for misalign in (0, 3, 9):
            if n > 20000 and misalign:
                continue
            data = bytes(rnd.getrandbits(8) for _ in range(n))
            seed = rnd.choice([0, rnd.getrandbits(64)])
            want = oracle.crc("crc64nvme", data, seed)
            got = braid64_model(br, data, 0x1000 + misalign, seed, rows)
            assert got == want, (rows, n, misalign, hex(seed))
