"""CPU: a Python model of crc64_xcd_kernel's walk (crc_kernels.hip), checked against
the oracle.  It restates the parts of the algebra that are new in that kernel; the row step, the lane
shares and the byte tables are test_braid64_model's:

  * all buffers' main regions in order form one sequence of chunks; XCD x of nx takes the x-th
    1/nx of it and its nwx waves take chunks j, j + nwx, ... (cut anywhere, also inside buffers);
  * inside a chunk every lane runs the braid step over its words (rows of 512 bytes);
  * a wave's next chunk of the same buffer: every lane's u <- u * J, J = x^(8 * chunk * (nwx - 1)),
    through the nibble tables the host builds (entry 16 n + v = (v << 4n) * J);
  * a part (a wave's chunks of one buffer) ends with the lane shares sum_l u_l K_l, moved to the
    buffer end by x^(8 * chunk * m) as one product per nonzero byte v of m (the host's byte-level
    columns of x^(8 * chunk * v * 256^L)), XORed into the buffer's accumulator with its chunk count;
    the part that completes the count finalises the buffer (tail bytes, complement);
  * a main region of no whole number of chunks is front-padded with virtual zeros (the kernel's
    buffer-resource loads return zeros there) and the head state enters lane (pad mod 512) / 8 of
    chunk 0 divided by X^(pad / 512), X = x^(8 * 512).

The kernel's chunk is 32 rows (16 KiB); the model takes a few rows per chunk (the algebra does not
depend on it) and small XCD / wave counts, so the cuts fall at every kind of place.
"""
import random

import pytest

from oracle import oracle
from tests.test_braid64_model import M64, ROW, Braid64, inv_mulx, mulmod, xpow8n


@pytest.fixture(scope="module")
def br():
    return Braid64()


def jump_tables(J):
    return [mulmod(v << (4 * n), J) for n in range(16) for v in range(16)]


def jump(tab, u):
    r = 0
    for n in range(16):
        r ^= tab[16 * n + ((u >> (4 * n)) & 15)]
    return r


def shift_bytes(r, m, chunk):
    """r * x^(8 * chunk * m): one product per nonzero byte v of m, by x^(8 * chunk * v * 256^L)"""
    L = 0
    while m:
        v = m & 255
        if v:
            r = mulmod(r, xpow8n(chunk * v * 256 ** L))
        m >>= 8
        L += 1
    return r


def xcd_model(br, data, ptrs, L, seeds, rows_per_chunk, nx, nwx):
    chunk = ROW * rows_per_chunk
    heads, mains = [], []
    for p in ptrs:
        H, E = (p + 15) & ~15, (p + L) & ~15
        assert E > H
        heads.append(H)
        mains.append(E - H)
    assert all(m == mains[0] for m in mains)
    cpb = -(-mains[0] // chunk)
    pad = cpb * chunk - mains[0]  # virtual zeros in front of every main region
    jr, l0 = pad // ROW, (pad % ROW) // 8
    xinv = 1 << 63  # X^(-jr), X = x^(8 * ROW)
    for _ in range(8 * ROW * jr):
        xinv = inv_mulx(xinv)
    nc = cpb * len(ptrs)
    J = xpow8n(chunk * (nwx - 1))
    jt = jump_tables(J)
    acc = [0] * len(ptrs)
    cnt = [0] * len(ptrs)
    out = [None] * len(ptrs)

    def head_state(b):
        p = ptrs[b]
        return br.bytes_(~seeds[b] & M64, data[p: heads[b]])

    def publish(b, r, n):
        acc[b] ^= r
        cnt[b] += n
        if cnt[b] == cpb:
            p = ptrs[b]
            fin = br.bytes_(acc[b], data[heads[b] + mains[b]: p + L])
            out[b] = ~fin & M64

    for x in range(nx):
        xlo, xhi = x * nc // nx, (x + 1) * nc // nx
        for j in range(nwx):
            u = [0] * 64
            pb, pk, pn = None, 0, 0
            c = xlo + j
            while c < xhi:
                b, k = divmod(c, cpb)
                if pn and b == pb:
                    u = [jump(jt, v) for v in u]
                else:
                    if pn:
                        r = 0
                        for lane in range(64):
                            r ^= br.mulK(u[lane], lane)
                        publish(pb, shift_bytes(r, cpb - 1 - pk, chunk), pn)
                    pb, pn = b, 0
                    u = [0] * 64
                    if k == 0:
                        u[l0] = mulmod(head_state(b), xinv)
                pn += 1
                pk = k
                base = heads[b] - pad + k * chunk
                for row in range(rows_per_chunk):
                    for lane in range(64):
                        a = base + ROW * row + 8 * lane
                        w = int.from_bytes(data[a: a + 8], "little") if a >= heads[b] else 0
                        u[lane] = br.step(u[lane] ^ w)
                c += nwx
            if pn:
                r = 0
                for lane in range(64):
                    r ^= br.mulK(u[lane], lane)
                publish(pb, shift_bytes(r, cpb - 1 - pk, chunk), pn)
    return out


def test_jump_tables_and_byte_shifts():
    """the nibble tables reproduce u * J for any u; the byte-level shift reproduces x^(8 chunk m)"""
    rng = random.Random(5)
    J = xpow8n(16384 * 511)
    jt = jump_tables(J)
    for _ in range(50):
        u = rng.getrandbits(64)
        assert jump(jt, u) == mulmod(u, J)
    for m in (0, 1, 255, 256, 511, 4095, 65537, (1 << 24) + 3):
        r = rng.getrandbits(64)
        assert shift_bytes(r, m, 16384) == mulmod(r, xpow8n(16384 * m)), m


@pytest.mark.parametrize("count,cpb,head,tail,nx,nwx,extra", [
    (3, 5, 13, 7, 2, 3, 0),     # eighths (here halves) cut inside buffers; a wave's chunks span buffers
    (2, 7, 0, 0, 3, 2, 0),      # jumps inside buffers; three "XCDs"
    (5, 2, 5, 11, 2, 4, 0),     # more waves than a buffer's chunks: a wave's next chunk two buffers on
    (3, 4, 13, 7, 2, 3, 16),    # front pad of a chunk less 16 bytes: the head enters the last row's lane 62
    (2, 5, 0, 9, 3, 2, 528),    # front pad 496: row 0, lane 62
    (4, 3, 5, 0, 2, 3, 512),    # front pad 512: row 1, lane 0
])
def test_xcd_walk_matches_oracle(br, count, cpb, head, tail, nx, nwx, extra):
    rows = 2
    chunk = ROW * rows
    L = head + cpb * chunk + extra + tail
    stride = (L + 15) // 16 * 16
    off = (16 - head) % 16
    rng = random.Random(count * 131 + cpb)
    data = bytes(rng.getrandbits(8) for _ in range(off + stride * count + 16))
    ptrs = [off + i * stride for i in range(count)]
    seeds = [rng.getrandbits(64) for _ in range(count)]
    got = xcd_model(br, data, ptrs, L, seeds, rows, nx, nwx)
    want = [oracle.crc("crc64nvme", data[p: p + L], s) for p, s in zip(ptrs, seeds)]
    assert got == want
