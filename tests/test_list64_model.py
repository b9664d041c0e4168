"""CPU: a Python model of crc64_list_stream_kernel (crc_kernels.hip), checked against
the oracle on ragged CRC64NVME lists.  The work split is test_list_partition_model's (the host cuts the
list's sequence of groups evenly over the waves, cut anywhere, also inside buffers); the row step, the
lane shares and the byte tables are test_braid64_model's.  New at W = 64:

  * a buffer's main region (round 5: the 8-byte words covering it, bytes outside it masked) is front-padded to whole groups with virtual zeros (the
    kernel's buffer-resource loads return zeros there); the head state enters lane (pad mod 512) / 8
    of group 0 divided by X^j, X = x^(8 * 512), j = pad // 512 (the host's X^(-j) columns);
  * a part (a wave's groups ga..gz of one buffer) ends with the lane shares sum_l u_l K_l moved to the
    buffer end by x^(8 * group * (vg - gz)), one product per set bit (the host's x^(8 * group * 2^i)
    columns), XORed into the buffer's accumulator; the part completing the group count finalises.

The kernel's group is 8 rows (4 KiB); the model takes 2 rows per group (the algebra does not depend
on it), so pads land on both rows and on every lane class at small sizes.
"""
import random

import pytest

from oracle import oracle
from tests.test_braid64_model import M64, ROW, Braid64, inv_mulx, mulmod, xpow8n
from tests.test_list_partition_model import host_split, kernel_walk

ROWS = 2
GROUP = ROWS * ROW


@pytest.fixture(scope="module")
def br():
    return Braid64()


def shift_bits(r, m):
    i = 0
    while m:
        if m & 1:
            r = mulmod(r, xpow8n(GROUP << i))
        m >>= 1
        i += 1
    return r


def xneg8(s, t):
    """s * x^(-8 t)"""
    for _ in range(8 * t):
        s = inv_mulx(s)
    return s


def list64_model(br, data, ptrs, lens, seeds, nw):
    # round 5: a buffer of >= 16 bytes is scanned as the 8-byte words [p & ~7, end & ~7); the o bytes in
    # front are cleared (the kernel masks its registers) and the head state enters times x^(-8 o); the
    # tail (< 8 bytes) is folded; shorter buffers fold whole
    edges = []
    for p, L in zip(ptrs, lens):
        if L >= 16:
            H, E = p & ~7, (p + L) & ~7
            main = E - H
        else:
            H, main = p + L, 0
        vg = -(-main // GROUP)
        edges.append((H, main, vg, vg * GROUP - main))
    groups = [e[2] for e in edges]
    acc = [0] * len(ptrs)
    cnt = [0] * len(ptrs)
    out = [None] * len(ptrs)

    def head_state(b):
        if edges[b][1]:
            return xneg8(~seeds[b] & M64, ptrs[b] - edges[b][0])
        return br.bytes_(~seeds[b] & M64, data[ptrs[b]: ptrs[b] + lens[b]])

    def finalize(b, s):
        H, main = edges[b][0], edges[b][1]
        if main:
            s = br.bytes_(s, data[H + main: ptrs[b] + lens[b]])
        out[b] = ~s & M64

    wbuf, woff, wq = host_split(groups, nw)
    for w in range(nw):
        _, empties, parts = kernel_walk(groups, wbuf, woff, wq, w)
        for b in empties:
            finalize(b, head_state(b))
        for b, ga, gz in parts:
            H, main, vg, pad = edges[b]
            u = [0] * 64
            if ga == 0:
                s = head_state(b)
                for _ in range(8 * ROW * (pad // ROW)):  # divided by X^j
                    s = inv_mulx(s)
                u[(pad % ROW) // 8] = s
            for g in range(ga, gz):
                base = H - pad + g * GROUP
                for row in range(ROWS):
                    for lane in range(64):
                        a = base + ROW * row + 8 * lane
                        wd = 0
                        if a >= H:  # the buffer's own bytes only (the kernel's masks)
                            p, e = ptrs[b], ptrs[b] + lens[b]
                            wd = int.from_bytes(bytes(data[x] if p <= x < e else 0 for x in range(a, a + 8)), "little")
                        u[lane] = br.step(u[lane] ^ wd)
            r = 0
            for lane in range(64):
                r ^= br.mulK(u[lane], lane)
            r = shift_bits(r, vg - gz)
            if ga == 0 and gz == vg:
                finalize(b, r)
                continue
            acc[b] ^= r
            cnt[b] += gz - ga
            if cnt[b] == vg:
                finalize(b, acc[b])
    return out


def test_inverse_column_entry():
    """dividing by X^j and stepping j rows of zeros restores the state (the head entry's premise)"""
    rng = random.Random(3)
    for j in (1, 3, 7):
        s = rng.getrandbits(64)
        t = s
        for _ in range(8 * ROW * j):
            t = inv_mulx(t)
        assert mulmod(t, xpow8n(ROW * j)) == s


@pytest.mark.parametrize("seed", range(6))
def test_list64_walk_matches_oracle(br, seed):
    rng = random.Random(0x64 + seed)
    count = rng.choice([3, 5, 8])
    lens = [rng.choice([0, 5, 16, 31, GROUP - 16, GROUP, GROUP + 8, 2 * GROUP + 40, 3 * GROUP - 520,
                        rng.randrange(1, 4 * GROUP)]) for _ in range(count)]
    if not any(L >= 32 for L in lens):
        lens[0] = 2 * GROUP + 40
    ptrs, off = [], rng.randrange(16)
    for L in lens:
        ptrs.append(off)
        off += L + rng.randrange(24)
    data = bytes(rng.getrandbits(8) for _ in range(off + 24))
    seeds = [rng.getrandbits(64) for _ in range(count)]
    nw = rng.choice([1, 2, 3, 7])
    got = list64_model(br, data, ptrs, lens, seeds, nw)
    want = [oracle.crc("crc64nvme", data[p: p + L], s) for p, L, s in zip(ptrs, lens, seeds)]
    assert got == want
