"""CPU model of the balanced event-stream framing kernel (round 6, VERDICT r05 item 6: "one flat word
loop per lane over its balanced span"), checked against zlib.  The algebra eventstream_flat_kernel in
crc_kernels.hip relies on, restated in Python.

Two forms.  `flat_wave` (first built, not kept): no resets, every message's register assembled after
the loop from two records and corrections -- about 80 table lookups per message after the scan, which
measured 3.3 us of a 27.5 us call.  `flat_wave_patched` (the kernel): each message's end patch -- its
stored CRC's four bytes XORed with themselves (cleared) and the next message's first four bytes XORed
with 0xFF (CRC32's ~0 start) -- is applied to the bytes before they are folded, and the lane's register
restarts at every end word (hi4 for a <= 4, else 0), so a record is its message's own register and
only the pieces of messages spanning chunks need products.

A wave takes 64 consecutive messages packed back to back.  Its region [rs, re) is the messages' bytes
widened to 64-byte alignment; lane l folds the l-th chunk [l C, (l + 1) C) of it (C = whole 64-byte
blocks, the same for every lane) as one flat loop of 8-byte words from register 0, with no masks and
no resets: the stored CRCs and the next message's first bytes are folded along.  Only the bytes in
front of the first message (lane 0's first block) are cleared.  Message i's CRC'd span is
[s_i, e_i), e_i = s_i + total_i - 4; its end word starts at P_i = (e_i - 1) & ~7, a_i = e_i - P_i in
1..8.  At its end word the lane records the fold's two halves: lo4 = the lookups of bytes 0..3 (the
register and the word's low half), hi4 = bytes 4..7.  Then

  rec_i = lo4 (a_i <= 4: bytes 4..7 hold only the stored CRC's tail and message i + 1's head) or
          lo4 ^ hi4 (a_i >= 5)
  Y_i   = word(rec_(i-1) ^ word(0, V1_i), V2_i)     (rec_(-1) = 0, B_i = P_(i-1) or s_0 & ~7)
  Z_i   = rec_i ^ G_i ^ Y_i x^(8 (P_i - B_i - 8)) ^ sum_(k = lane(B_i)) ^ (lane(P_i) - 1) end_k x^(8 (P_i + 8 - c0_(k+1)))
  CRC_i = ~(Z_i x^(-8 (8 - a_i)))

V1_i, V2_i are the words at B_i and B_i + 8 holding the previous message's stored-CRC bytes not
inside rec_(i-1) (cancelled) and 0xFF over message i's first four bytes (CRC32's ~0 start); G_i =
word(0, the stored-CRC bytes of message i inside rec_i).  end_k is lane k's register at its chunk end
(the pieces of a message spread over several chunks).  Every product is by x^(64 m) for a whole
number of words m, or by x^(-8 t), t < 8.
"""
import random
import zlib

M = 0xFFFFFFFF


def fold(v, data):
    """the reflected CRC-32 register after `data` from register v (zlib: crc32(d, c) = ~F(~c, d))"""
    return ~zlib.crc32(bytes(data), ~v & M) & M


def shift(r, nbytes):
    return fold(r, b"\0" * nbytes)


def word(v, w):
    """one slice-by-8 step: register v (entering bytes 0..3) and the little-endian word w"""
    return fold(v, int(w).to_bytes(8, "little"))


def halves(v, w):
    x = (v ^ w) & ((1 << 64) - 1)
    return word(0, x & M), word(0, x & ~M & ((1 << 64) - 1))


def _matrix_inverse_shift(t):
    """columns of x^(-8 t): solve shift(c, t) = e_j by Gaussian elimination over GF(2)"""
    cols = [shift(1 << j, t) for j in range(32)]  # image of basis vector j
    # rows of the augmented system A x = b with A's column j = cols[j]
    inv = []
    for target in range(32):
        rows = [(sum(((cols[j] >> r) & 1) << j for j in range(32)), (1 << target >> r) & 1) for r in range(32)]
        # solve for x (32 bits) with sum_j x_j cols[j] = e_target
        piv = []
        rows = list(rows)
        for bit in range(32):
            for k in range(len(piv), 32):
                if (rows[k][0] >> bit) & 1:
                    rows[len(piv)], rows[k] = rows[k], rows[len(piv)]
                    break
            else:
                continue
            p = len(piv)
            for k in range(32):
                if k != p and (rows[k][0] >> bit) & 1:
                    rows[k] = (rows[k][0] ^ rows[p][0], rows[k][1] ^ rows[p][1])
            piv.append(bit)
        x = 0
        for p, bit in enumerate(piv):
            if rows[p][1]:
                x |= 1 << bit
        inv.append(x)
    return inv


_INV = {t: _matrix_inverse_shift(t) for t in range(1, 8)}


def unshift(r, t):
    """r * x^(-8 t)"""
    if t == 0:
        return r
    out = 0
    for j in range(32):
        if (r >> j) & 1:
            out ^= _INV[t][j]
    return out


def bytes_word(pairs):
    """a little-endian word from {byte position: value}"""
    w = 0
    for pos, val in pairs.items():
        w |= (val & 0xFF) << (8 * pos)
    return w


def flat_wave(mem, base, offs, totals):
    """the kernel's walk over one wave of messages at mem[base + offs[i]], back to back.  Returns the
    message CRCs and the chunk size."""
    n = len(offs)
    assert all(offs[i] + totals[i] == offs[i + 1] for i in range(n - 1))
    rs = (base + offs[0]) & ~63
    re = (base + offs[-1] + totals[-1] + 63) & ~63
    units = (re - rs) // 64
    C = -(-units // 64) * 64
    s = [base + o - rs for o in offs]
    e = [s[i] + totals[i] - 4 for i in range(n)]
    P = [(x - 1) & ~7 for x in e]
    a = [e[i] - P[i] for i in range(n)]
    region = bytearray(mem[rs:rs + 64 * C])
    region += bytes(64 * C - len(region))
    for j in range(s[0]):  # lane 0 clears the bytes in front of the first message
        region[j] = 0
    rec = {}
    end_at = {p: i for i, p in enumerate(P)}
    end = []
    for lane in range(64):
        c0 = lane * C
        u = 0
        for p in range(c0, c0 + C, 8):
            w = int.from_bytes(region[p:p + 8], "little")
            lo4, hi4 = halves(u, w)
            if p in end_at:
                rec[end_at[p]] = (lo4, hi4)
            u = lo4 ^ hi4
        end.append(u)

    def lane_of(p):
        return p // C

    crcs = []
    for i in range(n):
        lo4, hi4 = rec[i]
        r = lo4 if a[i] <= 4 else lo4 ^ hi4
        stored = region[e[i]:e[i] + 4]
        # G_i: the stored-CRC bytes inside rec_i
        g = {q: stored[q - a[i]] for q in range(a[i], 4 if a[i] <= 4 else 8) if q - a[i] < 4}
        G = word(0, bytes_word(g))
        if i == 0:
            B, prev = s[0] & ~7, 0
            h = s[0] - B
            v1 = bytes_word({q: 0xFF for q in range(h, min(h + 4, 8))})
            v2 = bytes_word({q: 0xFF for q in range(0, h + 4 - 8)})
        else:
            B = P[i - 1]
            lo4p, hi4p = rec[i - 1]
            ap = a[i - 1]
            prev = lo4p if ap <= 4 else lo4p ^ hi4p
            stp = region[e[i - 1]:e[i - 1] + 4]
            if ap <= 4:
                v1 = bytes_word({**{q: stp[q - ap] for q in range(4, ap + 4)}, **{q: 0xFF for q in range(ap + 4, 8)}})
                v2 = bytes_word({q: 0xFF for q in range(0, ap)})
            else:
                v1 = 0
                v2 = bytes_word({**{q: stp[q + 8 - ap] for q in range(0, ap - 4)}, **{q: 0xFF for q in range(ap - 4, ap)}})
        y = word(prev ^ word(0, v1), v2)
        z = r ^ G ^ shift(y, P[i] - B - 8)
        for k in range(lane_of(B) if i else 0, lane_of(P[i])):
            z ^= shift(end[k], P[i] + 8 - (k + 1) * C)
        crcs.append(~unshift(z, 8 - a[i]) & M)
    return crcs, C


def flat_wave_patched(mem, base, offs, totals, chunk16=True):
    """the kernel's walk: end patches applied to the bytes, registers restarted at end words.  The
    region from message 0's start rounded down to 16 (the kernel) or 64, chunks of C bytes, a multiple
    of 16 (the kernel) or 64."""
    n = len(offs)
    assert all(offs[i] + totals[i] == offs[i + 1] for i in range(n - 1))
    align = 16 if chunk16 else 64
    rs = (base + offs[0]) & ~(align - 1)
    re = (base + offs[-1] + totals[-1] + align - 1) & ~(align - 1)
    rel = re - rs
    g = 16 if chunk16 else 64
    C = -(-(-(-rel // 64)) // g) * g
    s = [base + o - rs for o in offs]
    e = [s[i] + totals[i] - 4 for i in range(n)]
    P = [(x - 1) & ~7 for x in e]
    a = [e[i] - P[i] for i in range(n)]
    region = bytearray(mem[rs:rs + 64 * C])
    region += bytes(64 * C + 16 - len(region))
    for j in range(s[0]):  # bytes in front of message 0 cleared, its first four flipped
        region[j] = 0
    for j in range(s[0], s[0] + 4):
        region[j] ^= 0xFF
    for i in range(n):  # end patches (the stored CRC XORed with itself, the next start with 0xFF)
        stored = bytes(region[e[i]:e[i] + 4])
        for t in range(4):
            region[e[i] + t] ^= stored[t]
            region[e[i] + 4 + t] ^= 0xFF
    rec, end = {}, []
    end_at = {p: i for i, p in enumerate(P)}
    for lane in range(64):
        u = 0
        for p in range(lane * C, lane * C + C, 8):
            lo4, hi4 = halves(u, int.from_bytes(region[p:p + 8], "little"))
            if p in end_at:
                i = end_at[p]
                rec[i] = lo4 if a[i] <= 4 else lo4 ^ hi4
                u = hi4 if a[i] <= 4 else 0
            else:
                u = lo4 ^ hi4
        end.append(u)
    crcs = []
    for i in range(n):
        z = rec[i]
        B = P[i - 1] if i else 0
        for k in range(B // C, P[i] // C):
            z ^= shift(end[k], P[i] + 8 - (k + 1) * C)
        crcs.append(~unshift(z, 8 - a[i]) & M)
    return crcs, C


def _check(rng, mem, lens, base_off):
    offs, pos = [], base_off
    for t in lens:
        offs.append(pos)
        pos += t
    got, C = flat_wave(mem, 0, offs, lens)
    for chunk16 in (True, False):
        got2, _ = flat_wave_patched(mem, 0, offs, lens, chunk16)
        assert got2 == got
    for i, (o, t) in enumerate(zip(offs, lens)):
        assert got[i] == zlib.crc32(mem[o:o + t - 4]), (i, o, t, C)
    return C


def test_flat_algebra_matches_zlib():
    rng = random.Random(0xF1A7)
    mem = rng.randbytes(1 << 17)
    for _ in range(12):
        lens = [rng.randint(16, 1024) for _ in range(64)]
        _check(rng, mem, lens, rng.randrange(0, 4096))


def test_flat_algebra_edges():
    """every alignment of the first message, every end offset a = 1..8 on both sides of a chunk
    boundary, the shortest messages (several ends in one block), one message spanning many chunks"""
    rng = random.Random(5)
    mem = rng.randbytes(1 << 19)
    for h in range(64):
        _check(rng, mem, [16] * 64, 256 + h)
    for h in range(0, 64, 7):
        _check(rng, mem, [rng.randint(16, 40) for _ in range(64)], 1000 + h)
        _check(rng, mem, [16 + (i % 9) for i in range(64)], 333 + h)
        lens = [rng.randint(16, 64) for _ in range(64)]
        lens[17] = 20000  # spans ~30 chunks
        _check(rng, mem, lens, 77 + h)
        lens = [4096] * 63 + [16]
        _check(rng, mem, lens, 5 + h)
