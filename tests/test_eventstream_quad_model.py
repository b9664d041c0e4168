"""CPU model of the event-stream framing kernel's quad braid (crc_kernels.hip eventstream_kernel,
round 4): four lanes per message, each lane owning every fourth 8-byte word of the message body.

Lane j of a quad folds the words w(r, j) at body bytes 32 r + 8 j with the row step
    u_j <- T'(u_j ^ w(r, j)),   T'_t[e] = e * x^(8(t+1)) * x^(8*24)
(a slice-by-8 step whose tables also skip the quad's other 24 bytes of the row).  After R rows the
register of the 32 R body bytes is XOR_j u_j * x^(-64 j); the state entering the body (the prelude's
eight bytes folded from ~0) is XORed into lane 0's first word.  The last (body mod 32) bytes follow on
the plain slice-by-8 / byte path.  Checked against zlib's CRC32 (the oracle's CRC32 convention) on
random framed messages of every body length class, and the byte tables the kernel builds (T', the
lane-share tables) against their definitions.
"""
import random
import zlib

POLY = 0xEDB88320
M32 = 0xFFFFFFFF


def mulx(v):
    return (v >> 1) ^ (POLY if v & 1 else 0)


def mulmod(a, b):
    p, m = 0, 1 << 31
    while m:
        if a & m:
            p ^= b
        m >>= 1
        b = mulx(b)
    return p


def xpow8n(n):
    r, sq = 1 << 31, 1 << 23
    while n:
        if n & 1:
            r = mulmod(r, sq)
        sq = mulmod(sq, sq)
        n >>= 1
    return r


def inv_mulx(t):
    return (((t ^ POLY) << 1) | 1) & M32 if t & 0x80000000 else (t << 1) & M32


def table_entry(e, k):
    c = e
    for _ in range(8 * (k + 1)):
        c = mulx(c)
    return c


T0 = [table_entry(e, 0) for e in range(256)]
STD = [[table_entry(e, t) for e in range(256)] for t in range(8)]  # standard slice-by-8
SKIP = xpow8n(24)
TP = [[mulmod(STD[t][e], SKIP) for e in range(256)] for t in range(8)]  # T'_t


def kj(j):
    v = 1 << 31
    for _ in range(64 * j):
        v = inv_mulx(v)
    return v


K = [kj(j) for j in range(4)]
# lane-share byte tables of class j: M_j[k][e] = (e << 8k) * K_j
MJ = [[[mulmod(e << (8 * k), K[j]) for e in range(256)] for k in range(4)] for j in range(4)]


def word_step(tabs, s, w):
    """slice-by-8: byte i of (s ^ w) (little-endian, s in the low 32 bits) through table 7 - i"""
    a = w ^ s
    r = 0
    for i in range(8):
        r ^= tabs[7 - i][(a >> (8 * i)) & 0xFF]
    return r


def byte_step(s, b):
    return (s >> 8) ^ T0[(s ^ b) & 0xFF]


def quad_message_crc(msg):
    """(prelude CRC, message CRC) of a framed message the way the kernel computes them"""
    total = len(msg)
    s = M32
    s = word_step(STD, s, int.from_bytes(msg[0:8], "little"))  # prelude: the first 8 bytes
    pre = s ^ M32
    body = msg[8:total - 4]
    R = len(body) // 32
    u = [0, 0, 0, 0]
    for r in range(R):
        for j in range(4):
            w = int.from_bytes(body[32 * r + 8 * j: 32 * r + 8 * j + 8], "little")
            if r == 0 and j == 0:
                w ^= s  # the prelude state enters lane 0's first word
            u[j] = word_step(TP, u[j], w)
    if R:
        st = 0
        for j in range(4):
            share = 0
            for k in range(4):
                share ^= MJ[j][k][(u[j] >> (8 * k)) & 0xFF]
            st ^= share
        s = st
    off = 32 * R
    while off + 8 <= len(body):
        s = word_step(STD, s, int.from_bytes(body[off:off + 8], "little"))
        off += 8
    for b in body[off:]:
        s = byte_step(s, b)
    return pre, s ^ M32


def test_tables_match_definitions():
    rng = random.Random(3)
    for _ in range(200):
        e, t = rng.randrange(256), rng.randrange(8)
        # T'_t[e]: byte e, then t + 1 - 1 zero bytes to the end of its word, then 24 skipped bytes
        assert TP[t][e] == table_entry(e, t + 24)
        j, k = rng.randrange(4), rng.randrange(4)
        assert MJ[j][k][e] == mulmod((e << (8 * k)), K[j])
    # K_j * x^(64 j) = 1
    for j in range(4):
        assert mulmod(K[j], xpow8n(8 * j)) == 1 << 31


def test_quad_braid_vs_zlib():
    rng = random.Random(0xE5)
    lengths = list(range(16, 120)) + [16 + 32 * r + d for r in (1, 2, 5, 30, 31) for d in (0, 1, 7, 8, 9, 31)] + \
        [rng.randrange(16, 1025) for _ in range(60)]
    for total in lengths:
        msg = bytes(rng.randrange(256) for _ in range(total))
        pre, crc = quad_message_crc(msg)
        assert pre == zlib.crc32(msg[:8]), total
        assert crc == zlib.crc32(msg[:total - 4]), total
