"""CPU model of the chunked event-stream framing kernel (round 6; measured slower than
the lane kernel and kept as experiments/patches/eventstream_chunk.patch), checked against zlib: the
algebra the kernel relies on, restated in Python.

A message's CRC'd span [A, E) (A = its offset, E = A + total_length - 4) is cut on the 8-byte grid:
head [A, A8) with A8 = A rounded up to 8, whole words [A8, W) with W = E rounded down to 8, tail [W, E).
The words are cut into chunks of C bytes counted back from W: chunk k (k = 0 ending at W) covers
[max(A8, W - (k + 1) C), W - k C).  Any lane of the wave may fold any chunk: the message's first chunk
starts from the head's state (~0 folded over the head bytes), every other chunk from 0, and a chunk's
register moved to W is its register times x^(8 k C) (one nibble-image product per chunk, images for
k = 1 .. K - 1 in LDS).  The message's lane XORs the chunks' shares (state at W) and folds the tail.
With no whole word (a short message whose head ends at W), the state at W is the head's.
"""
import random
import zlib

M = 0xFFFFFFFF


def fold(v, data):
    """the reflected CRC-32 register after `data` from register v (no complements): zlib's
    crc32(d, c) = ~F(~c, d)"""
    return ~zlib.crc32(bytes(data), ~v & M) & M


def shift(r, nbytes):
    """r * x^(8 nbytes): the register moved past nbytes zero bytes"""
    return fold(r, b"\0" * nbytes)


def chunked_crc(mem, A, E, C):
    A8, W = (A + 7) & ~7, E & ~7
    if A8 > W:  # cannot happen for spans of >= 8 bytes
        raise AssertionError("span too short")
    nwords = (W - A8) // 8
    nch = -(-nwords * 8 // C) if nwords else 0
    head = fold(M, mem[A:A8])
    s = 0 if nch else head
    for k in range(nch):
        lo, hi = max(A8, W - (k + 1) * C), W - k * C
        r = fold(head if k == nch - 1 else 0, mem[lo:hi])
        s ^= shift(r, k * C)
    return ~fold(s, mem[W:E]) & M, nch


def test_chunk_algebra_matches_zlib():
    rng = random.Random(0xE56)
    mem = rng.randbytes(1 << 16)
    for C in (64, 128, 256):
        for _ in range(400):
            A = rng.randrange(0, 1 << 15)
            s = rng.randint(12, 1020)  # total_length 16 .. 1024
            got, _ = chunked_crc(mem, A, A + s, C)
            assert got == zlib.crc32(mem[A:A + s]), (C, A, s)


def test_chunk_algebra_edges():
    """every start and end alignment, spans around the chunk size and the shortest spans"""
    rng = random.Random(7)
    mem = rng.randbytes(1 << 12)
    for C in (64, 128):
        for A in range(64, 80):
            for s in list(range(12, 40)) + [C - 9, C - 1, C, C + 1, C + 7, C + 8, 2 * C + 3, 1020]:
                got, nch = chunked_crc(mem, A, A + s, C)
                assert got == zlib.crc32(mem[A:A + s]), (C, A, s)


def test_chunks_per_wave_balance():
    """the balance the kernel buys on the benchmark's mix (131,072 messages of 16..1024 bytes, 64 per
    wave): rounds of chunks per wave x C against the longest message of the wave (the lane kernel)"""
    rng = random.Random(0xE5)
    lens = [rng.randint(16, 1024) for _ in range(64 * 256)]
    for C in (128, 256):
        lane_words = chunk_words = 0
        for w in range(0, len(lens), 64):
            spans = [n - 4 for n in lens[w:w + 64]]
            lane_words += max(spans) / 8
            k = sum(-(-s // C) for s in spans)
            chunk_words += -(-k // 64) * C / 8
        assert chunk_words < 0.85 * lane_words, (C, chunk_words / lane_words)
