"""CPU suite: the streaming XXHash object (aws_xxhash_new/update/finalize, reference
include/aws/crt/checksum/XXHash.h:40-91, source/checksum/XXHash.cpp:50-71) keeps O(1) state --
the published XXH64 / XXH3 streaming states -- and agrees with the one-shot oracle for every way of
splitting the input, in particular at the length-class edges of XXH3 (16, 128, 240 bytes, 64-byte
stripes, 1 KiB blocks, the 256-byte internal buffer)."""
import ctypes
import os
import random
import resource

import numpy as np
import pytest

from oracle import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
from tests.libpaths import ENGINE as LIB, LOAD_SRC, load_engine  # noqa: E402


class Cursor(ctypes.Structure):
    _fields_ = [("len", ctypes.c_size_t), ("ptr", ctypes.c_void_p)]


class Buf(ctypes.Structure):
    _fields_ = [("len", ctypes.c_size_t), ("buffer", ctypes.c_void_p), ("capacity", ctypes.c_size_t),
                ("allocator", ctypes.c_void_p)]


@pytest.fixture(scope="module")
def L():
    lib = load_engine()
    for k in ("aws_xxhash64_new", "aws_xxhash3_64_new", "aws_xxhash3_128_new"):
        f = getattr(lib, k)
        f.restype, f.argtypes = ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_uint64]
    lib.aws_xxhash_update.argtypes = [ctypes.c_void_p, Cursor]
    lib.aws_xxhash_finalize.argtypes = [ctypes.c_void_p, ctypes.POINTER(Buf)]
    lib.aws_xxhash_destroy.argtypes = [ctypes.c_void_p]
    return lib


KINDS = {"xxh64": ("aws_xxhash64_new", 8), "xxh3_64": ("aws_xxhash3_64_new", 8), "xxh3_128": ("aws_xxhash3_128_new", 16)}


def stream(L, kind, chunks, seed=0):
    new, size = KINDS[kind]
    h = getattr(L, new)(None, seed)
    assert h
    try:
        for c in chunks:
            arr = c if isinstance(c, np.ndarray) else np.frombuffer(bytes(c), dtype=np.uint8)
            assert L.aws_xxhash_update(h, Cursor(arr.size, arr.ctypes.data if arr.size else None)) == 0
        out = ctypes.create_string_buffer(size)
        b = Buf(0, ctypes.cast(out, ctypes.c_void_p), size, None)
        assert L.aws_xxhash_finalize(h, ctypes.byref(b)) == 0
        assert b.len == size
        # finalize twice is an error (XXHash.h:40-42: unusable after Digest)
        b2 = Buf(0, ctypes.cast(out, ctypes.c_void_p), size, None)
        assert L.aws_xxhash_finalize(h, ctypes.byref(b2)) != 0
        return int.from_bytes(out.raw, "big")
    finally:
        L.aws_xxhash_destroy(h)


def splits(n, rng):
    edges = {0, 1, 15, 16, 17, 127, 128, 129, 239, 240, 241, 255, 256, 257, 511, 512, 513, 1023, 1024, 1025,
             1088, 2047, 2048, 2049, n - 1, n}
    cuts = sorted(e for e in edges if 0 <= e <= n)
    yield [cuts[i + 1] - cuts[i] for i in range(len(cuts) - 1)]
    for _ in range(4):
        sizes, left = [], n
        while left:
            s = min(left, rng.choice([1, 3, 16, 63, 64, 65, 200, 256, 300, 1024, 4097]))
            sizes.append(s)
            left -= s
        yield sizes


@pytest.mark.parametrize("kind", list(KINDS))
def test_every_split_matches_one_shot(L, kind):
    rng = random.Random(0x57EA + len(kind))
    for n in [0, 1, 3, 4, 8, 9, 16, 17, 100, 128, 129, 200, 240, 241, 255, 256, 257, 300, 1024, 1025, 1087,
              2048, 3000, 16384, 16385, 70000]:
        data = np.frombuffer(rng.randbytes(n), dtype=np.uint8)
        seed = rng.getrandbits(64) if n % 2 else 0
        want = oracle.checksum(kind, data, seed)
        for sizes in splits(n, rng):
            chunks, off = [], 0
            for s in sizes:
                chunks.append(data[off:off + s])
                off += s
            assert stream(L, kind, chunks, seed) == want, (kind, n, sizes)


def test_reference_streaming_vectors(L):
    # tests/XXHashTest.cpp:20-28 / :50-57 / :80-87: "Hello world", seed 0, streamed
    assert stream(L, "xxh64", [b"Hello ", b"world"]) == 0xC500B0C912B376D8
    assert stream(L, "xxh3_64", [b"Hello", b" wor", b"ld"]) == 0xB6ACB9D84A38FF74
    assert stream(L, "xxh3_128", [b"Hello world"]) == 0x7351F89812F97382B91D05B31E04DD7F


def test_bounded_memory_1gib_stream(L):
    """1 GiB fed in 1 MiB chunks: the state stays O(1) (peak RSS grows by far less than the stream)."""
    rng = np.random.default_rng(11)
    chunk = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    before = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss  # KiB
    for kind in ("xxh64", "xxh3_64"):
        new, size = KINDS[kind]
        h = getattr(L, new)(None, 7)
        for _ in range(1024):
            assert L.aws_xxhash_update(h, Cursor(chunk.size, chunk.ctypes.data)) == 0
        out = ctypes.create_string_buffer(size)
        b = Buf(0, ctypes.cast(out, ctypes.c_void_p), size, None)
        assert L.aws_xxhash_finalize(h, ctypes.byref(b)) == 0
        L.aws_xxhash_destroy(h)
    grown_kib = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss - before
    assert grown_kib < 1024, grown_kib
    # digest of the repeated chunk, cross-checked on a 64 MiB prefix-equivalent stream
    small = np.tile(chunk, 64)
    assert stream(L, "xxh64", [chunk] * 64, 7) == oracle.xxh64(small, 7)
    assert stream(L, "xxh3_64", [chunk] * 64, 7) == oracle.xxh3_64(small, 7)


def _dev_stream(L, kind, base, sizes, seed):
    """digest of the device bytes [base, base + sum(sizes)) streamed in `sizes` chunks"""
    new, size = KINDS[kind]
    h = getattr(L, new)(None, seed)
    assert h
    try:
        off = 0
        for s in sizes:
            assert L.aws_xxhash_update(h, Cursor(s, base + off if s else None)) == 0
            off += s
        out = ctypes.create_string_buffer(size)
        b = Buf(0, ctypes.cast(out, ctypes.c_void_p), size, None)
        assert L.aws_xxhash_finalize(h, ctypes.byref(b)) == 0
        return int.from_bytes(out.raw, "big")
    finally:
        L.aws_xxhash_destroy(h)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["xxh3_64", "xxh3_128"])
def test_device_stream_xxh3_every_edge(L, engine, kind):
    """Streaming XXH3 on device memory (abi_single.cpp aws_xxhash_update): chunks of >= 1 MiB are
    absorbed on the GPU (block sums over all CUs, then the scramble chain from the stream's
    accumulators), the bytes around them through the host state.  The first device chunk starts after
    host-sized prefixes at every XXH3 length-class edge (16, 128, 240 bytes, the 256-byte buffer, 1 KiB
    blocks, stripe positions), device chunks follow each other at shifted stripe positions, and every
    split digests to the oracle's one-shot value, with zero fallbacks (conftest)."""
    import torch

    M = 1 << 20
    g = torch.Generator(device="cuda")
    g.manual_seed(0xD5)
    n_max = 3 * M + 4096
    d = torch.randint(0, 256, (n_max,), dtype=torch.uint8, device="cuda", generator=g)
    h = d.cpu().numpy()
    prefixes = [0, 1, 16, 17, 128, 129, 240, 241, 255, 256, 257, 1000, 1023, 1024, 1025, 1087, 1088, 64 * 15 + 1, 4096]
    for n in (3 * M + 4096, 2 * M + 777, M + 64 * 16 + 5):
        for seed in (0, 0x9E3779B97F4A7C15):
            want = oracle.checksum(kind, h[:n], seed)
            for pre in prefixes:
                for tail in ([], [M + 13], [3, M - 1, 17, M + 64 * 7 + 1]):
                    sizes = [pre] + tail
                    if sum(sizes) > n:
                        continue
                    sizes.append(n - sum(sizes))
                    assert _dev_stream(L, kind, d.data_ptr(), sizes, seed) == want, (kind, n, seed, sizes)


@pytest.mark.gpu
def test_device_stream_xxh3_large_chunk(L, engine):
    """One 300 MiB device chunk (more than one 256 MiB absorb pass) after an unaligned 5-byte prefix,
    and 64 MiB chunks back to back, against the oracle's one-shot XXH3-64 / XXH3-128."""
    import torch

    n = 300 << 20
    g = torch.Generator(device="cuda")
    g.manual_seed(0xD6)
    d = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    h = d.cpu().numpy()
    for kind in ("xxh3_64", "xxh3_128"):
        want = oracle.checksum(kind, h, 7)
        assert _dev_stream(L, kind, d.data_ptr(), [5, n - 5], 7) == want
        assert _dev_stream(L, kind, d.data_ptr(), [64 << 20] * 4 + [n - (256 << 20)], 7) == want
