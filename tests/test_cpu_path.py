"""CPU suite: the engine's product host path (aws-crt-cpp_amd/csrc/cpu/) against the oracle and the
golden fixtures, and the dispatch contract of the value-only ABI (CRC.h:17-20: correct value,
hardware-selected implementation, never an error) -- all without a GPU.

The product host path is NOT the oracle: it is separate code (AVX-512 VPCLMULQDQ / PCLMULQDQ
folding, SSE4.2 crc32, slice-by-8, vectorised XXH3) in the shipped library; the oracle
(oracle/crc_oracle.c, test infrastructure) is the checker here.
"""
import ctypes
import json
import os
import random

import numpy as np
import pytest

from oracle import oracle
from tests.golden.patterns import pattern

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
from tests.libpaths import ENGINE as LIB, LOAD_SRC, load_engine  # noqa: E402
# the diagnostic build (make -C aws-crt-cpp_amd diag): the same host path plus a hook that runs one CRC
# on a chosen host tier, so every tier is checked on any host
from tests.libpaths import DIAG as DIAG_LIB  # noqa: E402
GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "vectors.json")))
ALG = {"crc32": 0, "crc32c": 1, "crc64nvme": 2, "xxh64": 3, "xxh3_64": 4, "xxh3_128": 5}
W64 = {"crc64nvme", "xxh64", "xxh3_64", "xxh3_128"}


@pytest.fixture(scope="module")
def L():
    lib = load_engine()
    vp, sz, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64
    lib.aws_crt_amd_cpu_batch.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(sz), sz,
                                          ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.c_int]
    lib.aws_crt_amd_cpu_tier.restype = ctypes.c_char_p
    for name, t in (("crc32", ctypes.c_uint32), ("crc32c", ctypes.c_uint32), ("crc64nvme", u64)):
        f = getattr(lib, f"aws_checksums_{name}_ex")
        f.restype, f.argtypes = t, [vp, sz, t]
    return lib


@pytest.fixture(scope="module")
def D():
    lib = ctypes.CDLL(DIAG_LIB)
    vp, sz, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64
    lib.aws_crt_amd_debug_cpu_crc.restype = u64
    lib.aws_crt_amd_debug_cpu_crc.argtypes = [ctypes.c_int, ctypes.c_int, vp, sz, u64]
    return lib


def cpu_batch(L, alg, bufs, seeds=None, threads=1):
    n = len(bufs)
    keep = [np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else b for b in bufs]
    P = (ctypes.c_void_p * max(n, 1))(*[k.ctypes.data if k.size else 0 for k in keep])
    S = (ctypes.c_size_t * max(n, 1))(*[k.size for k in keep])
    sd = (ctypes.c_uint64 * max(n, 1))(*(seeds or [0] * n))
    per = 2 if alg == "xxh3_128" else 1
    out = (ctypes.c_uint64 * max(n * per, 1))()
    assert L.aws_crt_amd_cpu_batch(ALG[alg], P, S, n, sd, out, threads) == 0
    if per == 2:
        return [(out[2 * i] << 64) | out[2 * i + 1] for i in range(n)]
    return [int(out[i]) for i in range(n)]


def test_cpu_tier_reported(L):
    assert L.aws_crt_amd_cpu_tier().decode() in ("avx512-vpclmulqdq", "pclmulqdq", "slice-by-8")


@pytest.mark.parametrize("alg", list(ALG))
def test_golden_vectors(L, alg):
    vs = [v for v in GOLDEN["vectors"] if v["alg"] == alg]
    got = cpu_batch(L, alg, [pattern(v["pattern"], v["len"]) for v in vs], [v["seed"] for v in vs])
    assert got == [v["expect"] for v in vs]


def test_reference_known_answers(L):
    # tests/CRCTest.cpp:16,29,42 (32 zero bytes, seed 0) through aws_checksums_*_ex, host memory
    z = ctypes.create_string_buffer(32)
    assert L.aws_checksums_crc32_ex(z, 32, 0) == 0x190A55AD
    assert L.aws_checksums_crc32c_ex(z, 32, 0) == 0x8A9136AA
    assert L.aws_checksums_crc64nvme_ex(z, 32, 0) == 0xCF3473434D4ECF3B
    for alg, want in GOLDEN["check_123456789"].items():
        b = ctypes.create_string_buffer(b"123456789", 9)
        assert getattr(L, f"aws_checksums_{alg}_ex")(b, 9, 0) == want


def test_config1_4k_crc32c(L):
    """BASELINE config 1: one 4 KiB splitmix64 (seed 0x5EED) buffer, CRC32C via the value-only ABI on
    the CPU, no GPU."""
    buf = pattern("splitmix:0x5EED", 4096)
    b = ctypes.create_string_buffer(buf, len(buf))
    got = L.aws_checksums_crc32c_ex(b, len(buf), 0)
    assert got == oracle.crc("crc32c", buf)
    assert got == oracle.crc("crc32c", buf, tier="bitwise")


@pytest.mark.parametrize("alg", ["crc32", "crc32c", "crc64nvme"])
@pytest.mark.parametrize("tier", [0, 1, 2])
def test_every_tier_lengths_alignments(D, alg, tier):
    """Every host tier (tables, PCLMULQDQ fold, AVX-512 fold) over lengths around every fold boundary
    (16/32/64/128/256-byte blocks), every alignment mod 16 and random seeds."""
    rng = random.Random(0xC0 + 7 * ALG[alg] + tier)
    base = np.frombuffer(rng.randbytes(1 << 16), dtype=np.uint8)
    lens = list(range(0, 600)) + [1023, 1024, 1025, 4095, 4096, 4097, 65536 - 17, 65536 - 16]
    for n in lens:
        off = rng.randrange(16)
        seed = rng.getrandbits(64 if alg in W64 else 32)
        chunk = base[off:off + n]
        got = D.aws_crt_amd_debug_cpu_crc(ALG[alg], tier, chunk.ctypes.data, n, seed)
        assert got == oracle.crc(alg, chunk, seed), (alg, tier, n, off)


@pytest.mark.parametrize("alg", list(ALG))
def test_fuzz_vs_oracle(L, alg):
    rng = random.Random(0xF00D + ALG[alg])
    bufs = [rng.randbytes(rng.choice([0, 1, 3, 8, 15, 16, 17, 100, 239, 240, 241, 1023, 1024, 1025, 5000,
                                      rng.randrange(1, 70000)])) for _ in range(300)]
    seeds = [rng.getrandbits(64 if alg in W64 else 32) for _ in bufs]
    assert cpu_batch(L, alg, bufs, seeds, threads=4) == [oracle.checksum(alg, b, s) for b, s in zip(bufs, seeds)]


def test_large_buffer_all_algs(L):
    rng = np.random.default_rng(5)
    buf = rng.integers(0, 256, (24 << 20) + 13, dtype=np.uint8)
    for alg in ALG:
        assert cpu_batch(L, alg, [buf]) == [oracle.checksum(alg, buf)], alg


def test_running_crc_and_combine(L):
    """Chunked running CRC (config 3 semantics) through the value-only ABI on the host path."""
    rng = random.Random(3)
    data = rng.randbytes(1 << 20)
    b = ctypes.create_string_buffer(data, len(data))
    for alg in ("crc32", "crc32c", "crc64nvme"):
        f = getattr(L, f"aws_checksums_{alg}_ex")
        one = f(b, len(data), 0)
        run, off = 0, 0
        for step in (1, 7, 64, 1000, 4096, 100000, len(data)):
            n = min(step, len(data) - off)
            run = f(ctypes.byref(b, off), n, run)
            off += n
            if off == len(data):
                break
        assert off == len(data) and run == one == oracle.crc(alg, data)


@pytest.mark.parametrize("alg", list(ALG))
def test_threaded_batch_splits_long_buffers(L, alg):
    """aws_crt_amd_cpu_batch with more threads than buffers: CRC buffers longer than a piece are
    checksummed in pieces on every thread and folded with Combine (the first piece from the caller's
    seed); hashes stay one item per buffer.  Few long buffers, ragged lengths, seeds, repeated calls
    on the persistent pool, and the same call from several Python threads at once (the pool is
    busy: those calls run on threads of their own)."""
    import threading

    rng = random.Random(0xBA7C + len(alg))
    bufs = [rng.randbytes(n) for n in (3 << 20, (5 << 20) + 13, 17, 0, (1 << 20) + 1)]
    seeds = [rng.getrandbits(64 if alg in ("crc64nvme", "xxh64", "xxh3_64", "xxh3_128") else 32) for _ in bufs]
    want = [oracle.checksum(alg, b, s) for b, s in zip(bufs, seeds)]
    for _ in range(3):
        assert cpu_batch(L, alg, bufs, seeds, threads=8) == want
    assert cpu_batch(L, alg, bufs[:1], seeds[:1], threads=16) == want[:1]
    errs = []

    def worker():
        try:
            for _ in range(3):
                assert cpu_batch(L, alg, bufs, seeds, threads=6) == want
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=worker) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
