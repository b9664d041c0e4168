"""GPU parity: the HIP engine (through its C ABI) against the oracle, bit-exact.

Covers the reference's known-answer tests (tests/CRCTest.cpp:16,29,42), the golden fixtures, the
BASELINE.json configs at full size where the oracle is fast enough (C2: 1024 x 64 KiB) and through
size-independent properties beyond that (C3: one-shot == chained running CRC == Combine of parts),
plus the edge cases the API admits: empty and tiny buffers, every alignment mod 16, ragged lengths,
non-zero previousCRC seeds, lengths not a multiple of the tile, repeated and concurrent launches.
"""
import json
import os
import random

import numpy as np
import pytest

from oracle import oracle
from tests.golden.patterns import pattern

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "vectors.json")))
ALG = {"crc32": 0, "crc32c": 1, "crc64nvme": 2, "xxh64": 3, "xxh3_64": 4, "xxh3_128": 5}
W64 = {"crc64nvme", "xxh64", "xxh3_64", "xxh3_128"}


def results(engine, alg, out):
    v = engine.as_unsigned(out)
    if alg == "xxh3_128":
        return [(v[2 * i] << 64) | v[2 * i + 1] for i in range(len(v) // 2)]
    return v


def dev_random(n, seed):
    import torch

    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.randint(0, 256, (max(n, 1),), dtype=torch.uint8, device="cuda", generator=g)


def host_bytes(t, off=0, n=None):
    a = t.cpu().numpy()
    return a[off: off + (len(a) - off if n is None else n)]


def seeds_tensor(alg, vals):
    import torch

    if alg in W64:
        return torch.tensor([v - (1 << 64) if v >= 1 << 63 else v for v in vals], dtype=torch.int64, device="cuda")
    return torch.tensor([v - (1 << 32) if v >= 1 << 31 else v for v in vals], dtype=torch.int32, device="cuda")


def test_reference_kats_single_abi(engine):
    # tests/CRCTest.cpp:12-42 through the aws_checksums_*_ex ABI, host memory
    z = bytes(32)
    assert engine.crc("crc32", z) == 0x190A55AD
    assert engine.crc("crc32c", z) == 0x8A9136AA
    assert engine.crc("crc64nvme", z) == 0xCF3473434D4ECF3B
    for alg, want in GOLDEN["check_123456789"].items():
        assert engine.crc(alg, b"123456789") == want


def test_single_abi_device_pointer(engine):
    t = dev_random(100003, 1)
    h = host_bytes(t)
    for alg in ("crc32", "crc32c", "crc64nvme"):
        assert engine.crc(alg, t, 77) == oracle.crc(alg, h, 77)


@pytest.mark.parametrize("alg", ["crc32", "crc32c", "crc64nvme", "xxh64", "xxh3_64", "xxh3_128"])
def test_golden_vectors_list(engine, alg):
    import torch

    vs = [v for v in GOLDEN["vectors"] if v["alg"] == alg]
    blobs = [pattern(v["pattern"], v["len"]) for v in vs]
    # pack with varying misalignment so the list path sees every offset mod 16
    offs, pos = [], 0
    for i, b in enumerate(blobs):
        pos += i % 16
        offs.append(pos)
        pos += len(b) + 16
    buf = np.zeros(pos + 16, dtype=np.uint8)
    for o, b in zip(offs, blobs):
        buf[o: o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    d = torch.from_numpy(buf).cuda()
    base = d.data_ptr()
    out = engine.checksum_list(ALG[alg], [base + o for o in offs], [len(b) for b in blobs],
                               seeds=seeds_tensor(alg, [v["seed"] for v in vs]))
    torch.cuda.synchronize()
    got = results(engine, alg, out)
    for v, g in zip(vs, got):
        assert g == v["expect"], v


@pytest.mark.parametrize("alg", ["crc32c", "crc32", "crc64nvme"])
def test_config2_full_size(engine, alg):
    """BASELINE config 2: 1024 x 64 KiB contiguous, device-resident, seed 0."""
    import torch

    n, L = 1024, 65536
    d = dev_random(n * L, 2)
    out = engine.checksum_strided(ALG[alg], d, L, L, n)
    torch.cuda.synchronize()
    h = host_bytes(d)
    ptrs = [h.ctypes.data + i * L for i in range(n)]
    want = oracle.batch(alg, ptrs, [L] * n, 8)
    assert engine.as_unsigned(out) == want


@pytest.mark.parametrize("alg", ["crc32", "crc32c", "crc64nvme"])
@pytest.mark.parametrize("L,off,count", [(8192, 0, 4096), (8192 + 16, 0, 300), (65536 + 48, 0, 200),
                                         (1000, 0, 257), (4096, 3, 1), (100, 0, 999), (1 << 20, 0, 16),
                                         ((1 << 20) + 5, 7, 1), (0, 0, 5), (1, 0, 33), (17, 0, 64),
                                         # streaming scan (main region a whole number of tiles): fewer
                                         # tiles than waves, head + tail bytes around whole tiles, and
                                         # buffers of many 32-tile groups
                                         (4096, 0, 5), (65554, 5, 300), (1 << 26, 0, 2)])
def test_strided_shapes_with_seeds(engine, alg, L, off, count):
    import torch

    stride = (L + 15) // 16 * 16 if count > 1 else L
    d = dev_random(stride * count + off + 16, 3 + L)
    rng = random.Random(L * 31 + count)
    seeds = [rng.getrandbits(64 if alg in W64 else 32) for _ in range(count)]
    out = engine.checksum_strided(ALG[alg], d, stride, L, count, seeds=seeds_tensor(alg, seeds), base_offset=off)
    torch.cuda.synchronize()
    h = host_bytes(d)
    want = [oracle.crc(alg, h[off + i * stride: off + i * stride + L], seeds[i]) for i in range(count)]
    assert engine.as_unsigned(out) == want


@pytest.mark.parametrize("L,off,count,stride_pad", [
    (0, 0, 5, 0), (31, 1, 3, 1), (32, 0, 7, 0), (33, 3, 17, 5), (511, 0, 1, 0), (512, 0, 2, 0), (513, 5, 3, 3),
    (32 * 16 * 12 * 3 + 100, 0, 4, 0), (32 * 16 * 12 + 32 * 5, 2, 3, 1), ((1 << 20) + 7, 1, 3, 9),
    (65536, 0, 1024, 0), (1000, 0, 1500, 0), (777, 4, 3000, 3), (300, 0, 6000, 0), (200, 1, 9000, 1)])
def test_xxh64_strided_wave_kernel(engine, L, off, count, stride_pad):
    """Strided XXH64 (xxh64_wave_kernel): B = 1, 2, 4, 8, 16 buffers per wave (by count), lengths
    with no full stripe, partial last slots and whole pipeline rounds, unaligned bases and strides,
    per-buffer seeds and seed 0."""
    import torch

    stride = L + stride_pad
    d = dev_random(stride * count + off + 16, 11 + L + count)
    rng = random.Random(L * 7 + count)
    seeds = [rng.getrandbits(64) for _ in range(count)]
    out = engine.checksum_strided(ALG["xxh64"], d, stride, L, count, seeds=seeds_tensor("xxh64", seeds), base_offset=off)
    out0 = engine.checksum_strided(ALG["xxh64"], d, stride, L, count, base_offset=off)
    torch.cuda.synchronize()
    h = host_bytes(d)
    ptrs = [h.ctypes.data + off + i * stride for i in range(count)]
    assert results(engine, "xxh64", out0) == oracle.batch("xxh64", ptrs, [L] * count, 8)
    assert results(engine, "xxh64", out) == [oracle.checksum("xxh64", h[off + i * stride: off + i * stride + L], s)
                                             for i, s in enumerate(seeds)]


def test_xxh64_overlapping_long_buffers(engine):
    """Few long XXH64 buffers whose stride is below their length -- stride 0 (one buffer under several
    seeds) and overlapping windows -- cannot be copied row by row (a 2D copy's pitch must cover its
    width): they stay on the kernels and equal the oracle."""
    L, n = (1 << 20) + 77, 6
    d = dev_random(L + n * 4096 + 64, 79)
    h = host_bytes(d)
    rng = random.Random(79)
    for stride in (0, 4096, 16):
        seeds = [rng.getrandbits(64) for _ in range(n)]
        out = engine.checksum_strided(ALG["xxh64"], d, stride, L, n, seeds=seeds_tensor("xxh64", seeds), base_offset=5)
        assert results(engine, "xxh64", out) == [oracle.checksum("xxh64", h[5 + i * stride: 5 + i * stride + L], s)
                                                 for i, s in enumerate(seeds)], stride


def test_xxh64_host_route_concurrent_streams(engine):
    """the host route hashes on its own worker threads, ordered against the streams
    by counters in signal memory (hipStreamWaitValue64 / hipStreamWriteValue64), not inside host
    callbacks.  Three streams each submit jobs back to back (more jobs than staging sets at first, and
    a job's input overwritten on its stream right after the call); every result equals the oracle."""
    import torch

    n, L = 4, (2 << 20) + 192
    streams = [torch.cuda.Stream() for _ in range(3)]
    data = [dev_random(n * L, 90 + k) for k in range(3)]
    want = []
    for k in range(3):
        h = host_bytes(data[k])
        want.append([oracle.checksum("xxh64", h[i * L:(i + 1) * L]) for i in range(n)])
    torch.cuda.synchronize()
    outs = []
    for rep in range(4):
        for k, st in enumerate(streams):
            with torch.cuda.stream(st):
                out = torch.empty(n, dtype=torch.int64, device="cuda")
                engine.checksum_strided(ALG["xxh64"], data[k], L, L, n, out=out, stream=st)
                outs.append((k, out))
    torch.cuda.synchronize()
    for k, out in outs:
        assert results(engine, "xxh64", out) == want[k], k
    # stream order: overwrite the input on the stream right after the call
    st = streams[0]
    with torch.cuda.stream(st):
        out = torch.empty(n, dtype=torch.int64, device="cuda")
        engine.checksum_strided(ALG["xxh64"], data[0], L, L, n, out=out, stream=st)
        data[0].fill_(0)
    torch.cuda.synchronize()
    assert results(engine, "xxh64", out) == want[0]


def test_xxh64_config5_on_the_kernels(engine, monkeypatch):
    """BASELINE C5's XXH64 half (8 x 64 MiB) on the GPU kernels (AWS_CRT_AMD_XXH64_ROUTE=0; by default
    the batch takes the host route): results equal the oracle and the default route's, seeds on half
    the buffers."""
    import torch

    n, L = 8, 64 << 20
    d = dev_random(n * L, 0xC5)
    rng = random.Random(0xC5)
    seeds = [rng.getrandbits(64) if i % 2 else 0 for i in range(n)]
    monkeypatch.setenv("AWS_CRT_AMD_XXH64_ROUTE", "0")
    kern = engine.checksum_strided(ALG["xxh64"], d, L, L, n, seeds=seeds_tensor("xxh64", seeds))
    torch.cuda.synchronize()
    monkeypatch.delenv("AWS_CRT_AMD_XXH64_ROUTE")
    route = engine.checksum_strided(ALG["xxh64"], d, L, L, n, seeds=seeds_tensor("xxh64", seeds))
    torch.cuda.synchronize()
    h = host_bytes(d)
    want = [oracle.checksum("xxh64", h[i * L:(i + 1) * L], s) for i, s in enumerate(seeds)]
    assert results(engine, "xxh64", kern) == want
    assert results(engine, "xxh64", route) == want


def test_xxh64_few_long_buffers_host_route(engine):
    """Strided XXH64 batches of at most 32 buffers of >= 1 MiB take the stream-ordered host route
    (engine.cpp xxh64_host_route: D2H slices, host threads, results H2D on the caller's stream; a
    serial XXH64 chain runs about 13x faster on a host core than on a gfx950 SIMD).
    The call stays asynchronous and stream-ordered: the input is overwritten on the same stream right
    after the call and the results are still those of the original bytes.  Seeds, an unaligned base,
    a stride that is not a multiple of 64, and the single-buffer ABI on a device buffer (whose result
    slot is pinned host memory) are covered."""
    import ctypes

    import torch

    n, Lb, off = 5, (3 << 20) + 13, 3
    d = dev_random(n * Lb + 64, 77)
    h = host_bytes(d).copy()
    rng = random.Random(77)
    seeds = [rng.getrandbits(64) for _ in range(n)]
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        out = torch.empty(n, dtype=torch.int64, device="cuda")
        engine.checksum_strided(ALG["xxh64"], d, Lb, Lb, n, seeds=seeds_tensor("xxh64", seeds), out=out, stream=st,
                                base_offset=off)
        d.zero_()  # queued behind the hash on the same stream
    st.synchronize()
    assert results(engine, "xxh64", out) == [oracle.checksum("xxh64", h[off + i * Lb: off + (i + 1) * Lb], s)
                                             for i, s in enumerate(seeds)]
    # the single-buffer ABI (aws_xxhash64_compute) on a 2 MiB device buffer
    d2 = dev_random(2 << 20, 78)
    torch.cuda.synchronize()

    class Cur(ctypes.Structure):
        _fields_ = [("len", ctypes.c_size_t), ("ptr", ctypes.c_void_p)]

    class Buf(ctypes.Structure):
        _fields_ = [("len", ctypes.c_size_t), ("buffer", ctypes.c_void_p), ("capacity", ctypes.c_size_t),
                    ("allocator", ctypes.c_void_p)]

    Lc = engine.lib()
    Lc.aws_xxhash64_compute.argtypes = [ctypes.c_uint64, Cur, ctypes.POINTER(Buf)]
    o = ctypes.create_string_buffer(8)
    b = Buf(0, ctypes.cast(o, ctypes.c_void_p), 8, None)
    assert Lc.aws_xxhash64_compute(99, Cur(d2.numel(), d2.data_ptr()), ctypes.byref(b)) == 0
    assert int.from_bytes(o.raw, "big") == oracle.checksum("xxh64", host_bytes(d2), 99)


def test_crc64_short_strided_batches_lane_path(engine):
    """Strided CRC64NVME launches of >= 65536 buffers of <= 4 KiB take the lane-per-buffer scan with
    per-batch bases, seeds and results: three queued batches of 30000 x 3000 B (stride 3008), seeds
    on two of them."""
    import torch

    L, stride, count, nb = 3000, 3008, 30000, 3
    d = dev_random(nb * stride * count + 64, 0x640)
    rng = random.Random(0x64)
    seeds = [[rng.getrandbits(64) for _ in range(count)] if j != 1 else None for j in range(nb)]
    outs = [torch.empty(count, dtype=torch.int64, device="cuda") for _ in range(nb)]
    batches = [(d.data_ptr() + j * stride * count, seeds_tensor("crc64nvme", seeds[j]) if seeds[j] else None, outs[j])
               for j in range(nb)]
    engine.checksum_batches(ALG["crc64nvme"], batches, stride, L, count)
    torch.cuda.synchronize()
    h = host_bytes(d)
    for j in range(nb):
        base = j * stride * count
        ptrs = [h.ctypes.data + base + i * stride for i in range(count)]
        if seeds[j] is None:
            assert engine.as_unsigned(outs[j]) == oracle.batch("crc64nvme", ptrs, [L] * count, 8), j
        else:
            got = engine.as_unsigned(outs[j])
            for i in range(0, count, 997):
                assert got[i] == oracle.crc("crc64nvme", h[base + i * stride: base + i * stride + L], seeds[j][i]), (j, i)


@pytest.mark.parametrize("count,L,stride,off,seeded", [
    (16384, 8192, 8192, 0, False),          # the C4 shard's buffer size, exactly a set of four per wave slot
    (16387, 8212, 8224, 3, True),           # a partial last set; 13 head and 7 tail bytes per buffer; seeds
    (20000, 2048, 2048, 0, True),           # two groups per buffer
    (16400, 65552, 65552, 5, False),        # 64 KiB main regions, 11 head and 5 tail bytes
])
def test_crc64_rows16_short_buffers(engine, count, L, stride, off, seeded):
    """Strided CRC64NVME batches of >= 16384 short buffers whose main regions are whole 1 KiB groups
    take crc64_rows16_kernel (16 lanes per buffer, four buffers per wave): whole sets, a partial last
    set, unaligned heads and tails, seeds."""
    import torch

    d = dev_random(stride * count + off + 64, 0x1616 + count)
    rng = random.Random(count)
    seeds = [rng.getrandbits(64) for _ in range(count)] if seeded else None
    out = engine.checksum_strided(ALG["crc64nvme"], d, stride, L, count,
                                  seeds=seeds_tensor("crc64nvme", seeds) if seeded else None, base_offset=off)
    torch.cuda.synchronize()
    h = host_bytes(d)
    got = engine.as_unsigned(out)
    ptrs = [h.ctypes.data + off + i * stride for i in range(count)]
    if not seeded:
        assert got == oracle.batch("crc64nvme", ptrs, [L] * count, 8)
    else:
        for i in list(range(0, count, 211)) + [count - 1, count - 2, count - 3]:
            assert got[i] == oracle.crc("crc64nvme", h[off + i * stride: off + i * stride + L], seeds[i]), i


@pytest.mark.parametrize("count,chunks,head,tail,seeded,extra", [
    (3, 300, 13, 7, True, 0),     # unaligned heads and tails, seeds; XCD eighths cut inside buffers
    (5, 256, 0, 0, False, 0),     # the fewest chunks taken: a wave's next chunk is two buffers on
    (2, 4099, 11, 5, True, 0),    # 64 MiB + 3 chunks: parts of 8-9 chunks per wave, ragged eighths
    (9, 1024, 0, 9, False, 0),    # nine 16 MiB buffers over eight XCDs
    (1, 4101, 3, 9, True, 0),     # one buffer over all eight XCDs: every eighth a part, shifts up to 3.6 K chunks
    (3, 300, 13, 7, True, 16),    # front pad 16368: the head enters lane 62 at row 31
    (2, 260, 0, 0, False, 2608),  # front pad 13776: lane 58, row 26
    (1, 4096, 5, 3, True, 8192),  # front pad 8192: lane 0, row 16 (two whole groups of zeros)
    (4, 256, 11, 0, False, 4080), # front pad 12304: lane 2, row 24
])
def test_crc64_xcd_long_buffers(engine, count, chunks, head, tail, seeded, extra):
    """Strided CRC64NVME batches with main regions of at least 256 chunks of 16 KiB take
    crc64_xcd_kernel: XCD-window chunk order, the chunk jump from nibble tables, parts moved to the
    buffer end and joined by chunk count; a main region of no whole number of chunks is front-padded
    with virtual zeros (buffer-resource loads) and the head state enters behind the pad."""
    import torch

    off = (16 - head) % 16
    L = head + chunks * 16384 + extra + tail
    stride = (L + 15) // 16 * 16
    d = dev_random(stride * count + off + 64, 0x5CD + count)
    rng = random.Random(chunks)
    seeds = [rng.getrandbits(64) for _ in range(count)] if seeded else None
    out = engine.checksum_strided(ALG["crc64nvme"], d, stride, L, count,
                                  seeds=seeds_tensor("crc64nvme", seeds) if seeded else None, base_offset=off)
    torch.cuda.synchronize()
    h = host_bytes(d)
    got = engine.as_unsigned(out)
    for i in range(count):
        want = oracle.crc("crc64nvme", h[off + i * stride: off + i * stride + L], seeds[i] if seeded else 0)
        assert got[i] == want, i


def test_crc64_xcd_multi_batch(engine):
    """Three queued batches of 2 x 16 MiB through aws_crt_amd_checksum_batches (one crc64_xcd_kernel
    launch over six buffers), seeds on one batch."""
    import torch

    L, count, nb = 16 << 20, 2, 3
    d = dev_random(nb * L * count, 0x5CE)
    rng = random.Random(0x5CE)
    seeds = [[rng.getrandbits(64) for _ in range(count)] if j == 1 else None for j in range(nb)]
    outs = [torch.empty(count, dtype=torch.int64, device="cuda") for _ in range(nb)]
    engine.checksum_batches(ALG["crc64nvme"], [(d.data_ptr() + j * L * count, seeds_tensor("crc64nvme", seeds[j]) if seeds[j] else None,
                                                outs[j]) for j in range(nb)], L, L, count)
    torch.cuda.synchronize()
    h = host_bytes(d)
    for j in range(nb):
        got = engine.as_unsigned(outs[j])
        for i in range(count):
            o = (j * count + i) * L
            assert got[i] == oracle.crc("crc64nvme", h[o:o + L], seeds[j][i] if seeds[j] else 0), (j, i)


@pytest.mark.parametrize("count,nb", [(2048, 1), (768, 3)])
def test_crc64_xcd_part_table_overflow(engine, count, nb):
    """crc64_xcd_kernel joins a workgroup's parts in an LDS table of 64 buffers (round 5); a workgroup
    meeting more buffers publishes the rest straight to the accumulators.  Overlapping 4 MiB windows
    at a 64 KiB + 16 stride put ~256 buffers on every XCD (and ~128 in every workgroup's walk): all
    results against the ragged-list kernel (crc64_list_stream_kernel) over the same windows, a sample
    against the oracle; seeds on the last batch."""
    import torch

    L, stride = 256 * 16384, 65536 + 16
    span = stride * (count - 1) + L
    d = dev_random(nb * span + 64, 0x7AB + count)
    rng = random.Random(count)
    seeds = [[rng.getrandbits(64) for _ in range(count)] if j == nb - 1 else None for j in range(nb)]
    outs = [torch.empty(count, dtype=torch.int64, device="cuda") for _ in range(nb)]
    engine.checksum_batches(ALG["crc64nvme"], [(d.data_ptr() + j * span, seeds_tensor("crc64nvme", seeds[j]) if seeds[j] else None,
                                                outs[j]) for j in range(nb)], stride, L, count)
    torch.cuda.synchronize()
    h = host_bytes(d)
    for j in range(nb):
        got = engine.as_unsigned(outs[j])
        ptrs = [d.data_ptr() + j * span + i * stride for i in range(count)]
        lst = engine.checksum_list(ALG["crc64nvme"], ptrs, [L] * count,
                                   seeds=seeds_tensor("crc64nvme", seeds[j]) if seeds[j] else None)
        torch.cuda.synchronize()
        assert got == engine.as_unsigned(lst), j
        for i in (0, 1, count // 2, count - 1):
            o = j * span + i * stride
            assert got[i] == oracle.crc("crc64nvme", h[o:o + L], seeds[j][i] if seeds[j] else 0), (j, i)


def test_crc64_rows16_multi_batch(engine):
    """Three queued batches of 16384 x 8 KiB through aws_crt_amd_checksum_batches (one rows16 launch
    over 49152 buffers, sets crossing batch boundaries), seeds on one batch."""
    import torch

    L, count, nb = 8192, 16384, 3
    d = dev_random(nb * L * count, 0x1617)
    rng = random.Random(0x1617)
    seeds = [[rng.getrandbits(64) for _ in range(count)] if j == 2 else None for j in range(nb)]
    outs = [torch.empty(count, dtype=torch.int64, device="cuda") for _ in range(nb)]
    engine.checksum_batches(ALG["crc64nvme"], [(d.data_ptr() + j * L * count, seeds_tensor("crc64nvme", seeds[j]) if seeds[j] else None,
                                                outs[j]) for j in range(nb)], L, L, count)
    torch.cuda.synchronize()
    h = host_bytes(d)
    for j in range(nb):
        ptrs = [h.ctypes.data + (j * count + i) * L for i in range(count)]
        if seeds[j] is None:
            assert engine.as_unsigned(outs[j]) == oracle.batch("crc64nvme", ptrs, [L] * count, 8), j
        else:
            got = engine.as_unsigned(outs[j])
            for i in range(0, count, 331):
                assert got[i] == oracle.crc("crc64nvme", h[(j * count + i) * L:(j * count + i + 1) * L], seeds[j][i]), i


def test_xxh64_list_many_buffers_per_wave(engine):
    """Ragged XXH64 lists of more than 1024 buffers put several buffers in one wave
    (xxh64_quad_kernel, bpw = ceil(n / 1024)): 5000 buffers of random length 0..3000 at random
    alignments, with per-buffer seeds, so the last wave is partly idle."""
    import torch

    rng = random.Random(0x64_5000)
    lens = [rng.randrange(0, 3001) for _ in range(5000)]
    offs, pos = [], 0
    for ln in lens:
        pos += rng.randrange(0, 16)
        offs.append(pos)
        pos += ln
    d = dev_random(pos + 64, 0x5000)
    seeds = [rng.getrandbits(64) for _ in lens]
    out = engine.checksum_list(ALG["xxh64"], [d.data_ptr() + o for o in offs], lens, seeds=seeds_tensor("xxh64", seeds))
    torch.cuda.synchronize()
    h = host_bytes(d)
    assert results(engine, "xxh64", out) == [oracle.checksum("xxh64", h[o: o + ln], s) for o, ln, s in zip(offs, lens, seeds)]


@pytest.mark.parametrize("alg", ["crc32", "crc32c", "crc64nvme", "xxh64", "xxh3_64", "xxh3_128"])
def test_ragged_list_random(engine, alg):
    import torch

    rng = random.Random(ALG[alg] + 100)
    lens = [rng.choice([0, 1, 3, 15, 16, 31, 33, 255, 4097, 8192, 30000, 65536, 65557, 200001, 1 << 20])
            for _ in range(300)]
    offs, pos = [], 0
    for ln in lens:
        pos += rng.randrange(0, 64)
        offs.append(pos)
        pos += ln
    d = dev_random(pos + 64, 5)
    seeds = [rng.getrandbits(64 if alg in W64 else 32) for _ in lens]
    out = engine.checksum_list(ALG[alg], [d.data_ptr() + o for o in offs], lens, seeds=seeds_tensor(alg, seeds))
    torch.cuda.synchronize()
    h = host_bytes(d)
    want = [oracle.checksum(alg, h[o: o + ln], s) for o, ln, s in zip(offs, lens, seeds)]
    assert results(engine, alg, out) == want


@pytest.mark.gpu
@pytest.mark.parametrize("alg", ["crc32c", "crc64nvme"])
def test_list_long_buffers_cut_over_all_waves(engine, alg):
    """list streaming scans (crc32_list_stream_kernel, crc64_list_stream_kernel): a 300 MiB buffer cut
    into parts on thousands of waves (part shifts of up to 2^16 groups, accumulator and count joins)
    beside empty, short and 64 MiB buffers, at every kind of front pad; seeds on all."""
    import torch

    lens = [(300 << 20) + 13, 0, 17, (64 << 20) - 8, (5 << 20) + 4095, 4096, 1]
    offs, pos = [], 3
    for ln in lens:
        offs.append(pos)
        pos += ln + 7
    d = dev_random(pos + 64, 0x1A)
    rng = random.Random(0x1A + ALG[alg])
    seeds = [rng.getrandbits(64 if alg in W64 else 32) for _ in lens]
    out = engine.checksum_list(ALG[alg], [d.data_ptr() + o for o in offs], lens, seeds=seeds_tensor(alg, seeds))
    torch.cuda.synchronize()
    h = host_bytes(d)
    want = [oracle.checksum(alg, h[o: o + ln], s) for o, ln, s in zip(offs, lens, seeds)]
    assert results(engine, alg, out) == want


@pytest.mark.gpu
@pytest.mark.parametrize("alg", ["crc32c", "crc64nvme"])
@pytest.mark.parametrize("nbuf,lo,hi", [(1024, 32 << 10, 96 << 10), (3000, 4097, 40000), (200, 200 << 10, 1 << 20)])
def test_ragged_list_workgroup_joins(engine, alg, nbuf, lo, hi):
    """Ragged lists on the list streaming scans where most buffers are cut between waves (the
    list probe's shape, scaled): a cut buffer's parts inside one workgroup join in LDS slots and
    finish there, or publish the workgroup's share when the buffer continues into another
    workgroup (slot 8 for a buffer begun in an earlier one); buffers over one, two and many waves.
    Random starts and lengths, seeds on all."""
    import torch

    rng = random.Random(nbuf + lo + ALG[alg])
    lens = [rng.randrange(lo, hi) for _ in range(nbuf)]
    offs, pos = [], 5
    for ln in lens:
        offs.append(pos)
        pos += ln + rng.randrange(0, 64)
    d = dev_random(pos + 64, nbuf + 0x70)
    seeds = [rng.getrandbits(64 if alg in W64 else 32) for _ in lens]
    out = engine.checksum_list(ALG[alg], [d.data_ptr() + o for o in offs], lens, seeds=seeds_tensor(alg, seeds))
    torch.cuda.synchronize()
    h = host_bytes(d)
    want = [oracle.crc(alg, h[o: o + ln], s) for o, ln, s in zip(offs, lens, seeds)]
    assert results(engine, alg, out) == want


@pytest.mark.parametrize("alg", ["crc32", "crc32c", "crc64nvme"])
def test_list_masked_edges(engine, alg):
    """Round 5: the list streaming scans read a buffer of >= 16 bytes as the 8-byte words covering it
    and clear the bytes in front of it in the registers (the head state enters times x^(-8 o)); the
    tail (< 8 bytes past the last whole word) is folded.  Every start offset mod 8 against lengths at the threshold
    (15, 16, 17), around one and two words, around a 4 KiB group and a 512-byte row, neighbours
    packed with no gap (the masked bytes are the neighbours' data), one 1 MiB buffer so that the
    list takes the streaming scan; seeds on all."""
    import torch

    rng = random.Random(0x3A5C + ALG[alg])
    base_lens = [15, 16, 17, 23, 24, 25, 31, 511, 512, 513, 4095, 4096, 4097, 4103, 8191, 12289]
    lens, offs, pos = [], [], 3
    for L in base_lens:
        for o in range(8):
            pos += (o - pos) % 8  # start at offset o mod 8, right after the previous buffer
            offs.append(pos)
            lens.append(L)
            pos += L
    offs.append(pos + 5)
    lens.append(1 << 20)
    pos += 5 + (1 << 20)
    d = dev_random(pos + 64, 0x3A5C)
    seeds = [rng.getrandbits(64 if alg in W64 else 32) for _ in lens]
    out = engine.checksum_list(ALG[alg], [d.data_ptr() + o for o in offs], lens, seeds=seeds_tensor(alg, seeds))
    torch.cuda.synchronize()
    h = host_bytes(d)
    want = [oracle.crc(alg, h[o: o + ln], s) for o, ln, s in zip(offs, lens, seeds)]
    assert results(engine, alg, out) == want


@pytest.mark.parametrize("alg", ["crc32", "crc32c", "crc64nvme", "xxh64", "xxh3_64", "xxh3_128"])
def test_fuzz_lengths_alignments_seeds(engine, alg):
    """GPU-vs-oracle differential fuzzing: 2000 buffers of uniformly random length
    0..4200, every start alignment mod 16, random seeds, one ragged batch (fixed RNG seed)."""
    import torch

    rng = random.Random(0xF022 + ALG[alg])
    lens = [rng.randrange(0, 4201) for _ in range(2000)]
    offs, pos = [], 0
    for ln in lens:
        pos = (pos + 15) // 16 * 16 + rng.randrange(16)
        offs.append(pos)
        pos += ln
    d = dev_random(pos + 64, 11 + ALG[alg])
    seeds = [rng.getrandbits(64 if alg in W64 else 32) for _ in lens]
    out = engine.checksum_list(ALG[alg], [d.data_ptr() + o for o in offs], lens, seeds=seeds_tensor(alg, seeds))
    torch.cuda.synchronize()
    h = host_bytes(d)
    want = [oracle.checksum(alg, h[o: o + ln], s) for o, ln, s in zip(offs, lens, seeds)]
    assert results(engine, alg, out) == want


@pytest.mark.parametrize("alg", ["crc32c", "crc64nvme"])
def test_list_front_pads_at_group_boundaries(engine, alg):
    """Braided list scans start a buffer's first tile at the 4 KiB group holding its front pad's end
    (DESIGN.md §3.3).  A 64 MiB list of 16 KiB buffers sets 16 KiB tiles (four groups); buffers of
    T tiles minus pads of 4096 k + {0, 16, 4080} bytes (k < 4) put the pad's end on, just past and
    just before every group boundary, at aligned and unaligned starts, with seeds.  Starts 9..15
    bytes past 16-byte alignment put the head's last bytes next to a group boundary."""
    import torch

    rng = random.Random(0x9AD + ALG[alg])
    special = [16384 * T - (4096 * k + dl) for T in (1, 2, 3) for k in range(4) for dl in (0, 16, 4080)
               if 16384 * T - (4096 * k + dl) > 0]
    lens = [16384] * 4000 + special * 4
    rng.shuffle(lens)
    offs, pos = [], 0
    for ln in lens:
        pos = (pos + 15) // 16 * 16 + rng.choice([0, 0, 3, 9, 13, 15])
        offs.append(pos)
        pos += ln
    d = dev_random(pos + 64, 0x9AD)
    seeds = [rng.getrandbits(64 if alg in W64 else 32) for _ in lens]
    out = engine.checksum_list(ALG[alg], [d.data_ptr() + o for o in offs], lens, seeds=seeds_tensor(alg, seeds))
    torch.cuda.synchronize()
    h = host_bytes(d)
    want = [oracle.crc(alg, h[o: o + ln], s) for o, ln, s in zip(offs, lens, seeds)]
    assert results(engine, alg, out) == want


@pytest.mark.parametrize("shape", ["long_and_short", "empties_between", "odd_lengths", "one_buffer"])
@pytest.mark.parametrize("alg", ["crc32", "crc32c"])
def test_list_stream_shapes(engine, alg, shape):
    """Ragged CRC32 / CRC32C lists on the list streaming scan: buffers of more than 32
    tiles beside short ones (cross-tile combine through the group slots and the buffer word), empty
    and sub-16-byte buffers between long ones (tiles without a main region on the waves' range
    edges), lengths just past a tile at every alignment (front pads of nearly a whole tile), and one
    buffer alone; seeds on every buffer."""
    import torch

    rng = random.Random(0x5712 + ALG[alg] + len(shape))
    if shape == "long_and_short":
        lens = [rng.choice([40 << 20, (24 << 20) + 48]) for _ in range(3)] + [rng.randrange(4097, 70000) for _ in range(120)]
    elif shape == "empties_between":
        lens = [rng.choice([0, 1, 7, 15, 16, 17, 31, 65536, 65536 + 16, 131072 - 16]) for _ in range(3000)]
    elif shape == "odd_lengths":
        lens = [rng.choice([4097, 4096 * 3 + 1, 65537, 65536 + 4095, 131073]) + rng.randrange(0, 32) for _ in range(1500)]
    else:
        lens = [(96 << 20) + 4096 + 13]
    rng.shuffle(lens)
    offs, pos = [], 0
    for ln in lens:
        pos = (pos + 15) // 16 * 16 + rng.randrange(16)
        offs.append(pos)
        pos += ln
    d = dev_random(pos + 64, 0x5712 + len(lens))
    seeds = [rng.getrandbits(32) for _ in lens]
    out = engine.checksum_list(ALG[alg], [d.data_ptr() + o for o in offs], lens, seeds=seeds_tensor(alg, seeds))
    torch.cuda.synchronize()
    h = host_bytes(d)
    want = [oracle.crc(alg, h[o: o + ln], s) for o, ln, s in zip(offs, lens, seeds)]
    assert results(engine, alg, out) == want


@pytest.mark.parametrize("alg", ["crc32", "crc32c", "crc64nvme", "xxh64"])
def test_checksum_batches(engine, alg):
    """aws_crt_amd_checksum_batches: 37 batches of one shape (more than one launch holds), each with its
    own base, seeds (some none) and results; bases of mixed alignment mod 16 split the launches.
    Shapes: whole-tile buffers (streaming scans), ragged lengths (braided scans), C2's 64 KiB."""
    import torch

    rng = random.Random(0xBA7C + ALG[alg])
    for L, count in [(65536, 64), (8192, 200), (4096 * 3 + 20, 33), (100, 7)]:
        stride = (L + 15) // 16 * 16 + 16
        nb = 37
        d = dev_random(nb * (stride * count + 64), 41 + L % 13)
        offs = [j * (stride * count + 64) + (0 if j % 5 else rng.choice([0, 16, 3, 8])) for j in range(nb)]
        seeds = [[rng.getrandbits(64 if alg in W64 else 32) for _ in range(count)] if j % 3 else None for j in range(nb)]
        outs = [torch.full((count,), 7, dtype=torch.int64 if alg in W64 else torch.int32, device="cuda") for _ in range(nb)]
        batches = [(d.data_ptr() + o, seeds_tensor(alg, sd) if sd else None, out) for o, sd, out in zip(offs, seeds, outs)]
        engine.checksum_batches(ALG[alg], batches, stride, L, count)
        torch.cuda.synchronize()
        h = host_bytes(d)
        for j in range(nb):
            want = [oracle.checksum(alg, h[offs[j] + i * stride: offs[j] + i * stride + L], seeds[j][i] if seeds[j] else 0)
                    for i in range(count)]
            assert engine.as_unsigned(outs[j]) == want, (L, j)


@pytest.mark.parametrize("alg", ["crc32c", "crc64nvme", "xxh64"])
def test_plan_launch(engine, alg):
    """aws_crt_amd_plan_*: a prepared submission launched twice, on two streams, equals the oracle
    each time; shapes whose kernels need the per-stream cross-tile workspace (multi-tile buffers,
    CRC64NVME XCD-window chunks) take it from the launch's stream."""
    import torch

    rng = random.Random(0x91A + ALG[alg])
    for L, count, nb in [(65536, 64, 5), (1 << 20, 40, 3), (4 << 20, 3, 2), (4096 * 3 + 20, 33, 4)]:
        stride = (L + 15) // 16 * 16 + 16
        d = dev_random(nb * (stride * count + 64), 77 + L % 11)
        offs = [j * (stride * count + 64) + (3 if j == 1 else 0) for j in range(nb)]
        seeds = [[rng.getrandbits(64 if alg in W64 else 32) for _ in range(count)] if j % 2 else None for j in range(nb)]
        outs = [torch.full((count,), 7, dtype=torch.int64 if alg in W64 else torch.int32, device="cuda") for _ in range(nb)]
        batches = [(d.data_ptr() + o, seeds_tensor(alg, sd) if sd else None, out) for o, sd, out in zip(offs, seeds, outs)]
        plan = engine.BatchSet(ALG[alg], batches, stride, L, count)
        assert plan.launches >= 1
        h = host_bytes(d)
        want = [[oracle.checksum(alg, h[offs[j] + i * stride: offs[j] + i * stride + L], seeds[j][i] if seeds[j] else 0)
                 for i in range(count)] for j in range(nb)]
        for st in (torch.cuda.Stream(), torch.cuda.Stream()):
            for o in outs:
                o.fill_(7)
            torch.cuda.synchronize()
            plan.run(st)
            torch.cuda.synchronize()
            for j in range(nb):
                assert engine.as_unsigned(outs[j]) == want[j], (L, j)


@pytest.mark.parametrize("alg", ["xxh3_64", "xxh3_128"])
def test_xxh3_split_long_strided(engine, alg):
    """Strided XXH3 over buffers of >= 4096 full blocks takes the split path (block-sum pass, then
    the scramble pass over the sums): lengths at, around and past the threshold and not a multiple
    of the block, aligned and unaligned bases, per-buffer seeds and seed 0."""
    import torch

    rng = random.Random(0x5A1 + ALG[alg])
    for L, count, off in [(4096 * 1024 + 1, 3, 0), (4097 * 1024 + 777, 2, 5), (8 << 20, 2, 16),
                          (3 * (1 << 20) + 100, 2, 3), (9 * (1 << 20) + 63, 1, 1)]:
        stride = L + 16
        d = dev_random(off + stride * count + 64, 31 + L % 97)
        seeds = [rng.getrandbits(64) for _ in range(count)]
        out = engine.checksum_strided(ALG[alg], d, stride, L, count, seeds=seeds_tensor(alg, seeds), base_offset=off)
        out0 = engine.checksum_strided(ALG[alg], d, stride, L, count, base_offset=off)
        torch.cuda.synchronize()
        h = host_bytes(d)
        bufs = [h[off + k * stride: off + k * stride + L] for k in range(count)]
        assert results(engine, alg, out) == [oracle.checksum(alg, b, sd) for b, sd in zip(bufs, seeds)], (L, off)
        assert results(engine, alg, out0) == [oracle.checksum(alg, b) for b in bufs], (L, off)


@pytest.mark.parametrize("alg", ["crc32", "crc32c", "crc64nvme"])
def test_fuzz_short_lists_lane_path(engine, alg):
    """Lists whose buffers are all <= 4096 bytes take the lane-per-buffer scan (crc_lanes_kernel):
    3000 buffers of random length 0..4096 (plus 0..8 and exactly 4096) at every alignment mod 16,
    with random seeds and with no seeds (seed 0)."""
    import torch

    rng = random.Random(0x1A4E + ALG[alg])
    lens = [rng.randrange(0, 4097) for _ in range(2990)] + list(range(9)) + [4096]
    rng.shuffle(lens)
    offs, pos = [], 0
    for ln in lens:
        pos = (pos + 15) // 16 * 16 + rng.randrange(16)
        offs.append(pos)
        pos += ln
    d = dev_random(pos + 64, 23 + ALG[alg])
    ptrs = [d.data_ptr() + o for o in offs]
    seeds = [rng.getrandbits(64 if alg in W64 else 32) for _ in lens]
    out = engine.checksum_list(ALG[alg], ptrs, lens, seeds=seeds_tensor(alg, seeds))
    out0 = engine.checksum_list(ALG[alg], ptrs, lens)
    torch.cuda.synchronize()
    h = host_bytes(d)
    assert results(engine, alg, out) == [oracle.checksum(alg, h[o: o + ln], s) for o, ln, s in zip(offs, lens, seeds)]
    assert results(engine, alg, out0) == [oracle.checksum(alg, h[o: o + ln]) for o, ln in zip(offs, lens)]


@pytest.mark.parametrize("alg", ["crc32", "crc32c", "crc64nvme"])
def test_fuzz_strided_shapes(engine, alg):
    """Random uniform batches (count, length, base alignment, stride slack), half of them whole-tile
    shapes that take the streaming scans, with random seeds (fixed RNG seed)."""
    import torch

    rng = random.Random(0x5712 + ALG[alg])
    for _ in range(12):
        L = 4096 * rng.choice([1, 2, 3, 8, 16, 24]) if rng.random() < 0.5 else rng.randrange(1, 70000)
        count = rng.randrange(1, 1500)
        off = rng.choice([0, 0, rng.randrange(16)])
        stride = (L + 15) // 16 * 16 + 16 * rng.randrange(3) if count > 1 else L
        d = dev_random(stride * count + off + 16, rng.randrange(1 << 30))
        seeds = [rng.getrandbits(64 if alg in W64 else 32) for _ in range(count)]
        out = engine.checksum_strided(ALG[alg], d, stride, L, count, seeds=seeds_tensor(alg, seeds), base_offset=off)
        torch.cuda.synchronize()
        h = host_bytes(d)
        want = [oracle.crc(alg, h[off + i * stride: off + i * stride + L], seeds[i]) for i in range(count)]
        assert engine.as_unsigned(out) == want, (L, count, off, stride)


def test_config3_full_chunked_running_crc(engine):
    """BASELINE config 3 at full size: 16 x 256 MiB, CRC32 and CRC32C.  One-shot == chained running
    CRC over 8 MiB chunks (seeded on device) == Combine of the chunk CRCs, and the oracle on all 16."""
    import torch

    L, chunk, nbuf = 256 << 20, 8 << 20, 16
    d = dev_random(L * nbuf, 9)
    h = host_bytes(d)
    for alg in ("crc32", "crc32c"):
        one = engine.as_unsigned(engine.checksum_strided(ALG[alg], d, L, L, nbuf))
        prev = None
        parts = []
        for c in range(L // chunk):
            prev = engine.checksum_strided(ALG[alg], d, L, chunk, nbuf, seeds=prev, base_offset=c * chunk)
            parts.append(engine.checksum_strided(ALG[alg], d, L, chunk, nbuf, base_offset=c * chunk))
        torch.cuda.synchronize()
        assert engine.as_unsigned(prev) == one
        pv = [engine.as_unsigned(p) for p in parts]
        for b in range(nbuf):
            acc = pv[0][b]
            for p in pv[1:]:
                acc = engine.combine(alg, acc, p[b], chunk)
            assert acc == one[b]
        want = oracle.batch(alg, [h.ctypes.data + b * L for b in range(nbuf)], [L] * nbuf, 16)
        assert one == want, alg


def test_combine_batch_device(engine):
    import torch

    rng = random.Random(4)
    for alg in ("crc32", "crc32c", "crc64nvme"):
        bits = 64 if alg in W64 else 32
        n = 1000
        c1 = [rng.getrandbits(bits) for _ in range(n)]
        c2 = [rng.getrandbits(bits) for _ in range(n)]
        l2 = [rng.choice([0, 1, 7, 1 << 20, rng.getrandbits(40)]) for _ in range(n)]
        out = engine.combine_batch(ALG[alg], seeds_tensor(alg, c1), seeds_tensor(alg, c2), l2)
        torch.cuda.synchronize()
        assert engine.as_unsigned(out) == [oracle.combine(alg, a, b, l) for a, b, l in zip(c1, c2, l2)]


def test_host_path_chunked(engine):
    rng = random.Random(8)
    bufs = [rng.randbytes(n) for n in (0, 1, 5000, (16 << 20) + 77, (40 << 20) + 3)]
    for alg in ("crc32", "crc32c", "crc64nvme", "xxh64", "xxh3_64", "xxh3_128"):
        seeds = [rng.getrandbits(64 if alg in W64 else 32) for _ in bufs]
        got = engine.checksum_host(ALG[alg], bufs, seeds)
        assert got == [oracle.checksum(alg, b, s) for b, s in zip(bufs, seeds)]


def test_repeat_and_concurrent_streams(engine):
    """multi-tile buffers use per-stream self-cleaning workspaces: repeat + overlap must agree"""
    import torch

    L, n = (3 << 20) + 16, 12
    d = dev_random(L * n, 12)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs = []
    for i in range(6):
        st = s1 if i % 2 == 0 else s2
        outs.append(engine.checksum_strided(ALG["crc32c"], d, L, L, n, stream=st))
    torch.cuda.synchronize()
    h = host_bytes(d)
    want = [oracle.crc("crc32c", h[i * L:(i + 1) * L]) for i in range(n)]
    for o in outs:
        assert engine.as_unsigned(o) == want


def test_config4_full_shard(engine):
    """BASELINE config 4's per-GPU shard at full size: 1M x 8 KiB round-robin over 8 GPUs leaves
    131072 x 8 KiB (1 GiB) on each; the batch is checked buffer by buffer against the oracle (CRC32C),
    and a CRC64NVME pass (S3's default algorithm) on the same shard."""
    import torch

    total, L, G = 1 << 20, 8192, 8
    n = total // G
    d = dev_random(n * L, 13)
    out = engine.checksum_strided(ALG["crc32c"], d, L, L, n)
    out64 = engine.checksum_strided(ALG["crc64nvme"], d, L, L, n)
    torch.cuda.synchronize()
    h = host_bytes(d)
    ptrs = [h.ctypes.data + i * L for i in range(n)]
    assert engine.as_unsigned(out) == oracle.batch("crc32c", ptrs, [L] * n, 16)
    assert engine.as_unsigned(out64) == oracle.batch("crc64nvme", ptrs, [L] * n, 16)


def test_config5_crc64_xxh64_8x64mib(engine):
    """BASELINE config 5: a batch of 8 x 64 MiB buffers, CRC64NVME and XXH64 (and XXH3-64 on the
    split path), against the oracle on all 8."""
    import torch

    L, n = 64 << 20, 8
    d = dev_random(L * n, 14)
    crc = engine.as_unsigned(engine.checksum_strided(ALG["crc64nvme"], d, L, L, n))
    xx = engine.as_unsigned(engine.checksum_strided(ALG["xxh64"], d, L, L, n))
    x3 = engine.as_unsigned(engine.checksum_strided(ALG["xxh3_64"], d, L, L, n))
    torch.cuda.synchronize()
    h = host_bytes(d)
    ptrs = [h.ctypes.data + i * L for i in range(n)]
    assert crc == oracle.batch("crc64nvme", ptrs, [L] * n, 8)
    assert xx == oracle.batch("xxh64", ptrs, [L] * n, 8)
    assert x3 == [oracle.xxh3_64(h[i * L:(i + 1) * L]) for i in range(n)]


@pytest.mark.parametrize("alg,n,L", [
    ("crc32c", 24, (3 << 20) + 16),   # multi-tile buffers: the cross-tile combine inside the graph
    ("crc64nvme", 4, 8 << 20),        # crc64_xcd_kernel: parts joined by chunk count inside the graph
])
def test_graph_capture_replay(engine, alg, n, L):
    """A scan captured into a HIP graph (torch.cuda.graph) after one eager warm-up on the capture
    stream replays correctly on that stream, also after the input bytes change (the captured launch
    keeps the capture stream's self-cleaning workspace)."""
    import torch

    d = dev_random(n * L, 51)
    s = torch.cuda.Stream()
    out = torch.empty(n, dtype=torch.int64 if alg in W64 else torch.int32, device="cuda")
    with torch.cuda.stream(s):
        engine.checksum_strided(ALG[alg], d, L, L, n, out=out, stream=s)  # warm-up: tables, workspace
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        engine.checksum_strided(ALG[alg], d, L, L, n, out=out, stream=s)
    for it in range(3):
        if it:
            d.copy_(dev_random(n * L, 60 + it))
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            g.replay()
        torch.cuda.synchronize()
        h = host_bytes(d)
        assert engine.as_unsigned(out) == [oracle.crc(alg, h[i * L:(i + 1) * L]) for i in range(n)], it
