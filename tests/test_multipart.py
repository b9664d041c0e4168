"""GPU: S3 multipart checksum composition through the C ABI
aws_crt_amd_multipart_crc -- part checksums from one batched scan, Combine-folded into the
full-object checksum, and its base64 wire form.  Checked against the oracle on the concatenated
object (parity of the full-object value is the CRC of the concatenation by definition) and against
Python's base64 of the big-endian bytes."""
import base64
import random

import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

ALGS = {"crc32": 0, "crc32c": 1, "crc64nvme": 2}


def _parts(sizes, seed, misalign=0):
    import torch

    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    total = sum(sizes) + 16 * len(sizes) + misalign
    blob = torch.randint(0, 256, (max(total, 1),), dtype=torch.uint8, device="cuda", generator=g)
    parts, off = [], misalign
    for n in sizes:
        parts.append((blob.data_ptr() + off, n))
        off += n + 7  # gaps: parts need not be contiguous or aligned
    return blob, parts


@pytest.mark.parametrize("alg", list(ALGS))
@pytest.mark.parametrize("case", ["s3_like", "ragged", "single", "with_empty"])
def test_multipart_full_object(engine, alg, case):
    rnd = random.Random(hash((alg, case)) & 0xFFFF)
    if case == "s3_like":  # 5 MiB parts and a short last part, as an S3 upload splits an object
        sizes = [5 << 20] * 3 + [1234567]
    elif case == "ragged":
        sizes = [rnd.randrange(0, 300000) for _ in range(37)]
    elif case == "single":
        sizes = [65536]
    else:
        sizes = [0, 17, 0, 4096, 0]
    blob, parts = _parts(sizes, seed=len(sizes) * 31 + ALGS[alg], misalign=rnd.randrange(16))
    part_vals, obj, b64 = engine.multipart_crc(ALGS[alg], parts)
    host = blob.cpu().numpy()
    base = blob.data_ptr()
    obj_bytes = bytearray()
    for (addr, n), v in zip(parts, part_vals):
        chunk = host[addr - base: addr - base + n].tobytes()
        assert v == oracle.crc(alg, chunk), (alg, case, n)
        obj_bytes += chunk
    assert obj == oracle.crc(alg, bytes(obj_bytes))
    width = 8 if alg == "crc64nvme" else 4
    assert b64 == base64.b64encode(obj.to_bytes(width, "big")).decode()


def test_multipart_no_parts(engine):
    vals, obj, b64 = engine.multipart_crc(ALGS["crc32c"], [])
    assert vals == [] and obj == 0 and b64 == "AAAAAA=="


def test_multipart_rejects_hashes(engine):
    with pytest.raises(Exception):
        engine.multipart_crc(3, [])


ALL = {"crc32": 0, "crc32c": 1, "crc64nvme": 2, "xxh64": 3, "xxh3_64": 4, "xxh3_128": 5}
WIDTH = {"crc32": 4, "crc32c": 4, "crc64nvme": 8, "xxh64": 8, "xxh3_64": 8, "xxh3_128": 16}


@pytest.mark.parametrize("alg", list(ALL))
@pytest.mark.parametrize("case", ["s3_like", "ragged", "with_empty"])
def test_multipart_composite(engine, alg, case):
    """VERDICT r04 missing #2: the S3 hash algorithms (S3.h:78-80) compose as COMPOSITE -- the same
    algorithm over the concatenated big-endian part digests, wire form base64 + "-N" (parity unpinned:
    checked against the oracle's digests of the parts and of their concatenation)"""
    rnd = random.Random(hash(("c", alg, case)) & 0xFFFF)
    sizes = {"s3_like": [5 << 20] * 2 + [777777], "ragged": [rnd.randrange(1, 200000) for _ in range(23)],
             "with_empty": [0, 33, 0, 70000]}[case]
    blob, parts = _parts(sizes, seed=len(sizes) * 17 + ALL[alg], misalign=rnd.randrange(16))
    vals, obj, wire = engine.multipart_checksum(ALL[alg], parts)
    host = blob.cpu().numpy()
    base = blob.data_ptr()
    cat = bytearray()
    for (addr, n), v in zip(parts, vals):
        want = oracle.checksum(alg, host[addr - base: addr - base + n].tobytes())
        assert v == want, (alg, case, n)
        cat += v.to_bytes(WIDTH[alg], "big")
    want_obj = oracle.checksum(alg, bytes(cat))
    assert obj == want_obj
    assert wire == base64.b64encode(want_obj.to_bytes(WIDTH[alg], "big")).decode() + f"-{len(sizes)}"


@pytest.mark.parametrize("alg", ["crc32", "crc32c", "crc64nvme"])
def test_multipart_checksum_full_object_matches_multipart_crc(engine, alg):
    blob, parts = _parts([100000, 3, 65536], seed=5)
    assert engine.multipart_checksum(ALL[alg], parts, engine.MULTIPART_FULL_OBJECT) == engine.multipart_crc(ALL[alg], parts)


def test_multipart_full_object_rejects_hashes(engine):
    with pytest.raises(Exception):
        engine.multipart_checksum(ALL["xxh64"], [], engine.MULTIPART_FULL_OBJECT)
