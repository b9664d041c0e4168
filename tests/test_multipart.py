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
