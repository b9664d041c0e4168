"""The submission queue (include/aws_crt_amd/checksums_batch.h, aws_crt_amd_queue_*): batches of one
shape pushed one at a time are launched together -- at 32 queued batches, at flush and at destroy --
so a producer that gets one part batch at a time (aws-c-s3's part Write, source/s3/S3.cpp:1133-1149)
reaches the multi-batch launch rate without building batch arrays itself.

CPU: the queue's host logic with no device visible (pushes queue without launching, a flush then
reports AWS_CRT_AMD_ERR_NO_DEVICE and empties the queue, argument checks).  GPU: results of queued
batches against the oracle, the automatic launch at 32, CRC64NVME long buffers, hashes, seeds.
"""
import os
import random
import subprocess
import sys

import pytest

from oracle import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "aws-crt-cpp_amd", "lib", "libaws-crt-cpp-amd.so")
ALG = {"crc32": 0, "crc32c": 1, "crc64nvme": 2, "xxh64": 3, "xxh3_64": 4, "xxh3_128": 5}


def test_queue_host_logic_without_device():
    code = (
        "import ctypes\n"
        f"L=ctypes.CDLL({LIB!r})\n"
        "vp=ctypes.c_void_p; sz=ctypes.c_size_t\n"
        "L.aws_crt_amd_queue_create.argtypes=[ctypes.c_int,sz,sz,sz,vp,ctypes.POINTER(vp)]\n"
        "L.aws_crt_amd_queue_push.argtypes=[vp,vp,vp,vp]\n"
        "L.aws_crt_amd_queue_flush.argtypes=[vp]\n"
        "L.aws_crt_amd_queue_pending.argtypes=[vp]; L.aws_crt_amd_queue_pending.restype=sz\n"
        "L.aws_crt_amd_queue_destroy.argtypes=[vp]\n"
        "q=vp()\n"
        "print('bad_alg', L.aws_crt_amd_queue_create(9,65536,65536,4,None,ctypes.byref(q)))\n"
        "print('bad_stride', L.aws_crt_amd_queue_create(1,65540,65536,4,None,ctypes.byref(q)))\n"
        "print('create', L.aws_crt_amd_queue_create(1,65536,65536,4,None,ctypes.byref(q)))\n"
        "print('null_out', L.aws_crt_amd_queue_push(q,4096,None,None))\n"
        "for i in range(5): L.aws_crt_amd_queue_push(q,4096*(i+1),None,8192*(i+1))\n"
        "print('pending', L.aws_crt_amd_queue_pending(q))\n"
        "print('flush', L.aws_crt_amd_queue_flush(q))\n"
        "print('pending_after', L.aws_crt_amd_queue_pending(q))\n"
        "print('destroy_empty', L.aws_crt_amd_queue_destroy(q))\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, HIP_VISIBLE_DEVICES="-1"))
    assert r.returncode == 0, r.stderr
    got = dict(line.split() for line in r.stdout.split("\n") if line)
    assert got == {"bad_alg": "-2", "bad_stride": "-2", "create": "0", "null_out": "-2", "pending": "5",
                   "flush": "-1", "pending_after": "0", "destroy_empty": "0"}


def _dev_random(n, seed):
    import torch

    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)


@pytest.mark.gpu
def test_queue_crc32c_auto_launch_and_flush(engine):
    """40 batches of 32 x 64 KiB pushed one by one: the 32nd push launches the first 32 (nothing
    pending after it), flush launches the other 8; every result equals the oracle; seeds on some."""
    import torch

    n, L, nb = 32, 65536, 40
    d = _dev_random(n * L * nb, 0x9E)
    rng = random.Random(0x9E)
    seeds = {j: [rng.getrandbits(32) for _ in range(n)] for j in (3, 33)}
    outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(nb)]
    q = engine.Queue(ALG["crc32c"], L, L, n)
    for j in range(nb):
        st = torch.tensor([v - (1 << 32) if v >= 1 << 31 else v for v in seeds[j]], dtype=torch.int32,
                          device="cuda") if j in seeds else None
        q.push(d[j * n * L:], outs[j], seeds=st)
        assert q.pending() == (j + 1) % 32, j
    q.flush()
    assert q.pending() == 0
    q.close()
    torch.cuda.synchronize()
    h = d.cpu().numpy()
    for j in range(nb):
        got = engine.as_unsigned(outs[j])
        for i in range(0, n, 7):
            o = (j * n + i) * L
            want = oracle.crc("crc32c", h[o:o + L], seeds[j][i] if j in seeds else 0)
            assert got[i] == want, (j, i)


@pytest.mark.gpu
@pytest.mark.parametrize("alg,n,L", [("crc64nvme", 2, 8 << 20), ("xxh64", 4, 65536), ("xxh3_64", 4, 65536)])
def test_queue_close_flushes(engine, alg, n, L):
    """close() launches what is queued: CRC64NVME long buffers (crc64_xcd_kernel), hashes (one launch
    per batch)."""
    import torch

    nb = 3
    d = _dev_random(n * L * nb, 0x9F)
    outs = [torch.empty(n, dtype=torch.int64, device="cuda") for _ in range(nb)]
    q = engine.Queue(ALG[alg], L, L, n)
    for j in range(nb):
        q.push(d[j * n * L:], outs[j])
    assert q.pending() == nb
    q.close()
    torch.cuda.synchronize()
    h = d.cpu().numpy()
    for j in range(nb):
        got = engine.as_unsigned(outs[j])
        for i in range(n):
            o = (j * n + i) * L
            assert got[i] == oracle.checksum(alg, h[o:o + L]), (j, i)
