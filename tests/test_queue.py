"""The submission queue (include/aws_crt_amd/checksums_batch.h, aws_crt_amd_queue_*): batches of one
shape pushed one at a time are launched together, so a producer that gets one part batch at a time
(aws-c-s3's part Write, source/s3/S3.cpp:1133-1149) reaches the multi-batch launch rate without
building batch arrays itself.  Eager policy (default, round 6): a push that finds the queue's stream
free launches at once; pushes made while a launch runs coalesce into the next one.  Batched policy: at
32 queued batches, at flush and at destroy only.

CPU: the queue's host logic with no device visible (batched: pushes queue without launching, a flush
then reports AWS_CRT_AMD_ERR_NO_DEVICE and empties the queue; eager: every push launches -- refused --
at once; argument checks).  GPU: results of queued batches against the oracle, the automatic launch at
32, CRC64NVME long buffers, hashes, seeds, eager launches and their tickets.
"""
import os
import random
import subprocess
import sys

import pytest

from oracle import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
from tests.libpaths import ENGINE as LIB, LOAD_SRC, load_engine  # noqa: E402
ALG = {"crc32": 0, "crc32c": 1, "crc64nvme": 2, "xxh64": 3, "xxh3_64": 4, "xxh3_128": 5}


def test_queue_host_logic_without_device():
    """the batched policy without a device: pushes queue, the flush's launch is refused"""
    code = (
        LOAD_SRC +
        "vp=ctypes.c_void_p; sz=ctypes.c_size_t; u64=ctypes.c_uint64\n"
        "class O(ctypes.Structure): _fields_=[('max_batches',sz),('max_age_us',u64),('policy',ctypes.c_uint32),('max_inflight',ctypes.c_uint32),('min_launch',ctypes.c_uint32),('reserved',ctypes.c_uint32)]\n"
        "L.aws_crt_amd_queue_create_ex.argtypes=[ctypes.c_int,sz,sz,sz,vp,ctypes.POINTER(O),ctypes.POINTER(vp)]\n"
        "L.aws_crt_amd_queue_create=lambda a,st,l,c,s_,q: L.aws_crt_amd_queue_create_ex(a,st,l,c,s_,ctypes.byref(O(0,0,1,0,0,0)),q)\n"
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


def test_queue_eager_policy_without_device():
    """the eager policy without a device: nothing of the queue is running, so with min_launch 1 every
    push launches at once -- refused (AWS_CRT_AMD_ERR_NO_DEVICE), reported by the push and by its
    ticket -- and nothing stays pending; with the default minimum of two, every second push launches
    (destroy then flushes the last one, refused); unknown policies, depths and minimums are refused"""
    code = (
        LOAD_SRC +
        "vp=ctypes.c_void_p; sz=ctypes.c_size_t; u64=ctypes.c_uint64\n"
        "class O(ctypes.Structure): _fields_=[('max_batches',sz),('max_age_us',u64),('policy',ctypes.c_uint32),('max_inflight',ctypes.c_uint32),('min_launch',ctypes.c_uint32),('reserved',ctypes.c_uint32)]\n"
        "L.aws_crt_amd_queue_create.argtypes=[ctypes.c_int,sz,sz,sz,vp,ctypes.POINTER(vp)]\n"
        "L.aws_crt_amd_queue_create_ex.argtypes=[ctypes.c_int,sz,sz,sz,vp,ctypes.POINTER(O),ctypes.POINTER(vp)]\n"
        "L.aws_crt_amd_queue_push_ex.argtypes=[vp,vp,vp,vp,ctypes.POINTER(u64)]\n"
        "L.aws_crt_amd_queue_status.argtypes=[vp,u64]\n"
        "L.aws_crt_amd_queue_pending.argtypes=[vp]; L.aws_crt_amd_queue_pending.restype=sz\n"
        "L.aws_crt_amd_queue_launches.argtypes=[vp]; L.aws_crt_amd_queue_launches.restype=u64\n"
        "L.aws_crt_amd_queue_destroy.argtypes=[vp]\n"
        "q=vp(); t=u64()\n"
        "print('bad_policy', L.aws_crt_amd_queue_create_ex(1,65536,65536,4,None,ctypes.byref(O(0,0,2,0,0,0)),ctypes.byref(q)))\n"
        "print('bad_depth', L.aws_crt_amd_queue_create_ex(1,65536,65536,4,None,ctypes.byref(O(0,0,0,9,0,0)),ctypes.byref(q)))\n"
        "print('create', L.aws_crt_amd_queue_create_ex(1,65536,65536,4,None,ctypes.byref(O(0,0,0,0,1,0)),ctypes.byref(q)))\n"
        "r=[L.aws_crt_amd_queue_push_ex(q,4096*(i+1),None,8192*(i+1),ctypes.byref(t)) for i in range(5)]\n"
        "print('push_rcs', ','.join(map(str,r)), 'pending', L.aws_crt_amd_queue_pending(q), 'launches', L.aws_crt_amd_queue_launches(q))\n"
        "print('st', ','.join(str(L.aws_crt_amd_queue_status(q,k)) for k in range(1,6)))\n"
        "print('destroy', L.aws_crt_amd_queue_destroy(q))\n"
        "print('create_default', L.aws_crt_amd_queue_create(1,65536,65536,4,None,ctypes.byref(q)))\n"
        "r=[L.aws_crt_amd_queue_push_ex(q,4096*(i+1),None,8192*(i+1),ctypes.byref(t)) for i in range(5)]\n"
        "print('dpush_rcs', ','.join(map(str,r)), 'dpending', L.aws_crt_amd_queue_pending(q), 'dlaunches', L.aws_crt_amd_queue_launches(q))\n"
        "print('bad_min', L.aws_crt_amd_queue_create_ex(1,65536,65536,4,None,ctypes.byref(O(0,0,0,0,33,0)),ctypes.byref(vp())))\n"
        "print('bad_reserved', L.aws_crt_amd_queue_create_ex(1,65536,65536,4,None,ctypes.byref(O(0,0,0,0,0,1)),ctypes.byref(vp())))\n"
        "print('destroy2', L.aws_crt_amd_queue_destroy(q))\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, HIP_VISIBLE_DEVICES="-1"))
    assert r.returncode == 0, r.stderr
    got = {}
    for line in r.stdout.split("\n"):
        f = line.split()
        for i in range(0, len(f) - 1, 2):
            got[f[i]] = f[i + 1]
    assert got["bad_policy"] == "-2" and got["bad_depth"] == "-2" and got["create"] == "0"
    assert got["push_rcs"] == "-1,-1,-1,-1,-1" and got["pending"] == "0" and got["launches"] == "5"
    assert got["st"] == "-1,-1,-1,-1,-1" and got["destroy"] == "0"
    # the default minimum of two batches per eager launch: every second push launches
    assert got["create_default"] == "0" and got["dpush_rcs"] == "0,-1,0,-1,0"
    assert got["dpending"] == "1" and got["dlaunches"] == "2" and got["destroy2"] == "-1"
    assert got["bad_min"] == "-2" and got["bad_reserved"] == "-2"


def test_queue_tickets_refused_launch_and_age_flush_without_device():
    """Tickets and completion without a device: every batch of a refused launch reports the launch's
    error (AWS_CRT_AMD_ERR_NO_DEVICE) through its ticket, queued tickets report QUEUED, unknown
    tickets are refused; max_batches launches early; the age bound launches without a further push."""
    code = (
        LOAD_SRC + "import time\n"
        "vp=ctypes.c_void_p; sz=ctypes.c_size_t; u64=ctypes.c_uint64\n"
        "class O(ctypes.Structure): _fields_=[('max_batches',sz),('max_age_us',u64),('policy',ctypes.c_uint32),('max_inflight',ctypes.c_uint32),('min_launch',ctypes.c_uint32),('reserved',ctypes.c_uint32)]\n"
        "L.aws_crt_amd_queue_create_ex.argtypes=[ctypes.c_int,sz,sz,sz,vp,ctypes.POINTER(O),ctypes.POINTER(vp)]\n"
        "L.aws_crt_amd_queue_push_ex.argtypes=[vp,vp,vp,vp,ctypes.POINTER(u64)]\n"
        "L.aws_crt_amd_queue_status.argtypes=[vp,u64]; L.aws_crt_amd_queue_wait.argtypes=[vp,u64]\n"
        "L.aws_crt_amd_queue_pending.argtypes=[vp]; L.aws_crt_amd_queue_pending.restype=sz\n"
        "L.aws_crt_amd_queue_first_pending.argtypes=[vp]; L.aws_crt_amd_queue_first_pending.restype=u64\n"
        "L.aws_crt_amd_queue_destroy.argtypes=[vp]\n"
        "q=vp(); t=u64()\n"
        "print('too_many', L.aws_crt_amd_queue_create_ex(1,65536,65536,4,None,ctypes.byref(O(33,0,1,0,0,0)),ctypes.byref(q)))\n"
        "print('create', L.aws_crt_amd_queue_create_ex(1,65536,65536,4,None,ctypes.byref(O(3,0,1,0,0,0)),ctypes.byref(q)))\n"
        "r=[L.aws_crt_amd_queue_push_ex(q,4096*(i+1),None,8192*(i+1),ctypes.byref(t)) for i in range(4)]\n"
        "print('push_rcs', ','.join(map(str,r)), 'last_ticket', t.value)\n"
        "print('st', ','.join(str(L.aws_crt_amd_queue_status(q,k)) for k in range(1,5)))\n"
        "print('bad_ticket', L.aws_crt_amd_queue_status(q,0), L.aws_crt_amd_queue_status(q,9))\n"
        "print('first_pending', L.aws_crt_amd_queue_first_pending(q))\n"
        "print('wait4', L.aws_crt_amd_queue_wait(q,4), 'pending', L.aws_crt_amd_queue_pending(q))\n"
        "print('destroy', L.aws_crt_amd_queue_destroy(q))\n"
        "print('create_age', L.aws_crt_amd_queue_create_ex(1,65536,65536,4,None,ctypes.byref(O(0,2000,1,0,0,0)),ctypes.byref(q)))\n"
        "for i in range(3): L.aws_crt_amd_queue_push_ex(q,4096*(i+1),None,8192*(i+1),ctypes.byref(t))\n"
        "dl=time.time()+5\n"
        "while L.aws_crt_amd_queue_pending(q) and time.time()<dl: time.sleep(0.002)\n"
        "print('age_pending', L.aws_crt_amd_queue_pending(q), 'age_st', ','.join(str(L.aws_crt_amd_queue_status(q,k)) for k in range(1,4)))\n"
        "print('destroy_age', L.aws_crt_amd_queue_destroy(q))\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, HIP_VISIBLE_DEVICES="-1"))
    assert r.returncode == 0, r.stderr
    got = {}
    for line in r.stdout.split("\n"):
        f = line.split()
        for i in range(0, len(f) - 1, 2):
            got[f[i]] = f[i + 1]
    assert got["too_many"] == "-2" and got["create"] == "0"
    assert got["push_rcs"] == "0,0,-1,0" and got["last_ticket"] == "4"  # the 3rd push launched (max_batches 3): refused
    assert got["st"] == "-1,-1,-1,1"  # the refused launch's three tickets; ticket 4 still queued
    assert got["bad_ticket"] == "-2" and got["first_pending"] == "4"
    assert got["wait4"] == "-1" and got["pending"] == "0"  # wait launched it (refused) and reports that
    assert got["destroy"] == "0" and got["create_age"] == "0"
    assert got["age_pending"] == "0" and got["age_st"] == "-1,-1,-1"  # the flusher launched them, no push needed
    assert got["destroy_age"] == "0"


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
    q = engine.Queue(ALG["crc32c"], L, L, n, policy=engine.QUEUE_BATCHED)
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
    q = engine.Queue(ALG[alg], L, L, n, policy=engine.QUEUE_BATCHED)
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


@pytest.mark.gpu
def test_queue_tickets_age_bound_and_refused_flush(engine):
    """Per-push completion on the GPU: tickets complete (0) once their launch has run, with correct
    results; an age-bounded queue launches a lone push by itself; and a flush the engine refuses --
    queued on a stream under graph capture, whose batch needs a workspace the engine may not allocate
    during capture -- reports the error to every batch it dropped."""
    import time

    import torch

    n, L = 16, 65536
    d = _dev_random(n * L * 4, 0xA1)
    h = d.cpu().numpy()
    outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(4)]
    q = engine.Queue(ALG["crc32c"], L, L, n, max_batches=2, policy=engine.QUEUE_BATCHED)
    t = [q.push(d[j * n * L:], outs[j]) for j in range(3)]
    assert t == [1, 2, 3] and q.status(3) == engine.TICKET_QUEUED
    assert q.wait(1) == 0 and q.wait(3) == 0 and q.status(2) == 0
    for j in range(3):
        assert engine.as_unsigned(outs[j])[5] == oracle.crc("crc32c", h[(j * n + 5) * L:(j * n + 6) * L]), j
    q.close()
    # age bound: a single push is launched by the flusher
    qa = engine.Queue(ALG["crc32c"], L, L, n, max_age_us=500, policy=engine.QUEUE_BATCHED)
    ta = qa.push(d[3 * n * L:], outs[3])
    deadline = time.time() + 5
    while qa.pending() and time.time() < deadline:
        time.sleep(0.001)
    assert qa.pending() == 0 and qa.wait(ta) == 0
    assert engine.as_unsigned(outs[3])[0] == oracle.crc("crc32c", h[3 * n * L:(3 * n + 1) * L])
    qa.close()
    # refused flush: one 6 GiB buffer is 24,576 tiles, whose tile-shift columns the engine has never
    # built (nothing else scans a buffer that long); on a stream that is capturing the engine refuses
    # to build them (no allocation under capture), so the launch is refused.  The bytes are never read.
    big = torch.empty(6 << 30, dtype=torch.uint8, device="cuda")
    bo = [torch.empty(1, dtype=torch.int32, device="cuda") for _ in range(2)]
    cs = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    qr = None
    with torch.cuda.graph(g, stream=cs):
        qr = engine.Queue(ALG["crc32c"], 6 << 30, 6 << 30, 1, stream=cs, policy=engine.QUEUE_BATCHED)
        tr = [qr.push(big, bo[j]) for j in range(2)]
        with pytest.raises(engine.EngineError):
            qr.flush()
    assert [qr.status(x) for x in tr] == [-2, -2]  # AWS_CRT_AMD_ERR_INVALID_ARG, for both batches
    assert qr.wait(tr[1]) == -2
    qr.close()
    del big


@pytest.mark.gpu
@pytest.mark.parametrize("depth,min_launch", [(1, 1), (2, 1), (1, 0)])
def test_queue_eager_launches(engine, depth, min_launch):
    """the eager policy launches a push at once when nothing of the queue runs
    (the first push leaves nothing pending), coalesces the pushes made while launches run (fewer
    launches than pushes: a one-batch launch of 64 MiB takes ~15 us, a push a few), and every ticket
    completes with results equal to the oracle; the flush launches the rest."""
    import torch

    n, L, nb = 1024, 65536, 60  # C2 batches (64 MiB), 6 resident ones reused (the results are per push)
    d = _dev_random(n * L * 6, 0xE1)
    outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(nb)]
    q = engine.Queue(ALG["crc32c"], L, L, n, max_inflight=depth, min_launch=min_launch)
    first = 1 if min_launch == 1 else 2  # the default minimum is two batches
    tickets = []
    for j in range(nb):
        tickets.append(q.push(d[(j % 6) * n * L:], outs[j]))
        if j + 1 < first:
            assert q.pending() == j + 1 and q.launches() == 0
        elif j + 1 == first:
            assert q.pending() == 0 and q.launches() == 1
    q.flush()
    assert q.pending() == 0
    launches = q.launches()
    assert 2 <= launches < nb, launches
    assert all(q.wait(t) == 0 for t in tickets)
    assert all(q.status(t) == 0 for t in tickets)
    q.close()
    h = d.cpu().numpy()
    for j in range(0, nb, 7):
        got = engine.as_unsigned(outs[j])
        for i in (0, n // 2, n - 1):
            o = ((j % 6) * n + i) * L
            assert got[i] == oracle.crc("crc32c", h[o:o + L]), (j, i)


def test_queue_refused_tickets_never_report_complete():
    """beyond 1024 pruned refused launches the oldest records used to be dropped and their
    tickets then read 0 (complete, results written).  Adjacent refused launches now share a record, so
    3,000 refused one-batch launches all still report the refusal; a ticket whose record is gone would
    report AWS_CRT_AMD_ERR_TICKET_EXPIRED (-5), never 0."""
    code = (
        LOAD_SRC +
        "vp=ctypes.c_void_p; sz=ctypes.c_size_t; u64=ctypes.c_uint64\n"
        "class O(ctypes.Structure): _fields_=[('max_batches',sz),('max_age_us',u64),('policy',ctypes.c_uint32),('max_inflight',ctypes.c_uint32),('min_launch',ctypes.c_uint32),('reserved',ctypes.c_uint32)]\n"
        "L.aws_crt_amd_queue_create_ex.argtypes=[ctypes.c_int,sz,sz,sz,vp,ctypes.POINTER(O),ctypes.POINTER(vp)]\n"
        "L.aws_crt_amd_queue_push_ex.argtypes=[vp,vp,vp,vp,ctypes.POINTER(u64)]\n"
        "L.aws_crt_amd_queue_status.argtypes=[vp,u64]\n"
        "L.aws_crt_amd_queue_destroy.argtypes=[vp]\n"
        "q=vp(); t=u64()\n"
        "assert L.aws_crt_amd_queue_create_ex(1,65536,65536,4,None,ctypes.byref(O(1,0,1,0,0,0)),ctypes.byref(q))==0\n"
        "rc=[L.aws_crt_amd_queue_push_ex(q,4096,None,8192,ctypes.byref(t)) for i in range(3000)]\n"
        "st=[L.aws_crt_amd_queue_status(q,k) for k in range(1,3001)]\n"
        "print('pushes', set(rc), 'status', sorted(set(st)), 'last', t.value)\n"
        "print('destroy', L.aws_crt_amd_queue_destroy(q))\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, HIP_VISIBLE_DEVICES="-1"))
    assert r.returncode == 0, r.stderr
    assert "pushes {-1} status [-1] last 3000" in r.stdout, r.stdout
    assert "destroy 0" in r.stdout
