"""Host ingest (aws_crt_amd_host_submit / aws_crt_amd_job_wait) and the
in-process multi-device fan-out (aws_crt_amd_checksum_list_devices / aws_crt_amd_checksum_devices),
against the oracle.

CPU suite: with no device visible a host job runs on the engine's host path (the API never needs a
GPU for host memory).  GPU suite: pinned (torch pin_memory / hipHostRegister'ed) and pageable
buffers, buffers longer than a 32 MiB pipeline slot (pieces folded with Combine), seeds, xxHash
routed to the host path, and device-resident lists over every visible device."""
import ctypes
import random

import numpy as np
import pytest

from oracle import oracle

ALG = {"crc32": 0, "crc32c": 1, "crc64nvme": 2, "xxh64": 3, "xxh3_64": 4, "xxh3_128": 5}
W64 = {"crc64nvme", "xxh64", "xxh3_64", "xxh3_128"}


def _bufs(rng, sizes):
    return [np.frombuffer(rng.randbytes(n), dtype=np.uint8) if n else np.zeros(0, dtype=np.uint8) for n in sizes]


def _addr(a):
    return a.ctypes.data if a.size else 0


def test_host_job_without_device_uses_host_path():
    import aws_crt_amd as eng

    if eng.device_count() > 0:
        pytest.skip("device present: covered by the gpu tests")
    rng = random.Random(21)
    # buffers past a piece (8 MiB) are cut, spread over the host threads and joined with Combine
    bufs = _bufs(rng, [0, 1, 100, 4096, 70000, 1 << 20, (8 << 20) + 5, (17 << 20) + 3, 8 << 20])
    for alg in ALG:
        seeds = [rng.getrandbits(64 if alg in W64 else 32) for _ in bufs]
        got = eng.host_job(ALG[alg], [_addr(b) for b in bufs], [b.size for b in bufs], seeds)
        assert got == [oracle.checksum(alg, b, s) for b, s in zip(bufs, seeds)], alg


@pytest.mark.gpu
@pytest.mark.parametrize("host_threads", [-1, 0])
@pytest.mark.parametrize("alg", list(ALG))
def test_host_job_pageable(engine, alg, host_threads):
    """hybrid (host threads beside the device lane, the default) and devices only"""
    rng = random.Random(0x1A + ALG[alg])
    sizes = [0, 1, 15, 4096, 65536, 65537, (32 << 20) - 3, (32 << 20) + 17, (70 << 20) + 5] + \
            [rng.randrange(1, 300000) for _ in range(200)]
    bufs = _bufs(rng, sizes)
    seeds = [rng.getrandbits(64 if alg in W64 else 32) for _ in bufs]
    got = engine.host_job(ALG[alg], [_addr(b) for b in bufs], [b.size for b in bufs], seeds, host_threads=host_threads)
    assert got == [oracle.checksum(alg, b, s) for b, s in zip(bufs, seeds)]


@pytest.mark.gpu
@pytest.mark.parametrize("alg", ["crc32c", "crc64nvme"])
def test_host_job_hybrid_split(engine, alg):
    """A hybrid job's pieces go to the host threads and the device lane (both take some), a
    devices-only job's all to the lane, a split with a fixed thread count beside the lane, and the
    default policy (host path alone on a CPU share of 12+ threads); buffers cut into 8 MiB pieces at
    odd offsets join with Combine."""
    import torch

    rng = random.Random(0x4B + ALG[alg])
    lens = [(8 << 20) + 5, 3, (24 << 20) - 7, 65536] * 6 + [rng.randrange(1, 1 << 20) for _ in range(64)]
    total = sum(lens)
    host = torch.randint(0, 256, (total + 64,), dtype=torch.uint8).pin_memory()
    a = host.numpy()
    offs, o = [], 1
    for n in lens:
        offs.append(o)
        o += n
    ptrs = [host.data_ptr() + o for o in offs]
    seeds = [rng.getrandbits(64 if alg in W64 else 32) for _ in lens]
    want = [oracle.checksum(alg, a[o:o + n], s) for o, n, s in zip(offs, lens, seeds)]
    import os
    share = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    # (ndevices, host_threads): hybrid asked for, devices only, a fixed thread count beside the lane,
    # and the default -- device lanes only for a CPU share under 12 threads (ingest.cpp)
    for nd, ht, check in ((1, -1, lambda d: 0 < d < total), (0, 0, lambda d: d == total), (0, 3, lambda d: 0 < d < total),
                          (0, -1, (lambda d: d == 0) if share >= 12 else (lambda d: 0 <= d <= total))):
        job = engine.HostJob(ALG[alg], ptrs, lens, seeds, ndevices=nd, host_threads=ht)
        job.run()  # the first job may find the lane still being set up (it claims once it is ready)
        assert job.results() == want, ht
        job.run()
        assert job.results() == want, ht
        assert check(job.device_bytes), (nd, ht, job.device_bytes, total)


@pytest.mark.gpu
@pytest.mark.parametrize("alg", ["crc32", "crc32c", "crc64nvme"])
def test_host_job_pinned_and_registered(engine, alg):
    """A pinned batch (one allocation, contiguous parts: one DMA per slot) and a registered pageable
    part pool (hipHostRegister through aws_crt_amd_register_host)."""
    import torch

    count, L = 2048, 65536
    host = torch.randint(0, 256, (count * L,), dtype=torch.uint8).pin_memory()
    a = host.numpy()
    ptrs = [host.data_ptr() + i * L for i in range(count)]
    got = engine.host_job(ALG[alg], ptrs, [L] * count)
    assert got == oracle.batch(alg, [a.ctypes.data + i * L for i in range(count)], [L] * count, 16)
    pool = np.frombuffer(random.Random(5).randbytes(48 << 20), dtype=np.uint8).copy()
    engine.register_host(pool.ctypes.data, pool.nbytes)
    try:
        parts = [(0, 8 << 20), (8 << 20, 40 << 20), (1, 1000), (3, (48 << 20) - 3)]
        got = engine.host_job(ALG[alg], [pool.ctypes.data + o for o, _ in parts], [n for _, n in parts])
        assert got == [oracle.crc(alg, pool[o:o + n]) for o, n in parts]
    finally:
        engine.unregister_host(pool.ctypes.data)


@pytest.mark.gpu
def test_list_devices_and_devices_batches(engine):
    """Buffers on every visible device in one call, results in caller order; per-device uniform
    batches all at once (one stream per device)."""
    import torch

    ndev = torch.cuda.device_count()
    rng = random.Random(99)
    datas = []
    ptrs, lens, want = [], [], []
    for dev in range(ndev):
        d = torch.randint(0, 256, (4 << 20,), dtype=torch.uint8, device=f"cuda:{dev}")
        h = d.cpu().numpy()
        datas.append((d, h))
    for i in range(600):
        dev = rng.randrange(ndev)
        d, h = datas[dev]
        o, n = rng.randrange(0, 1 << 20), rng.choice([0, 5, 4096, 65536, rng.randrange(1, 3 << 20)])
        ptrs.append(d.data_ptr() + o)
        lens.append(n)
        want.append(h[o:o + n])
    for alg in ("crc32c", "crc64nvme", "xxh64"):
        seeds = [rng.getrandbits(64 if alg in W64 else 32) for _ in ptrs]
        got = engine.checksum_list_devices(ALG[alg], ptrs, lens, seeds)
        assert got == [oracle.checksum(alg, w, s) for w, s in zip(want, seeds)], alg
    entries, outs = [], []
    for dev, (d, h) in enumerate(datas):
        out = torch.empty(64, dtype=torch.int32, device=f"cuda:{dev}")
        outs.append(out)
        entries.append((dev, d, 65536, 65536, 64, None, out, None))
    engine.checksum_devices(ALG["crc32c"], entries)
    for dev, (d, h) in enumerate(datas):
        assert engine.as_unsigned(outs[dev]) == [oracle.crc("crc32c", h[i * 65536:(i + 1) * 65536]) for i in range(64)]


_NUMA_SCRIPT = r"""
import json, random, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import aws_crt_amd as eng
rng = random.Random(7)
sizes = [3, 70000, (9 << 20) + 5, 1 << 20, (6 << 20) + 1] + [rng.randrange(1, 1 << 20) for _ in range(40)]
bufs = [np.frombuffer(rng.randbytes(n), dtype=np.uint8) for n in sizes]
ptrs, lens = [b.ctypes.data for b in bufs], [b.size for b in bufs]
out = {}
for alg in (0, 1, 2, 3):
    out[alg] = {"batch": eng.cpu_batch(alg, ptrs, lens, threads=4),
                "job": eng.host_job(alg, ptrs, lens, ndevices=-1, host_threads=4)}
np.save(sys.argv[2], np.concatenate(bufs))
print(json.dumps({"sizes": sizes, "out": out}))
"""


def test_numa_placed_host_path(tmp_path):
    """Host-path jobs placed on a NUMA node (AWS_CRT_AMD_NUMA=force places them on a one-node host:
    every index on pool workers moved onto the node's CPUs, the caller waiting) give the oracle's
    values, for the batch call and the host-ingest job; the job's trace names the node."""
    import json
    import os
    import subprocess
    import sys

    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "aws-crt-cpp_amd")
    env = dict(os.environ, AWS_CRT_AMD_NUMA="force", AWS_CRT_AMD_INGEST_TRACE="1", HIP_VISIBLE_DEVICES="")
    blob = tmp_path / "bytes.npy"
    r = subprocess.run([sys.executable, "-c", _NUMA_SCRIPT, pkg, str(blob)], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    data, off, bufs = np.load(blob), 0, []
    for n in rec["sizes"]:
        bufs.append(data[off:off + n])
        off += n
    names = {0: "crc32", 1: "crc32c", 2: "crc64nvme", 3: "xxh64"}
    for alg, got in rec["out"].items():
        want = [oracle.checksum(names[int(alg)], b, 0) for b in bufs]
        assert got["batch"] == want and got["job"] == want, names[int(alg)]
    # the CRC jobs' host threads (an xxHash job runs a thread per buffer outside the pool)
    traces = [json.loads(l) for l in r.stderr.splitlines() if l.startswith('{"ingest_trace"')]
    crc = [t for t in traces if t["host_threads"] > 0]
    assert len(crc) == 3 and all(t["numa_node"] == 0 for t in crc), traces


def test_runner_runs_concurrent_jobs_concurrently():
    """the coordinator threads (csrc/runner.h) give every queued job a thread of its own,
    so two jobs submitted together overlap (tests/cpp/runner_test.cpp under TSan)"""
    import os
    import subprocess

    cpp = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp")
    subprocess.run(["make", "-s", "-C", cpp, "build/runner_tsan"], check=True, capture_output=True, text=True)
    r = subprocess.run([os.path.join(cpp, "build", "runner_tsan")], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "[PASS] RunnerConcurrent" in r.stdout, r.stdout + r.stderr
