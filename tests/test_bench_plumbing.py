"""bench.py's rank plumbing (CPU, no GPU call): `--gpus N` without a launcher spawns N rank
processes; under torch.distributed.run `--gpus` must equal WORLD_SIZE; RCCL ranks each need their own
device, gloo ranks may share (the one-GPU rehearsal).  --plumbing-check DEVICES makes every rank print
its layout and exit before touching the GPU (BASELINE.json north_star: 1, 2, 4 and 8 GPUs)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
sys.path.insert(0, ROOT)


def _run(args, env=None, launcher=None):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env or {})
    cmd = (launcher or [sys.executable]) + [BENCH] + args
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=180, env=e)
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, sorted(lines, key=lambda d: d["rank"]), r.stderr


@pytest.mark.parametrize("n", [2, 4, 8])
def test_gpus_n_spawns_n_ranks(n):
    rc, lines, err = _run(["--gpus", str(n), "--plumbing-check", "8"])
    assert rc == 0, err[-2000:]
    assert [d["rank"] for d in lines] == list(range(n))
    assert all(d["world"] == n for d in lines)
    assert [d["device_index"] for d in lines] == list(range(n))  # one GPU per rank
    assert not any(d["shared"] for d in lines)
    assert len({d["master"] for d in lines}) == 1 and lines[0]["master"].startswith("127.0.0.1:")


def test_gpus_1_is_one_process():
    rc, lines, err = _run(["--plumbing-check", "8"])
    assert rc == 0, err[-2000:]
    assert len(lines) == 1 and lines[0]["world"] == 1 and lines[0]["device_index"] == 0


def test_rccl_refuses_ranks_without_a_gpu():
    rc, lines, err = _run(["--gpus", "2", "--plumbing-check", "1"])
    assert rc == 2 and "no GPU of its own" in err


def test_gloo_rehearsal_shares_the_device():
    rc, lines, err = _run(["--gpus", "2", "--plumbing-check", "1", "--dist-backend", "gloo"])
    assert rc == 0, err[-2000:]
    assert [d["device_index"] for d in lines] == [0, 0] and all(d["shared"] for d in lines)


def test_gpus_must_match_the_launchers_world():
    rc, _, err = _run(["--gpus", "3", "--plumbing-check", "8"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert rc == 2 and "WORLD_SIZE=2" in err


def test_under_torchrun():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    launcher = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(port)]
    rc, lines, err = _run(["--gpus", "2", "--plumbing-check", "8"], launcher=launcher)
    assert rc == 0, err[-2000:]
    assert [(d["rank"], d["world"], d["device_index"]) for d in lines] == [(0, 2, 0), (1, 2, 1)]


def test_rank_layout_and_device_count():
    import bench

    a = bench.parse(["--gpus", "4"])
    assert bench.rank_layout(a, {"WORLD_SIZE": "4", "RANK": "3", "LOCAL_RANK": "3"}, 8) == (4, 3, 3, 3, False)
    with pytest.raises(SystemExit):
        bench.rank_layout(a, {"WORLD_SIZE": "2", "RANK": "0"}, 8)
    assert bench.distinct_devices([{"uuid": "a"}, {"uuid": "a"}]) == 1
    assert bench.distinct_devices([{"uuid": None, "pci_bus_id": 3}, {"uuid": None, "pci_bus_id": 4}]) == 2


def test_split_is_weak_scaling_per_rank():
    """every rank / device runs the full --steps (weak scaling): the launch split of K steps"""
    import bench

    assert bench.split(20, 32) == [0, 20]
    assert bench.split(20, 1) == list(range(21))
    assert bench.widest(200, 32) == 29


class _HostEngine:
    """The engine with checksum_strided served by its own host path on CPU tensors: bench.py's C4 leg
    driven without a GPU (the record's plumbing, not a measurement)"""

    def __init__(self):
        import aws_crt_amd

        self._e = aws_crt_amd

    def __getattr__(self, k):
        return getattr(self._e, k)

    def checksum_strided(self, alg, base, stride, length, count, seeds=None, out=None, stream=None):
        import torch

        vals = self._e.cpu_batch(alg, [base.data_ptr() + i * stride for i in range(count)], [length] * count, threads=4)
        bits = 64 if out.dtype == torch.int64 else 32
        out.copy_(torch.tensor([v - (1 << bits) if v >> (bits - 1) else v for v in vals], dtype=out.dtype))
        return out


def _c4_golden(n, L):
    from aws_crt_amd import synth
    from oracle import oracle

    buf = synth.buffers_np(0, n, L)
    g = {}
    for alg, w in (("crc32c", "<u4"), ("crc64nvme", "<u8")):
        res = oracle.batch(alg, [buf.ctypes.data + i * L for i in range(n)], [L] * n, 4)
        import numpy as np

        g[alg] = {"digest": hex(oracle.crc("crc64nvme", np.asarray(res, dtype=np.uint64).astype(w).tobytes()))}
    return g


def _c4_args():
    import argparse

    return argparse.Namespace(c4_passes=1, timing_launches=8, no_cpu_baseline=False, cpu_seconds=0.05,
                              c4_preload_ms=5.0, c4_window_ms=0.0)


def _fake_timer(eng, launch, st, nt):
    launch(0, st)
    return 0.5, 0.5


def _check_c4_records(recs, world, n):
    assert set(recs) == {"C4_crc32c", "C4_crc64nvme"}
    for r in recs.values():
        assert r["digest_match"] is True and r["parity"] is True, r
        assert r["scaling"] == "strong" and r["n_gpus"] == world and r["value"] > 0
        assert [x["rank"] for x in r["ranks"]] == list(range(world))
        assert sum(x["buffers"] for x in r["ranks"]) == n
        assert r["cpu_baseline"] is not None and r["cpu_baseline"]["value"] > 0
        assert r["cpu_baseline"]["parity_with_gpu"] is True
        assert r["roofline"]["bound"] == "hbm" and 0 < r["roofline"]["frac"]


def test_c4_leg_record_world1_cpu():
    """bench.py's C4 leg (the fixed set, buffer i on rank i mod N) assembles its
    record -- digest of the gathered results against the golden rule, per-rank records, cpu_baseline --
    here on a 2,048-buffer set with the host path standing in for the kernels"""
    import torch

    import bench

    n, L = 2048, 8192
    recs = bench.c4_leg(_HostEngine(), _c4_args(), torch.device("cpu"), 0, 1, [None], lambda x: x, lambda: None, None,
                        n=n, L=L, golden=_c4_golden(n, L), timer=_fake_timer)
    _check_c4_records(recs, 1, n)


def _c4_rank(rank, world, port, q, golden):
    import torch
    import torch.distributed as dist

    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def mx(x):
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    try:
        recs = bench.c4_leg(_HostEngine(), _c4_args(), torch.device("cpu"), rank, world, [None], mx, dist.barrier, None,
                            n=2047, L=8192, golden=golden, timer=_fake_timer)
        q.put((rank, recs))
    except Exception as e:
        q.put((rank, repr(e)))
    dist.destroy_process_group()


def test_c4_leg_record_two_gloo_ranks_cpu():
    """the same leg at world 2 over gloo: each rank builds and scans its own shard (odd set size:
    unequal shards), rank 0 gathers every result and carries both ranks' records"""
    import random

    import torch.multiprocessing as mp

    n, L = 2047, 8192
    golden = _c4_golden(n, L)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 32800 + random.Random().randrange(1000)
    procs = [ctx.Process(target=_c4_rank, args=(r, 2, port, q, golden)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=240) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert res[1] is None, res[1]
    assert isinstance(res[0], dict), res[0]
    _check_c4_records(res[0], 2, n)
