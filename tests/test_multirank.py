"""CPU, world_size 2 over gloo: the round-robin sharding and result gather used for multi-GPU
batches (BASELINE.json config 4).  Each rank computes its shard through the engine's own C ABI
(aws_crt_amd_host_submit / aws_checksums_*_ex: with no device visible the library serves host memory
on its host path, exactly as it would on a rank whose GPU failed); the gathered, re-ordered results
must equal the oracle's single-rank answer."""
import os
import random

import pytest
import torch.multiprocessing as mp

from aws_crt_amd import sharding


def test_shard_partition_is_exact():
    for n in (0, 1, 7, 8, 1000, 1 << 20):
        for world in (1, 2, 4, 8):
            seen = []
            for r in range(world):
                seen.extend(sharding.shard_indices(n, r, world))
            assert sorted(seen) == list(range(n))
            counts = [sharding.shard_count(n, r, world) for r in range(world)]
            assert max(counts) - min(counts) <= 1  # balanced


def _worker(rank, world, port, q):
    import ctypes

    import torch.distributed as dist

    import aws_crt_amd as eng
    from oracle import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = random.Random(1234)  # same buffers on every rank
    bufs = [rng.randbytes(rng.choice([0, 5, 100, 8192])) for _ in range(101)]
    keep = [ctypes.create_string_buffer(b, max(len(b), 1)) for b in bufs]

    def shard(idx):
        idx = list(idx)
        return eng.host_job(eng.CRC32C, [ctypes.addressof(keep[i]) for i in idx], [len(bufs[i]) for i in idx])

    got = sharding.sharded_checksums(len(bufs), shard)
    want = [oracle.crc("crc32c", b) for b in bufs]
    q.put((rank, got == want))
    dist.destroy_process_group()


def test_slice_bounds_partition_is_exact():
    for total in (0, 1, 4095, 4096, 4097, 10 ** 6, 1 << 30):
        for world in (1, 2, 3, 8):
            sl = [sharding.slice_bounds(total, r, world) for r in range(world)]
            assert sl[0].start == 0 and sl[-1].stop == total
            assert all(a.stop == b.start for a, b in zip(sl, sl[1:]))
            assert all(s.start % 4096 == 0 for s in sl if len(s))


def _split_worker(rank, world, port, q):
    import torch.distributed as dist

    import aws_crt_amd as eng
    from oracle import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = random.Random(99).randbytes(3 * 1000 * 1000 + 17)  # same buffer on every rank
    ok = []
    for alg in ("crc32", "crc32c", "crc64nvme"):
        got = sharding.split_buffer_crc(alg, len(data), lambda sl: eng.crc(alg, data[sl.start:sl.stop]))
        ok.append(got == oracle.crc(alg, data))
    q.put((rank, all(ok)))
    dist.destroy_process_group()


def test_gloo_world2_split_buffer_combine():
    """One huge buffer split into contiguous per-rank slices, slice CRCs (the engine's
    aws_checksums_*_ex) folded with the engine's host-side Combine."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30600 + random.Random().randrange(1000)
    procs = [ctx.Process(target=_split_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res


@pytest.mark.parametrize("world", [2])
def test_gloo_world2_gather_matches_single_rank(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + random.Random().randrange(1000)
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res
