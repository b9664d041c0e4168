"""CPU, world_size 2 over gloo: the round-robin sharding and result gather used for multi-GPU
batches (BASELINE.json config 4).  Each rank 'computes' its shard with the oracle standing in for
its GPU (test infrastructure); the gathered, re-ordered results must equal a single-rank run."""
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
    import torch.distributed as dist
    from oracle import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = random.Random(1234)  # same buffers on every rank
    bufs = [rng.randbytes(rng.choice([0, 5, 100, 8192])) for _ in range(101)]
    got = sharding.sharded_checksums(len(bufs), lambda idx: [oracle.crc("crc32c", bufs[i]) for i in idx])
    want = [oracle.crc("crc32c", b) for b in bufs]
    q.put((rank, got == want))
    dist.destroy_process_group()


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
