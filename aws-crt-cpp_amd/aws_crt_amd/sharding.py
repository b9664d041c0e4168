"""Multi-GPU sharding of a checksum batch: buffer i is owned by rank i % world
(BASELINE.json config 4: 1M x 8 KiB parts round-robin over the GPUs of a node).  Buffers are
independent, so the data path has no collective; each rank scans its shard on its own GPU and
stream.  The only cross-rank traffic is the optional gather of 4-8 byte results back into the
caller's order (an all_gather of per-rank result vectors), never payload bytes.
"""
from __future__ import annotations

from typing import Callable, List, Sequence


def shard_indices(n: int, rank: int, world: int) -> range:
    """Indices of the buffers rank `rank` owns under round-robin assignment."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return range(rank, n, world)


def shard_count(n: int, rank: int, world: int) -> int:
    return len(shard_indices(n, rank, world))


def interleave(per_rank: Sequence[Sequence[int]], n: int) -> List[int]:
    """Inverse of the round-robin split: per-rank result lists -> results in buffer order."""
    world = len(per_rank)
    out = [0] * n
    for r, vals in enumerate(per_rank):
        for j, v in enumerate(vals):
            out[r + j * world] = v
    return out


def sharded_checksums(n: int, compute_shard: Callable[[range], Sequence[int]], group=None) -> List[int]:
    """Run `compute_shard(indices)` on this rank's shard, then gather every rank's results (a
    small all_gather of result words) and return them in buffer order.  With no process group
    initialised this is the single-GPU case."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return list(compute_shard(range(n)))
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    mine = list(compute_shard(shard_indices(n, rank, world)))
    width = max(shard_count(n, r, world) for r in range(world))
    t = torch.zeros(width, dtype=torch.int64)
    for j, v in enumerate(mine):
        t[j] = v - (1 << 64) if v >= 1 << 63 else v
    bufs = [torch.zeros(width, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(bufs, t, group=group)
    per_rank = [[int(x) & ((1 << 64) - 1) for x in b.tolist()[: shard_count(n, r, world)]] for r, b in enumerate(bufs)]
    return interleave(per_rank, n)
