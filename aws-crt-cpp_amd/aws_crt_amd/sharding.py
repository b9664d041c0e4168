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


def slice_bounds(total: int, rank: int, world: int, align: int = 4096) -> range:
    """Contiguous byte slice [lo, hi) of one huge buffer owned by `rank` (slices in rank order,
    boundaries on `align`-byte multiples so every rank's slice starts aligned)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    units = (total + align - 1) // align
    lo = min(total, units * rank // world * align)
    hi = min(total, units * (rank + 1) // world * align)
    return range(lo, hi)


def split_buffer_crc(alg_name: str, total: int, compute_slice: Callable[[range], int], group=None) -> int:
    """SURVEY.md 8(e), single huge buffer: each rank computes the finalised CRC of its contiguous
    slice on its own GPU, the 8-byte (crc, length) pairs are all_gathered, and every rank folds them
    in order with Combine (CRC(A||B) = Combine(CRC(A), CRC(B), |B|), CRC.h:38-51) -- the engine's
    host-side GF(2) combine.  No payload bytes cross GPUs."""
    import torch
    import torch.distributed as dist

    from . import combine

    if not (dist.is_available() and dist.is_initialized()):
        return compute_slice(range(0, total))
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    sl = slice_bounds(total, rank, world)
    mine = compute_slice(sl)
    t = torch.tensor([mine - (1 << 64) if mine >= 1 << 63 else mine, len(sl)], dtype=torch.int64)
    bufs = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(bufs, t, group=group)
    crc = None
    for b in bufs:
        c, n = int(b[0]) & ((1 << 64) - 1), int(b[1])
        if n == 0:
            continue
        crc = c if crc is None else combine(alg_name, crc, c, n)
    return crc if crc is not None else compute_slice(range(0, 0))


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
