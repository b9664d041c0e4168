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


def gather_round_robin(local, n: int, group=None):
    """Every rank's results (rank r holds buffers r, r + world, ...: a 1-D tensor of result words) ->
    all n results in buffer order, on every rank.  One all_gather of the padded result vectors (4-8
    bytes per buffer, never payload), then a strided scatter.  `local` lives where the group's
    backend wants it (CPU for gloo, the rank's GPU for RCCL); the result is on the same device.
    With no process group initialised this is the single-GPU case."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return local[:n]
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if local.numel() != shard_count(n, rank, world):
        raise ValueError("local results do not match this rank's shard")
    width = shard_count(n, 0, world)  # rank 0's shard is the largest
    pad = torch.zeros(width, dtype=local.dtype, device=local.device)
    pad[: local.numel()] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    out = torch.empty(n, dtype=local.dtype, device=local.device)
    for r, b in enumerate(bufs):
        out[r::world] = b[: shard_count(n, r, world)]
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
    mine = [v - (1 << 64) if v >= 1 << 63 else v for v in compute_shard(shard_indices(n, rank, world))]
    got = gather_round_robin(torch.tensor(mine, dtype=torch.int64), n, group)
    return [int(x) & ((1 << 64) - 1) for x in got.tolist()]


class RoundRobinShard:
    """One rank's part of a uniform set of n device buffers of `length` bytes sharded round-robin over
    the ranks (BASELINE.json config 4: buffer i on GPU i mod N).  The rank's buffers lie back to back
    in its own GPU's memory (`data`, uint8, stride = length); `launch` scans them with one strided
    call on the rank's stream; `gather` brings every rank's result words together in buffer order.
    No payload byte leaves its GPU and the data path has no collective."""

    def __init__(self, eng, alg: int, data, n: int, length: int, rank: int = 0, world: int = 1):
        import torch

        self.eng, self.alg, self.data, self.n, self.length = eng, alg, data, n, length
        self.rank, self.world = rank, world
        self.count = shard_count(n, rank, world)
        if data.numel() < self.count * length:
            raise ValueError("shard data smaller than the rank's buffers")
        wide = alg in (eng.CRC64NVME, eng.XXH64, eng.XXH3_64)
        if alg == eng.XXH3_128:
            raise ValueError("one result word per buffer: XXH3-128 is not sharded this way")
        self.out = torch.empty(self.count, dtype=torch.int64 if wide else torch.int32, device=data.device)
        self.width = 8 if wide else 4

    def launch(self, stream=None):
        self.eng.checksum_strided(self.alg, self.data, self.length, self.length, self.count, out=self.out, stream=stream)

    def gather(self, group=None, device=None):
        """all n results in buffer order as int64 bit patterns (4-byte results zero-extended) on
        `device` (default: CPU, as gloo wants; RCCL groups pass the rank's GPU)"""
        import torch

        local = self.out.to(device or "cpu").to(torch.int64)
        if self.width == 4:
            local = torch.bitwise_and(local, 0xFFFFFFFF)
        return gather_round_robin(local, self.n, group)


def results_digest(eng, results, width: int) -> int:
    """The set's "checksum of checksums" (tests/golden/c4_digest.json): CRC64NVME, on the engine's host
    path, over the results in buffer order as little-endian words of `width` bytes."""
    import numpy as np

    arr = results.cpu().numpy().astype("<u8" if width == 8 else "<u4")
    return eng.crc("crc64nvme", arr.tobytes())
