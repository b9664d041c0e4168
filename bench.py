#!/usr/bin/env python3
"""Headline benchmark: GiB/s of CRC32C over device-resident buffers (BASELINE.json `metric`),
on BASELINE.json configs[1]: batches of 1024 x 64 KiB independent buffers per GPU.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...   (one rank per GPU)

A step = one launch of the batched CRC32C scan over one 64 MiB batch already resident in HBM.
Each rank scans its own batches (buffers shard across GPUs with no collective: weak scaling).
Steps rotate over --batches distinct batches (default 8 = 512 MiB per GPU, twice the 256 MiB
Infinity Cache) so every launch streams from HBM, not from the on-die cache.

Timed region: K eager launches, alternating over --branches HIP streams so that a launch's
workgroups start on CUs as the previous launch's workgroups retire (its prologue overlaps the other
launch.s tail; 3 streams by default).  --mode graph replays a captured HIP graph instead (one
launch per batch, batches split over graph branches; measured slower on ROCm 7.2: every replay
starts with a ~20 us bubble).  Kernel duration for the roofline: a separate pass queues
--timing-launches eager launches on one stream behind a GPU-side hold; each launch stamps HIP
events with its own dispatch start / end (hipExtLaunchKernel through the engine's diagnostics
hook), the interval rocprofv3's kernel trace reports for the same dispatches.

End-to-end (PCIe-inclusive): the same batches start in pinned host memory; H2D copies
on a copy stream overlap the scans on a compute stream through a 3-slot device ring, results come
back D2H.  Reported as `e2e_pinned` next to `value`, never as `value`.

North-star shape (`target_shape`, rank 0 at N=1): BASELINE.json's target, CRC32C over batches of
16 x 64 MiB device-resident buffers (>= 80 % of HBM peak), measured the same two ways; reported
beside `value`, never as `value`.  The profiling passes run with --target-buffers 0.

Prints one JSON line (rank 0).  `roofline.achieved` = algorithmic bytes per launch (1 byte read per
payload byte) / mean kernel duration from HIP events recorded on the launch stream.
`roofline.read_ceiling` = the same two measurements for a read-only XOR-reduce kernel of the same
launch shape over the same batches (the achievable streaming read for this bytes-per-launch).
`cpu_baseline` = the oracle's SSE4.2 crc32q 3-way path (the technique class of aws-checksums)
timed on this host over a bounded sample, rank 0 at N=1 only.
"""
import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "aws-crt-cpp_amd"))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md chip table
ALG = {"crc32": 0, "crc32c": 1, "crc64nvme": 2, "xxh64": 3, "xxh3_64": 4, "xxh3_128": 5}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--alg", default="crc32c", choices=list(ALG))
    ap.add_argument("--buffers", type=int, default=1024)
    ap.add_argument("--buffer-bytes", type=int, default=65536)
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--branches", type=int, default=3)
    ap.add_argument("--mode", default="eager", choices=["graph", "eager"])
    ap.add_argument("--timing-launches", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-read-ceiling", action="store_true", help="skip the streaming-read ceiling kernel")
    ap.add_argument("--e2e-batches", type=int, default=64, help="batches through the pinned-host pipeline (0: skip)")
    ap.add_argument("--target-buffers", type=int, default=16,
                    help="north-star shape leg: batches of this many 64 MiB buffers (0: skip)")
    return ap.parse_args()


def cpu_baseline(alg, host_batch, count, L, gpu_results, seconds, threads):
    """Oracle (kind "port") on a bounded sample: one batch, repeated passes for ~`seconds`."""
    from oracle import oracle

    base = host_batch.ctypes.data
    ptrs = [base + i * L for i in range(count)]
    lens = [L] * count
    first = oracle.batch(alg, ptrs, lens, threads)
    parity = first == gpu_results
    passes, t0 = 0, time.perf_counter()
    while True:
        oracle.batch(alg, ptrs, lens, threads)
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    rate = passes * count * L / el / 2**30
    # single-thread rate on a smaller slice, for reference
    t1, n1 = time.perf_counter(), 0
    while time.perf_counter() - t1 < min(2.0, seconds / 5):
        oracle.batch(alg, ptrs[:64], lens[:64], 1)
        n1 += 1
    rate1 = n1 * 64 * L / (time.perf_counter() - t1) / 2**30
    return {"value": round(rate, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{passes} passes over one {count} x {L // 1024} KiB batch ({count * L >> 20} MiB) "
                      f"copied to host, {threads} threads, oracle SSE4.2 crc32q 3-way "
                      f"({'PCLMUL fold' if alg != 'crc32c' else 'crc32q'}) tier",
            "single_thread_gibs": round(rate1, 3), "parity_with_gpu": parity}


def e2e_pinned(eng, alg_id, dev_data, count, L, nb, iters, wide):
    """Pinned host -> device -> scan -> results to host, copies overlapped with scans (3-slot ring)."""
    import torch

    step = count * L
    host = torch.empty(nb * step, dtype=torch.uint8, pin_memory=True)
    host.copy_(dev_data[: nb * step])
    odt = torch.int64 if wide else torch.int32
    slots = [torch.empty(step, dtype=torch.uint8, device=dev_data.device) for _ in range(3)]
    per = 2 if alg_id == 5 else 1
    outs = [torch.empty(count * per, dtype=odt, device=dev_data.device) for _ in range(3)]
    hres = torch.empty((iters, count * per), dtype=odt, pin_memory=True)
    cs, ks = torch.cuda.Stream(device=dev_data.device), torch.cuda.Stream(device=dev_data.device)
    copied = [torch.cuda.Event() for _ in range(3)]
    freed = [torch.cuda.Event() for _ in range(3)]

    def run(n):
        for i in range(n):
            k, b = i % 3, i % nb
            with torch.cuda.stream(cs):
                if i >= 3:
                    cs.wait_event(freed[k])
                slots[k].copy_(host[b * step:(b + 1) * step], non_blocking=True)
                copied[k].record(cs)
            ks.wait_event(copied[k])
            eng.checksum_strided(alg_id, slots[k], L, L, count, out=outs[k], stream=ks)
            with torch.cuda.stream(ks):
                hres[i].copy_(outs[k], non_blocking=True)
            freed[k].record(ks)

    run(min(iters, 6))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(iters)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # H2D alone through the same pinned buffers (the PCIe ceiling of this pipeline)
    t1 = time.perf_counter()
    with torch.cuda.stream(cs):
        for i in range(iters):
            slots[i % 3].copy_(host[(i % nb) * step:((i % nb) + 1) * step], non_blocking=True)
    torch.cuda.synchronize()
    el_h2d = time.perf_counter() - t1
    return {"value": round(iters * step / el / 2**30, 2), "unit": "GiB/s", "h2d_only_gibs": round(iters * step / el_h2d / 2**30, 2),
            "sample": f"{iters} batches of {count} x {L // 1024} KiB from {nb * step >> 20} MiB pinned host memory, "
                      f"H2D on a copy stream overlapped with the scans, results D2H"}


def target_shape(eng, alg_id, dev, streams, nbuf, steps=20, nb=2, timing=6):
    """BASELINE.json north_star target shape, reported beside `value` (never as `value`): CRC32C over
    batches of `nbuf` device-resident 64 MiB buffers, pipelined over the same streams as the headline
    leg, plus the dispatch-stamped duration of `timing` serialized launches."""
    import torch

    L = 64 << 20
    step_bytes = nbuf * L
    g = torch.Generator(device=dev)
    g.manual_seed(0x7A26)
    data = torch.randint(0, 256, (nb * step_bytes,), dtype=torch.uint8, device=dev, generator=g)
    outs = [torch.empty(nbuf, dtype=torch.int32, device=dev) for _ in range(nb)]

    def launch(i, st):
        eng.checksum_strided(alg_id, data, L, L, nbuf, out=outs[i % nb], stream=st, base_offset=(i % nb) * step_bytes)

    for i in range(max(nb * len(streams), 3)):
        launch(i, streams[i % len(streams)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        launch(i, streams[i % len(streams)])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st = streams[0]
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(timing)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(timing)]
    with torch.cuda.stream(st):
        torch.cuda._sleep(int(40e6))
    for i in range(timing):
        starts[i].record(st)
        ends[i].record(st)
        eng.time_next_launch(starts[i], ends[i])
        launch(i, st)
    torch.cuda.synchronize()
    kms = sum(eng.event_ms(s_, e_) for s_, e_ in zip(starts, ends)) / timing
    gibs = steps * step_bytes / el / 2**30
    del data
    return {"workload": f"{nbuf} x 64 MiB buffers per step, CRC32C, device-resident, {nb} rotating batches",
            "value": round(gibs, 2), "unit": "GiB/s", "steps": steps,
            "pct_hbm_peak": round(100.0 * gibs * 2**30 / 1e9 / HBM_PEAK_GBS, 2),
            "kernel_ms": round(kms, 4), "roofline_frac": round(step_bytes / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "target_pct": 80.0}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import aws_crt_amd as eng

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    eng.init()

    alg, count, L = args.alg, args.buffers, args.buffer_bytes
    step_bytes = count * L
    nb = max(1, args.batches)
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED + rank)
    data = torch.randint(0, 256, (nb * step_bytes,), dtype=torch.uint8, device=dev, generator=g)
    wide = alg in ("crc64nvme", "xxh64", "xxh3_64", "xxh3_128")
    per = 2 if alg == "xxh3_128" else 1  # XXH3-128: {high, low} per buffer
    outs = [torch.empty(count * per, dtype=torch.int64 if wide else torch.int32, device=dev) for _ in range(nb)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(max(1, args.branches))]

    def launch(i, st=None):
        b = i % nb
        st = st or streams[i % len(streams)]
        eng.checksum_strided(ALG[alg], data, L, L, count, out=outs[b], stream=st, base_offset=b * step_bytes)

    torch.cuda.synchronize()
    # every batch once and, when there is a timed region, every stream (per-stream workspaces are
    # allocated on first use); with --steps 0 (profiling the timing pass) stream 0 only, so every
    # launch of the run is a serialized one
    for i in range(max(args.warmup, nb if args.steps == 0 else nb * len(streams))):
        launch(i, streams[0] if args.steps == 0 else None)
    torch.cuda.synchronize()

    graph = None
    if args.mode == "graph":
        graph = torch.cuda.CUDAGraph()
        cap = streams[0]
        with torch.cuda.graph(graph, stream=cap):
            for st in streams[1:]:
                st.wait_stream(cap)
            for i in range(nb):
                launch(i, streams[i % len(streams)])
            for st in streams[1:]:
                cap.wait_stream(st)
        for _ in range(2):
            graph.replay()
        torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if graph is not None:
        for _ in range(args.steps // nb):
            graph.replay()
        for i in range(args.steps % nb):
            launch(i)
    else:
        for i in range(args.steps):
            launch(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = world * args.steps * step_bytes / elapsed / 2**30

    # kernel duration: eager launches on one stream, each between two HIP events, queued while
    # the stream is held by a GPU sleep so the events bracket back-to-back kernels
    st = streams[0]
    nt = max(1, args.timing_launches)
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(nt)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(nt)]
    with torch.cuda.stream(st):
        torch.cuda._sleep(int(40e6))
    for i in range(nt):
        starts[i].record(st)  # creates the events; the launch below re-stamps them
        ends[i].record(st)
        eng.time_next_launch(starts[i], ends[i])  # hipExtLaunchKernel: the dispatch's own timestamps
        launch(i, st)
    torch.cuda.synchronize()
    durs = sorted(eng.event_ms(s_, e_) for s_, e_ in zip(starts, ends))
    kernel_ms = sum(durs) / nt
    achieved_gbs = step_bytes / (kernel_ms * 1e-3) / 1e9

    # secondary denominator: the streaming-read ceiling of this launch shape -- the
    # same batches read by an XOR-reduce kernel with the W=32 scan's geometry, timed the same two ways
    ceiling = None
    if not args.no_read_ceiling:
        with torch.cuda.stream(st):
            torch.cuda._sleep(int(40e6))
        for i in range(nt):
            starts[i].record(st)
            ends[i].record(st)
            eng.time_next_launch(starts[i], ends[i])
            eng.read_ceiling(data, step_bytes, stream=st, base_offset=(i % nb) * step_bytes)
        torch.cuda.synchronize()
        rc_ms = sum(eng.event_ms(s_, e_) for s_, e_ in zip(starts, ends)) / nt
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(args.steps):
            eng.read_ceiling(data, step_bytes, stream=streams[i % len(streams)], base_offset=(i % nb) * step_bytes)
        torch.cuda.synchronize()
        rc_el = time.perf_counter() - t1
        rc_gbs = step_bytes / (rc_ms * 1e-3) / 1e9
        ceiling = {"kernel_ms": round(rc_ms, 5), "achieved": round(rc_gbs, 1), "unit": "GB/s",
                   "pipelined_gibs": round(args.steps * step_bytes / max(rc_el, 1e-9) / 2**30, 2),
                   "scan_frac_of_ceiling": round(achieved_gbs / rc_gbs, 4),
                   "kernel": "read_ceiling_kernel: same launch shape, 256-B non-temporal rows XOR-reduced"}

    traffic = None
    pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            rec = json.load(open(pmc))
            if rec.get("workload") == f"{alg}:{count}x{L}":
                traffic = rec.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    e2e = None
    if rank == 0 and world == 1 and args.e2e_batches > 0:
        e2e = e2e_pinned(eng, ALG[alg], data, count, L, nb, args.e2e_batches, wide)

    target = None
    if rank == 0 and world == 1 and alg == "crc32c" and args.target_buffers > 0:
        target = target_shape(eng, ALG[alg], dev, streams, args.target_buffers)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and alg in ("crc32", "crc32c", "crc64nvme", "xxh64"):
        host = data[:step_bytes].cpu().numpy()
        torch.cuda.synchronize()
        gpu0 = eng.as_unsigned(outs[0])
        threads = min(args.cpu_threads, os.cpu_count() or 1)
        cpu = cpu_baseline(alg, host, count, L, gpu0, args.cpu_seconds, threads)

    if rank == 0:
        rec = {
            "metric": "GiB/s CRC32C over device-resident buffers; % of HBM read peak" if alg == "crc32c"
            else f"GiB/s {alg.upper()} over device-resident buffers; % of HBM read peak",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / max(args.steps, 1) * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (torch.randint bytes on device)",
            "config": {"workload": f"C2: {count} x {L // 1024} KiB independent buffers, {alg.upper()}, "
                                   f"device-resident, per GPU per step",
                       "buffers_per_step": count, "buffer_bytes": L, "rotating_batches": nb,
                       "resident_bytes_per_gpu": nb * step_bytes, "launch": args.mode,
                       "streams": len(streams),
                       "parallelism": f"buffers sharded over {world} GPU(s), no collective"},
            "pct_hbm_peak": round(100.0 * value * 2**30 / 1e9 / world / HBM_PEAK_GBS, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved_gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel_ms": round(kernel_ms, 5), "kernel_ms_median": round(durs[nt // 2], 5),
                         "bytes_per_launch": step_bytes, "timing_launches": nt, "read_ceiling": ceiling},
            "cpu_baseline": cpu,
            "e2e_pinned": e2e,
            "target_shape": target,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
