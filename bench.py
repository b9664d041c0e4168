#!/usr/bin/env python3
"""Headline benchmark: GiB/s of CRC32C over device-resident buffers (BASELINE.json `metric`),
on BASELINE.json configs[1]: batches of 1024 x 64 KiB independent buffers per GPU.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...   (one rank per GPU)

A step = one launch of the batched CRC32C scan over one 64 MiB batch already resident in HBM.
Each rank scans its own batches (buffers shard across GPUs with no collective: weak scaling).
Steps rotate over --batches distinct batches (default 8 = 512 MiB per GPU, twice the 256 MiB
Infinity Cache) so every launch streams from HBM, not from the on-die cache.

Timed region: the K launches are replayed from a captured HIP graph (one launch per batch, the
batches split over --branches independent graph branches so consecutive launches overlap their
ramp-up and tail); any K % batches remainder is launched eagerly.  Kernel duration for the
roofline: a separate pass queues --timing-launches eager launches bracketed by HIP events behind a
GPU-side hold (so host launch latency never sits between an event pair).

Prints one JSON line (rank 0).  `roofline.achieved` = algorithmic bytes per launch (1 byte read per
payload byte) / mean kernel duration from HIP events recorded on the launch stream.
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
ALG = {"crc32": 0, "crc32c": 1, "crc64nvme": 2, "xxh64": 3}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--alg", default="crc32c", choices=list(ALG))
    ap.add_argument("--buffers", type=int, default=1024)
    ap.add_argument("--buffer-bytes", type=int, default=65536)
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--branches", type=int, default=2)
    ap.add_argument("--mode", default="graph", choices=["graph", "eager"])
    ap.add_argument("--timing-launches", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
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
    wide = alg in ("crc64nvme", "xxh64")
    outs = [torch.empty(count, dtype=torch.int64 if wide else torch.int32, device=dev) for _ in range(nb)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(max(1, args.branches))]

    def launch(i, st=None):
        b = i % nb
        st = st or streams[i % len(streams)]
        eng.checksum_strided(ALG[alg], data, L, L, count, out=outs[b], stream=st, base_offset=b * step_bytes)

    torch.cuda.synchronize()
    for i in range(max(args.warmup, 2 * nb)):  # every (batch, stream) pair once: caches + workspaces
        launch(i)
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
        starts[i].record(st)
        launch(i, st)
        ends[i].record(st)
    torch.cuda.synchronize()
    durs = sorted(s_.elapsed_time(e_) for s_, e_ in zip(starts, ends))
    kernel_ms = sum(durs) / nt
    achieved_gbs = step_bytes / (kernel_ms * 1e-3) / 1e9

    traffic = None
    pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            rec = json.load(open(pmc))
            if rec.get("workload") == f"{alg}:{count}x{L}":
                traffic = rec.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
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
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (torch.randint bytes on device)",
            "config": {"workload": f"C2: {count} x {L // 1024} KiB independent buffers, {alg.upper()}, "
                                   f"device-resident, per GPU per step",
                       "buffers_per_step": count, "buffer_bytes": L, "rotating_batches": nb,
                       "resident_bytes_per_gpu": nb * step_bytes, "launch": args.mode,
                       "graph_branches": len(streams) if graph is not None else 1,
                       "parallelism": f"buffers sharded over {world} GPU(s), no collective"},
            "pct_hbm_peak": round(100.0 * value * 2**30 / 1e9 / world / HBM_PEAK_GBS, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved_gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel_ms": round(kernel_ms, 5), "kernel_ms_median": round(durs[nt // 2], 5),
                         "bytes_per_launch": step_bytes, "timing_launches": nt},
            "cpu_baseline": cpu,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
