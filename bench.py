#!/usr/bin/env python3
"""Headline benchmark: GiB/s of CRC32C over device-resident buffers (BASELINE.json `metric`), on
BASELINE.json configs[1] (C2): batches of 1024 x 64 KiB independent buffers per GPU.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...   (one rank per GPU)

A step = one C2 batch (1024 x 64 KiB, its own base and its own 1024 results) checksummed on the GPU,
inputs already resident in HBM.  Each rank scans its own batches (buffers shard across GPUs with no
collective: weak scaling).  Steps rotate over --batches distinct batches (8 = 512 MiB per GPU, twice
the 256 MiB Infinity Cache) so every launch streams from HBM.

Launches: steps are submitted through aws_crt_amd_checksum_batches, which puts up to --coalesce
queued batches (same shape, separate bases / results) into ONE launch, so back-to-back batches do
not each pay a launch's ramp and tail (DESIGN.md §3 "multi-batch launches"); the K steps are split
into ceil(K / coalesce) near-equal launches, alternating over --branches HIP streams.  --coalesce 1 is
one launch per batch.  The resident pool holds at least as many distinct batches as one launch
(32 x 64 MiB = 2 GiB at the default), so no launch reads any byte twice.

Roofline (`roofline`): the dominant kernel's algorithmic bytes per launch (1 byte read per payload
byte) / its mean dispatch duration, from HIP events stamped by the dispatch itself
(hipExtLaunchKernel via the engine's measurement hook) over --timing-launches launches serialised on
one stream -- the interval rocprofv3's kernel trace reports.  `single_batch` gives the same figures
for one-batch launches.  `traffic` is HBM bytes per launch from the committed rocprofv3 --pmc pass
named in `traffic_source` (not measured in this run).

C4 (`configs.C4_crc32c`, `configs.C4_crc64nvme`; every N, every rank): the fixed set of 1,048,576 x
8 KiB buffers, buffer i on rank i mod N (strong scaling), each rank's shard built on its own GPU; per-rank
kernel fraction and parity sample, the gathered results' digest checked on rank 0, cpu_baseline on rank
0's shard.  Config legs (rank 0, N = 1; `configs`): C3 (16 x 256 MiB, CRC32 and CRC32C), C5 (8 x 64 MiB,
CRC64NVME and XXH64: the XXH64 host route's roofline is the PCIe D2H rate measured in the run, the kernel
route beside it) and the north-star target shape (16 x 64 MiB CRC32C), each with value, kernel duration,
roofline and cpu_baseline.  Never `value`.

CPU baseline (`cpu_baseline`; rank 0 at every N, after the timed region): the engine's own host path (csrc/cpu/: AVX-512
VPCLMULQDQ / PCLMULQDQ folding, SSE4.2 crc32, vectorised XXH3 -- aws-checksums' technique class;
aws-checksums itself cannot be built here) over a bounded sample of the same buffers, 1 thread and
the box's CPU share (std::threads, buffers round-robin), median of >= 5 reps, CPU model stated,
results checked against the GPU's.  The oracle's hw tier is reported beside it.

End-to-end (`e2e_pinned`): the same batches start in pinned host memory; H2D copies on
a copy stream overlap the scans through a 3-slot device ring, results come back D2H.  Never `value`.

Prints one JSON line (rank 0).
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "aws-crt-cpp_amd"))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md chip table
ALG = {"crc32": 0, "crc32c": 1, "crc64nvme": 2, "xxh64": 3, "xxh3_64": 4, "xxh3_128": 5}
WIDE = {"crc64nvme", "xxh64", "xxh3_64", "xxh3_128"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of the job; default: WORLD_SIZE under a launcher, else 1.  N > 1 without a "
                         "launcher spawns N rank processes (one per GPU) before any GPU call")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (RCCL; gloo only to rehearse the rank path)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--alg", default="crc32c", choices=list(ALG))
    ap.add_argument("--buffers", type=int, default=1024)
    ap.add_argument("--buffer-bytes", type=int, default=65536)
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--coalesce", type=int, default=32, help="queued batches per launch (1..32)")
    ap.add_argument("--branches", type=int, default=3)
    ap.add_argument("--timing-launches", type=int, default=32)
    ap.add_argument("--cpu-seconds", type=float, default=1.0, help="per CPU-baseline rep")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-read-ceiling", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the C3 / C5 / target-shape legs")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 leg (the 1M x 8 KiB set sharded over the ranks)")
    ap.add_argument("--c4-passes", type=int, default=3, help="least timed passes over the C4 set")
    ap.add_argument("--c4-preload-ms", type=float, default=60.0,
                    help="continuous scanning of the C4 set before its timed window (past the power-management dip)")
    ap.add_argument("--c4-window-ms", type=float, default=30.0, help="least length of the C4 timed window")
    ap.add_argument("--e2e-batches", type=int, default=64, help="batches through the pinned-host pipeline (0: skip)")
    ap.add_argument("--inproc", action="store_true",
                    help="one process drives --gpus devices (the engine's in-process fan-out: one HIP stream per GPU, "
                         "batches sharded round-robin, no collective) instead of one rank per GPU")
    ap.add_argument("--only-coalesced", action="store_true",
                    help="profiling runs: every scan launch has the timed region's shape (no one-batch warm-up or timing "
                         "launches), so a kernel-trace average is the dominant kernel's duration")
    ap.add_argument("--plumbing-check", type=int, default=None, metavar="DEVICES",
                    help="tests: assume DEVICES visible GPUs; each rank prints its rank / world / device assignment as "
                         "JSON and exits, with no GPU call")
    return ap.parse_args(argv)


class PlumbingError(SystemExit):
    """A launch whose ranks or devices do not match --gpus (exit status 2)."""

    def __init__(self, msg):
        print(f"bench.py: {msg}", file=sys.stderr, flush=True)
        super().__init__(2)


def rank_layout(args, env, device_count):
    """Where this process sits in the job, before any GPU call: (world, rank, local rank, device index,
    shared).  `--gpus` must equal the launcher's WORLD_SIZE; with RCCL every rank needs its own device,
    with --dist-backend gloo ranks beyond the visible devices share them round-robin (a rehearsal of
    the rank path on fewer GPUs, reported as such).  device_count: torch.cuda.device_count(), which on
    this image counts without initialising the GPU."""
    world = int(env.get("WORLD_SIZE", "1"))
    rank = int(env.get("RANK", "0"))
    local = int(env.get("LOCAL_RANK", str(rank)))
    gpus = world if args.gpus is None else args.gpus
    if gpus != world:
        raise PlumbingError(f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
    if device_count < 1:
        raise PlumbingError("no GPU visible")
    if local >= device_count and args.dist_backend == "nccl":
        raise PlumbingError(f"rank {rank} (local {local}) has no GPU of its own: {device_count} visible, RCCL needs one "
                            f"per rank (--dist-backend gloo rehearses the rank path on shared devices)")
    return world, rank, local, local % device_count, world > device_count


def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv=None):
    """--gpus N > 1 with no launcher: start N rank processes of this script (fresh interpreters, one
    per GPU: RANK = LOCAL_RANK = i, WORLD_SIZE = N, rendezvous on 127.0.0.1) and wait for them.  This
    process makes no GPU call.  The first rank to fail ends the others; the exit status is the first
    non-zero one.  Rank 0 prints the JSON line."""
    import subprocess

    argv = sys.argv[1:] if argv is None else argv
    port = str(free_port())
    procs = []
    for i in range(n):
        env = dict(os.environ, RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 1
                for q in live:
                    q.terminate()
        if live:
            time.sleep(0.05)
    return rc


def cpu_topology():
    """Sockets and physical cores of the machine (/proc/cpuinfo), the cgroup CPU quota (cgroup v2
    cpu.max, in cores, None when unlimited), the affinity mask and the pool's share (OMP_NUM_THREADS)."""
    model, phys, cur = "unknown", set(), {}
    try:
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and model == "unknown":
                model = v
            elif k in ("physical id", "core id"):
                cur[k] = v
            elif not k and cur:
                phys.add((cur.get("physical id"), cur.get("core id")))
                cur = {}
        if cur:
            phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    return {"cpu_model": model, "sockets": len({p for p, _ in phys}) or None, "physical_cores": len(phys) or None,
            "logical_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_cpu_quota_cores": quota,
            "pool_share_threads": share}


def cpu_share():
    """Threads for the CPU baseline: every physical core this process may use -- the
    affinity mask, capped by the cgroup CPU quota and by the share the GPU pool gives one GPU
    (OMP_NUM_THREADS, 16 on the pool's boxes; the pool's rules forbid using more).  The machine's
    topology is reported beside it."""
    topo = cpu_topology()
    limits = [topo["affinity_cpus"]]
    if topo["cgroup_cpu_quota_cores"]:
        limits.append(max(1, int(topo["cgroup_cpu_quota_cores"])))
    if topo["pool_share_threads"]:
        limits.append(topo["pool_share_threads"])
    if topo["physical_cores"]:
        limits.append(topo["physical_cores"])
    threads = min(limits)
    limit = ("pool share (OMP_NUM_THREADS)" if topo["pool_share_threads"] == threads else
             "cgroup CPU quota" if topo["cgroup_cpu_quota_cores"] and int(topo["cgroup_cpu_quota_cores"]) == threads else
             "physical cores" if topo["physical_cores"] == threads else "affinity mask")
    return threads, topo, limit


def host_sample(dev_data, nbytes, pinned=None):
    """The CPU baseline's bytes in host memory: the e2e leg's pinned copy of them when there is one
    (the same pages the host-ingest legs read, so the two figures differ only by the path), else a
    pageable copy written by this thread (its pages on one NUMA node, where the engine's host path
    places its threads: cpu::home_node)."""
    import numpy as np

    if pinned is not None:
        return pinned[:nbytes].numpy()
    host = np.empty(nbytes, dtype=np.uint8)
    np.copyto(host, dev_data[:nbytes].cpu().numpy())
    return host


def interleaved(legs, reps):
    """Median GiB/s of each leg over `reps` reps; a leg's rep runs its callable until >= its seconds
    have passed.  legs: (name, fn, nbytes, seconds).  Each leg is warmed up once; within a rep the
    legs run one after another, the starting leg rotating with the rep."""
    for _, fn, _, _ in legs:
        fn()
    rs = {name: [] for name, _, _, _ in legs}
    for r in range(reps):
        for k in range(len(legs)):
            name, fn, nbytes, secs = legs[(r + k) % len(legs)]
            passes, t0 = 0, time.perf_counter()
            while True:
                fn()
                passes += 1
                el = time.perf_counter() - t0
                if el >= secs:
                    break
            rs[name].append(passes * nbytes / el / 2**30)
    return {name: statistics.median(v) for name, v in rs.items()}


def cpu_baseline(eng, alg, host, count, L, gpu_results, rep_seconds, reps=5, step_buffers=None, paired=None):
    """Engine host path (kind "port") on a bounded sample: `count` buffers of L bytes from `host`
    (numpy), 1 thread and the box's CPU share, median of `reps` reps of >= rep_seconds each.
    gpu_results: the GPU's results for the first buffers.  step_buffers: also time the first
    step_buffers buffers alone (one step, which may sit in the host's last-level cache) beside it.
    paired: an IngestLegs whose host-ingest legs are timed in the same reps as the share-thread
    figure (interleaved, order rotated per rep), so that `value` and the e2e legs see the same
    state of the shared host (other tenants' memory traffic moves both by up to 2x between runs)."""
    from oracle import oracle  # checker and secondary figure only

    threads, topo, limit = cpu_share()
    base = host.ctypes.data
    ptrs = [base + i * L for i in range(count)]
    lens = [L] * count
    first = eng.cpu_batch(ALG[alg], ptrs, lens, threads=threads)
    parity = first[:len(gpu_results)] == gpu_results[:count]

    def rate(fn, nbytes):
        return interleaved([("r", fn, nbytes, rep_seconds)], reps)["r"]

    n1 = count  # the same sample on one thread
    # argument arrays prepared once: the timed calls are the C calls alone
    many, one = eng.CpuBatch(ALG[alg], ptrs, lens, threads=threads), eng.CpuBatch(ALG[alg], ptrs[:n1], lens[:n1], threads=1)
    legs = [("cpu", many.run, count * L, rep_seconds)] + (paired.legs() if paired is not None else [])
    rates = interleaved(legs, reps)
    if paired is not None:
        paired.rates = rates
    v = rates["cpu"]
    v1 = rate(one.run, n1 * L)
    ov = None
    if alg in oracle.ALG_INDEX:
        ov = rate(oracle.prepared_batch(alg, ptrs, lens, threads), count * L)
    cached = None
    if step_buffers and step_buffers < count:
        cached = round(rate(eng.CpuBatch(ALG[alg], ptrs[:step_buffers], lens[:step_buffers], threads=threads).run,
                            step_buffers * L), 2)
    third = third_party_rates(alg, host, min(count, len(gpu_results)), L, threads, gpu_results, rate)
    hashed = alg in ("xxh64", "xxh3_64", "xxh3_128")
    busy = min(threads, count) if hashed else threads
    return {"value": round(v, 2), "unit": "GiB/s", "cores": busy, "kind": "port",
            "impl": f"engine host path ({eng.cpu_tier()} tier)",
            "sample": f"{count} x {L >> 10} KiB ({count * L >> 20} MiB) in "
                      f"{'the e2e legs pinned host pages' if paired is not None else 'pageable host memory'}, median of {reps} reps "
                      f"of >= {rep_seconds:g} s{' interleaved with the e2e legs' if paired is not None else ''}, "
                      f"{threads} persistent threads claiming work items "
                      + ("(one per buffer: a hash is one serial chain)" if hashed else
                         "(buffers cut into >= 1 MiB pieces folded with Combine, so every thread is busy)"),
            "threads_limit": limit, "single_thread_gibs": round(v1, 2), "topology": topo,
            "one_step_gibs": cached,
            "oracle_hw_tier_gibs": round(ov, 2) if ov is not None else None, "parity_with_gpu": parity,
            "third_party": third}


def third_party_rates(alg, host, count, L, threads, gpu_results, rate):
    """SURVEY.md §8(d) extra CPU data points: zlib crc32 for CRC32, libxxhash XXH64 for XXH64 (the
    system libraries; their calls release the GIL, so Python threads run them in parallel), 1 thread
    and `threads` threads over the same buffers, checked against the GPU results."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor

    mv = memoryview(host)
    bufs = [mv[i * L:(i + 1) * L] for i in range(count)]
    if alg == "crc32":
        import zlib

        fn, name = zlib.crc32, f"zlib {zlib.ZLIB_RUNTIME_VERSION} crc32"
    elif alg == "xxh64":
        try:
            lib = ctypes.CDLL("libxxhash.so.0")
        except OSError:
            return None
        lib.XXH64.restype = ctypes.c_uint64
        lib.XXH64.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
        base = host.ctypes.data
        addrs = [base + i * L for i in range(count)]
        fn, name = (lambda a: lib.XXH64(a, L, 0)), "libxxhash XXH64 (system libxxhash.so.0)"
        bufs = addrs
    else:
        return None
    if [fn(b) for b in bufs] != list(gpu_results[:count]):
        return {"impl": name, "parity_with_gpu": False}
    pool = ThreadPoolExecutor(max_workers=threads)
    try:
        v1 = rate(lambda: [fn(b) for b in bufs[: max(1, min(count, (64 << 20) // L))]], max(1, min(count, (64 << 20) // L)) * L)
        vn = rate(lambda: list(pool.map(fn, bufs)), count * L)
    finally:
        pool.shutdown()
    return {"impl": name, "gibs": round(vn, 2), "threads": threads, "single_thread_gibs": round(v1, 2), "parity_with_gpu": True}


def pmc_traffic(alg, nbuf, L, batches_per_launch):
    """HBM bytes per launch of this shape from the committed rocprofv3 FETCH_SIZE passes
    (profiles/pmc_traffic.json), with its source, or None"""
    pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        for rec in json.load(open(pmc))["records"]:
            if rec.get("workload") == f"{alg}:{nbuf}x{L}" and rec.get("batches_per_launch", 1) == batches_per_launch:
                return rec.get("hbm_bytes_per_launch"), rec.get("source", "profiles/pmc_traffic.json")
    except (OSError, ValueError, KeyError):
        pass
    return None


def time_launches(eng, launch, st, nt, stamps=False):
    """Mean dispatch duration (ms) of nt launches serialised on stream st behind a GPU-side hold.
    stamps: launch(i, st, start_event, stop_event) stamps its own dispatch (the diagnostic library's
    read-ceiling kernel); otherwise the engine's profiling hook stamps the next launch."""
    import torch

    starts = [torch.cuda.Event(enable_timing=True) for _ in range(nt)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(nt)]
    with torch.cuda.stream(st):
        torch.cuda._sleep(int(40e6))
    for i in range(nt):
        starts[i].record(st)  # creates the events; the launch below re-stamps them
        ends[i].record(st)
        if stamps:
            launch(i, st, starts[i], ends[i])
        else:
            eng.time_next_launch(starts[i], ends[i])
            launch(i, st)
    torch.cuda.synchronize()
    durs = sorted(eng.event_ms(s_, e_) for s_, e_ in zip(starts, ends))
    return sum(durs) / nt, durs[nt // 2]


def timed_passes(launch, st, npre, nmeas, hold_ms=10.0):
    """(mean ms per pass of the first npre passes, mean ms per pass of the next nmeas), all issued back
    to back on stream st after a GPU-side idle hold of hold_ms and timed with events on st (or on the
    host clock when st is None: the CPU plumbing tests)"""
    if st is None:
        t0 = time.perf_counter()
        for _ in range(npre):
            launch()
        t1 = time.perf_counter()
        for _ in range(nmeas):
            launch()
        t2 = time.perf_counter()
        return ((t1 - t0) * 1e3 / npre if npre else 0.0), (t2 - t1) * 1e3 / nmeas
    import torch

    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    if hold_ms > 0:
        with torch.cuda.stream(st):
            torch.cuda._sleep(int(hold_ms * 2e6))
    ev[0].record(st)
    for _ in range(npre):
        launch()
    ev[1].record(st)
    for _ in range(nmeas):
        launch()
    ev[2].record(st)
    torch.cuda.synchronize()
    return (ev[0].elapsed_time(ev[1]) / npre if npre else 0.0), ev[1].elapsed_time(ev[2]) / nmeas


def roofline(bytes_per_launch, kernel_ms, kernel_name):
    ach = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "kernel": kernel_name, "kernel_ms": round(kernel_ms, 5),
            "bytes_per_launch": bytes_per_launch}


def split(k, g):
    """k steps into ceil(k / g) near-equal consecutive launches"""
    n = max(1, -(-k // max(1, g)))
    return [k * i // n for i in range(n + 1)]


def widest(k, g):
    """batches in the largest launch of split(k, g)"""
    c = split(k, g)
    return max(b - a for a, b in zip(c, c[1:]))


def kernel_name(alg, nbuf, L):
    """the dominant kernel (or route) of a uniform batch of nbuf x L bytes (engine.cpp dispatch)"""
    if alg in ("crc32", "crc32c"):
        return "crc32_stream_kernel"
    if alg == "crc64nvme":
        if L <= 4096 and nbuf >= 65536:
            return "crc_lanes_kernel"
        if nbuf >= 16384 and L % 1024 == 0 and 1024 <= L <= 256 << 10:
            return "crc64_rows16_kernel"
        if L >= 256 * 16384:
            return "crc64_xcd_kernel"
        return "crc64_stream4_kernel"
    if alg == "xxh64":
        if nbuf <= 16 and L >= 1 << 20:
            return "xxh64 host route (D2H slices + host threads, stream-ordered; DESIGN.md §3.4)"
        return "xxh64_row_kernel" if nbuf <= 1024 else "xxh64_wave_kernel"
    return "xxh3_blocksum_kernel + xxh3_wave_kernel"


class IngestLegs:
    """One host-ingest job over host buffers, four ways: the default (aws_crt_amd_host_submit with no
    options: device lanes only for a CPU-poor share, the host path on the pool's 16-CPU share), hybrid
    asked for explicitly (one lane beside the share less four threads), devices only (the PCIe-bound
    pipeline) and the host path alone on the same bytes.  legs() are timed by interleaved() (beside
    cpu_baseline's share-thread figure when paired with it, else alone): GiB/s is the median of the
    reps, each rep re-running the job for >= `seconds`."""

    def __init__(self, eng, alg_id, ptrs, lens, seconds=0.25):
        self.nbytes = sum(lens)
        share = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        self.jobs = {name: eng.HostJob(alg_id, ptrs, lens, ndevices=nd, host_threads=ht)
                     for name, nd, ht in (("default", 0, -1), ("hybrid", 1, max(1, share - 4)),
                                          ("devices_only", 0, 0), ("host_only", -1, -1))}
        self.seconds = seconds
        self.rates = None

    def legs(self):
        return [(name, job.run, self.nbytes, self.seconds) for name, job in self.jobs.items()]

    def record(self, reps=5):
        if self.rates is None:
            self.rates = interleaved(self.legs(), reps)
        share = {name: round(job.device_bytes / max(self.nbytes, 1), 4) for name, job in self.jobs.items()}
        gibs = {name: round(self.rates[name], 2) for name in self.jobs}
        return {"value": gibs["default"], "unit": "GiB/s", "device_share": share["default"],
                "hybrid_gibs": gibs["hybrid"], "hybrid_device_share": share["hybrid"],
                "devices_only_gibs": gibs["devices_only"], "host_only_gibs": gibs["host_only"],
                "timing": f"median of reps of >= {self.seconds:g} s per leg"
                          + (", interleaved with cpu_baseline's reps" if "cpu" in self.rates else ""),
                "api": "aws_crt_amd_host_submit (default policy) + aws_crt_amd_job_wait"}

    def results(self):
        return self.jobs["default"].results()


def config_label(alg, count, L):
    """the BASELINE.json config a bench shape is, or "custom" """
    if alg == "crc32c" and count == 1024 and L == 65536:
        return "C2"
    if alg in ("crc64nvme", "xxh64") and L == 64 << 20:
        return "C5"
    if alg in ("crc32", "crc32c") and count == 16 and L == 256 << 20:
        return "C3"
    if count == 131072 and L == 8192:
        return "C4 per-GPU shard"
    return "custom"


class E2EStep:
    """One config step from pinned host memory through the host-ingest API (SURVEY.md §8(d)
    end-to-end row): results in host memory, checked against the device-resident results; beside it
    the H2D-only rate of the same bytes (the PCIe ceiling).  `ingest` is timed by record() or,
    paired, inside cpu_baseline."""

    def __init__(self, eng, alg, dev_step, nbuf, L):
        import torch

        self.host = torch.empty(nbuf * L, dtype=torch.uint8, pin_memory=True)
        self.host.copy_(dev_step[: nbuf * L])
        self.dev, self.nbuf, self.L = dev_step.device, nbuf, L
        self.ingest = IngestLegs(eng, ALG[alg], [self.host.data_ptr() + i * L for i in range(nbuf)], [L] * nbuf)

    def record(self, gpu_results):
        import torch

        hy = self.ingest.record()
        parity = self.ingest.results()[: self.nbuf] == gpu_results[: self.nbuf]
        total = self.nbuf * self.L
        slot = torch.empty(min(total, 256 << 20), dtype=torch.uint8, device=self.dev)
        cs = torch.cuda.Stream(device=self.dev)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        with torch.cuda.stream(cs):
            for off in range(0, total, slot.numel()):
                n = min(slot.numel(), total - off)
                slot[:n].copy_(self.host[off:off + n], non_blocking=True)
        torch.cuda.synchronize()
        el_h2d = time.perf_counter() - t1
        self.host = None
        return dict(hy, h2d_only_gibs=round(total / el_h2d / 2**30, 2), parity_with_device_path=parity,
                    sample=f"one step ({self.nbuf} x {self.L} B) from pinned host memory, results to host memory")


def d2h_rate(data, nbytes, dev, reps=3):
    """GiB/s of plain device-to-pinned-host copies of nbytes (64 MiB pieces on one stream): the PCIe D2H
    ceiling of this box, right now"""
    import torch

    piece = 64 << 20
    host = torch.empty(min(nbytes, piece), dtype=torch.uint8, pin_memory=True)
    cs = torch.cuda.Stream(device=dev)
    rates = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(cs):
            for off in range(0, nbytes, piece):
                n = min(piece, nbytes - off)
                host[:n].copy_(data[off:off + n], non_blocking=True)
        torch.cuda.synchronize()
        rates.append(nbytes / (time.perf_counter() - t0) / 2**30)
    return statistics.median(rates[1:])


def xxh64_route_roofline(eng, roof, data, step_bytes, per, dev):
    """the XXH64 host route reads each byte once over PCIe (stream-ordered D2H
    slices hashed by host threads), so its bound is the link's device-to-host rate, not
    HBM.  peak = the D2H-only rate of the same bytes measured now; frac = the route's rate / that.  The
    HBM fraction stays beside it as a side field."""
    d2h = d2h_rate(data, per * step_bytes, dev)
    ach = roof["achieved"]
    peak = d2h * 2**30 / 1e9
    return dict(roof, bound="pcie_d2h", peak=round(peak, 1), frac=round(ach / peak, 4), hbm_frac=roof["frac"],
                peak_source="D2H-only rate of the same bytes into pinned host memory, measured in this run "
                            f"({round(d2h, 2)} GiB/s)")


def xxh64_kernel_route(eng, launch_group, outs, nb, steps, coalesce, streams, timing, step_bytes, per, nbuf, L):
    """The same XXH64 leg on the gfx950 kernels (AWS_CRT_AMD_XXH64_ROUTE=0, read per call): the "same
    kernel template" figure BASELINE configs[4] names, measured beside the route, with its results
    checked against the route's"""
    import torch

    ref = [eng.as_unsigned(o) for o in outs]
    os.environ["AWS_CRT_AMD_XXH64_ROUTE"] = "0"
    try:
        for o in outs:
            o.zero_()
        cuts = split(steps, coalesce)
        for j in range(len(cuts) - 1):
            launch_group(cuts[j], cuts[j + 1], streams[j % len(streams)])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for j in range(len(cuts) - 1):
            launch_group(cuts[j], cuts[j + 1], streams[j % len(streams)])
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        kms, _ = time_launches(eng, lambda i, st: launch_group(i * per, i * per + per, st), streams[0], timing)
        same = [eng.as_unsigned(o) for o in outs] == ref
    finally:
        del os.environ["AWS_CRT_AMD_XXH64_ROUTE"]
    kn = "xxh64_row_kernel" if nbuf <= 1024 else "xxh64_wave_kernel"
    return {"value": round(steps * step_bytes / el / 2**30, 2), "unit": "GiB/s",
            "roofline": roofline(per * step_bytes, kms, kn), "parity_with_route": same,
            "note": "AWS_CRT_AMD_XXH64_ROUTE=0: every buffer's serial XXH64 chain on the GPU (one wave per buffer); "
                    "chain-latency bound, DESIGN.md §3.4"}


def config_leg(eng, name, alg, nbuf, L, streams, dev, coalesce=1, steps=12, nb=2, timing=6, cpu_bufs=None,
               cpu_seconds=0.5, do_cpu=True, do_e2e=True):
    """One BASELINE config: `steps` steps of `nbuf` x L bytes (nb rotating batches), pipelined over
    the streams; roofline from `timing` serialised launches; CPU baseline on `cpu_bufs` buffers."""
    import torch

    step_bytes = nbuf * L
    nb = max(nb, widest(steps, coalesce))  # no launch reads a batch twice
    g = torch.Generator(device=dev)
    g.manual_seed(hash(name) & 0xFFFF)
    data = torch.randint(0, 256, (nb * step_bytes,), dtype=torch.uint8, device=dev, generator=g)
    odt = torch.int64 if alg in WIDE else torch.int32
    outs = [torch.empty(nbuf, dtype=odt, device=dev) for _ in range(nb)]

    def launch_group(i0, i1, st):
        eng.checksum_batches(ALG[alg], [(data.data_ptr() + (i % nb) * step_bytes, None, outs[i % nb]) for i in range(i0, i1)],
                             L, L, nbuf, stream=st)

    cuts = split(steps, coalesce)
    for j in range(len(cuts) - 1):
        launch_group(cuts[j], cuts[j + 1], streams[j % len(streams)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(len(cuts) - 1):
        launch_group(cuts[j], cuts[j + 1], streams[j % len(streams)])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    per = cuts[1] - cuts[0]
    kms, _ = time_launches(eng, lambda i, st: launch_group(i * per, i * per + per, st), streams[0], timing)
    gibs = steps * step_bytes / el / 2**30
    rec = {"workload": f"{name}: {nbuf} x {L >> 20 if L >= 1 << 20 else L >> 10} {'MiB' if L >= 1 << 20 else 'KiB'} "
                       f"{alg.upper()}, device-resident, {nb} rotating batches, {per} per launch",
           "value": round(gibs, 2), "unit": "GiB/s", "steps": steps, "ms_per_step": round(el / steps * 1e3, 4),
           "pct_hbm_peak": round(100.0 * gibs * 2**30 / 1e9 / HBM_PEAK_GBS, 2),
           "roofline": dict(roofline(per * step_bytes, kms, kernel_name(alg, nbuf, L)), timing_launches=timing)}
    if alg == "xxh64":  # the host route is PCIe-bound: the link's state right after the timed launches
        bx = box_state(torch.cuda.get_device_properties(dev))
        rec["pcie_after"] = {"dpm": (bx.get("pcie") or {}).get("current"), "link": bx.get("link")}
        if "host route" in rec["roofline"]["kernel"]:
            rec["roofline"] = xxh64_route_roofline(eng, rec["roofline"], data, step_bytes, per, dev)
            rec["kernel_route"] = xxh64_kernel_route(eng, launch_group, outs, nb, steps, coalesce, streams, timing,
                                                     step_bytes, per, nbuf, L)
    trf = pmc_traffic(alg, nbuf, L, per)
    if trf:
        rec["roofline"]["traffic"], rec["roofline"]["traffic_source"] = trf
    e2e = None
    if do_e2e and alg not in ("xxh64", "xxh3_64", "xxh3_128"):  # host-ingest hash jobs run on the host path
        torch.cuda.synchronize()
        e2e = E2EStep(eng, alg, data, nbuf, L)
    if do_cpu:
        # the whole step's buffers (buffers round-robin over the threads, so a sample
        # of fewer buffers than threads would leave cores idle)
        cpu_bufs = nbuf if cpu_bufs is None else cpu_bufs
        torch.cuda.synchronize()
        gpu0 = eng.as_unsigned(outs[0])
        host = host_sample(data, cpu_bufs * L, e2e.host if e2e is not None else None)
        rec["cpu_baseline"] = cpu_baseline(eng, alg, host, cpu_bufs, L, gpu0, cpu_seconds,
                                           paired=e2e.ingest if e2e is not None else None)
        del host
    if e2e is not None:
        rec["e2e_pinned"] = e2e.record(eng.as_unsigned(outs[0]))
    del data
    torch.cuda.empty_cache()
    return rec


def c4_leg(eng, args, dev, rank, world, streams, max_over_ranks, barrier, group_device, n=None, L=None, golden=None,
           timer=None):
    """BASELINE.json configs[3] as stated: the fixed set of 1,048,576 x 8 KiB
    buffers (8 GiB), buffer i on rank i mod N -- strong scaling of one set over the job's GPUs.  Every
    rank builds its shard on its own GPU (aws_crt_amd/synth.py: bytes are a function of the global
    position, so every N scans the same set), scans it with one strided launch per pass, and reports
    its kernel fraction and a parity sample (the engine's host path); rank 0 gathers every result in
    buffer order (4-8 bytes per buffer) and checks the set's digest against tests/golden/c4_digest.json
    (computed by the oracle on the CPU).  value = 8 GiB / the slowest rank's time per pass in the
    sustained regime: back-to-back passes after >= --c4-preload-ms of the same scan, past the
    power-management dip that slows compute-heavy scans 2-30 ms into a burst from idle;
    the burst (one pass after an idle hold) and the mean pass from idle are reported beside it.
    Returns {alg: record} on rank 0, None elsewhere.  (n, L, golden, timer: a smaller set and stand-ins
    for the CPU plumbing test, tests/test_bench_plumbing.py.)"""
    import torch

    from aws_crt_amd import sharding, synth

    n, L = n or synth.C4_COUNT, L or synth.C4_LEN
    if golden is None:
        golden = json.load(open(os.path.join(REPO, "tests", "golden", "c4_digest.json")))
    timer = timer or time_launches
    cnt = sharding.shard_count(n, rank, world)
    data = torch.empty(cnt * L, dtype=torch.uint8, device=dev)
    synth.fill_shard(data, rank, world, count=n, length=L)
    sync = torch.cuda.synchronize if data.is_cuda else (lambda: None)
    sync()
    st = streams[0]
    recs = {}
    for alg in ("crc32c", "crc64nvme"):
        sh = sharding.RoundRobinShard(eng, ALG[alg], data, n, L, rank, world)
        sh.launch(st)  # warm-up (first launch of the shape)
        sync()
        reps = max(1, args.c4_passes)
        # three regimes: one pass after an idle hold (burst), the mean pass of the first
        # pre_ms of continuous scanning (the power-management dip 2-30 ms into a burst lies there), and
        # the sustained pass after it (`value`)
        pre_ms, win_ms = getattr(args, "c4_preload_ms", 60.0), getattr(args, "c4_window_ms", 30.0)
        barrier()
        sync()
        _, burst_ms = timed_passes(lambda: sh.launch(st), st, 0, 1, hold_ms=10.0)
        npre = -(-int(pre_ms * 1000) // max(1, int(burst_ms * 1000))) if pre_ms > 0 else 0
        nmeas = max(reps, -(-int(win_ms * 1000) // max(1, int(burst_ms * 1000))))
        barrier()
        sync()
        pre_pass_ms, own_ms = timed_passes(lambda: sh.launch(st), st, npre, nmeas, hold_ms=10.0)
        own = own_ms * 1e-3
        elapsed = max_over_ranks(own)
        kms, _ = timer(eng, lambda i, s_: sh.launch(s_), st, max(2, args.timing_launches // 8))
        # parity: a sample of this rank's buffers on the engine's host path; the whole set by digest
        nchk = min(cnt, 1024)
        hs = data[: nchk * L].cpu().numpy()
        want = eng.cpu_batch(ALG[alg], [hs.ctypes.data + i * L for i in range(nchk)], [L] * nchk, threads=8)
        sample_ok = eng.as_unsigned(sh.out)[:nchk] == want
        allr = sh.gather(device=group_device)
        digest = sharding.results_digest(eng, allr, sh.width) if rank == 0 else None
        roof = roofline(cnt * L, own_ms, kernel_name(alg, cnt, L))
        roof_burst = roofline(cnt * L, kms, kernel_name(alg, cnt, L))
        mine = {"rank": rank, "buffers": cnt, "value": round(cnt * L / own / 2**30, 2), "kernel_ms": roof["kernel_ms"],
                "frac": roof["frac"], "burst_frac": round(cnt * L / (burst_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "from_idle_frac": round(cnt * L / (pre_pass_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if npre else None,
                "parity_sample_buffers": nchk, "parity": sample_ok}
        ranks = [None] * world
        if world > 1:
            import torch.distributed as dist

            dist.all_gather_object(ranks, mine)
        else:
            ranks = [mine]
        if rank == 0:
            want_digest = int(golden[alg]["digest"], 16)
            value = n * L / elapsed / 2**30
            recs[f"C4_{alg}"] = {
                "workload": f"C4: {n} x {L >> 10} KiB {alg.upper()} ({n * L / 2**30:g} GiB), buffer i on rank i mod {world}, "
                            f"device-resident, "
                            f"one strided launch of {sharding.shard_count(n, 0, world)} buffers per rank per pass",
                "value": round(value, 2), "unit": "GiB/s", "scaling": "strong", "n_gpus": world,
                "per_gpu_gibs": round(value / world, 2), "passes": nmeas, "ms_per_pass": round(elapsed * 1e3, 4),
                "pct_hbm_peak": round(100.0 * value * 2**30 / 1e9 / world / HBM_PEAK_GBS, 2),
                "timing": f"sustained: {nmeas} back-to-back passes timed with events after {npre} passes "
                          f"(>= {pre_ms:g} ms) of the same scan; slowest rank",
                "regimes": {"burst_ms_per_pass": round(burst_ms, 4),
                            "burst_gibs_per_gpu": round(cnt * L / (burst_ms * 1e-3) / 2**30, 2),
                            "from_idle_ms_per_pass": round(pre_pass_ms, 4) if npre else None,
                            "preload_passes": npre, "note": "rank 0; burst = one pass after a 10 ms idle hold; "
                            "from_idle = mean pass of the first passes after the hold (burst + the 2-30 ms dip)"},
                "roofline": dict(roof, timing="sustained passes (events)", rank=0),
                "roofline_burst": dict(roof_burst, timing_launches=max(2, args.timing_launches // 8), rank=0,
                                       timing="serialised launches after a 40 ms hold, stamped by the dispatch"),
                "ranks": ranks,
                "digest": hex(digest), "digest_expected": hex(want_digest), "digest_match": digest == want_digest,
                "parity": digest == want_digest and all(r["parity"] for r in ranks),
                "parity_rule": "gathered results in buffer order, CRC64NVME of the result words == "
                               "tests/golden/c4_digest.json (oracle, CPU); plus 1024 buffers per rank on the host path"}
            if not args.no_cpu_baseline:
                # rank 0's shard (up to 131,072 buffers = 1 GiB, the 8-GPU shard) on the host cores,
                # while the other ranks wait at the barrier below
                cb = min(cnt, 131072)
                host = host_sample(data, cb * L)
                recs[f"C4_{alg}"]["cpu_baseline"] = cpu_baseline(eng, alg, host, cb, L, eng.as_unsigned(sh.out)[:cb],
                                                                 args.cpu_seconds / 2, reps=3)
                del host
        barrier()
        del sh
    del data
    if dev.type == "cuda":
        torch.cuda.empty_cache()
    return recs if rank == 0 else None


class E2EPinned:
    """Pinned host memory -> results in host memory through the engine's host-ingest API
    (aws_crt_amd_host_submit / aws_crt_amd_job_wait: device lanes with a 3-slot pipeline, H2D on a copy
    stream overlapping the scans, results D2H, beside the host path), `iters` C2 batches of parts in
    one job; checked against the device-resident results of the same bytes.  Also the H2D-only rate of
    the same bytes (the PCIe ceiling of the pipeline).  `ingest` is timed by record() or, paired,
    inside cpu_baseline."""

    def __init__(self, eng, alg_id, dev_data, count, L, nb, iters):
        import torch

        self.eng, self.alg_id, self.dev_data, self.count, self.L, self.nb, self.iters = eng, alg_id, dev_data, count, L, nb, iters
        step = count * L
        self.host = torch.empty(nb * step, dtype=torch.uint8, pin_memory=True)
        self.host.copy_(dev_data[: nb * step])
        base = self.host.data_ptr()
        self.ptrs = [base + (i % nb) * step + j * L for i in range(iters) for j in range(count)]
        self.ingest = IngestLegs(eng, alg_id, self.ptrs, [L] * len(self.ptrs))

    def record(self):
        import torch

        eng, count, L, nb, iters = self.eng, self.count, self.L, self.nb, self.iters
        step = count * L
        first = eng.host_job(self.alg_id, self.ptrs[:count], [L] * count)
        hy = self.ingest.record()
        res = self.ingest.results()
        dev_out = eng.checksum_strided(self.alg_id, self.dev_data, L, L, count)
        torch.cuda.synchronize()
        parity = first == eng.as_unsigned(dev_out) and res[:count] == first
        slot = torch.empty(step, dtype=torch.uint8, device=self.dev_data.device)
        cs = torch.cuda.Stream(device=self.dev_data.device)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        with torch.cuda.stream(cs):
            for i in range(iters):
                slot.copy_(self.host[(i % nb) * step:((i % nb) + 1) * step], non_blocking=True)
        torch.cuda.synchronize()
        el_h2d = time.perf_counter() - t1
        self.host = self.dev_data = None
        return dict(hy, h2d_only_gibs=round(iters * step / el_h2d / 2**30, 2), parity_with_device_path=parity,
                    sample=f"{iters} C2 batches ({iters * count} parts of {L // 1024} KiB) from {nb * step >> 20} MiB pinned host "
                           f"memory in one host job, results to host memory")


def box_state(props):
    """The GPU's clocks and partition modes as the kernel driver reports them (sysfs of the device's
    PCI function: pp_dpm_sclk / pp_dpm_mclk / pp_dpm_fclk / pp_dpm_pcie with the current level marked
    '*', the PCIe link's current speed and width, the compute and memory partition modes), so that a
    box-to-box spread in the kernel fractions (or in the PCIe-bound XXH64 route) can be traced to its
    clocks, link or memory mode.  Fields the box does not expose are null."""
    import glob

    bus = getattr(props, "pci_bus_id", None)
    dom = getattr(props, "pci_domain_id", 0) or 0
    devid = getattr(props, "pci_device_id", 0) or 0
    cands = []
    if bus is not None:
        cands.append(f"/sys/bus/pci/devices/{dom:04x}:{bus:02x}:{devid:02x}.0")
    cands += sorted(glob.glob("/sys/class/drm/card*/device"))
    path = next((c for c in cands if os.path.exists(os.path.join(c, "pp_dpm_sclk"))), None)

    def rd(name, cur_only=False):
        if path is None:
            return None
        try:
            txt = open(os.path.join(path, name)).read().strip()
        except OSError:
            return None
        if cur_only:
            cur = [ln.split(":", 1)[-1].replace("*", "").strip() for ln in txt.splitlines() if ln.rstrip().endswith("*")]
            return {"current": cur[0] if cur else None, "levels": [ln.strip() for ln in txt.splitlines()]}
        return txt

    return {"sysfs": path, "sclk": rd("pp_dpm_sclk", True), "mclk": rd("pp_dpm_mclk", True),
            "fclk": rd("pp_dpm_fclk", True), "pcie": rd("pp_dpm_pcie", True),
            "link": {"speed": rd("current_link_speed"), "width": rd("current_link_width")},
            "compute_partition": rd("current_compute_partition"),
            "memory_partition": rd("current_memory_partition"),
            "power_profile": (rd("pp_power_profile_mode") or "").splitlines()[:1] or None}


class Rig:
    """One GPU's share of the job (one rank, or one device of the in-process fan-out): its resident
    batches -- at least --batches and never fewer than one launch holds, so every launch streams from
    HBM and no launch reads a batch twice (aliased batches would hit in L2 / the Infinity Cache) --
    their result buffers and streams, and the launch plans over them."""

    def __init__(self, eng, dev, args, seed):
        import torch

        self.eng, self.dev, self.args = eng, dev, args
        self.alg, self.count, self.L = args.alg, args.buffers, args.buffer_bytes
        # hash batches run one launch per batch (aws_crt_amd_checksum_batches coalesces CRC scans only)
        self.G = 1 if self.alg in ("xxh64", "xxh3_64", "xxh3_128") else max(1, min(32, args.coalesce))
        self.step_bytes = self.count * self.L
        self.nb = max(1, args.batches, widest(max(args.steps, 1), self.G), widest(max(args.warmup, 1), self.G))
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        self.data = torch.randint(0, 256, (self.nb * self.step_bytes,), dtype=torch.uint8, device=dev, generator=g)
        self.per = 2 if self.alg == "xxh3_128" else 1
        odt = torch.int64 if self.alg in WIDE else torch.int32
        self.outs = [torch.empty(self.count * self.per, dtype=odt, device=dev) for _ in range(self.nb)]
        self.streams = [torch.cuda.Stream(device=dev) for _ in range(max(1, args.branches))]

    def batch(self, i):
        b = i % self.nb
        return (self.data.data_ptr() + b * self.step_bytes, None, self.outs[b])

    def launch_group(self, i0, i1, st):
        self.eng.checksum_batches(ALG[self.alg], [self.batch(i) for i in range(i0, i1)], self.L, self.L, self.count,
                                  stream=st)

    def prepare(self, k, g_):
        """the submissions of k steps in launches of <= g_ batches (descriptors built up front, as a
        producer fills a submission queue), alternating over the streams"""
        cuts = split(k, g_)
        return [(self.eng.BatchSet(ALG[self.alg], [self.batch(i) for i in range(cuts[j], cuts[j + 1])], self.L, self.L,
                                   self.count), self.streams[j % len(self.streams)]) for j in range(len(cuts) - 1)]

    def warm(self):
        """every batch and every stream once (per-stream workspaces are allocated on first use), then
        the requested warm-up steps the same way as the timed ones"""
        if not self.args.only_coalesced:
            for j in range(self.nb * len(self.streams)):
                self.launch_group(j, j + 1, self.streams[j % len(self.streams)])
        if self.args.warmup > 0:
            for bs, st in self.prepare(self.args.warmup, self.G):
                bs.run(st)

    def parity_sample(self):
        """the first 64 buffers of the first resident batch (written by the warm-up and the timed
        region) against the engine's host path"""
        nchk = min(self.count, 64)
        hs = self.data[: nchk * self.L].cpu().numpy()
        got = self.eng.as_unsigned(self.outs[0])[: nchk * self.per]
        want = self.eng.cpu_batch(ALG[self.alg], [hs.ctypes.data + i * self.L for i in range(nchk)], [self.L] * nchk,
                                  threads=8)
        if self.alg == "xxh3_128":
            got = [(got[2 * i] << 64) | got[2 * i + 1] for i in range(nchk)]
        return nchk, got == want

    def roofline(self):
        """dominant kernel: launches of the timed region's shape, then (unless --only-coalesced) one-batch
        launches, each stamped by its own dispatch"""
        args = self.args
        nt = max(1, args.timing_launches)
        gsz = widest(max(args.steps, 1), self.G)  # batches per launch in the timed region
        kms, kmed = time_launches(self.eng, lambda i, st: self.launch_group(i * gsz, i * gsz + gsz, st), self.streams[0], nt)
        roof = roofline(gsz * self.step_bytes, kms, kernel_name(self.alg, self.count, self.L))
        roof["kernel_ms_median"] = round(kmed, 5)
        roof["timing_launches"] = nt
        if not args.only_coalesced:
            kms1, _ = time_launches(self.eng, lambda i, st: self.launch_group(i, i + 1, st), self.streams[0], nt)
            roof["single_batch"] = {"kernel_ms": round(kms1, 5), "frac": roofline(self.step_bytes, kms1, "")["frac"],
                                    "bytes_per_launch": self.step_bytes}
        roof["traffic"] = None
        trf = pmc_traffic(self.alg, self.count, self.L, gsz)
        if trf:
            roof["traffic"], roof["traffic_source"] = trf
        return roof, gsz

    def device_record(self):
        import torch

        props = torch.cuda.get_device_properties(self.dev)
        return {"device": torch.cuda.get_device_name(self.dev), "device_index": self.dev.index,
                "pci_bus_id": getattr(props, "pci_bus_id", None), "uuid": str(getattr(props, "uuid", "")) or None}


def distinct_devices(recs):
    """devices actually used by the ranks / fan-out entries (by UUID, else PCI bus, else index)"""
    return len({r.get("uuid") or r.get("pci_bus_id") or r.get("device_index") for r in recs})


def metric_name(alg):
    return ("GiB/s CRC32C over device-resident buffers; % of HBM read peak" if alg == "crc32c"
            else f"GiB/s {alg.upper()} over device-resident buffers; % of HBM read peak")


def main_inproc(args):
    """In-process multi-device mode (the engine's in-process fan-out: one HIP stream per GPU, no
    collective).  Weak scaling, as the rank path: every device holds its own rotating batches and runs
    the full --steps of them (each device's steps submitted as prepared launches on its own stream,
    the devices' launches interleaved); the timed region ends when every device is done.  value = all
    devices' bytes / that time.  Every device's kernel fraction and parity sample are reported."""
    import torch
    import aws_crt_amd as eng

    n = args.gpus or 1
    vis = torch.cuda.device_count()
    if n > vis:
        raise PlumbingError(f"--inproc --gpus {n} but {vis} GPU(s) visible")
    rigs = []
    for dv in range(n):
        torch.cuda.set_device(dv)
        eng.init()
        rigs.append(Rig(eng, torch.device("cuda", dv), args, 0x5EED + dv))
    for dv, rig in enumerate(rigs):
        torch.cuda.set_device(dv)
        rig.warm()
    per_dev = [rig.prepare(args.steps, rig.G) if args.steps > 0 else [] for rig in rigs]
    order = [(dv, per_dev[dv][j]) for j in range(max(len(p) for p in per_dev)) for dv in range(n) if j < len(per_dev[dv])]
    for dv in range(n):
        torch.cuda.synchronize(dv)
    t0 = time.perf_counter()
    for dv, (bs, st) in order:
        torch.cuda.set_device(dv)
        bs.run(st)
    for dv in range(n):
        torch.cuda.synchronize(dv)
    el = time.perf_counter() - t0
    step_bytes = rigs[0].step_bytes
    value = n * args.steps * step_bytes / max(el, 1e-9) / 2**30
    devs = []
    for dv, rig in enumerate(rigs):
        with torch.cuda.device(dv):
            nchk, ok = rig.parity_sample()
            roof, _ = rig.roofline()
        devs.append(dict(rig.device_record(), kernel_ms=roof["kernel_ms"], frac=roof["frac"],
                         roofline={k: roof[k] for k in ("achieved", "frac", "kernel_ms", "bytes_per_launch")},
                         parity_sample_buffers=nchk, parity=ok))
    used = distinct_devices(devs)
    gsz = widest(max(args.steps, 1), rigs[0].G)
    rec = {
        "metric": metric_name(args.alg), "value": round(value, 2), "unit": "GiB/s", "n_gpus": n,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / max(args.steps, 1) * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (torch.randint bytes on device)",
        "config": {"workload": f"{config_label(args.alg, args.buffers, args.buffer_bytes)}: {args.buffers} x "
                               f"{args.buffer_bytes // 1024} KiB independent buffers per step, {args.alg.upper()}, "
                               f"device-resident, {args.steps} steps per GPU",
                   "launch": f"in-process fan-out: each device's steps in launches of up to {rigs[0].G} batches "
                             f"({gsz} per launch) on its own HIP stream",
                   "parallelism": f"one process, {n} device(s), no collective"},
        "pct_hbm_peak": round(100.0 * value * 2**30 / 1e9 / n / HBM_PEAK_GBS, 2),
        "per_gpu_gibs": round(value / n, 2), "devices_used": used,
        "parity": all(d["parity"] for d in devs), "devices": devs,
        "roofline": dict(devs[0]["roofline"], bound="hbm", peak=HBM_PEAK_GBS, unit="GB/s",
                         kernel=kernel_name(args.alg, args.buffers, args.buffer_bytes)),
    }
    print(json.dumps(rec), flush=True)
    if used != n:
        raise PlumbingError(f"--inproc --gpus {n} ran on {used} distinct device(s)")
    if not rec["parity"]:
        raise SystemExit(1)


def main_rank(args):
    import torch

    ndev = torch.cuda.device_count() if args.plumbing_check is None else args.plumbing_check
    world, rank, local, devidx, shared = rank_layout(args, os.environ, ndev)
    if args.plumbing_check is not None:
        print(json.dumps({"rank": rank, "world": world, "local_rank": local, "device_index": devidx, "shared": shared,
                          "master": f"{os.environ.get('MASTER_ADDR', '')}:{os.environ.get('MASTER_PORT', '')}"}),
              flush=True)
        return
    import torch.distributed as dist
    import aws_crt_amd as eng

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(devidx)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", devidx))
        else:
            dist.init_process_group(args.dist_backend, rank=rank, world_size=world)
    dev = torch.device("cuda", devidx)
    torch.cuda.set_device(dev)
    eng.init()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    rig = Rig(eng, dev, args, 0x5EED + rank)
    alg, count, L, G, nb, step_bytes = args.alg, rig.count, rig.L, rig.G, rig.nb, rig.step_bytes
    data, outs, streams = rig.data, rig.outs, rig.streams
    torch.cuda.synchronize()
    rig.warm()
    torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    subs = rig.prepare(args.steps, G) if args.steps > 0 else []
    torch.cuda.synchronize()
    w0 = time.time()
    t0 = time.perf_counter()
    for bs, st in subs:
        bs.run(st)
    torch.cuda.synchronize()
    # each rank's clock stops when its own GPU is done; the closing barrier follows, and the slowest
    # rank's time (max over ranks) is the job's, so the barrier's own latency is not counted as work
    own = time.perf_counter() - t0
    w1 = time.time()
    if world > 1:
        dist.barrier()
        torch.cuda.synchronize()
    elapsed = max_over_ranks(own)
    # the job's wall-clock span on this node (first rank's start to last rank's end): equal to
    # `elapsed` when the ranks start together; on a gloo rehearsal with shared devices the ranks'
    # regions need not overlap, so there `value` is no N-GPU rate and the span is reported beside it
    span = max_over_ranks(w1) + max_over_ranks(-w0)
    value = world * args.steps * step_bytes / max(elapsed, 1e-9) / 2**30

    # the same K steps submitted one launch per batch (--coalesce 1), timed the same way: the rate a
    # caller that never queues batches together sees (reported beside `value`, never as it)
    one_per_launch = None
    if G > 1 and args.steps > 0:
        subs1 = rig.prepare(args.steps, 1)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for bs, st in subs1:
            bs.run(st)
        torch.cuda.synchronize()
        el1 = max_over_ranks(time.perf_counter() - t0)
        one_per_launch = {"value": round(world * args.steps * step_bytes / max(el1, 1e-9) / 2**30, 2), "unit": "GiB/s",
                          "ms_per_step": round(el1 / args.steps * 1e3, 4),
                          "launch": f"one launch per batch, {args.steps} launches over {len(streams)} streams"}

    # the same K steps pushed one at a time into a submission queue (aws_crt_amd_queue_*): the rate a
    # producer of one batch at a time gets.  The default (eager) policy launches a push at once when
    # none of the queue's launches runs and coalesces pushes made while one does; beside it, a second
    # launch allowed in flight, and round 5's batched policy (launch at 32 queued and at the flush).
    # Median of 5 interleaved runs each; the eager default is the reported value.
    queued = None
    if G > 1 and args.steps > 0:
        policies = (("eager", eng.QUEUE_EAGER, 0, 0), ("eager_min2", eng.QUEUE_EAGER, 1, 2),
                    ("eager_min4", eng.QUEUE_EAGER, 1, 4), ("eager_inflight2", eng.QUEUE_EAGER, 2, 1),
                    ("batched", eng.QUEUE_BATCHED, 0, 0))
        runs = {name: [] for name, _, _, _ in policies}
        nl = {}
        for rep in range(5):
            for name, pol, depth, mn in policies:
                q = eng.Queue(ALG[alg], L, L, count, stream=streams[0], policy=pol, max_inflight=depth, min_launch=mn)
                if world > 1:
                    dist.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(args.steps):
                    b = rig.batch(i)
                    q.push(b[0], b[2])
                q.flush()
                torch.cuda.synchronize()
                runs[name].append(max_over_ranks(time.perf_counter() - t0))
                nl.setdefault(name, []).append(q.launches())
                q.close()

        def qrec(name):
            el = statistics.median(runs[name])
            return {"value": round(world * args.steps * step_bytes / max(el, 1e-9) / 2**30, 2), "unit": "GiB/s",
                    "ms_per_step": round(el / args.steps * 1e3, 4), "launches": nl[name]}

        queued = dict(qrec("eager"), launch=f"{args.steps} pushes of one batch into aws_crt_amd_queue, eager policy "
                                           f"(launch on a push when none of the queue's launches runs; pushes made "
                                           f"while one runs coalesce), then flush; median of 5",
                      policies={name: qrec(name) for name, _, _, _ in policies})

    # every rank checks a sample of its own results against the engine's host path
    torch.cuda.synchronize()
    nchk, rank_parity = rig.parity_sample()
    roof, gsz = rig.roofline()

    # secondary denominator: the streaming-read ceiling of a one-batch launch and
    # of a launch of the timed region's size (the same bytes, read by an XOR-reduce kernel)
    if not args.no_read_ceiling and not args.only_coalesced:
        nt = max(1, args.timing_launches)
        rc_ms, _ = time_launches(eng, lambda i, st, e0, e1: eng.read_ceiling(data, step_bytes, stream=st,
                                                                             base_offset=(i % nb) * step_bytes,
                                                                             start_event=e0, stop_event=e1),
                                 streams[0], nt, stamps=True)
        roof["single_batch"]["read_ceiling_kernel_ms"] = round(rc_ms, 5)
        roof["single_batch"]["read_ceiling_frac"] = roofline(step_bytes, rc_ms, "")["frac"]
        rcg_ms, _ = time_launches(eng, lambda i, st, e0, e1: eng.read_ceiling(data, gsz * step_bytes, stream=st,
                                                                              start_event=e0, stop_event=e1),
                                  streams[0], max(2, nt // 4), stamps=True)
        roof["read_ceiling"] = {"kernel_ms": round(rcg_ms, 5), "frac": roofline(gsz * step_bytes, rcg_ms, "")["frac"],
                                "timing_launches": max(2, nt // 4),
                                "scan_frac_of_ceiling": round(rcg_ms / roof["kernel_ms"], 4),
                                "kernel": "read_ceiling_kernel: the scan's launch shape, 256-B non-temporal rows XOR-reduced"}

    # per-rank record (device, own rate, kernel time and fraction, parity), gathered on rank 0
    mine = dict({"rank": rank, "local_rank": local}, **rig.device_record())
    mine.update({"value": round(args.steps * step_bytes / max(own, 1e-9) / 2**30, 2), "unit": "GiB/s",
                 "kernel_ms": roof["kernel_ms"], "frac": roof["frac"],
                 "roofline": {k: roof[k] for k in ("achieved", "frac", "kernel_ms", "bytes_per_launch")},
                 "parity_sample_buffers": nchk, "parity": rank_parity})
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
    else:
        ranks = [mine]
    parity_all = all(r["parity"] for r in ranks)
    used = distinct_devices(ranks)

    def barrier():
        if world > 1:
            dist.barrier()

    # BASELINE configs[3] at every N: the fixed 1M x 8 KiB set, buffer i on rank i mod N (all ranks)
    configs = {}
    if not args.no_c4:
        c4 = c4_leg(eng, args, dev, rank, world, streams, max_over_ranks, barrier,
                    dev if world > 1 and args.dist_backend == "nccl" else None)
        if rank == 0:
            configs.update(c4)
            parity_all = parity_all and all(v["parity"] for v in c4.values())

    cpu = e2e = None
    if rank == 0:
        # the CPU baseline on rank 0's host cores at every N (the other ranks wait at the barrier below);
        # the pinned-host legs and the single-GPU config legs at N = 1
        e2e_legs = (E2EPinned(eng, ALG[alg], data, count, L, nb, args.e2e_batches)
                    if args.e2e_batches > 0 and world == 1 else None)
        if not args.no_cpu_baseline:
            # the sample: every resident batch (as many bytes as the timed region streams, more than
            # the host's last-level cache, as the GPU's reads are beyond its caches), with one step
            # alone (cache-resident on the host) reported beside it
            torch.cuda.synchronize()
            host = host_sample(data, nb * step_bytes, e2e_legs.host if e2e_legs is not None else None)
            cpu = cpu_baseline(eng, alg, host, nb * count, L, eng.as_unsigned(outs[0]), args.cpu_seconds,
                               step_buffers=count, paired=e2e_legs.ingest if e2e_legs is not None else None)
            del host
        if e2e_legs is not None:
            e2e = e2e_legs.record()
            del e2e_legs
    barrier()
    if rank == 0 and world == 1:
        if not args.no_configs:
            del data, rig
            torch.cuda.empty_cache()
            do_cpu = not args.no_cpu_baseline
            legs = {"do_cpu": do_cpu, "do_e2e": args.e2e_batches > 0}
            configs["C3_crc32c"] = config_leg(eng, "C3", "crc32c", 16, 256 << 20, streams, dev, **legs)
            configs["C3_crc32"] = config_leg(eng, "C3", "crc32", 16, 256 << 20, streams, dev, **legs)
            configs["C5_crc64nvme"] = config_leg(eng, "C5", "crc64nvme", 8, 64 << 20, streams, dev, **legs)
            configs["C5_xxh64"] = config_leg(eng, "C5", "xxh64", 8, 64 << 20, streams, dev, steps=4, timing=2, **legs)
            configs["target_16x64MiB_crc32c"] = config_leg(eng, "north-star target", "crc32c", 16, 64 << 20, streams, dev,
                                                           steps=20, **legs)
            configs["target_16x64MiB_crc32c"]["target_pct"] = 80.0
            # the same C5 steps through the multi-batch launch (12 queued batches = 6 GiB per launch, as the
            # headline coalesces C2): the batched API's rate for S3's default algorithm.  Last: the XXH64
            # host route measured right after these launches runs at ~17 GiB/s instead of 41-50 for the
            # next ~0.3 s (tools/x64_leg_order.py, profiles/r06/x64order), so no leg follows them.
            configs["C5_crc64nvme_multi_batch"] = config_leg(eng, "C5", "crc64nvme", 8, 64 << 20, streams, dev,
                                                             coalesce=12, timing=2, do_cpu=False, do_e2e=False)

    if rank == 0:
        rec = {
            "metric": metric_name(alg),
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
            "config": {"workload": f"{config_label(alg, count, L)}: {count} x {L // 1024} KiB independent buffers per step, "
                                   f"{alg.upper()}, device-resident, per GPU",
                       "buffers_per_step": count, "buffer_bytes": L, "rotating_batches": nb,
                       "resident_bytes_per_gpu": nb * step_bytes,
                       "launch": f"aws_crt_amd_checksum_batches, up to {G} queued batches per launch "
                                 f"({len(split(max(args.steps, 1), G)) - 1} launches for {args.steps} steps)",
                       "streams": len(streams),
                       "parallelism": f"buffers sharded over {world} rank(s) on {used} GPU(s), no collective"
                                      + (" (gloo rehearsal: ranks share devices)" if shared else "")},
            "pct_hbm_peak": round(100.0 * value * 2**30 / 1e9 / world / HBM_PEAK_GBS, 2),
            "per_gpu_gibs": round(value / world, 2),
            "devices_used": used,
            "shared_devices": shared,
            "span_ms": round(span * 1e3, 4),
            "parity": parity_all,
            "ranks": ranks,
            **({"note": "gloo rehearsal on shared devices: value is not an N-GPU rate"} if shared else {}),
            "box": box_state(torch.cuda.get_device_properties(dev)),
            "one_batch_per_launch": one_per_launch,
            "queued_one_at_a_time": queued,
            "roofline": roof,
            "cpu_baseline": cpu,
            "e2e_pinned": e2e,
            "configs": configs or None,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()
    # RCCL ranks each need their own GPU (rank_layout refused a rank without one); a job whose ranks
    # ran on fewer distinct devices than --gpus without asking for the gloo rehearsal is not an N-GPU
    # measurement
    if used != world and not shared:
        raise PlumbingError(f"{world} ranks ran on {used} distinct GPU(s)")
    if not parity_all:
        raise SystemExit(1)


def main(argv=None):
    args = parse(argv)
    if args.inproc:
        return main_inproc(args)
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        # no launcher: one fresh rank process per GPU, started before this process touches the GPU
        raise SystemExit(spawn_ranks(args.gpus, sys.argv[1:] if argv is None else argv))
    return main_rank(args)


if __name__ == "__main__":
    main()
