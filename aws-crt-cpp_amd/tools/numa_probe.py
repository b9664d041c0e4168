#!/usr/bin/env python3
"""NUMA probe for the host path: where the pages of a pinned (hipHostMalloc through torch) and a
pageable buffer live, and the CRC32C GiB/s of aws_crt_amd_cpu_batch and of a host-only ingest job
over each, with the process's threads allowed on every CPU, or only on one node's CPUs.

Each affinity runs in its own child process (the engine's thread pool inherits the mask of the thread
that creates it), started before anything touches the GPU.  Output: one JSON line per affinity."""
import ctypes
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))


def node_cpus():
    base = "/sys/devices/system/node"
    out = {}
    for d in sorted(os.listdir(base)) if os.path.isdir(base) else []:
        if d.startswith("node") and d[4:].isdigit():
            cpus = set()
            for part in open(os.path.join(base, d, "cpulist")).read().strip().split(","):
                if part:
                    a, _, b = part.partition("-")
                    cpus.update(range(int(a), int(b or a) + 1))
            out[int(d[4:])] = cpus
    return out


def page_nodes(addr, nbytes, samples=256):
    """node id -> count over `samples` pages spread over the buffer (move_pages with nodes=NULL)"""
    libc = ctypes.CDLL(None, use_errno=True)
    page = os.sysconf("SC_PAGE_SIZE")
    n = min(samples, max(1, nbytes // page))
    pages = (ctypes.c_void_p * n)(*[(addr + (i * (nbytes // n))) & ~(page - 1) for i in range(n)])
    status = (ctypes.c_int * n)()
    rc = libc.syscall(279, 0, ctypes.c_ulong(n), pages, None, status, 0)
    if rc != 0:
        return {"error": ctypes.get_errno()}
    hist = {}
    for s in status:
        hist[str(s)] = hist.get(str(s), 0) + 1
    return hist


def rate(fn, nbytes, reps=5, secs=0.25):
    fn()
    rs = []
    for _ in range(reps):
        passes, t0 = 0, time.perf_counter()
        while True:
            fn()
            passes += 1
            el = time.perf_counter() - t0
            if el >= secs:
                break
        rs.append(passes * nbytes / el / 2**30)
    rs.sort()
    return round(rs[len(rs) // 2], 1)


def child(mode, total_mib):
    nodes = node_cpus()
    allowed = os.sched_getaffinity(0)
    if mode != "all":
        cpus = nodes[int(mode[4:])] & allowed
        os.sched_setaffinity(0, cpus)
    sys.path.insert(0, os.path.dirname(HERE))
    import torch

    import aws_crt_amd as eng

    eng.init()
    total = total_mib << 20
    threads = int(os.environ.get("OMP_NUM_THREADS", "16"))
    pinned = torch.randint(0, 256, (total,), dtype=torch.uint8).pin_memory()
    pageable = torch.empty(total, dtype=torch.uint8)
    pageable.copy_(pinned)
    row = {"mode": mode, "cpus": len(os.sched_getaffinity(0))}
    part = 64 << 10
    n = total // part
    for mem, host in (("pinned", pinned), ("pageable", pageable)):
        row[mem + "_pages"] = page_nodes(host.data_ptr(), total)
        ptrs, lens = [host.data_ptr() + i * part for i in range(n)], [part] * n
        cb = eng.CpuBatch(eng.CRC32C, ptrs, lens, threads=threads)
        row[mem + "_cpu_batch"] = rate(cb.run, total)
        job = eng.HostJob(eng.CRC32C, ptrs, lens, ndevices=-1, host_threads=-1)
        row[mem + "_host_only"] = rate(job.run, total)
    print(json.dumps(row), flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2], int(os.environ.get("NUMA_PROBE_MIB", "1280")))
        return
    nodes = node_cpus()
    print(json.dumps({"nodes": {k: len(v) for k, v in nodes.items()},
                      "allowed": len(os.sched_getaffinity(0))}), flush=True)
    rc = 0
    modes = os.environ.get("NUMA_PROBE_MODES") or ",".join(["all"] + [f"node{k}" for k in sorted(nodes)] + ["all"])
    for mode in modes.split(","):
        r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", mode], timeout=240)
        rc = rc or r.returncode
        if r.returncode:
            break
    sys.exit(rc)


if __name__ == "__main__":
    main()
