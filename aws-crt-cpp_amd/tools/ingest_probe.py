#!/usr/bin/env python3
"""Host-ingest throughput probe: GiB/s of one CRC32C job over host memory, for several part shapes,
pinned and pageable, through

  cpu_batch     aws_crt_amd_cpu_batch (the CPU baseline's call: persistent pool, the CPU share)
  host_only     aws_crt_amd_host_submit_ex, ndevices < 0
  hybrid        aws_crt_amd_host_submit_ex (host threads beside the device lane; the default)
  devices_only  aws_crt_amd_host_submit_ex, host_threads 0

median of `reps` reps of >= 0.2 s after a warm-up each, and the plain H2D rate of the same bytes."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

import aws_crt_amd as eng  # noqa: E402


def best(fn, reps, secs=0.2):
    """seconds per call: the median over `reps` reps of >= secs each (after a warm-up call)"""
    fn()
    ts = []
    for _ in range(reps):
        passes, t0 = 0, time.perf_counter()
        while True:
            fn()
            passes += 1
            el = time.perf_counter() - t0
            if el >= secs:
                break
        ts.append(el / passes)
    ts.sort()
    return ts[len(ts) // 2]


def main(total_mib=1280, reps=5):
    eng.init()
    total = total_mib << 20
    threads = int(os.environ.get("OMP_NUM_THREADS", "16"))
    pinned = torch.randint(0, 256, (total,), dtype=torch.uint8).pin_memory()
    pageable = torch.empty(total, dtype=torch.uint8)
    pageable.copy_(pinned)
    res = []
    mems = os.environ.get("INGEST_PROBE_MEM", "pinned,pageable").split(",")
    for mem, host in ((m, h) for m, h in (("pinned", pinned), ("pageable", pageable)) if m in mems):
        for part in (64 << 10, 8 << 20):
            n = total // part
            ptrs, lens = [host.data_ptr() + i * part for i in range(n)], [part] * n
            row = {"memory": mem, "part_bytes": part, "parts": n}
            cb = eng.CpuBatch(eng.CRC32C, ptrs, lens, threads=threads)
            row["cpu_batch"] = round(total / best(cb.run, reps) / 2**30, 1)
            legs = [("host_only", -1, -1), ("hybrid", 0, -1), ("devices_only", 0, 0)]
            legs += [(f"hybrid_h{h}", 0, h) for h in (int(x) for x in os.environ.get("INGEST_PROBE_H", "").split(",") if x)]
            if os.environ.get("INGEST_PROBE_AGAIN"):
                legs.append(("hybrid_again", 0, -1))  # the default once more, after the other legs
            for name, nd, ht in legs:
                job = eng.HostJob(eng.CRC32C, ptrs, lens, ndevices=nd, host_threads=ht)
                row[name] = round(total / best(job.run, reps) / 2**30, 1)
                if name.startswith("hybrid"):
                    row[name + "_device_share"] = round(job.device_bytes / total, 3)
            res.append(row)
            print(json.dumps(row), flush=True)
    dev = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(total // (256 << 20)):
        dev.copy_(pinned[i * (256 << 20):(i + 1) * (256 << 20)], non_blocking=True)
    torch.cuda.synchronize()
    print(json.dumps({"h2d_only_gibs": round(total / (time.perf_counter() - t0) / 2**30, 1), "threads": threads,
                      "results": res}))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
