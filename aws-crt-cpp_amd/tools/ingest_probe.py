#!/usr/bin/env python3
"""Host-ingest throughput probe (aws_crt_amd_host_submit / job_wait): GiB/s for several part shapes
from pinned and pageable host memory, beside the plain H2D rate of the same bytes."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

import aws_crt_amd as eng  # noqa: E402


def main():
    eng.init()
    total = 4 << 30
    pinned = torch.randint(0, 256, (total,), dtype=torch.uint8).pin_memory()
    pageable = torch.empty(512 << 20, dtype=torch.uint8)
    pageable.copy_(pinned[: 512 << 20])
    out = []
    for name, host, part in [("pinned 64 KiB parts", pinned, 64 << 10), ("pinned 1 MiB parts", pinned, 1 << 20),
                             ("pinned 32 MiB parts", pinned, 32 << 20), ("pinned 256 MiB parts", pinned, 256 << 20),
                             ("pageable 1 MiB parts", pageable, 1 << 20), ("pinned 8 KiB parts (C4 shape)", pinned, 8 << 10)]:
        n = host.numel() // part
        job = eng.HostJob(eng.CRC32C, [host.data_ptr() + i * part for i in range(n)], [part] * n)
        job.run()  # warm
        t0 = time.perf_counter()
        job.run()
        el = time.perf_counter() - t0
        out.append({"shape": name, "bytes": n * part, "gibs": round(n * part / el / 2**30, 2)})
        print(out[-1], flush=True)
    dev = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(total // (256 << 20)):
        dev.copy_(pinned[i * (256 << 20):(i + 1) * (256 << 20)], non_blocking=True)
    torch.cuda.synchronize()
    out.append({"shape": "H2D only (torch, 256 MiB copies)", "bytes": total, "gibs": round(total / (time.perf_counter() - t0) / 2**30, 2)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
