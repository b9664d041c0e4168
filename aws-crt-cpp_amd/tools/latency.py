#!/usr/bin/env python3
"""Single-call latency of the value-only ABI (aws_checksums_crc32c_ex / crc64nvme_ex, the call
Aws::Crt::Checksum::ComputeCRC32C makes, source/checksum/CRC.cpp:20-23) for host buffers on the host
path and on the GPU path (dispatch forced), and for device-resident buffers (always the GPU).
The dispatch crossover in DESIGN.md §1 comes from this table.

    python aws-crt-cpp_amd/tools/latency.py > profiles/r02/latency.json
"""
import ctypes
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402

import aws_crt_amd as eng  # noqa: E402


def timed(fn, min_s=0.3, max_calls=200000):
    fn()
    ts = []
    t_end = time.perf_counter() + min_s
    while time.perf_counter() < t_end and len(ts) < max_calls:
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def main():
    L = eng.lib()
    gpu = eng.device_count() > 0
    if gpu:
        import torch

        eng.init()
    rows = []
    for alg in ("crc32c", "crc64nvme"):
        f = getattr(L, f"aws_checksums_{alg}_ex")
        for n in (32, 4096, 1 << 20, 64 << 20):
            h = np.frombuffer(np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes(), dtype=np.uint8)
            p = h.ctypes.data
            row = {"alg": alg, "bytes": n}
            eng.set_dispatch(eng.DISPATCH_CPU)
            cpu_s = timed(lambda: f(p, n, 0))
            want = f(p, n, 0)
            row["host_buffer_cpu_us"] = round(cpu_s * 1e6, 3)
            row["host_buffer_cpu_gibs"] = round(n / cpu_s / 2**30, 2)
            if gpu:
                eng.set_dispatch(eng.DISPATCH_GPU)
                before = eng.fallback_count()
                g_s = timed(lambda: f(p, n, 0))
                assert f(p, n, 0) == want and eng.fallback_count() == before
                row["host_buffer_gpu_us"] = round(g_s * 1e6, 3)
                row["host_buffer_gpu_gibs"] = round(n / g_s / 2**30, 2)
                d = torch.from_numpy(h.copy()).cuda()
                torch.cuda.synchronize()
                dp = d.data_ptr()
                dev_s = timed(lambda: f(dp, n, 0))
                assert f(dp, n, 0) == want
                row["device_buffer_gpu_us"] = round(dev_s * 1e6, 3)
                row["device_buffer_gpu_gibs"] = round(n / dev_s / 2**30, 2)
            rows.append(row)
    eng.set_dispatch(eng.DISPATCH_AUTO)
    print(json.dumps({"cpu_tier": eng.cpu_tier(), "rows": rows,
                      "note": "median wall time of one synchronous call from Python (ctypes ~0.3 us included)"}, indent=1))


if __name__ == "__main__":
    main()
