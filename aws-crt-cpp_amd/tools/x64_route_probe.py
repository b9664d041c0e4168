"""Where the XXH64 host route's time goes on this box: the C5 shape (8 x 64 MiB) as
  d2h_1d    one 512 MiB device-to-host copy into pinned memory
  d2h_2d    the route's copies alone: 16 slices, each one hipMemcpy2DAsync of 8 rows x 4 MiB (source
            pitch 64 MiB) into one of two 32 MiB pinned halves, back to back on one stream
  d2h_rows  the same slices as 8 one-dimensional copies each
  host      the route's hashing alone: 8 host threads (the engine's pool), 64 MiB each, from pinned
  route     the route itself (aws_crt_amd checksum_batches, XXH64), AWS_CRT_AMD_X64_TRACE=1 on stderr
GiB/s of the 512 MiB per rep, median of --reps.

    python aws-crt-cpp_amd/tools/x64_route_probe.py [--reps 5]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

os.environ.setdefault("AWS_CRT_AMD_X64_TRACE", "1")
import torch  # noqa: E402

import aws_crt_amd as eng  # noqa: E402
import bench  # noqa: E402

N, L = 8, 64 << 20
HALF = 32 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    eng.init()
    dev = torch.device("cuda", 0)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy2DAsync.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                     ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    D2H = 2
    st = torch.cuda.Stream()
    data = torch.randint(0, 256, (N * L,), dtype=torch.uint8, device=dev)
    pin = torch.empty(N * L, dtype=torch.uint8, pin_memory=True)
    halves = torch.empty(2 * HALF, dtype=torch.uint8, pin_memory=True)
    sl = HALF // N

    def timed(fn):
        out = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            out.append(time.perf_counter() - t0)
        return round(N * L / statistics.median(out) / 2**30, 2)

    def d2h_1d():
        assert hip.hipMemcpyAsync(pin.data_ptr(), data.data_ptr(), N * L, D2H, st.cuda_stream) == 0

    def d2h_2d():
        for k in range(L // sl):
            dst = halves.data_ptr() + (k & 1) * HALF
            assert hip.hipMemcpy2DAsync(dst, sl, data.data_ptr() + k * sl, L, sl, N, D2H, st.cuda_stream) == 0

    def d2h_rows():
        for k in range(L // sl):
            dst = halves.data_ptr() + (k & 1) * HALF
            for i in range(N):
                assert hip.hipMemcpyAsync(dst + i * sl, data.data_ptr() + i * L + k * sl, sl, D2H, st.cuda_stream) == 0

    def host():
        eng.cpu_batch(bench.ALG["xxh64"], [pin.data_ptr() + i * L for i in range(N)], [L] * N, threads=N)

    out = torch.empty(N, dtype=torch.int64, device=dev)

    def route():
        eng.checksum_batches(bench.ALG["xxh64"], [(data.data_ptr(), None, out)], L, L, N, stream=st)

    d2h_1d()
    rec = {"d2h_1d": timed(d2h_1d), "d2h_2d": timed(d2h_2d), "d2h_rows": timed(d2h_rows), "host": timed(host)}
    route()
    torch.cuda.synchronize()
    rec["route"] = timed(route)
    want = eng.cpu_batch(bench.ALG["xxh64"], [pin.data_ptr() + i * L for i in range(N)], [L] * N)
    rec["route_parity"] = eng.as_unsigned(out) == want
    rec["host_threads"] = os.environ.get("OMP_NUM_THREADS")
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
