#!/usr/bin/env python3
"""Hash paths on device-resident data, one JSON line:

  * xxh64_strided: strided XXH64 batches of N buffers of L bytes through aws_crt_amd_checksum_strided
    (whatever route the library takes: the stream-ordered host route for few long buffers, the
    gfx950 kernels otherwise), GiB/s over `reps` synchronised calls, for each N of --counts;
  * xxh3_stream: the streaming XXH3 object (aws_xxhash3_64_new / update / finalize) fed one device
    chunk of --stream-mib MiB, GiB/s of the update;
  * xxh3_batch: the same bytes as a one-buffer strided XXH3-64 batch (block sums + scramble).

Every result is checked against the engine's host path on the same bytes (copied to host).

    python aws-crt-cpp_amd/tools/hash_probe.py [--counts 8,16,32,48,64] [--mib 16]
"""
import argparse
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import aws_crt_amd as eng  # noqa: E402


class Cursor(ctypes.Structure):
    _fields_ = [("len", ctypes.c_size_t), ("ptr", ctypes.c_void_p)]


class Buf(ctypes.Structure):
    _fields_ = [("len", ctypes.c_size_t), ("buffer", ctypes.c_void_p), ("capacity", ctypes.c_size_t),
                ("allocator", ctypes.c_void_p)]


def main():
    import torch

    ap = argparse.ArgumentParser()
    ap.add_argument("--counts", default="4,8,16,24,32,48,64")
    ap.add_argument("--mib", type=int, default=16, help="bytes per XXH64 buffer (MiB)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--stream-mib", type=int, default=512)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    eng.init()
    L = eng.lib()
    out = {"variant": os.environ.get("VARIANT"), "xxh64_strided": {}}
    Lb = args.mib << 20
    counts = [int(c) for c in args.counts.split(",")]
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    d = torch.randint(0, 256, (max(counts) * Lb,), dtype=torch.uint8, device="cuda", generator=g)
    for n in counts:
        res = eng.checksum_strided(eng.XXH64, d, Lb, Lb, n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            res = eng.checksum_strided(eng.XXH64, d, Lb, Lb, n)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / args.reps
        h = d[: n * Lb].cpu().numpy()
        want = eng.cpu_batch(eng.XXH64, [h.ctypes.data + i * Lb for i in range(n)], [Lb] * n, threads=16)
        out["xxh64_strided"][str(n)] = {"gibs": round(n * Lb / el / 2**30, 2), "ms": round(el * 1e3, 3),
                                        "parity": eng.as_unsigned(res) == want}
    del d
    torch.cuda.empty_cache()
    # streaming XXH3 over one device chunk
    n = args.stream_mib << 20
    d = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    torch.cuda.synchronize()
    L.aws_xxhash3_64_new.restype = ctypes.c_void_p
    L.aws_xxhash3_64_new.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    L.aws_xxhash_update.argtypes = [ctypes.c_void_p, Cursor]
    L.aws_xxhash_finalize.argtypes = [ctypes.c_void_p, ctypes.POINTER(Buf)]
    L.aws_xxhash_destroy.argtypes = [ctypes.c_void_p]

    def stream_once():
        hnd = L.aws_xxhash3_64_new(None, 0)
        t0 = time.perf_counter()
        assert L.aws_xxhash_update(hnd, Cursor(n, d.data_ptr())) == 0
        el = time.perf_counter() - t0
        o = ctypes.create_string_buffer(8)
        b = Buf(0, ctypes.cast(o, ctypes.c_void_p), 8, None)
        assert L.aws_xxhash_finalize(hnd, ctypes.byref(b)) == 0
        L.aws_xxhash_destroy(hnd)
        return int.from_bytes(o.raw, "big"), el

    stream_once()
    els = []
    for _ in range(args.reps):
        v, el = stream_once()
        els.append(el)
    h = d.cpu().numpy()
    want = eng.cpu_batch(eng.XXH3_64, [h.ctypes.data], [n], threads=1)[0]
    out["xxh3_stream"] = {"chunk_mib": args.stream_mib, "gibs": round(n / min(els) / 2**30, 2), "parity": v == want}
    r = eng.checksum_strided(eng.XXH3_64, d, n, n, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        r = eng.checksum_strided(eng.XXH3_64, d, n, n, 1)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / args.reps
    out["xxh3_batch_one_buffer"] = {"gibs": round(n / el / 2**30, 2), "parity": eng.as_unsigned(r)[0] == want}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
