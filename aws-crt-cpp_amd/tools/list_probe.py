#!/usr/bin/env python3
"""Ragged-list scans (crc32_braid_kernel<LIST>) against the strided streaming scan on the same bytes:
dispatch-stamped kernel time (median of `reps`) for a few list shapes."""
import json
import os
import random
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

import aws_crt_amd as eng  # noqa: E402


def timed(fn, reps=12):
    out = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        e1.record()
        eng.time_next_launch(e0, e1)
        fn()
        torch.cuda.synchronize()
        out.append(eng.event_ms(e0, e1) * 1e3)
    return statistics.median(out)


def main(alg_name="crc32c"):
    eng.init()
    alg = {"crc32": eng.CRC32, "crc32c": eng.CRC32C, "crc64nvme": eng.CRC64NVME}[alg_name]
    odt = torch.int64 if alg_name == "crc64nvme" else torch.int32
    total = 256 << 20
    data = torch.randint(0, 256, (2 * total + 4096,), dtype=torch.uint8, device="cuda")
    base = data.data_ptr()
    rnd = random.Random(1)
    res = {}
    L = 65536
    n = total // L
    out = torch.empty(n, dtype=odt, device="cuda")
    res["strided_4096x64KiB"] = timed(lambda: eng.checksum_strided(alg, data, L, L, n, out=out))
    ptrs, lens = [base + i * L for i in range(n)], [L] * n
    res["list_4096x64KiB_aligned"] = timed(lambda: eng.checksum_list(alg, ptrs, lens, out=out))
    lens2 = [rnd.randrange(32 << 10, 96 << 10) for _ in range(n)]
    ptrs2, a = [], base + 5
    for ln in lens2:
        ptrs2.append(a)
        a += ln + rnd.randrange(0, 64)
    res["list_4096_ragged_32-96KiB_unaligned"] = timed(lambda: eng.checksum_list(alg, ptrs2, lens2, out=out))
    res["list_ragged_bytes"] = sum(lens2)
    # which of the two costs: raggedness (aligned starts, lengths a multiple of 16) or misalignment
    # (uniform 64 KiB buffers starting 5 bytes past 16-byte alignment)
    lens3 = [16 * rnd.randrange(2 << 10, 6 << 10) for _ in range(n)]
    ptrs3, a = [], base
    for ln in lens3:
        ptrs3.append(a)
        a += ln
    res["list_4096_ragged_aligned"] = timed(lambda: eng.checksum_list(alg, ptrs3, lens3, out=out))
    res["list_4096_ragged_aligned_gibs"] = round(sum(lens3) / (res["list_4096_ragged_aligned"] * 1e-6) / 2**30, 1)
    ptrs4 = [base + 5 + i * L for i in range(n)]
    res["list_4096x64KiB_unaligned"] = timed(lambda: eng.checksum_list(alg, ptrs4, lens, out=out))
    res["list_4096x64KiB_unaligned_gibs"] = round(total / (res["list_4096x64KiB_unaligned"] * 1e-6) / 2**30, 1)
    for k in ("strided_4096x64KiB", "list_4096x64KiB_aligned"):
        res[k + "_gibs"] = round(total / (res[k] * 1e-6) / 2**30, 1)
    res["list_4096_ragged_32-96KiB_unaligned_gibs"] = round(sum(lens2) / (res["list_4096_ragged_32-96KiB_unaligned"] * 1e-6) / 2**30, 1)
    # short ragged lists (the lane-per-buffer scan's domain): 65536 buffers of 1..4 KiB and of 256 B..1 KiB
    for name, lo, hi in (("short_1-4KiB", 1024, 4096), ("short_256B-1KiB", 256, 1024)):
        ls = [rnd.randrange(lo, hi + 1) for _ in range(65536)]
        ps, a = [], base
        for ln in ls:
            ps.append(a)
            a += ln
        o2 = torch.empty(len(ls), dtype=odt, device="cuda")
        res[name] = timed(lambda: eng.checksum_list(alg, ps, ls, out=o2))
        res[name + "_gibs"] = round(sum(ls) / (res[name] * 1e-6) / 2**30, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:])
