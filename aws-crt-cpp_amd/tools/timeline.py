#!/usr/bin/env python3
"""Diagnostics: per-wave timeline of the braided CRC32C scan (AMDCRC_DEBUG bit 4).

Launches the C2 batch (1024 x 64 KiB by default) a few times, then reads the 4 s_memrealtime
stamps (100 MHz, chip-wide) each wave wrote on the last launch: start, LDS tables built, scan
loop done, exit.  Prints the phase durations and the start/end skew across waves.
"""
import argparse
import ctypes
import os
import sys

os.environ["AMDCRC_DEBUG"] = str(int(os.environ.get("AMDCRC_DEBUG", "0")) | 16)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import aws_crt_amd as A  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buffers", type=int, default=1024)
    ap.add_argument("--buffer-bytes", type=int, default=65536)
    ap.add_argument("--launches", type=int, default=20)
    a = ap.parse_args()
    n, L = a.buffers, a.buffer_bytes
    data = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    for _ in range(a.launches):
        A.checksum_strided(A.CRC32C, data, L, L, n, out=out)
    torch.cuda.synchronize()
    lib = A.lib()
    lib.aws_crt_amd_debug_timeline.restype = ctypes.c_size_t
    lib.aws_crt_amd_debug_timeline.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    cap = 256 * 16
    buf = np.zeros(cap * 4, dtype=np.uint64)
    w = lib.aws_crt_amd_debug_timeline(buf.ctypes.data, cap)
    t = buf[: w * 4].reshape(w, 4).astype(np.int64)
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    us = (t - t0) * 0.01  # 100 MHz ticks -> us
    ph = np.diff(us, axis=1)
    pct = lambda v: " ".join(f"{q:6.2f}" for q in np.percentile(v, [0, 10, 50, 90, 100]))
    print(f"waves {len(t)}   (percentiles 0/10/50/90/100, microseconds)")
    print(f"start offset      {pct(us[:, 0])}")
    print(f"prologue (tables) {pct(ph[:, 0])}")
    print(f"scan loop         {pct(ph[:, 1])}")
    print(f"finish/combine    {pct(ph[:, 2])}")
    print(f"end offset        {pct(us[:, 3])}")
    print(f"kernel span (first start -> last end) {us[:, 3].max():.2f} us")


if __name__ == "__main__":
    main()
