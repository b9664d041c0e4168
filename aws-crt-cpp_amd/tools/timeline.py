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
    buf = np.zeros(cap * 8, dtype=np.uint64)
    w = lib.aws_crt_amd_debug_timeline(buf.ctypes.data, cap)
    t8 = buf[: w * 8].reshape(w, 8).astype(np.int64)
    valid = t8[:, 0] > 0
    t = t8[valid][:, :4]
    cst = (t8[valid][:, 4] - t8[valid][:, 0]) * 0.01
    t0 = t[:, 0].min()
    us = (t - t0) * 0.01  # 100 MHz ticks -> us
    ph = np.diff(us, axis=1)
    pct = lambda v: " ".join(f"{q:6.2f}" for q in np.percentile(v, [0, 10, 50, 90, 100]))
    print(f"waves {len(t)}   (percentiles 0/10/50/90/100, microseconds)")
    print(f"start offset      {pct(us[:, 0])}")
    print(f"constants arrived {pct(cst)}")
    print(f"prologue (tables) {pct(ph[:, 0])}")
    print(f"scan loop         {pct(ph[:, 1])}")
    print(f"finish/combine    {pct(ph[:, 2])}")
    print(f"end offset        {pct(us[:, 3])}")
    print(f"kernel span (first start -> last end) {us[:, 3].max():.2f} us")
    # where does the spread live?  by workgroup (CU) and by XCD (workgroups go round-robin to the
    # 8 XCDs), and by position of the wave's tile in the address space
    scan = ph[:, 1]
    wid = np.nonzero(valid)[0]
    blk = wid // 16
    nb = blk.max() + 1
    blk_mean = np.array([scan[blk == b].mean() for b in range(nb)])
    within = np.mean([scan[blk == b].std() for b in range(nb)])
    print(f"scan by workgroup: mean-of-means {blk_mean.mean():.1f}, spread of WG means (std) {blk_mean.std():.1f}, "
          f"mean within-WG std {within:.1f}")
    for x in range(8):
        sel = (blk % 8) == x
        print(f"  xcd {x}: scan mean {scan[sel].mean():7.1f}  p90 {np.percentile(scan[sel], 90):7.1f}  "
              f"end max {us[sel, 3].max():7.1f}")
    q = len(scan) // 8
    print("scan by address octile (wave order):", " ".join(f"{scan[i*q:(i+1)*q].mean():.1f}" for i in range(8)))
    slow = np.argsort(blk_mean)[-8:]
    print("slowest WGs:", " ".join(f"{b}({blk_mean[b]:.0f})" for b in slow))


if __name__ == "__main__":
    main()
