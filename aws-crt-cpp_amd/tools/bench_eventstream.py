#!/usr/bin/env python3
"""Event-stream framing CRCs: N framed messages of random length packed
back to back in one device buffer, 2N CRC32 spans per call through the ragged list path
(aws_crt_amd/eventstream.py).  Prints one JSON line: pipelined GiB/s of CRC'd bytes (Σ span
lengths), messages/s, host time per call (descriptor staging included) and the isolated kernel time.

  python aws-crt-cpp_amd/tools/bench_eventstream.py [--messages 131072 --min-bytes 16 --max-bytes 1024]
"""
import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
import aws_crt_amd as A  # noqa: E402
from aws_crt_amd.eventstream import FrameBatch  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--messages", type=int, default=131072)
    ap.add_argument("--min-bytes", type=int, default=16)
    ap.add_argument("--max-bytes", type=int, default=1024)
    ap.add_argument("--batches", type=int, default=6, help="rotating copies (6 x 65 MiB exceeds the 256 MiB Infinity Cache)")
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--timing-launches", type=int, default=8)
    ap.add_argument("--timing-only", action="store_true",
                    help="skip the zlib check (A/B builds whose results are wrong by design: experiments/patches)")
    ap.add_argument("--no-hold", action="store_true",
                    help="time the launches without the GPU-side hold in front of them (the probe's way)")
    ap.add_argument("--gap-max", type=int, default=0,
                    help="random gaps of 0..N bytes between messages (frames not packed back to back)")
    ap.add_argument("--device-frames", action="store_true",
                    help="aws_crt_amd_eventstream_crcs: device offsets, lengths read from the preludes, CRCs checked")
    a = ap.parse_args()
    A.init()
    rng = random.Random(0xE5)
    lens = [rng.randint(a.min_bytes, a.max_bytes) for _ in range(a.messages)]
    offs, pos = [], 0
    for n in lens:
        offs.append(pos)
        pos += n + (rng.randint(0, a.gap_max) if a.gap_max else 0)
    data = torch.randint(0, 256, (a.batches * pos,), dtype=torch.uint8, device="cuda")
    fbs = [FrameBatch(data.data_ptr() + b * pos, offs, lens) for b in range(a.batches)]
    for fb in fbs:
        fb.device = data.device
    outs = [torch.empty(fbs[0].n, dtype=torch.int32, device="cuda") for _ in range(a.batches)]
    if a.device_frames:
        # write each message's total_length into its prelude (big-endian), one batch copy per slot
        import numpy as np
        import ctypes

        # prelude: total_length (big-endian) and headers_length = 0, so every frame is well formed and
        # is CRC'd (a random headers_length > total - 16 would be flagged malformed and skipped)
        hdr = np.zeros(pos, dtype=np.uint8)
        be = np.concatenate([np.array(lens, dtype=">u4").view(np.uint8).reshape(-1, 4),
                             np.zeros((len(lens), 4), dtype=np.uint8)], axis=1)
        idx = np.array(offs, dtype=np.int64)[:, None] + np.arange(8)[None, :]
        hdr[idx.ravel()] = be.ravel()
        hd = torch.from_numpy(hdr).cuda()
        mask = torch.zeros(pos, dtype=torch.bool, device="cuda")
        mask[torch.from_numpy(idx.ravel()).cuda()] = True
        for b in range(a.batches):
            data[b * pos:(b + 1) * pos][mask] = hd[mask]
        o_dev = torch.tensor(offs, dtype=torch.int64, device="cuda")
        f = A.lib().aws_crt_amd_eventstream_crcs
        f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t] + [ctypes.c_void_p] * 4
        res = [[torch.empty(a.messages, dtype=torch.int32, device="cuda") for _ in range(3)] for _ in range(a.batches)]

        class _Dev:
            def __init__(self, b):
                self.b = b
                self.n = 2 * a.messages
                self.payload_bytes = sum(lens) - 4 * a.messages  # bytes CRC'd: [0, total - 4) of each message

            def run(self, out, stream):
                r = res[self.b]
                A._check(f(data.data_ptr() + self.b * pos, pos, o_dev.data_ptr(), a.messages, r[0].data_ptr(),
                           r[1].data_ptr(), r[2].data_ptr(), stream.cuda_stream))

        fbs = [_Dev(b) for b in range(a.batches)]
    streams = [torch.cuda.Stream() for _ in range(a.streams)]
    for i in range(max(a.batches, a.streams) * 2):
        fbs[i % a.batches].run(outs[i % a.batches], streams[i % a.streams])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = 0.0
    for i in range(a.steps):
        h0 = time.perf_counter()
        fbs[i % a.batches].run(outs[i % a.batches], streams[i % a.streams])
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st = streams[0]
    nt = a.timing_launches
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(nt)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(nt)]
    if not a.no_hold:  # queue the timed launches behind a GPU-side hold so they run back to back
        with torch.cuda.stream(st):
            torch.cuda._sleep(int(40e6))
    for i in range(nt):
        starts[i].record(st)
        ends[i].record(st)
        A.time_next_launch(starts[i], ends[i])
        fbs[i % a.batches].run(outs[i % a.batches], st)
    torch.cuda.synchronize()
    kms = sum(A.event_ms(s, e) for s, e in zip(starts, ends)) / nt
    nbytes = fbs[0].payload_bytes
    if a.device_frames:
        # spot check of batch 0 against zlib (the library build under test may be an A/B variant)
        import zlib
        host_b = data[:pos].cpu().numpy().tobytes()
        pre_d, msg_d = (res[0][k].cpu().numpy().view("uint32") for k in (0, 1))
        for m in rng.sample(range(a.messages), min(4096, a.messages)):
            o, n = offs[m], lens[m]
            if not a.timing_only and (zlib.crc32(host_b[o:o + 8]) != int(pre_d[m]) or
                                      zlib.crc32(host_b[o:o + n - 4]) != int(msg_d[m])):
                raise SystemExit(f"event-stream CRC mismatch at message {m} (offset {o}, {n} bytes)")
    print(json.dumps({
        "workload": f"event-stream framing: {a.messages} messages of {a.min_bytes}..{a.max_bytes} B "
                    f"({pos / 2**20:.1f} MiB), {fbs[0].n} CRC32 spans per call, "
                    + ("device framing check (eventstream_crcs)" if a.device_frames else "list path"),
        "value": round(a.steps * nbytes / el / 2**30, 2), "unit": "GiB/s (CRC'd bytes)",
        "messages_per_s": round(a.steps * a.messages / el), "host_ms_per_call": round(host / a.steps * 1e3, 4),
        "ms_per_call": round(el / a.steps * 1e3, 4), "kernel_ms": round(kms, 4),
        "kernel_gbs": round(nbytes / (kms * 1e-3) / 1e9, 1),
        "roofline_frac": round(nbytes / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "streams": a.streams}), flush=True)


if __name__ == "__main__":
    main()
