#!/usr/bin/env python3
"""Where the time of a driver-shaped timed region goes (C2, 20 queued batches in one launch):
host time inside the submission call, dispatch duration (hipExtLaunchKernel events), and the
synchronised wall time of the whole region, each the median of `reps` repetitions."""
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

import aws_crt_amd as eng  # noqa: E402


def main(nbatch=20, reps=30):
    eng.init()
    L, count = 65536, 1024
    step = L * count
    data = torch.randint(0, 256, (nbatch * step,), dtype=torch.uint8, device="cuda")
    outs = [torch.empty(count, dtype=torch.int32, device="cuda") for _ in range(nbatch)]
    st = torch.cuda.Stream()
    bs = eng.BatchSet(eng.CRC32C, [(data.data_ptr() + i * step, None, outs[i]) for i in range(nbatch)], L, L, count)
    small = eng.BatchSet(eng.CRC32C, [(data.data_ptr(), None, outs[0])], 4096, 4096, 16)
    for _ in range(5):
        bs.run(st)
        small.run(st)
    torch.cuda.synchronize()
    res = {}
    for name, b in (("c2_20_batches", bs), ("tiny_16x4KiB", small)):
        call, wall, kern = [], [], []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            b.run(st)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            call.append((t1 - t0) * 1e6)
            wall.append((t2 - t0) * 1e6)
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            e1.record(st)
            eng.time_next_launch(e0, e1)
            b.run(st)
            torch.cuda.synchronize()
            kern.append(eng.event_ms(e0, e1) * 1e3)
        # one repetition measured every way: marker events before / after the launch on the stream,
        # the dispatch's own start / end stamps, and the host wall time
        pre, post, gap0, gap1, same = [], [], [], [], []
        for _ in range(reps):
            m0, m1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            e1.record(st)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m0.record(st)
            eng.time_next_launch(e0, e1)
            b.run(st)
            m1.record(st)
            torch.cuda.synchronize()
            w = (time.perf_counter() - t0) * 1e6
            k = eng.event_ms(e0, e1) * 1e3
            same.append(w - k)
            pre.append(m0.elapsed_time(m1) * 1e3)
            gap0.append(eng.event_ms(m0, e0) * 1e3)
            gap1.append(eng.event_ms(e1, m1) * 1e3)
        res[name] = {"host_call_us": round(statistics.median(call), 2), "wall_us": round(statistics.median(wall), 2),
                     "kernel_us": round(statistics.median(kern), 2),
                     "same_rep_wall_minus_kernel_us": round(statistics.median(same), 2),
                     "marker_to_marker_us": round(statistics.median(pre), 2),
                     "marker_to_dispatch_start_us": round(statistics.median(gap0), 2),
                     "dispatch_end_to_marker_us": round(statistics.median(gap1), 2)}
        res[name]["wall_minus_kernel_us"] = round(res[name]["wall_us"] - res[name]["kernel_us"], 2)
        print(name, res[name], flush=True)
    # the synchronise round trip alone
    sy = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        sy.append((time.perf_counter() - t0) * 1e6)
    res["idle_synchronize_us"] = round(statistics.median(sy), 2)
    print(json.dumps(res))


def set_sched(mode):
    """hipSetDeviceFlags before the device's context exists (AMDCRC_PROBE_SCHED=spin|yield|blocking):
    how the host waits in hipDeviceSynchronize -- the completion-to-host leg of a timed region"""
    import ctypes

    flags = {"auto": 0, "spin": 1, "yield": 2, "blocking": 4}[mode]
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(flags))
    print(json.dumps({"sched": mode, "hipSetDeviceFlags_rc": rc}), flush=True)


if __name__ == "__main__":
    if os.environ.get("AMDCRC_PROBE_SCHED"):
        set_sched(os.environ["AMDCRC_PROBE_SCHED"])
    main(*(int(a) for a in sys.argv[1:]))
