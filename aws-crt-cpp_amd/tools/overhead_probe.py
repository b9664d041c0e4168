#!/usr/bin/env python3
"""Where the time of a driver-shaped timed region goes (C2, 20 batches in one launch), per submission
path, each figure the median of `reps` repetitions:

  host_call_us   Python + C ABI + HIP launch call (perf_counter around the submission)
  wall_us        synchronize; t0; submit; synchronize; t1  (bench.py's timed region)
  kernel_us      the dispatch's own interval (hipExtLaunchKernel events, aws_crt_amd_debug_time_next_launch)
  outside_us     wall - kernel of the same repetition

Paths: "batches" = aws_crt_amd_checksum_batches with prepared ctypes arguments (round 3's bench),
"plan" = aws_crt_amd_plan_launch of a prepared plan (round 4's bench).  The process's HIP runtime
settings (environment) are printed with the result, so runs under different settings compare.

    python aws-crt-cpp_amd/tools/overhead_probe.py [nbatch] [reps]
"""
import ctypes
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def set_sched(mode):
    """hipSetDeviceFlags before the device's context exists (AMDCRC_PROBE_SCHED=spin|yield|blocking):
    how the host waits in hipDeviceSynchronize -- the completion-to-host leg of a timed region"""
    flags = {"auto": 0, "spin": 1, "yield": 2, "blocking": 4}[mode]
    import torch  # noqa: F401  (loads torch's HIP runtime; no device call yet)
    hip = ctypes.CDLL("libamdhip64.so")
    return hip.hipSetDeviceFlags(ctypes.c_uint(flags))


def main(nbatch=20, reps=40):
    sched_rc = set_sched(os.environ["AMDCRC_PROBE_SCHED"]) if os.environ.get("AMDCRC_PROBE_SCHED") else None
    import torch

    import aws_crt_amd as eng

    eng.init()
    L, count = 65536, 1024
    step = L * count
    data = torch.randint(0, 256, (nbatch * step,), dtype=torch.uint8, device="cuda")
    outs = [torch.empty(count, dtype=torch.int32, device="cuda") for _ in range(nbatch)]
    st = torch.cuda.Stream()
    batches = [(data.data_ptr() + i * step, None, outs[i]) for i in range(nbatch)]
    plan = eng.BatchSet(eng.CRC32C, batches, L, L, count)
    lib = eng.lib()
    arr = (eng._Batch * nbatch)()
    for i, (b, _, o) in enumerate(batches):
        arr[i].d_base, arr[i].d_seeds, arr[i].d_out = b, None, o.data_ptr()
    fn = lib.aws_crt_amd_checksum_batches
    fn.argtypes = [ctypes.c_int, ctypes.POINTER(eng._Batch), ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                   ctypes.c_size_t, ctypes.c_void_p]
    sh = st.cuda_stream
    paths = {"batches": lambda: fn(eng.CRC32C, arr, nbatch, L, L, count, sh),
             "plan": lambda: plan.fn(plan._plan, sh),
             "batchset_run": lambda: plan.run(st)}  # bench.py's call: the plan plus record_stream
    for f in paths.values():
        for _ in range(3):
            f()
    torch.cuda.synchronize()
    res = {"env": {k: os.environ[k] for k in sorted(os.environ) if k.startswith(("ROC_", "HIP_", "HSA_", "DEBUG_CLR", "AMDCRC_"))},
           "sched_rc": sched_rc}
    acc = {name: ([], [], [], [], []) for name in paths}
    for _ in range(reps):  # the paths interleaved rep by rep (clock and box drift hit both alike)
        for name, f in paths.items():
            call, wall, outside, kern, wall_plain = acc[name]
            # as bench.py's timed region: no events on the launch
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f()
            torch.cuda.synchronize()
            wall_plain.append((time.perf_counter() - t0) * 1e6)
            # the same with the dispatch stamping its own start / end
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            e1.record(st)
            torch.cuda.synchronize()
            eng.time_next_launch(e0, e1)
            t0 = time.perf_counter()
            f()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            k = eng.event_ms(e0, e1) * 1e3
            call.append((t1 - t0) * 1e6)
            wall.append((t2 - t0) * 1e6)
            kern.append(k)
            outside.append((t2 - t0) * 1e6 - k)
    for name in paths:
        call, wall, outside, kern, wall_plain = acc[name]
        med = lambda v: round(statistics.median(v), 2)  # noqa: E731
        res[name] = {"host_call_us": med(call), "wall_us": med(wall_plain), "wall_min_us": round(min(wall_plain), 2),
                     "gibs_median": round(nbatch * step / (statistics.median(wall_plain) * 1e-6) / 2**30, 1),
                     "timed_wall_us": med(wall), "kernel_us": med(kern), "outside_us": med(outside)}
    sy = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        sy.append((time.perf_counter() - t0) * 1e6)
    res["idle_synchronize_us"] = round(statistics.median(sy), 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
