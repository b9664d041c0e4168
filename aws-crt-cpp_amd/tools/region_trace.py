#!/usr/bin/env python3
"""Decompose bench.py's timed region from a rocprofv3 kernel + HIP API trace of the same command
(DESIGN.md §5 "Where the timed region goes").

    rocprofv3 --kernel-trace --hip-trace -d DIR -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5
    python aws-crt-cpp_amd/tools/region_trace.py DIR/.../run_kernel_trace.csv DIR/.../run_hip_api_trace.csv

bench.py's timed region is `torch.cuda.synchronize(); t0; <submission calls>; torch.cuda.synchronize(); t1`.
The headline launch is the first dispatch of the dominant kernel longer than --min-us.  Its HIP API
launch call is found by correlation id; the region is bracketed by the hipDeviceSynchronize that
ends before that call and the first one that ends after the kernel.  Printed (us):

  host_pre      previous synchronize returns -> launch API call begins (Python, ctypes, engine planning)
  launch_api    the launch API call itself
  api_to_kernel launch call returns -> the kernel starts (command processor, dispatch)
  kernel        the dispatch's own interval
  kernel_to_sync_end  kernel ends -> the closing synchronize returns (completion signal, wake-up)
  region        previous synchronize end -> closing synchronize end (what bench.py's clock sees)
"""
import argparse
import csv
import json


def rows(path):
    return list(csv.DictReader(open(path)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel_trace")
    ap.add_argument("hip_trace")
    ap.add_argument("--kernel", default="crc32_stream_kernel")
    ap.add_argument("--min-us", type=float, default=100.0)
    ap.add_argument("--nth", type=int, default=0, help="which qualifying dispatch (0 = the first: the timed region)")
    a = ap.parse_args()
    ks = sorted(rows(a.kernel_trace), key=lambda r: int(r["Start_Timestamp"]))
    hs = sorted(rows(a.hip_trace), key=lambda r: int(r["Start_Timestamp"]))
    hits = [r for r in ks if a.kernel in r["Kernel_Name"]
            and (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 >= a.min_us]
    k = hits[a.nth]
    kb, ke = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
    corr = k["Correlation_Id"]
    launch = next(r for r in hs if r["Correlation_Id"] == corr)
    lb, le = int(launch["Start_Timestamp"]), int(launch["End_Timestamp"])
    syncs = [r for r in hs if r["Function"] in ("hipDeviceSynchronize", "hipStreamSynchronize")]
    pre = max((r for r in syncs if int(r["End_Timestamp"]) <= lb), key=lambda r: int(r["End_Timestamp"]))
    post = min((r for r in syncs if int(r["End_Timestamp"]) >= ke), key=lambda r: int(r["End_Timestamp"]))
    t0, t1 = int(pre["End_Timestamp"]), int(post["End_Timestamp"])
    between = [r for r in hs if t0 <= int(r["Start_Timestamp"]) <= t1]
    calls = {}
    for r in between:
        c = calls.setdefault(r["Function"], [0, 0.0])
        c[0] += 1
        c[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    out = {
        "kernel": k["Kernel_Name"][:80], "launch_function": launch["Function"],
        "host_pre_us": (lb - t0) / 1e3, "launch_api_us": (le - lb) / 1e3, "api_to_kernel_us": (kb - le) / 1e3,
        "kernel_us": (ke - kb) / 1e3, "kernel_to_sync_end_us": (t1 - ke) / 1e3,
        "sync_call_us": (t1 - int(post["Start_Timestamp"])) / 1e3, "region_us": (t1 - t0) / 1e3,
        "api_calls_in_region": {f: {"n": n, "us": round(us, 2)} for f, (n, us) in sorted(calls.items())},
    }
    for key in list(out):
        if key.endswith("_us"):
            out[key] = round(out[key], 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
