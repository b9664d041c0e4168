"""Does a preceding leg change the XXH64 host route's rate?  Runs bench.py's C5_xxh64 leg alone, then
after the C5 CRC64NVME multi-batch leg (6 GiB launches at the power limit), then after the C5
CRC64NVME leg with its CPU baseline and host-ingest legs, then alone again; prints each leg's value
and roofline fraction (of the D2H rate measured in the same leg).

    python aws-crt-cpp_amd/tools/x64_leg_order.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import torch  # noqa: E402

import aws_crt_amd as eng  # noqa: E402
import bench  # noqa: E402


def x64(tag, streams, dev):
    r = bench.config_leg(eng, "C5", "xxh64", 8, 64 << 20, streams, dev, steps=4, timing=2, do_cpu=False, do_e2e=False)
    print(json.dumps({"order": tag, "value": r["value"], "frac_d2h": r["roofline"]["frac"], "d2h_peak_gbs": r["roofline"]["peak"],
                      "kernel_route": (r.get("kernel_route") or {}).get("value")}), flush=True)


def main():
    eng.init()
    dev = torch.device("cuda:0")
    streams = [torch.cuda.Stream(device=dev) for _ in range(3)]
    x64("alone", streams, dev)
    bench.config_leg(eng, "C5", "crc64nvme", 8, 64 << 20, streams, dev, coalesce=12, timing=2, do_cpu=False, do_e2e=False)
    x64("after C5 multi-batch", streams, dev)
    bench.config_leg(eng, "C5", "crc64nvme", 8, 64 << 20, streams, dev, do_cpu=True, do_e2e=True)
    x64("after C5 crc64nvme with CPU baseline and e2e", streams, dev)
    x64("alone again", streams, dev)


if __name__ == "__main__":
    main()
