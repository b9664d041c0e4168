#!/usr/bin/env python3
"""Median per-dispatch SQ counters of one kernel from a rocprofv3 --pmc CSV, with the wave-cycle
buckets as fractions (SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~ SQ_WAVE_CYCLES)."""
import csv
import statistics
import sys
from collections import defaultdict


def main(path, kernel):
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    names = sorted({c for d in per.values() for c in d})
    med = {c: statistics.median(d[c] for d in per.values()) for c in names}
    wc = med.get("SQ_WAVE_CYCLES", 0)
    print(f"{kernel}: {len(per)} dispatches")
    for c in names:
        frac = f"  ({med[c] / wc:.3f} of wave cycles)" if wc and c.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
        print(f"  {c:24s} {med[c]:16.0f}{frac}")
    if "SQ_INSTS_VALU" in med and "SQ_INSTS_LDS" in med:
        print(f"  VALU / LDS instructions: {med['SQ_INSTS_VALU'] / max(med['SQ_INSTS_LDS'], 1):.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
