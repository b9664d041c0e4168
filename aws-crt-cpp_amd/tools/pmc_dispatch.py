#!/usr/bin/env python3
"""Per-dispatch view of a rocprofv3 --pmc counter CSV: duration, effective shader clock
(GRBM_GUI_ACTIVE / 8 XCDs / duration) and the wave-cycle fractions, one line per dispatch of the scan
kernels (grid >= --min-grid), so that sustained launches' clock-down shows dispatch by dispatch.

    python aws-crt-cpp_amd/tools/pmc_dispatch.py <run_counter_collection.csv> [--min-grid 100000]
"""
import csv
import sys
from collections import defaultdict


def main(path, min_grid):
    rows = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if int(r["Grid_Size"]) < min_grid:
            continue
        d = rows[int(r["Dispatch_Id"])]
        d["name"] = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")[:44]
        d["dur_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for k in sorted(rows):
        d = rows[k]
        if "at::" in d["name"] or "rocclr" in d["name"]:
            continue
        wc = max(d.get("SQ_WAVE_CYCLES", 0.0), 1.0)
        clk = d.get("GRBM_GUI_ACTIVE", 0.0) / 8 / (d["dur_us"] * 1e3)
        extra = "  ".join(f"{c[3:].lower()} {d[c] / wc:.3f}" for c in ("SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if c in d)
        print(f"{k:4d}  {d['name']:44s}  {d['dur_us']:9.1f} us  clk {clk:5.2f} GHz  {extra}")


if __name__ == "__main__":
    mg = int(sys.argv[sys.argv.index("--min-grid") + 1]) if "--min-grid" in sys.argv else 100000
    main(sys.argv[1], mg)
