#!/usr/bin/env python3
"""Per-kernel-shape medians of a rocprofv3 --pmc counter CSV (one or more passes over the same
program): dispatches grouped by (kernel, grid size), counters summed over a dispatch's rows (XCDs /
shader engines), then the median over the group's dispatches, with derived figures:

    clk_ghz_est   GRBM_GUI_ACTIVE / 8 XCDs / the dispatch's duration (when the CSV carries timestamps)
    wave_busy     SQ_BUSY_CYCLES per wave cycle, issue and wait buckets as fractions of SQ_WAVE_CYCLES
    lds_conflict  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra LDS cycles per LDS-array cycle)
    valu_per_lds  SQ_INSTS_VALU / SQ_INSTS_LDS

    python aws-crt-cpp_amd/tools/pmc_group.py <counter_collection.csv> [more.csv ...] [--min-grid N]
"""
import csv
import json
import re
import statistics
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    return re.sub(r"\(.*", "", name).strip()


def main(paths, min_grid=0):
    groups = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # (kernel, grid) -> dispatch -> counter
    dur = defaultdict(dict)
    for path in paths:
        for r in csv.DictReader(open(path)):
            key = (short(r["Kernel_Name"]), int(r.get("Grid_Size", 0) or 0))
            if key[1] < min_grid:
                continue
            did = (path, r["Dispatch_Id"])
            groups[key][did][r["Counter_Name"]] += float(r["Counter_Value"])
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                dur[key][did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = []
    for key, per in sorted(groups.items()):
        names = sorted({c for d in per.values() for c in d})
        med = {c: statistics.median(d[c] for d in per.values() if c in d) for c in names}
        rec = {"kernel": key[0], "grid": key[1], "dispatches": len(per), "counters": {c: round(v) for c, v in med.items()}}
        ds = list(dur[key].values())
        if ds:
            rec["duration_us"] = round(statistics.median(ds) * 1e6, 2)
            if "GRBM_GUI_ACTIVE" in med:
                rec["clk_ghz_est"] = round(med["GRBM_GUI_ACTIVE"] / 8 / statistics.median(ds) / 1e9, 3)
        wc = med.get("SQ_WAVE_CYCLES")
        if wc:
            rec["of_wave_cycles"] = {c: round(med[c] / wc, 4) for c in names if c.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_BUSY"))}
        if med.get("SQ_LDS_IDX_ACTIVE"):
            rec["lds_conflict"] = round(med.get("SQ_LDS_BANK_CONFLICT", 0) / med["SQ_LDS_IDX_ACTIVE"], 4)
        if med.get("SQ_INSTS_LDS") and med.get("SQ_INSTS_VALU"):
            rec["valu_per_lds"] = round(med["SQ_INSTS_VALU"] / med["SQ_INSTS_LDS"], 3)
        out.append(rec)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    mg = 0
    if "--min-grid" in sys.argv:
        mg = int(sys.argv[sys.argv.index("--min-grid") + 1])
        args = [a for a in args if a != str(mg)]
    main(args, mg)
