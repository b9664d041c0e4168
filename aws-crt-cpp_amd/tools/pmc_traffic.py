#!/usr/bin/env python3
"""HBM bytes per scan launch from a rocprofv3 counter pass, for bench.py's `roofline.traffic`.

    rocprofv3 --pmc FETCH_SIZE -d D -o run --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d D2 ...
    python3 tools/pmc_traffic.py --fetch D/run_counter_collection.csv --rdreq D2/run_counter_collection.csv \
        --workload crc32c:1024x65536 --bytes-per-launch 67108864 --update profiles/pmc_traffic.json

profiles/pmc_traffic.json holds one record per (workload, batches per launch); --update replaces the
record of the same shape and keeps the others.

Corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): FETCH_SIZE is in KiB and on gfx950
reports half the bytes of a wide coalesced streaming read, so bytes = 2 * 1024 * FETCH_SIZE; the
raw fabric read requests cross-check it: bytes = 128 * (RDREQ - RDREQ_32B) + 32 * RDREQ_32B.
"""
import argparse
import csv
import json
import statistics


def per_dispatch(path, kernel_substr, grid=None):
    vals = {}
    for r in csv.DictReader(open(path)):
        if kernel_substr not in r["Kernel_Name"] or (grid and int(r["Grid_Size"]) != grid):
            continue
        vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--rdreq")
    ap.add_argument("--kernel", default="crc32_stream_kernel")
    ap.add_argument("--grid", type=int, help="only dispatches of this grid size (work-items): the launch shape measured")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--bytes-per-launch", type=int, required=True)
    ap.add_argument("--batches-per-launch", type=int, default=1)
    ap.add_argument("--source", default="", help="where the counter CSV came from (recorded in the output)")
    ap.add_argument("--update", help="JSON file of records to add this record to (replacing the same shape)")
    a = ap.parse_args()
    f = per_dispatch(a.fetch, a.kernel, a.grid)["FETCH_SIZE"]
    fetch_bytes = 2 * 1024 * statistics.median(f)
    rec = {"workload": a.workload, "batches_per_launch": a.batches_per_launch, "source": a.source,
           "kernel": a.kernel, "grid_size": a.grid, "dispatches": len(f),
           "hbm_bytes_per_launch": round(fetch_bytes), "algorithmic_bytes_per_launch": a.bytes_per_launch,
           "traffic_over_algorithmic": round(fetch_bytes / a.bytes_per_launch, 4),
           "method": "2 x 1024 x median FETCH_SIZE per dispatch (gfx950 half-count correction)"}
    if a.rdreq:
        r = per_dispatch(a.rdreq, a.kernel, a.grid)
        req = statistics.median(r["TCC_EA0_RDREQ_sum"])
        req32 = statistics.median(r.get("TCC_EA0_RDREQ_32B_sum", [0.0]))
        rec["rdreq_bytes_per_launch"] = round(128 * (req - req32) + 32 * req32)
    print(json.dumps(rec, indent=1))
    if a.update:
        try:
            doc = json.load(open(a.update))
        except FileNotFoundError:
            doc = {"records": []}
        recs = doc["records"] if "records" in doc else [doc]
        recs = [r for r in recs if (r.get("workload"), r.get("batches_per_launch", 1)) !=
                (rec["workload"], rec["batches_per_launch"])] + [rec]
        with open(a.update, "w") as fh:
            json.dump({"records": recs}, fh, indent=1)
            fh.write("\n")


if __name__ == "__main__":
    main()
