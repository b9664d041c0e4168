"""Effective shader clock per dispatch from a rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES pass
(scripts/gpu_session.sh clk64 / clk32): GRBM_GUI_ACTIVE / dispatch duration / 8 XCDs ~ MHz for
dispatches long enough that the counting window's edges do not matter (>= 150 us).  Finds power
or current throttling of long launches (back-to-back 10 GiB CRC64 launches).

  python aws-crt-cpp_amd/tools/clock_summary.py <run_counter_collection.csv> [...]
"""
import collections
import csv
import sys


def dispatches(path):
    per = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        d = per.setdefault(int(r["Dispatch_Id"]), {})
        d["name"] = r["Kernel_Name"].replace("void (anonymous namespace)::", "").split("(")[0][:40]
        d["grid"] = int(r["Grid_Size"])
        d["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        d[r["Counter_Name"]] = float(r["Counter_Value"])
    return per


def main():
    for path in sys.argv[1:]:
        print("==", path)
        for k, d in dispatches(path).items():
            if d["us"] < 150 or not ("crc" in d["name"] or "read_ceiling" in d["name"]):
                continue
            print(f"dispatch {k:5d} {d['name']:40s} {d['us']:9.1f} us  ~{d.get('GRBM_GUI_ACTIVE', 0) / d['us'] / 8:6.0f} MHz"
                  f"  SQ_BUSY_CYCLES/us {d.get('SQ_BUSY_CYCLES', 0) / d['us']:7.0f}")


if __name__ == "__main__":
    main()
