#!/usr/bin/env python3
"""Match bench.py's event-timed launches with rocprofv3's kernel trace of the same run (DESIGN.md §6
"rocprof cross-check").

bench.py times every roofline figure with time_launches(): a GPU-side hold (torch.cuda._sleep, the
`spin_kernel` dispatch) followed by N launches serialised on one stream, each stamped by its own
dispatch (hipExtLaunchKernel events).  In a kernel trace of the same command each such section is
therefore a spin_kernel dispatch followed by the section's launches on the same queue.  This script
cuts the trace into those sections, averages each section's dispatch durations and prints them next
to the bench line's kernel_ms values in the order bench.py took them: the headline launch, the
one-batch launch, the two read-ceiling launches, then every config leg.

    python aws-crt-cpp_amd/tools/trace_match.py <run_kernel_trace.csv> <bench log with the JSON line>
"""
import csv
import json
import sys


def sections(trace_csv):
    rows = list(csv.DictReader(open(trace_csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    out, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if "spin_kernel" in name:
            if cur is not None:
                out.append(cur)
            cur = []
            continue
        if cur is None or name.startswith("__amd_rocclr"):
            continue
        cur.append((name, int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    if cur is not None:
        out.append(cur)
    return out


def bench_entries(rec):
    """(label, events kernel_ms, launches timed) in the order bench.py timed them"""
    roof = rec["roofline"]
    nt = roof.get("timing_launches")
    ent = [("headline launch", roof["kernel_ms"], nt, roof.get("kernel"))]
    sb = roof.get("single_batch")
    if sb:
        ent.append(("one-batch launch", sb["kernel_ms"], nt, roof.get("kernel")))
        if "read_ceiling_kernel_ms" in sb:
            ent.append(("read ceiling, one batch", sb["read_ceiling_kernel_ms"], nt, "read_ceiling_kernel"))
    if roof.get("read_ceiling"):
        ent.append(("read ceiling, headline size", roof["read_ceiling"]["kernel_ms"],
                    roof["read_ceiling"].get("timing_launches", max(2, (nt or 8) // 4)), "read_ceiling_kernel"))
    for k, v in (rec.get("configs") or {}).items():
        ent.append((k, v["roofline"]["kernel_ms"], v["roofline"].get("timing_launches", 2 if "xxh64" in k else 6),
                    v["roofline"].get("kernel")))
    return ent


def main(trace_csv, bench_log):
    rec = next(json.loads(ln) for ln in open(bench_log) if ln.startswith("{"))
    secs = [s for s in sections(trace_csv) if s]
    ents = bench_entries(rec)
    rows = []
    for (label, ev_ms, k, kname), sec in zip(ents, secs):
        if kname and "host route" in str(kname):
            # no kernel dispatch: D2H copies and host hashing, bracketed by the bench's events
            rows.append({"section": label, "bench_events_ms": ev_ms, "rocprof_avg_ms": None, "kernels": [],
                         "note": "host route: no kernel dispatch to match"})
            continue
        # the section's timed launches: its first k dispatches of its first kernel (what follows the
        # launches -- the next leg's warm-up, copies -- is not part of it); a host-routed leg (XXH64
        # host route) has copies only, and its events bracket them
        sec = [x for x in sec if x[0] == sec[0][0]][: k or len(sec)]
        names = {n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0] for n, _ in sec}
        avg_ms = sum(d for _, d in sec) / len(sec) / 1e6
        rows.append({"section": label, "bench_events_ms": ev_ms, "rocprof_avg_ms": round(avg_ms, 5),
                     "dispatches": len(sec), "kernels": sorted(names),
                     "rocprof_over_events": round(avg_ms / ev_ms, 4) if ev_ms else None})
    print(json.dumps({"trace": trace_csv, "sections_in_trace": len(secs), "bench_entries": len(ents), "rows": rows}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
