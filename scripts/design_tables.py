#!/usr/bin/env python3
"""Regenerate DESIGN.md §6's config, CPU-baseline and end-to-end tables from the committed bench
records (profiles/r02/bench_default.json, bench_steps20*.json).  Documentation helper only."""
import json
import os

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def main():
    d = json.load(open(os.path.join(R, "profiles/r02/bench_default.json")))
    s20 = [json.load(open(os.path.join(R, f"profiles/r02/{f}"))) for f in ("bench_steps20.json", "bench_steps20_b.json")]
    C = d["configs"]
    r = d["roofline"]
    rows = [f"| C2 CRC32C, 29 batches per launch (200 steps) | {d['value']:.0f} | {d['pct_hbm_peak']:.1f} % | {r['kernel_ms'] * 1e3:.1f} | {r['frac']:.3f} |"]
    v = sorted(x["value"] for x in s20)
    p = sorted(x["pct_hbm_peak"] for x in s20)
    k = sorted(x["roofline"]["kernel_ms"] * 1e3 for x in s20)
    fr = sorted(x["roofline"]["frac"] for x in s20)
    rows.append(f"| C2 CRC32C, 20 batches per launch (20 steps) | {v[0]:.0f}–{v[1]:.0f} | {p[0]:.1f}–{p[1]:.1f} % | {k[0]:.1f}–{k[1]:.1f} | {fr[0]:.3f}–{fr[1]:.3f} |")
    sb = sorted(x["roofline"]["single_batch"]["kernel_ms"] * 1e3 for x in s20)
    sf = sorted(x["roofline"]["single_batch"]["frac"] for x in s20)
    rows.append(f"| C2 CRC32C, one batch per launch | — | — | {sb[0]:.1f}–{sb[1]:.1f} | {sf[0]:.3f}–{sf[1]:.3f} |")
    names = [("C3_crc32c", "C3 CRC32C 16 × 256 MiB"), ("C3_crc32", "C3 CRC32 16 × 256 MiB"),
             ("C4_shard_crc32c", "C4 shard 131,072 × 8 KiB (CRC32C)"),
             ("C4_shard_crc64nvme", "C4 shard 131,072 × 8 KiB (CRC64NVME, streaming scan, §3.6)"),
             ("C5_crc64nvme", "C5 CRC64NVME 8 × 64 MiB"), ("C5_xxh64", "C5 XXH64 8 × 64 MiB"),
             ("target_16x64MiB_crc32c", "north-star target 16 × 64 MiB CRC32C")]
    for key, label in names:
        c = C[key]
        rr = c["roofline"]
        if key == "C5_xxh64":
            rows.append(f"| {label} | {c['value']:.1f} (3 launches in flight) | {c['pct_hbm_peak']:.1f} % | {rr['kernel_ms'] * 1e3:,.0f} | {rr['frac']:.4f} (chain-bound, §3.4) |")
        else:
            rows.append(f"| {label} | {c['value']:.0f} | {c['pct_hbm_peak']:.1f} % | {rr['kernel_ms'] * 1e3:.1f} | {rr['frac']:.3f} |")
    cb = d["cpu_baseline"]
    crow = [f"| C2 CRC32C | {cb['value']:.1f} GiB/s | {cb['single_thread_gibs']:.1f} GiB/s | {cb['oracle_hw_tier_gibs']:.1f} | — | {d['value'] / cb['value']:.0f}× |"]
    lab = {"C3_crc32c": "C3 CRC32C", "C3_crc32": "C3 CRC32", "C4_shard_crc32c": "C4 shard CRC32C",
           "C4_shard_crc64nvme": "C4 shard CRC64NVME", "C5_crc64nvme": "C5 CRC64NVME", "C5_xxh64": "C5 XXH64",
           "target_16x64MiB_crc32c": "target 16 × 64 MiB"}
    for key, l in lab.items():
        c = C[key]
        b = c["cpu_baseline"]
        tp = b.get("third_party")
        tps = "—" if not tp else f"{tp['impl'].split(' (')[0]}: {tp['gibs']:.1f} / {tp['single_thread_gibs']:.1f} GiB/s"
        ratio = c["value"] / b["value"]
        rs = f"{ratio:.0f}×" if ratio >= 1 else f"{ratio:.1f}× (few-buffer XXH64 belongs on the CPU)"
        crow.append(f"| {l} | {b['value']:.1f} GiB/s | {b['single_thread_gibs']:.1f} GiB/s | {b['oracle_hw_tier_gibs']:.1f} | {tps} | {rs} |")
    e = d["e2e_pinned"]
    erow = [f"| C2, 64 batches (65,536 parts of 64 KiB) | {e['value']:.1f} GiB/s | {e['h2d_only_gibs']:.1f} GiB/s | {100 * e['value'] / e['h2d_only_gibs']:.0f} % |"]
    elab = {"C3_crc32c": "C3 CRC32C, 16 × 256 MiB", "C3_crc32": "C3 CRC32, 16 × 256 MiB",
            "C4_shard_crc32c": "C4 shard CRC32C, 131,072 × 8 KiB", "C4_shard_crc64nvme": "C4 shard CRC64NVME, 131,072 × 8 KiB",
            "C5_crc64nvme": "C5 CRC64NVME, 8 × 64 MiB", "target_16x64MiB_crc32c": "target 16 × 64 MiB"}
    for key, l in elab.items():
        x = C[key]["e2e_pinned"]
        erow.append(f"| {l} | {x['value']:.1f} GiB/s | {x['h2d_only_gibs']:.1f} GiB/s | {min(100, 100 * x['value'] / x['h2d_only_gibs']):.0f} % |")
    path = os.path.join(R, "DESIGN.md")
    s = open(path).read()

    def swap(s, header_prefix, body):
        i = s.index(header_prefix)
        j = s.index("\n", s.index("\n", i) + 1)
        k = s.index("\n\n", j)
        return s[:j + 1] + body + s[k:]

    s = swap(s, "| config (per GPU per step) | GiB/s |", "\n".join(rows))
    s = swap(s, "| config | 16 threads | 1 thread |", "\n".join(crow))
    s = swap(s, "| config step | through the host-ingest API |", "\n".join(erow))
    open(path, "w").write(s)


if __name__ == "__main__":
    main()
