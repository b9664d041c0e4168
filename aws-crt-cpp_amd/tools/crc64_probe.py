"""CRC64NVME against its read ceiling.  For the C5 shape (8 x 64 MiB) as one-batch
and 20-batch launches, and the C4 per-GPU shard (131,072 x 8 KiB), the dispatch duration of the CRC64
scan, of the CRC32C scan over the same bytes and of the read-ceiling kernel over the same byte count
(diagnostic build): which part of the CRC64 kernel's distance from the HBM peak is the stream's and
which is the scan's.  Each figure is the mean of serialised launches stamped by their own dispatch
(bench.py time_launches), launches alternating kernels so that clocks and caches treat them alike.
c4full is the whole C4 set (1,048,576 x 8 KiB, 8 GiB) in one launch: bench.py's C4 leg at N = 1.

    python aws-crt-cpp_amd/tools/crc64_probe.py [--reps 3] [--only c5_1|c5_20|c4]

One JSON line per shape: ms and frac of the HBM peak per kernel, scan / ceiling ratios.  Under
rocprofv3 --pmc the kernels are told apart by name and grid (tools/sq_summary.py).
"""
import argparse
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import torch  # noqa: E402

import aws_crt_amd as eng  # noqa: E402
import bench  # noqa: E402

PEAK = 8.0e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--launches", type=int, default=6)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    eng.init()
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream()
    shapes = {"c5_1": (8, 64 << 20, 1), "c5_20": (8, 64 << 20, 20), "c4": (131072, 8192, 1),
              "c4full": (1 << 20, 8192, 1)}
    for name, (n, L, nb) in shapes.items():
        if a.only and name != a.only:
            continue
        step = n * L
        g = torch.Generator(device=dev)
        g.manual_seed(0xC64)
        # nb distinct batches plus one: consecutive launches never read the same bytes
        data = torch.randint(0, 256, ((nb + 1) * step,), dtype=torch.uint8, device=dev, generator=g)
        outs = {w: [torch.empty(n, dtype=torch.int64 if w == "crc64nvme" else torch.int32, device=dev)
                    for _ in range(nb + 1)] for w in ("crc64nvme", "crc32c")}

        def scan(alg):
            def go(i, s_):
                o = i % 2
                eng.checksum_batches(bench.ALG[alg], [(data.data_ptr() + ((o + j) % (nb + 1)) * step, None,
                                                       outs[alg][(o + j) % (nb + 1)]) for j in range(nb)], L, L, n,
                                     stream=s_)
            return go

        def ceiling(i, s_, e0, e1):
            eng.read_ceiling(data, nb * step, stream=s_, base_offset=(i % 2) * step, start_event=e0, stop_event=e1)

        res = {"crc64nvme": [], "crc32c": [], "read_ceiling": []}
        for _ in range(a.reps):
            for k in ("crc64nvme", "crc32c", "read_ceiling"):
                if k == "read_ceiling":
                    ms, _ = bench.time_launches(eng, ceiling, st, a.launches, stamps=True)
                else:
                    ms, _ = bench.time_launches(eng, scan(k), st, a.launches)
                res[k].append(ms)
        torch.cuda.synchronize()
        # parity of the last launch's results against the host path (a sample)
        h = data[: min(step, 8 << 20)].cpu().numpy()
        m = max(1, min(n, (8 << 20) // L))
        want = eng.cpu_batch(eng.CRC64NVME, [h.ctypes.data + i * L for i in range(m)], [min(L, 8 << 20)] * m, threads=8) \
            if L <= 8 << 20 else None
        rec = {"shape": name, "buffers": n, "buffer_bytes": L, "batches_per_launch": nb,
               "bytes_per_launch": nb * step}
        for k, v in res.items():
            ms = statistics.median(v)
            rec[k] = {"ms": round(ms, 5), "frac": round(nb * step / (ms * 1e-3) / PEAK, 4), "reps_ms": [round(x, 5) for x in v]}
        rec["crc64_over_ceiling"] = round(rec["read_ceiling"]["ms"] / rec["crc64nvme"]["ms"], 4)
        rec["crc32c_over_ceiling"] = round(rec["read_ceiling"]["ms"] / rec["crc32c"]["ms"], 4)
        if want is not None:
            # outs[...][0] holds batch 0 of the last even launch: the first m buffers of `data`
            rec["parity_sample"] = eng.as_unsigned(outs["crc64nvme"][0])[:m] == want
        print(json.dumps(rec), flush=True)
        del data, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
