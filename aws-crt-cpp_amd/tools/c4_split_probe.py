"""The C4 set (1,048,576 x 8 KiB, 8 GiB) scanned as one launch against k back-to-back launches of
1/k of the buffers each (one stream, or round-robin over three), timed with events on the streams
around the whole pass: whether the long launch loses to its length (work drift between waves, which
splitting bounds) or to sustained load (clocks, which splitting does not change).

    python aws-crt-cpp_amd/tools/c4_split_probe.py [--reps 5] [--algs crc32c,crc64nvme]

One JSON line per (alg, form): ms per pass, GiB/s, fraction of the 8 TB/s HBM peak.
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
N, L = 1 << 20, 8192


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--algs", default="crc32c,crc64nvme")
    ap.add_argument("--splits", default="1,2,4,8,16,32")
    ap.add_argument("--alloc-gib", type=int, default=8, help="size of the one allocation holding the set")
    ap.add_argument("--offset-gib", type=int, default=0, help="where in it the set starts")
    ap.add_argument("--passes", type=int, default=1, help="passes back to back per timed rep (sustained load)")
    ap.add_argument("--hold-ms", type=float, default=10.0, help="GPU sleep before each timed rep (0: none)")
    ap.add_argument("--synth", action="store_true", help="fill with aws_crt_amd/synth.py (the bench's C4 data)")
    a = ap.parse_args()
    eng.init()
    dev = torch.device("cuda", 0)
    sts = [torch.cuda.Stream() for _ in range(3)]
    assert (a.offset_gib << 30) + N * L <= a.alloc_gib << 30
    whole = torch.empty(a.alloc_gib << 30, dtype=torch.uint8, device=dev)
    data = whole[a.offset_gib << 30:(a.offset_gib << 30) + N * L]
    if a.synth:
        from aws_crt_amd import synth
        synth.fill_shard(data, 0, 1, count=N, length=L)
    else:
        g = torch.Generator(device=dev)
        g.manual_seed(0xC4)
        data.copy_(torch.randint(0, 256, (N * L,), dtype=torch.uint8, device=dev, generator=g))
    for alg in a.algs.split(","):
        out = torch.empty(N, dtype=torch.int64 if alg == "crc64nvme" else torch.int32, device=dev)
        ref = None
        for nst in (1, 3):
            for k in [int(x) for x in a.splits.split(",")]:
                if nst == 3 and k < 3:
                    continue
                per = N // k

                def one_pass():
                    for j in range(k):
                        eng.checksum_batches(bench.ALG[alg], [(data.data_ptr() + j * per * L, None, out[j * per:(j + 1) * per])],
                                             L, L, per, stream=sts[j % nst])

                one_pass()  # warm-up (first launch of the shape)
                torch.cuda.synchronize()
                ms = []
                for _ in range(a.reps):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = [torch.cuda.Event(enable_timing=True) for _ in range(nst)]
                    if a.hold_ms > 0:
                        with torch.cuda.stream(sts[0]):
                            torch.cuda._sleep(int(a.hold_ms * 2e6))
                    e0.record(sts[0])
                    for s_ in sts[1:nst]:
                        s_.wait_event(e0)
                    for _ in range(a.passes):
                        one_pass()
                    for i in range(nst):
                        e1[i].record(sts[i])
                    torch.cuda.synchronize()
                    ms.append(max(e0.elapsed_time(e) for e in e1) / a.passes)
                torch.cuda.synchronize()
                res = eng.as_unsigned(out)
                if ref is None:
                    ref = res
                m = statistics.median(ms)
                print(json.dumps({"alloc_gib": a.alloc_gib, "offset_gib": a.offset_gib, "synth": a.synth, "passes": a.passes, "hold_ms": a.hold_ms, "alg": alg, "launches": k, "streams": nst, "buffers_per_launch": per, "ms": round(m, 4),
                                  "gibs": round(N * L / (m * 1e-3) / 2**30, 1), "frac": round(N * L / (m * 1e-3) / PEAK, 4),
                                  "reps_ms": [round(x, 4) for x in ms], "same_results": res == ref}), flush=True)
        del out


if __name__ == "__main__":
    main()
