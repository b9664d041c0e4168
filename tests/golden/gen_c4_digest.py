#!/usr/bin/env python3
"""Golden digest of BASELINE.json config 4 (1,048,576 x 8 KiB, aws_crt_amd/synth.py bytes), computed on
the CPU by the oracle (oracle/crc_oracle.c, hw tier), written to tests/golden/c4_digest.json.

For CRC32C and CRC64NVME: the per-buffer results in global buffer order, reduced to one value (a
"checksum of checksums": CRC64NVME over the result words, little-endian, 4 bytes each for CRC32C and 8
for CRC64NVME), plus the first and last results.  The GPU tests and bench.py's C4 leg gather their
results (any world size) and compare this digest: a size-independent parity check of the full set.

    python tests/golden/gen_c4_digest.py          # ~1 minute on 8 CPUs
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aws-crt-cpp_amd")]

from aws_crt_amd import synth  # noqa: E402
from oracle import oracle  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c4_digest.json")


def digest(results, width):
    """CRC64NVME over the results as little-endian words of `width` bytes"""
    arr = np.asarray(results, dtype=np.uint64 if width == 8 else np.uint32).astype("<u8" if width == 8 else "<u4")
    return oracle.crc("crc64nvme", arr.tobytes())


def main():
    n, L, chunk = synth.C4_COUNT, synth.C4_LEN, 1 << 14
    threads = min(8, os.cpu_count() or 1)
    res = {"crc32c": [], "crc64nvme": []}
    t0 = time.time()
    for k0 in range(0, n, chunk):
        k1 = min(n, k0 + chunk)
        buf = synth.buffers_np(k0, k1 - k0, L)
        ptrs = [buf.ctypes.data + i * L for i in range(k1 - k0)]
        for alg in res:
            res[alg].extend(oracle.batch(alg, ptrs, [L] * (k1 - k0), threads))
    rec = {"generator": "aws_crt_amd/synth.py (splitmix64 of the global word index, seed C4_SEED)",
           "count": n, "length": L, "seed": hex(synth.C4_SEED),
           "digest_rule": "crc64nvme over the per-buffer results in global order, little-endian, 4 bytes each "
                          "(crc32c) or 8 (crc64nvme)",
           "oracle": "oracle/crc_oracle.c batch, hw tier",
           "seconds": round(time.time() - t0, 1)}
    for alg, w in (("crc32c", 4), ("crc64nvme", 8)):
        v = res[alg]
        rec[alg] = {"digest": hex(digest(v, w)), "first": [hex(x) for x in v[:4]], "last": [hex(x) for x in v[-4:]]}
    json.dump(rec, open(OUT, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
