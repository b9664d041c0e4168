"""Generate tests/golden/vectors.json from implementations INDEPENDENT of the oracle under test:

  CRC32      zlib.crc32 (zlib 1.2.11; same convention as aws_checksums_crc32_ex incl. seeding)
  CRC32C     pure-Python bitwise definition, reflected 0x82F63B78 (Castagnoli)
  CRC64NVME  pure-Python bitwise definition, reflected 0x9A6C9329AC4BC9B5 (CRC.h:33-35)
  XXH64      python `xxhash` 3.8.1 (bundled libxxhash 0.8.2)

and checks each against the reference's own known-answer tests before writing anything:
  tests/CRCTest.cpp:16 (CRC32 of 32 zero bytes = 0x190A55AD), :29 (CRC32C = 0x8A9136AA),
  :42 (CRC64NVME = 0xCF3473434D4ECF3B); tests/XXHashTest.cpp:15 (XXH64("Hello world") =
  c500b0c912b376d8), :44 (XXH3-64 = b6acb9d84a38ff74), :73-74 (XXH3-128 =
  7351f89812f97382b91d05b31e04dd7f).
Run:  python tests/golden/gen_golden.py      (writes tests/golden/vectors.json)
"""
import json
import os
import sys
import zlib

import xxhash

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from patterns import pattern  # noqa: E402

POLY = {"crc32c": (0x82F63B78, 32), "crc64nvme": (0x9A6C9329AC4BC9B5, 64)}


def crc_bitwise(name, data, prev=0):
    if name == "crc32":
        return zlib.crc32(data, prev)
    poly, w = POLY[name]
    mask = (1 << w) - 1
    r = ~prev & mask
    for b in data:
        r ^= b
        for _ in range(8):
            r = (r >> 1) ^ poly if r & 1 else r >> 1
    return ~r & mask


REFERENCE_KATS = [
    # (algorithm, input description, expected, reference file:line)
    ("crc32", "zeros", 32, 0, 0x190A55AD, "tests/CRCTest.cpp:16"),
    ("crc32c", "zeros", 32, 0, 0x8A9136AA, "tests/CRCTest.cpp:29"),
    ("crc64nvme", "zeros", 32, 0, 0xCF3473434D4ECF3B, "tests/CRCTest.cpp:42"),
]
XXH_KATS = [
    ("xxh64", b"Hello world", 0xC500B0C912B376D8, "tests/XXHashTest.cpp:15"),
    ("xxh3_64", b"Hello world", 0xB6ACB9D84A38FF74, "tests/XXHashTest.cpp:44"),
    ("xxh3_128", b"Hello world", 0x7351F89812F97382B91D05B31E04DD7F, "tests/XXHashTest.cpp:73-74"),
]
CHECK = {"crc32": 0xCBF43926, "crc32c": 0xE3069283, "crc64nvme": 0xAE8B14860A799888}

LENGTHS = [0, 1, 2, 3, 4, 7, 8, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 255, 256, 1023, 1024, 4096, 8192,
           65536]
PATTERNS = ["zeros", "ff", "ramp", "splitmix:0x5EED"]
SEEDS32 = [0, 0xDEADBEEF]
SEEDS64 = [0, 0xDEADBEEFCAFEF00D]


def xxh(name, data, seed=0):
    if name == "xxh64":
        return xxhash.xxh64(data, seed=seed).intdigest()
    if name == "xxh3_64":
        return xxhash.xxh3_64(data, seed=seed).intdigest()
    return xxhash.xxh3_128(data, seed=seed).intdigest()


def main():
    for alg, pat, n, seed, want, where in REFERENCE_KATS:
        got = crc_bitwise(alg, pattern(pat, n), seed)
        assert got == want, (alg, where, hex(got))
    for alg, data, want, where in XXH_KATS:
        assert xxh(alg, data) == want, (alg, where)
    for alg, want in CHECK.items():
        assert crc_bitwise(alg, b"123456789") == want, alg

    vectors = []
    for alg in ("crc32", "crc32c", "crc64nvme"):
        seeds = SEEDS64 if alg == "crc64nvme" else SEEDS32
        for pat in PATTERNS:
            for n in LENGTHS:
                data = pattern(pat, n)
                for seed in seeds:
                    vectors.append({"alg": alg, "pattern": pat, "len": n, "seed": seed,
                                    "expect": crc_bitwise(alg, data, seed)})
    for alg in ("xxh64", "xxh3_64", "xxh3_128"):
        for pat in PATTERNS:
            for n in LENGTHS + [129, 240, 241, 1025, 2000]:
                data = pattern(pat, n)
                for seed in SEEDS64:
                    vectors.append({"alg": alg, "pattern": pat, "len": n, "seed": seed, "expect": xxh(alg, data, seed)})

    # chunk/combine triples: CRC(A||B) == Combine(CRC(A), CRC(B), |B|) == Compute(B, Compute(A))
    combines = []
    for alg in ("crc32", "crc32c", "crc64nvme"):
        for la, lb in [(0, 0), (0, 5), (5, 0), (1, 1), (17, 100), (1000, 24), (4096, 4096), (65536, 3)]:
            d = pattern("splitmix:0xC0B1", la + lb)
            a, b = d[:la], d[la:]
            combines.append({"alg": alg, "pattern": "splitmix:0xC0B1", "len_a": la, "len_b": lb,
                             "crc_a": crc_bitwise(alg, a), "crc_b": crc_bitwise(alg, b),
                             "crc_ab": crc_bitwise(alg, d)})

    # large buffers: stored as (pattern, len) + expected value, regenerated deterministically
    large = []
    for alg in ("crc32", "crc32c", "crc64nvme"):
        for seed_pat, n in [("splitmix:0x1A76E", 1 << 20), ("splitmix:0x1A76F", (1 << 20) + 13)]:
            large.append({"alg": alg, "pattern": seed_pat, "len": n, "seed": 0,
                          "expect": crc_bitwise(alg, pattern(seed_pat, n))})

    out = {"generator": "tests/golden/gen_golden.py", "reference_kats": REFERENCE_KATS, "xxh_kats": [
        (a, d.decode(), w, s) for a, d, w, s in XXH_KATS], "check_123456789": CHECK, "vectors": vectors,
        "combines": combines, "large": large}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vectors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print(f"wrote {path}: {len(vectors)} vectors, {len(combines)} combines, {len(large)} large")


if __name__ == "__main__":
    main()
