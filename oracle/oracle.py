"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of oracle/crc_oracle.c (the CPU restatement).

May be imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker / CPU baseline; never by the product (aws-crt-cpp_amd/).  See crc_oracle.c's header for
the reference file:line each function restates and how the restatement is pinned.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "build", "liboracle.so")

_L = None


def build() -> str:
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(os.path.join(HERE, "crc_oracle.c")):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return SO


def lib() -> ctypes.CDLL:
    global _L
    if _L is None:
        build()
        L = ctypes.CDLL(SO)
        vp, sz, u32, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64
        for tier in ("bitwise", "sw", "hw"):
            for name, t in (("crc32", u32), ("crc32c", u32), ("crc64nvme", u64)):
                f = getattr(L, f"oracle_{name}_{tier}")
                f.restype, f.argtypes = t, [vp, sz, t]
        L.oracle_crc32c_fold.restype, L.oracle_crc32c_fold.argtypes = u32, [vp, sz, u32]
        for name, t in (("crc32", u32), ("crc32c", u32), ("crc64nvme", u64)):
            f = getattr(L, f"oracle_{name}_combine")
            f.restype, f.argtypes = t, [t, t, u64]
        L.oracle_xxh64.restype, L.oracle_xxh64.argtypes = u64, [vp, sz, u64]
        L.oracle_xxh3_64.restype, L.oracle_xxh3_64.argtypes = u64, [vp, sz, u64]
        L.oracle_xxh3_128.restype, L.oracle_xxh3_128.argtypes = None, [vp, sz, u64, ctypes.POINTER(u64)]
        L.oracle_xpow8n.restype, L.oracle_xpow8n.argtypes = u64, [u64, ctypes.c_int]
        L.oracle_mulmod.restype, L.oracle_mulmod.argtypes = u64, [u64, u64, ctypes.c_int]
        L.oracle_hw_available.restype = ctypes.c_int
        L.oracle_batch.restype = ctypes.c_int
        L.oracle_batch.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(sz), ctypes.POINTER(u64), sz,
                                   ctypes.c_int]
        _L = L
    return _L


ALG_INDEX = {"crc32": 0, "crc32c": 1, "crc64nvme": 2, "xxh64": 3}


def _ptr(data):
    if hasattr(data, "ctypes"):  # numpy array
        return data.ctypes.data, data.nbytes, None
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    return ctypes.addressof(buf), len(data), buf


def crc(name: str, data, previous: int = 0, tier: str = "hw") -> int:
    p, n, keep = _ptr(data)
    return getattr(lib(), f"oracle_{name}_{tier}")(p, n, previous)


def xxh64(data, seed: int = 0) -> int:
    p, n, keep = _ptr(data)
    return lib().oracle_xxh64(p, n, seed)


def xxh3_64(data, seed: int = 0) -> int:
    p, n, keep = _ptr(data)
    return lib().oracle_xxh3_64(p, n, seed)


def xxh3_128(data, seed: int = 0) -> int:
    """128-bit value, high half first (canonical XXH128 digest order)"""
    p, n, keep = _ptr(data)
    out = (ctypes.c_uint64 * 2)()
    lib().oracle_xxh3_128(p, n, seed, out)
    return (out[0] << 64) | out[1]


def checksum(name: str, data, seed: int = 0) -> int:
    if name == "xxh64":
        return xxh64(data, seed)
    if name == "xxh3_64":
        return xxh3_64(data, seed)
    if name == "xxh3_128":
        return xxh3_128(data, seed)
    return crc(name, data, seed)


def combine(name: str, c1: int, c2: int, len2: int) -> int:
    return getattr(lib(), f"oracle_{name}_combine")(c1, c2, len2)


def xpow8n(name: str, nbytes: int) -> int:
    return lib().oracle_xpow8n(nbytes, ALG_INDEX[name])


def mulmod(name: str, a: int, b: int) -> int:
    return lib().oracle_mulmod(a, b, ALG_INDEX[name])


def batch(name: str, ptrs, lens, nthreads: int = 1):
    """Threaded batch over host buffers (the CPU baseline)."""
    n = len(ptrs)
    P = (ctypes.c_void_p * n)(*ptrs)
    S = (ctypes.c_size_t * n)(*lens)
    out = (ctypes.c_uint64 * n)()
    rc = lib().oracle_batch(ALG_INDEX[name], P, S, out, n, nthreads)
    if rc != 0:
        raise RuntimeError("oracle_batch failed")
    return list(out)


def prepared_batch(name: str, ptrs, lens, nthreads: int = 1):
    """oracle.batch with its argument arrays built once; returns a zero-argument callable (the CPU
    baseline's secondary figure times only the C call)."""
    n = len(ptrs)
    P = (ctypes.c_void_p * n)(*ptrs)
    S = (ctypes.c_size_t * n)(*lens)
    out = (ctypes.c_uint64 * n)()
    f, a = lib().oracle_batch, ALG_INDEX[name]

    def run():
        if f(a, P, S, out, n, nthreads) != 0:
            raise RuntimeError("oracle_batch failed")
    return run
