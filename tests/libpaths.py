"""Paths of the built libraries (aws-crt-cpp_amd/Makefile) and a loader for tests that call the C ABI
without the Python package.

libaws-checksums-amd.so exports the aws-checksums C ABI and aws_crt_amd_* only; its aws-c-common calls
bind to the process's aws-c-common, which standalone is libaws-c-common-shim.so, loaded globally first.
"""
import ctypes
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(REPO, "aws-crt-cpp_amd", "lib")
ENGINE = os.path.join(LIBDIR, "libaws-checksums-amd.so")
SHIM = os.path.join(LIBDIR, "libaws-c-common-shim.so")
SURFACE = os.path.join(LIBDIR, "libaws-crt-cpp-amd.so")
DIAG = os.path.join(LIBDIR, "libaws-crt-cpp-amd-diag.so")

# the same load as Python source, for tests that run it in a fresh interpreter (binds `L`)
LOAD_SRC = f"import ctypes\nctypes.CDLL({SHIM!r}, mode=ctypes.RTLD_GLOBAL)\nL=ctypes.CDLL({ENGINE!r})\n"


def load_engine() -> ctypes.CDLL:
    ctypes.CDLL(SHIM, mode=ctypes.RTLD_GLOBAL)
    return ctypes.CDLL(ENGINE)
