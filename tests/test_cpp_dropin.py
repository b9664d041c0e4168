"""The reference's own checksum test files and our C++ drop-in tests, built against the drop-in
headers (include/aws/...) and linked to the engine library.

CPU: compile and link -- tests/cpp/checksum_dropin_test.cpp always; the reference's
tests/CRCTest.cpp and tests/XXHashTest.cpp unmodified when /root/reference is present (proof that
they drop in; nothing of the reference is copied into this repo).
GPU: run the binaries (they compute on the device through the C ABI).
"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(REPO, "tests", "cpp")
REF_TESTS = "/root/reference/tests"


def _make(*extra):
    subprocess.run(["make", "-s", "-C", CPP, *extra], check=True, capture_output=True, text=True)


def test_dropin_tests_build():
    _make()
    assert os.path.exists(os.path.join(CPP, "build", "checksum_tests"))


@pytest.mark.skipif(not os.path.isdir(REF_TESTS), reason="reference checkout not mounted")
def test_reference_test_files_compile_unmodified():
    _make(f"REF_TESTS={REF_TESTS}")
    assert os.path.exists(os.path.join(CPP, "build", "reference_tests"))


@pytest.mark.gpu
def test_dropin_tests_run(engine):
    _make()
    r = subprocess.run([os.path.join(CPP, "build", "checksum_tests")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout


@pytest.mark.gpu
def test_reference_test_files_run_on_gpu(engine):
    """tests/CRCTest.cpp + tests/XXHashTest.cpp of the reference, compiled unmodified in the build
    container (test_reference_test_files_compile_unmodified) and shipped as a binary: every
    CRC32/CRC32C/CRC64NVME/XXH64/XXH3 known answer computed by the gfx950 engine."""
    exe = os.path.join(CPP, "build", "reference_tests")
    if not os.path.exists(exe):
        pytest.skip("reference_tests binary not built (needs the reference checkout at build time)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    for name in ("CRC32Piping", "CRC32CPiping", "CRC64NVMEPiping", "XXHash64Piping", "XXHash3_64Piping",
                 "XXHash3_128Piping"):
        assert f"[PASS] {name}" in r.stdout, r.stdout


def test_types_base64_cpu():
    """Base64 of the Types surface (Types.h:70-75): the reference's Base64RoundTrip vector
    (tests/TypesTest.cpp:17-31), RFC 4648 vectors, S3 wire forms of the CRC check values and
    malformed inputs.  Host code; no device needed."""
    _make()
    r = subprocess.run([os.path.join(CPP, "build", "types_tests")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "4 ran, 0 failed" in r.stdout, r.stdout
