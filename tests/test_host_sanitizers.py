"""CPU: the engine's whole host side under sanitizers (race detection / sanitizers;
the reference runs its tests under clang sanitizers, .github/workflows/ci.yml:416-431).

Kernels cannot be sanitized on this pool, so the host sources -- the Aws::Crt C++ surface, the
aws-c-common shim, the single-buffer ABI with its CPU / GPU dispatch (abi_single.cpp) and the host
checksum path (csrc/cpu/) -- are compiled straight into test binaries (no HIP engine: the device
stand-ins in tests/cpp/host_only_stubs.cpp report "no usable device"):
  * ASan + UBSan: our drop-in tests, the Types tests, the concurrency test and, when the reference
    checkout is present, the reference's own tests/CRCTest.cpp and tests/XXHashTest.cpp;
  * TSan: eight threads racing on first use and then checksumming concurrently.
"""
import os

import pytest
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(REPO, "tests", "cpp")
REF_TESTS = "/root/reference/tests"


def _build(target):
    extra = [f"REF_TESTS={REF_TESTS}"] if os.path.isdir(REF_TESTS) else []
    subprocess.run(["make", "-s", "-C", CPP, *extra, target], check=True, capture_output=True, text=True)


def test_host_side_under_asan_ubsan():
    _build("build/host_asan")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(CPP, "build", "host_asan")], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert ", 0 failed" in r.stdout, r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr


def test_concurrent_callers_under_tsan():
    _build("build/host_tsan")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(CPP, "build", "host_tsan")], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "[PASS] ConcurrentCallers" in r.stdout, r.stdout
    assert "ThreadSanitizer" not in r.stderr, r.stderr


@pytest.mark.parametrize("numa", ["", "force"])
@pytest.mark.parametrize("target,opts", [("build/ingest_tsan", {"TSAN_OPTIONS": "halt_on_error=1"}),
                                         ("build/ingest_asan", {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"})])
def test_concurrent_host_jobs_under_sanitizers(target, opts, numa):
    """Host-ingest jobs from six threads at once on the host path (tests/cpp/ingest_host_test.cpp):
    uncut jobs writing results directly, cut jobs joined with Combine, jobs and their vectors reused
    across threads, coordinators on the shared runner threads -- under TSan and under ASan; with
    AWS_CRT_AMD_NUMA=force the jobs of >= 16 MiB run on pool workers placed on the node."""
    _build(target)
    env = dict(os.environ, **opts)
    if numa:
        env["AWS_CRT_AMD_NUMA"] = numa
    r = subprocess.run([os.path.join(CPP, target)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "[PASS] ConcurrentHostJobs" in r.stdout, r.stdout
    assert "ThreadSanitizer" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr


def test_unreadable_device_buffer_raises():
    """A device buffer that neither the GPU nor a read-back can reach (tests/cpp/unreadable_stubs.cpp
    injects it) must not yield a silent CRC: the value-only calls raise AWS_ERROR_UNSUPPORTED_OPERATION
    into Aws::Crt::LastError() (reference source/Api.cpp:469-472), xxHash returns false, and a host
    buffer afterwards is served normally.  ASan + UBSan build."""
    _build("build/host_unreadable")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1")
    r = subprocess.run([os.path.join(CPP, "build", "host_unreadable")], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "[PASS] UnreadableDeviceBufferRaises" in r.stdout, r.stdout
    assert "is unreadable" in r.stderr  # the diagnostic line is printed too


def test_device_stream_xxh3_split_logic():
    """Streaming XXH3 over device chunks (abi_single.cpp, cpu::xxh3_update_source): with the engine
    stand-ins of tests/cpp/devstream_stubs.cpp (a readable "device" buffer; the GPU block absorb
    modelled on the host, then made to fail), every split of up to 4 MiB into host-sized and
    >= 1 MiB device chunks, at every buffer-fill and stripe-position class, digests to the one-shot
    XXH3-64 / XXH3-128 of the same bytes, with and without seed; failed absorbs fall back (counted)
    to the same value.  ASan + UBSan build."""
    _build("build/host_devstream")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1")
    r = subprocess.run([os.path.join(CPP, "build", "host_devstream")], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "[PASS] DeviceStreamXxh3Splits" in r.stdout and "[PASS] DeviceStreamXxh3Fallback" in r.stdout, r.stdout
