"""CPU: the host C++ of the drop-in surface under AddressSanitizer + UndefinedBehaviorSanitizer.

SURVEY.md §5 (race detection / sanitizers): the reference runs its tests under clang sanitizers
(.github/workflows/ci.yml:416-431).  Kernels cannot be sanitized on this pool, so the host sources
of the C++ surface -- Types (Base64, byte cursors), the aws-c-common shim and the ApiHandle -- are
compiled straight into a test binary with -fsanitize=address,undefined (no engine: the library
init / clean-up are no-op stubs, tests/cpp/host_only_stubs.cpp) and the Types tests run on it.
"""
import os
import subprocess

CPP = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "cpp")


def test_types_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", CPP, "build/types_tests_san"], check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(CPP, "build", "types_tests_san")], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "4 ran, 0 failed" in r.stdout, r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
