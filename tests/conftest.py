"""Shared test setup.  `-m gpu` tests need a gfx950 device and call the engine through its C ABI;
everything else runs on CPU (oracle, host logic, ABI exports, drop-in compilation, gloo ranks)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "aws-crt-cpp_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: longer CPU test")


def _ensure_built():
    lib = os.path.join(PKG, "lib", "libaws-checksums-amd.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", PKG, "-j8"], check=True)
    from oracle import oracle  # noqa: E402  (test infrastructure)

    oracle.build()


_ensure_built()


def gpu_available() -> bool:
    import aws_crt_amd

    try:
        return aws_crt_amd.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def engine():
    """The engine with the single-buffer ABI forced onto the GPU: host buffers passed to
    aws_checksums_*_ex / checksum_host run through the gfx950 kernels (the dispatch mode selects the
    processor only, never the arithmetic)."""
    import aws_crt_amd

    if not gpu_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    aws_crt_amd.init()
    aws_crt_amd.set_dispatch(aws_crt_amd.DISPATCH_GPU)
    return aws_crt_amd


@pytest.fixture(autouse=True)
def _no_silent_cpu_fallback(request):
    """GPU tests must be served by the kernels: a GPU failure that the dispatch absorbed by falling
    back to the host path fails the test."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    import aws_crt_amd

    before = aws_crt_amd.fallback_count()
    yield
    assert aws_crt_amd.fallback_count() == before, "a GPU call fell back to the host path"


def pytest_collection_modifyitems(config, items):
    """The bench-contract test (a subprocess run of bench.py) goes last, after every parity test."""
    items.sort(key=lambda it: it.nodeid.startswith("tests/test_bench_contract.py"))
