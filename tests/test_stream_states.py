"""Per-stream engine state has a bounded lifetime (csrc/stream_states.h, aws_crt_amd_stream_release).

CPU: the state cache under ASan + UBSan with host stand-ins (tests/cpp/stream_states_test.cpp):
1,000 streams created, used and destroyed -- some released, some not, some with work in flight --
never hold more than the bound's worth of states, busy states are never handed to another stream,
and recycled stream handles get their own.  GPU: 1,000 torch streams each running a scan that needs
the cross-tile workspace, against the engine's own counters, with correct results throughout."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(REPO, "tests", "cpp")


def test_stream_state_cache_bounded_under_asan():
    subprocess.run(["make", "-s", "-C", CPP, "build/stream_states"], check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1")
    r = subprocess.run([os.path.join(CPP, "build", "stream_states")], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "[PASS] StreamStatesBounded" in r.stdout, r.stdout


@pytest.mark.gpu
def test_thousand_streams_bounded_state(engine):
    import torch

    from oracle import oracle

    n, L = 8, 1 << 20  # 1 MiB buffers: several tiles each, so every launch uses the stream's workspace
    g = torch.Generator(device="cuda")
    g.manual_seed(0x51)
    d = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    h = d.cpu().numpy()
    want = [oracle.crc("crc32c", h[i * L:(i + 1) * L]) for i in range(n)]
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")  # torch's HIP runtime (already loaded): raw streams, not torch's pool
    hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    before = engine.stream_states()
    for i in range(1000):
        st = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(st), 1) == 0
        engine.checksum_strided(engine.CRC32C, d, L, L, n, out=out, stream=st.value)
        assert hip.hipStreamSynchronize(st) == 0
        if i % 97 == 0:
            assert engine.as_unsigned(out) == want, i
        if i % 2:
            engine.stream_release(st.value)
        assert hip.hipStreamDestroy(st) == 0
    torch.cuda.synchronize()
    after = engine.stream_states()
    assert after["live"] <= 64
    assert after["created"] - before["created"] <= 64 + 8, (before, after)
