"""CPU: the C-ABI shared library loads (no device needed) and exports every function the public
headers under include/ declare -- the drop-in boundary -- and nothing else: the
three libraries split as the reference's layers do (aws-checksums / aws-c-common / aws-crt-cpp,
reference CMakeLists.txt:149,388), so the checksum library can replace aws-checksums beside a real
aws-c-common and aws-crt-cpp without interposing on either."""
import ctypes
import os
import re
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
from tests.libpaths import ENGINE as LIB, LOAD_SRC, SHIM, SURFACE, load_engine  # noqa: E402
C_HEADERS = {LIB: ["include/aws_crt_amd/checksums_batch.h", "include/aws/checksums/crc.h", "include/aws/checksums/xxhash.h"],
             SHIM: ["include/aws/common/allocator.h", "include/aws/common/byte_buf.h", "include/aws/common/error.h"]}
# what the checksum library may leave to the process's aws-c-common (aws-checksums' own dependency)
COMMON_IMPORTS = {"aws_raise_error", "aws_mem_acquire", "aws_mem_release", "aws_default_allocator",
                  "aws_byte_buf_write_be64", "aws_byte_cursor_from_array"}


def declared_c_functions(path):
    text = open(os.path.join(REPO, path)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(aws_[a-z0-9_]+)\s*\(", text)
    return sorted(set(n for n in names if not n.endswith("_t")))


def exported(lib=LIB, demangle=False):
    out = subprocess.run(["nm", "-D", "--defined-only"] + (["-C"] if demangle else []) + [lib], capture_output=True,
                         text=True, check=True).stdout
    if demangle:
        return {line.split(None, 2)[-1] for line in out.splitlines() if line.strip()}
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def imported(lib):
    out = subprocess.run(["nm", "-D", "--undefined-only", lib], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1].split("@")[0] for line in out.splitlines() if line.strip()}


def needed(lib):
    out = subprocess.run(["readelf", "-d", lib], capture_output=True, text=True, check=True).stdout
    return re.findall(r"\(NEEDED\)\s+Shared library: \[([^\]]+)\]", out)


def test_library_loads_without_gpu():
    L = load_engine()
    assert L.aws_crt_amd_device_count() >= 0


def test_every_declared_c_symbol_is_exported():
    missing = []
    for lib, headers in C_HEADERS.items():
        syms = exported(lib)
        for h in headers:
            for fn in declared_c_functions(h):
                if fn not in syms:
                    missing.append((os.path.basename(lib), h, fn))
    assert not missing, missing


def test_checksum_library_exports_only_its_abi():
    """VERDICT r05 missing 2: libaws-checksums-amd.so exports the aws-checksums C ABI and aws_crt_amd_*
    only (exports/checksums.map) -- no aws-c-common, no Aws::Crt, no engine internals, no C++ runtime
    instantiations -- and imports from aws-c-common only what aws-checksums itself would."""
    syms = exported(LIB)
    stray = sorted(s for s in syms if not s.startswith(("aws_checksums_", "aws_xxhash", "aws_crt_amd_")))
    assert not stray, stray
    assert {"aws_checksums_crc32c_ex", "aws_xxhash64_compute", "aws_crt_amd_checksum_batches"} <= syms
    for bad in ("amdcrc", "_ZNSt", "_ZN3Aws", "aws_mem_", "aws_last_error", "aws_byte_buf_", "queue_flush_locked"):
        assert not any(bad in s for s in syms), bad
    imp = {s for s in imported(LIB) if s.startswith(("aws_", "_ZN3Aws"))}
    assert imp <= COMMON_IMPORTS, sorted(imp - COMMON_IMPORTS)
    # no aws-c-common provider is named: the process's own (real or the shim) satisfies the imports
    assert not any("aws" in n for n in needed(LIB)), needed(LIB)


def test_shim_and_surface_export_lists():
    """libaws-c-common-shim.so exports aws-c-common functions only; libaws-crt-cpp-amd.so (the Aws::Crt
    surface, hidden visibility as the reference builds it, CMakeLists.txt:326-351) exports Aws::Crt
    symbols only and reaches the engine through the aws-checksums C ABI."""
    shim = exported(SHIM)
    assert shim and all(s.startswith("aws_") and not s.startswith(("aws_checksums", "aws_xxhash", "aws_crt_amd"))
                        for s in shim), sorted(shim)
    surf = exported(SURFACE, demangle=True)
    stray = sorted(s for s in surf if not s.startswith(("Aws::Crt::", "typeinfo for Aws::Crt", "vtable for Aws::Crt")))
    assert not stray, stray
    assert set(needed(SURFACE)) >= {"libaws-checksums-amd.so", "libaws-c-common-shim.so"}
    imp = imported(SURFACE)
    assert not any(s.startswith(("aws_crt_amd_", "_ZN6amdcrc")) for s in imp), sorted(imp)


def test_cpp_api_symbols_exported():
    out = subprocess.run(["nm", "-DC", "--defined-only", SURFACE], capture_output=True, text=True, check=True).stdout
    for sig in ["Aws::Crt::Checksum::ComputeCRC32(aws_byte_cursor, unsigned int)",
                "Aws::Crt::Checksum::ComputeCRC32C(aws_byte_cursor, unsigned int)",
                "Aws::Crt::Checksum::ComputeCRC64NVME(aws_byte_cursor, unsigned long)",
                "Aws::Crt::Checksum::CombineCRC32(unsigned int, unsigned int, unsigned long)",
                "Aws::Crt::Checksum::CombineCRC32C(unsigned int, unsigned int, unsigned long)",
                "Aws::Crt::Checksum::CombineCRC64NVME(unsigned long, unsigned long, unsigned long)",
                "Aws::Crt::Checksum::ComputeXXHash64(aws_byte_cursor const&, aws_byte_buf&, unsigned long)",
                "Aws::Crt::Checksum::ComputeXXHash3_64(aws_byte_cursor const&, aws_byte_buf&, unsigned long)",
                "Aws::Crt::Checksum::ComputeXXHash3_128(aws_byte_cursor const&, aws_byte_buf&, unsigned long)",
                "Aws::Crt::Checksum::XXHash::Update(aws_byte_cursor const&)",
                "Aws::Crt::Checksum::XXHash::Digest(aws_byte_buf&)",
                "Aws::Crt::ApiHandle::ApiHandle(aws_allocator*)", "Aws::Crt::LastError()"]:
        assert sig in out, sig


def test_no_oracle_in_product():
    """The product libraries must not link or embed the test oracle."""
    for lib in (LIB, SHIM, SURFACE):
        out = subprocess.run(["nm", "-D", lib], capture_output=True, text=True, check=True).stdout
        assert "oracle_" not in out
        deps = subprocess.run(["readelf", "-d", lib], capture_output=True, text=True, check=True).stdout
        assert "liboracle" not in deps


def test_combine_scalar_abi_matches_oracle():
    """aws_checksums_*_combine is scalar GF(2) algebra (no payload) and callable without a device."""
    from oracle import oracle
    L = load_engine()
    for name, t in (("crc32", ctypes.c_uint32), ("crc32c", ctypes.c_uint32), ("crc64nvme", ctypes.c_uint64)):
        f = getattr(L, f"aws_checksums_{name}_combine")
        f.restype, f.argtypes = t, [t, t, ctypes.c_uint64]
        for a, b, n in [(0, 0, 0), (0x12345678, 0x9ABCDEF0, 1), (0xFFFFFFFF, 1, 1 << 33), (7, 11, 123456789)]:
            assert f(a, b, n) == oracle.combine(name, a, b, n)


def test_no_device_fails_loudly():
    """Without a device the device-pointer batch ABI returns AWS_CRT_AMD_ERR_NO_DEVICE (device
    addresses cannot be read by the host path)."""
    L = load_engine()
    if L.aws_crt_amd_device_count() > 0:
        import pytest
        pytest.skip("device present")
    L.aws_crt_amd_last_error.restype = ctypes.c_char_p
    rc = L.aws_crt_amd_checksum_strided(1, ctypes.c_void_p(0x1000), 16, 16, 1, None, ctypes.c_void_p(0x2000), None)
    assert rc == -1
    assert b"no HIP device" in L.aws_crt_amd_last_error()


def test_eventstream_abi_argument_checks():
    """aws_crt_amd_eventstream_crcs: count 0 is a no-op, null arrays are refused before any device
    work, and without a device a real call fails loudly."""
    L = load_engine()
    vp = ctypes.c_void_p
    f = L.aws_crt_amd_eventstream_crcs
    f.argtypes = [vp, ctypes.c_uint64, vp, ctypes.c_size_t, vp, vp, vp, vp]
    L.aws_crt_amd_last_error.restype = ctypes.c_char_p
    assert f(None, 0, None, 0, None, None, None, None) == 0
    rc = f(vp(0x1000), 64, None, 4, vp(0x2000), vp(0x3000), vp(0x4000), None)
    assert rc != 0 and b"null argument" in L.aws_crt_amd_last_error()
    if L.aws_crt_amd_device_count() == 0:
        rc = f(vp(0x1000), 64, vp(0x1800), 4, vp(0x2000), vp(0x3000), vp(0x4000), None)
        assert rc == -1 and b"no HIP device" in L.aws_crt_amd_last_error()


def test_release_library_has_no_diagnostics():
    """The shipped library carries no environment-driven diagnostics (no AMDCRC_* variables that could
    change geometry or results) and none of the measured-and-removed kernel variants."""
    strings = subprocess.run(["strings", "-a", LIB], capture_output=True, text=True, check=True).stdout
    assert "AMDCRC_" not in strings
    syms = subprocess.run(["nm", "-C", LIB], capture_output=True, text=True, check=True).stdout
    for gone in ("crc32_stream8_kernel", "crc64_stream_kernel<", "debug_timeline"):
        assert gone not in syms, gone
    # diagnostics (the read-ceiling kernel, test hooks) live only in the diagnostic build
    dyn = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    for gone in ("aws_crt_amd_debug", "read_ceiling", "amdcrc_debug"):
        assert gone not in dyn, gone
    assert "read_ceiling_kernel" not in syms
    # the only getenv in the product selects the processor for host memory, never the arithmetic
    assert "AWS_CRT_AMD_DISPATCH" in strings


def test_value_abi_never_aborts_without_device():
    """aws_checksums_*_ex are value-only and noexcept (CRC.h:20-51): with no usable device they are
    served by the host path (never abort, never a wrong value), even with the GPU dispatch forced."""
    from oracle import oracle
    code = (
        LOAD_SRC + "import sys\n"
        "f=L.aws_checksums_crc32c_ex; f.restype=ctypes.c_uint32; f.argtypes=[ctypes.c_void_p,ctypes.c_size_t,ctypes.c_uint32]\n"
        "b=ctypes.create_string_buffer(b'123456789',9)\n"
        "print(f(b,9,0))\n")
    for mode in ("auto", "cpu", "gpu"):
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                           env=dict(os.environ, AWS_CRT_AMD_DISPATCH=mode, HIP_VISIBLE_DEVICES="-1"))
        assert r.returncode == 0, r.stderr
        assert int(r.stdout.split()[-1]) == oracle.crc("crc32c", b"123456789") == 0xE3069283


def test_pointer_classifier_model():
    """csrc/ptr_class.h with a stand-in probe (tests/cpp/ptr_class_test.cpp, ASan): the common small host
    call never reaches the HIP runtime; device and runtime-known host memory always do; per thread;
    AWS_CRT_AMD_PTR_CACHE=0 probes every call"""
    cpp = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp")
    subprocess.run(["make", "-s", "-C", cpp, "build/ptr_class"], check=True, capture_output=True, text=True)
    exe = os.path.join(cpp, "build", "ptr_class")
    for env, args in (({}, []), ({"AWS_CRT_AMD_PTR_CACHE": "0"}, ["off"])):
        r = subprocess.run([exe] + args, capture_output=True, text=True, timeout=120, env=dict(os.environ, **env))
        assert r.returncode == 0 and "[PASS] PtrClass" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_value_abi_small_host_calls_skip_the_runtime_probe(engine):
    """AUTO-mode aws_checksums_crc32c_ex on small host buffers classifies the
    pointer without hipPointerGetAttributes after the first call in a 64 KiB window; a device
    pointer is still detected and served by the kernels (the diagnostic build counts the probes)"""
    import ctypes

    import torch

    from oracle import oracle

    D = engine.diag_lib()
    D.aws_crt_amd_debug_pointer_probes.restype = ctypes.c_ulonglong
    f = D.aws_checksums_crc32c_ex
    f.restype, f.argtypes = ctypes.c_uint32, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
    assert D.aws_crt_amd_init() == 0 and D.aws_crt_amd_set_dispatch(0) == 0
    buf = ctypes.create_string_buffer(bytes(range(256)) * 16, 4096)
    base = ctypes.addressof(buf)
    p0 = D.aws_crt_amd_debug_pointer_probes()
    vals = {}
    for i in range(1000):
        n = (8, 12, 32, 4096)[i % 4]
        vals[n] = f(base + (i % 64), n, 0) if i % 64 == 0 else f(base, n, 0)
    vals = {n: f(base, n, 0) for n in (8, 12, 32, 4096)}
    probes = D.aws_crt_amd_debug_pointer_probes() - p0
    assert probes <= 2, probes
    raw = (bytes(range(256)) * 16)
    assert vals == {n: oracle.crc("crc32c", raw[:n]) for n in (8, 12, 32, 4096)}
    d = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    torch.cuda.synchronize()
    p1 = D.aws_crt_amd_debug_pointer_probes()
    assert f(d.data_ptr(), 4096, 0) == oracle.crc("crc32c", raw)
    assert D.aws_crt_amd_debug_pointer_probes() - p1 >= 1  # device memory is always asked about


def test_release_build_rejects_ab_knobs():
    """an AMDCRC_* A/B knob outside a variant build is a compile error
    (csrc/variant_guard.h); the results-breaking timing switches are not in the source at all"""
    pkg = os.path.join(REPO, "aws-crt-cpp_amd")
    base = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only", "-D__HIP_PLATFORM_AMD__",
            "-I" + os.path.join(REPO, "include"), "-I" + os.path.join(pkg, "csrc"), os.path.join(pkg, "csrc", "engine.cpp")]
    r = subprocess.run(base + ["-DAMDCRC_XCD=0"], capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "not a variant build" in r.stderr
    r = subprocess.run(base + ["-DAMDCRC_XCD=0", "-DAMDCRC_VARIANT_BUILD=1"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    src = open(os.path.join(pkg, "csrc", "crc_kernels.hip")).read() + open(os.path.join(pkg, "csrc", "engine.cpp")).read()
    for gone in ("AMDCRC_XP_LIST_NOHEAD", "AMDCRC_XP_LIST_NOFINISH", "AMDCRC_XP_XCD_NOPUB", "AMDCRC_XP"):
        assert gone not in src, gone


def test_scan_kernels_keep_their_arguments_out_of_scratch(tmp_path):
    """Round 5: one more branch in a per-set helper made the compiler copy the whole ScanParams (1 KiB of
    kernel arguments) to scratch in crc64_rows16_kernel, so every batch base came from scratch memory
    (0.53 of the HBM peak instead of 0.79).  Every kernel of the release library keeps a private segment
    of at most a few words (the code object's own metadata, read with llvm-readelf).  Round 6: the
    event-stream kernels too (eventstream_flat_kernel holds ~125 VGPRs and no scratch)."""
    import glob
    import shutil

    llvm = "/opt/rocm/lib/llvm/bin"
    lib = shutil.copy(LIB, tmp_path / "lib.so")
    subprocess.run([f"{llvm}/llvm-objdump", "--offloading", str(lib)], cwd=tmp_path, check=True, capture_output=True)
    cos = glob.glob(str(tmp_path / "lib.so.*gfx950"))
    assert cos, "no gfx950 code object in the library"
    seen = 0
    for co in cos:
        notes = subprocess.run([f"{llvm}/llvm-readelf", "--notes", co], capture_output=True, text=True, check=True).stdout
        name = None
        for line in notes.splitlines():
            line = line.strip()
            if line.startswith(".name:"):
                name = line.split(":", 1)[1].strip()
            elif line.startswith(".private_segment_fixed_size:") and name and ("ScanParams" in name or "EventStreamParams" in name):
                seen += 1
                size = int(line.split(":", 1)[1])
                # crc32_braid_kernel<POLY, false> (strided batches that are not whole tiles) has kept 20
                # bytes since round 3; nothing may hold the argument block
                assert size <= 32, (name, size)
    assert seen >= 8
