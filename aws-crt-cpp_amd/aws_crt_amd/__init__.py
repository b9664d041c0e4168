"""ctypes binding of the MI355X checksum engine's C ABI (include/aws_crt_amd/checksums_batch.h,
include/aws/checksums/crc.h).  Used by tests/ and bench.py; torch supplies device memory and
streams only.  Every compute call goes through lib/libaws-checksums-amd.so -- there is no Python
checksum code: if the library is missing, calls raise; device-batch calls raise without a gfx950
device.  The library's own host path (csrc/cpu/) serves host memory per its dispatch mode.

Reference API being mirrored: Aws::Crt::Checksum (include/aws/crt/checksum/CRC.h:20-51,
XXHash.h:21-37) -> aws-checksums (source/checksum/CRC.cpp:17-42, XXHash.cpp:17-65).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_PKG_DIR), "lib", "libaws-checksums-amd.so")
# aws-c-common stand-in: the engine's few aws-c-common calls (aws_raise_error, aws_mem_*) bind to the
# process's aws-c-common, as aws-checksums' do; standalone that is this library, loaded globally first
SHIM_PATH = os.path.join(os.path.dirname(_PKG_DIR), "lib", "libaws-c-common-shim.so")

CRC32, CRC32C, CRC64NVME, XXH64, XXH3_64, XXH3_128 = 0, 1, 2, 3, 4, 5
DISPATCH_AUTO, DISPATCH_CPU, DISPATCH_GPU = 0, 1, 2
ALGORITHMS = {"crc32": CRC32, "crc32c": CRC32C, "crc64nvme": CRC64NVME, "xxh64": XXH64, "xxh3_64": XXH3_64,
              "xxh3_128": XXH3_128}
WIDE = {CRC64NVME, XXH64, XXH3_64, XXH3_128}  # 64-bit result words (XXH3_128: two per buffer)

_lib = None


class EngineError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load the native engine (raises if it was not built)."""
    global _lib
    if _lib is None:
        # torch ships its own HIP runtime (SONAME libamdhip64.so.7, loaded by the unversioned name).
        # Load it first so the engine's DT_NEEDED libamdhip64.so.7 binds to that same instance:
        # one HIP runtime per process, and torch's streams / allocations are valid handles for us.
        import torch  # noqa: F401
        for p in (SHIM_PATH, LIB_PATH):
            if not os.path.exists(p):
                raise EngineError(f"native engine not built: {p} missing (run __graft_entry__.build())")
        ctypes.CDLL(SHIM_PATH, mode=ctypes.RTLD_GLOBAL)
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, u32, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64
        L.aws_crt_amd_init.restype = ctypes.c_int
        L.aws_crt_amd_device_count.restype = ctypes.c_int
        L.aws_crt_amd_last_error.restype = ctypes.c_char_p
        L.aws_crt_amd_fallback_count.restype = ctypes.c_ulonglong
        L.aws_crt_amd_cpu_tier.restype = ctypes.c_char_p
        L.aws_crt_amd_cpu_batch.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(sz), sz,
                                            ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.c_int]
        L.aws_crt_amd_checksum_strided.argtypes = [ctypes.c_int, vp, sz, sz, sz, vp, vp, vp]
        L.aws_crt_amd_checksum_list.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(sz), sz, vp, vp, vp]
        L.aws_crt_amd_checksum_host.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(sz), sz, vp, vp]
        L.aws_crt_amd_crc_combine_batch.argtypes = [ctypes.c_int, vp, vp, ctypes.POINTER(u64), sz, vp, vp]
        L.aws_crt_amd_multipart_crc.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(sz), sz, vp, vp,
                                                ctypes.c_char_p, vp]
        for name, rt, st in (("crc32", u32, u32), ("crc32c", u32, u32), ("crc64nvme", u64, u64)):
            f = getattr(L, f"aws_checksums_{name}_ex")
            f.restype, f.argtypes = rt, [vp, sz, st]
            f = getattr(L, f"aws_checksums_{name}_combine")
            f.restype, f.argtypes = rt, [st, st, u64]
        _lib = L
    return _lib


def _check(rc: int) -> None:
    if rc != 0:
        raise EngineError(f"aws_crt_amd error {rc}: {lib().aws_crt_amd_last_error().decode()}")


def set_dispatch(mode: int) -> None:
    """Where the single-buffer ABI runs host-memory input (DISPATCH_AUTO / _CPU / _GPU)."""
    _check(lib().aws_crt_amd_set_dispatch(mode))


def fallback_count() -> int:
    """GPU calls that failed and were served by the host path instead (process-wide)."""
    return int(lib().aws_crt_amd_fallback_count())


def cpu_tier() -> str:
    return lib().aws_crt_amd_cpu_tier().decode()


class CpuBatch:
    """A prepared aws_crt_amd_cpu_batch call (argument arrays built once; `run()` is the C call only)."""

    def __init__(self, alg: int, ptrs: Sequence[int], lens: Sequence[int], seeds=None, threads: int = 1):
        n = len(ptrs)
        self.n, self.alg, self.threads = n, alg, threads
        self.P = (ctypes.c_void_p * max(n, 1))(*ptrs)
        self.S = (ctypes.c_size_t * max(n, 1))(*lens)
        self.sd = (ctypes.c_uint64 * max(n, 1))(*seeds) if seeds is not None else None
        self.out = (ctypes.c_uint64 * max(n * (2 if alg == XXH3_128 else 1), 1))()
        self.fn = lib().aws_crt_amd_cpu_batch

    def run(self) -> None:
        _check(self.fn(self.alg, self.P, self.S, self.n, self.sd, self.out, self.threads))

    def results(self) -> list:
        out, n = self.out, self.n
        if self.alg == XXH3_128:
            return [(out[2 * i] << 64) | out[2 * i + 1] for i in range(n)]
        return list(out[:n]) if n else []


def cpu_batch(alg: int, ptrs: Sequence[int], lens: Sequence[int], seeds=None, threads: int = 1) -> list:
    """The library's host path over host buffers (raw addresses), `threads` std::threads; one value
    per buffer (XXH3_128: 128-bit ints)."""
    n = len(ptrs)
    P = (ctypes.c_void_p * max(n, 1))(*ptrs)
    S = (ctypes.c_size_t * max(n, 1))(*lens)
    sd = (ctypes.c_uint64 * max(n, 1))(*seeds) if seeds is not None else None
    per = 2 if alg == XXH3_128 else 1
    out = (ctypes.c_uint64 * max(n * per, 1))()
    _check(lib().aws_crt_amd_cpu_batch(alg, P, S, n, sd, out, threads))
    if per == 2:
        return [(out[2 * i] << 64) | out[2 * i + 1] for i in range(n)]
    return [int(out[i]) for i in range(n)]


def device_count() -> int:
    return lib().aws_crt_amd_device_count()


def init() -> None:
    _check(lib().aws_crt_amd_init())


def _stream_handle(stream) -> Optional[int]:
    if stream is None:
        import torch

        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def _out_dtype(alg: int):
    import torch

    return torch.int64 if alg in WIDE else torch.int32


def time_next_launch(start_event, stop_event) -> None:
    """Profiling (aws_crt_amd_profile_next_launch): the next launch made by this thread stamps its own
    dispatch start / end into these torch.cuda.Event objects (created with enable_timing=True)."""
    L = lib()
    L.aws_crt_amd_profile_next_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.aws_crt_amd_profile_next_launch(start_event.cuda_event, stop_event.cuda_event)


DIAG_LIB_PATH = os.path.join(os.path.dirname(_PKG_DIR), "lib", "libaws-crt-cpp-amd-diag.so")
_diag = None


def diag_lib() -> ctypes.CDLL:
    """The diagnostic build of the engine (make diag: the same sources plus the read-ceiling kernel and
    the host-tier hook).  Measurement and tests only; checksums always go through lib()."""
    global _diag
    if _diag is None:
        lib()  # torch's HIP runtime first (one runtime per process)
        if not os.path.exists(DIAG_LIB_PATH):
            raise EngineError(f"diagnostic engine not built: {DIAG_LIB_PATH} missing (make -C aws-crt-cpp_amd diag)")
        _diag = ctypes.CDLL(DIAG_LIB_PATH)
    return _diag


def read_ceiling(base, nbytes: int, stream=None, base_offset: int = 0, start_event=None, stop_event=None) -> None:
    """Diagnostics (diagnostic library): one launch of the streaming-read ceiling kernel (the W=32
    streaming scan's launch shape, CRC removed) over nbytes of device memory, optionally stamping its
    dispatch into (start_event, stop_event)."""
    D = diag_lib()
    D.aws_crt_amd_debug_read_ceiling.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    if start_event is not None:
        D.aws_crt_amd_profile_next_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        D.aws_crt_amd_profile_next_launch(start_event.cuda_event, stop_event.cuda_event)
    addr = (base.data_ptr() if hasattr(base, "data_ptr") else int(base)) + base_offset
    rc = D.aws_crt_amd_debug_read_ceiling(addr, nbytes, _stream_handle(stream))
    if rc != 0:
        raise EngineError(f"read ceiling launch failed ({rc})")


def event_ms(start_event, stop_event) -> float:
    """Milliseconds between two events stamped by time_next_launch (aws_crt_amd_profile_elapsed_ms)."""
    L = lib()
    L.aws_crt_amd_profile_elapsed_ms.restype = ctypes.c_float
    L.aws_crt_amd_profile_elapsed_ms.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    ms = L.aws_crt_amd_profile_elapsed_ms(start_event.cuda_event, stop_event.cuda_event)
    if ms < 0:
        raise EngineError("event timing failed")
    return ms


def checksum_strided(alg: int, base, stride: int, length: int, count: int, seeds=None, out=None, stream=None,
                     base_offset: int = 0):
    """Batch of `count` device buffers [base + i*stride + base_offset, +length).  `base` is a torch
    device tensor (or raw address).  Returns the int32/int64 result tensor (reinterpret as unsigned)."""
    import torch

    addr = (base.data_ptr() if hasattr(base, "data_ptr") else int(base)) + base_offset
    dev = base.device if hasattr(base, "device") else torch.device("cuda")
    if out is None:
        out = torch.empty(count * (2 if alg == XXH3_128 else 1), dtype=_out_dtype(alg), device=dev)
    sp = seeds.data_ptr() if seeds is not None else None
    _check(lib().aws_crt_amd_checksum_strided(alg, addr, stride, length, count, sp, out.data_ptr(),
                                              _stream_handle(stream)))
    return out


def stream_release(stream) -> None:
    """aws_crt_amd_stream_release: the stream's engine state goes back for reuse (call before the
    stream is dropped, if it was used with the engine)."""
    L = lib()
    L.aws_crt_amd_stream_release.argtypes = [ctypes.c_void_p]
    _check(L.aws_crt_amd_stream_release(_stream_handle(stream)))


def stream_states() -> dict:
    """live / spare / ever-created per-stream engine states of the current device"""
    L = lib()
    sz = ctypes.c_size_t
    L.aws_crt_amd_stream_states.argtypes = [ctypes.POINTER(sz)] * 3
    a, b, c = sz(), sz(), sz()
    _check(L.aws_crt_amd_stream_states(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
    return {"live": a.value, "spare": b.value, "created": c.value}


class _Batch(ctypes.Structure):
    _fields_ = [("d_base", ctypes.c_void_p), ("d_seeds", ctypes.c_void_p), ("d_out", ctypes.c_void_p)]


class BatchSet:
    """A prepared submission of several uniform batches of one shape (aws_crt_amd_plan_create over
    the batches of aws_crt_amd_checksum_batches): the planning -- runs of batches, kernel, tile size,
    geometry, constants -- is done once, like a producer filling a submission queue, and `run()` only
    launches the plan (aws_crt_amd_plan_launch).  `batches`: (base address / tensor, seeds tensor or
    None, out tensor) per batch."""

    def __init__(self, alg: int, batches, stride: int, length: int, count: int):
        self.n = len(batches)
        # the tensors behind the raw addresses stay referenced as long as the prepared submission: a
        # temporary freed (and reused by the caching allocator) under a queued launch would be read or
        # written by it
        self._keep = [t for b in batches for t in b if hasattr(t, "data_ptr")]
        self._cuda = [t for t in self._keep if getattr(t, "is_cuda", False)]
        # streams the tensors are already recorded on, keyed by the stream OBJECT and holding it (ADVICE
        # r05): a raw handle can be reused by a new stream once the old one is destroyed, an object
        # kept alive here cannot be confused with another
        self._recorded = {}
        arr = (_Batch * max(self.n, 1))()
        for i, (base, seeds, out) in enumerate(batches):
            arr[i].d_base = base.data_ptr() if hasattr(base, "data_ptr") else int(base)
            arr[i].d_seeds = seeds.data_ptr() if seeds is not None else None
            arr[i].d_out = out.data_ptr()
        L = lib()
        L.aws_crt_amd_plan_create.argtypes = [ctypes.c_int, ctypes.POINTER(_Batch), ctypes.c_size_t, ctypes.c_size_t,
                                              ctypes.c_size_t, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]
        L.aws_crt_amd_plan_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.aws_crt_amd_plan_launches.argtypes = [ctypes.c_void_p]
        L.aws_crt_amd_plan_launches.restype = ctypes.c_size_t
        L.aws_crt_amd_plan_destroy.argtypes = [ctypes.c_void_p]
        self._destroy = L.aws_crt_amd_plan_destroy
        h = ctypes.c_void_p()
        _check(L.aws_crt_amd_plan_create(alg, arr, self.n, stride, length, count, ctypes.byref(h)))
        self._plan = h
        self.fn = L.aws_crt_amd_plan_launch
        self.launches = int(L.aws_crt_amd_plan_launches(h))

    def run(self, stream=None) -> None:
        rc = self.fn(self._plan, _stream_handle(stream))
        if rc != 0:
            _check(rc)
        if self._cuda and stream is not None and hasattr(stream, "cuda_stream") and id(stream) not in self._recorded:
            # a launch on a side stream: the caching allocator must not hand these blocks out again
            # before that stream has finished with them.  Once per stream: the allocator waits for every
            # recorded stream when the block is freed, so recording it again per launch only costs host
            # time between launches
            for t in self._cuda:
                t.record_stream(stream)
            self._recorded[id(stream)] = stream

    def __del__(self):
        if getattr(self, "_plan", None):
            self._destroy(self._plan)
            self._plan = None


def checksum_batches(alg: int, batches, stride: int, length: int, count: int, stream=None) -> None:
    """Several uniform batches of one shape, each (base address, seeds tensor or None, out tensor),
    coalesced into as few launches as the engine allows (aws_crt_amd_checksum_batches)."""
    n = len(batches)
    arr = (_Batch * max(n, 1))()
    for i, (base, seeds, out) in enumerate(batches):
        arr[i].d_base = base.data_ptr() if hasattr(base, "data_ptr") else int(base)
        arr[i].d_seeds = seeds.data_ptr() if seeds is not None else None
        arr[i].d_out = out.data_ptr()
    L = lib()
    L.aws_crt_amd_checksum_batches.argtypes = [ctypes.c_int, ctypes.POINTER(_Batch), ctypes.c_size_t, ctypes.c_size_t,
                                               ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p]
    _check(L.aws_crt_amd_checksum_batches(alg, arr, n, stride, length, count, _stream_handle(stream)))
    if stream is not None and hasattr(stream, "cuda_stream"):
        for b in batches:
            for t in b:
                if getattr(t, "is_cuda", False):
                    t.record_stream(stream)


class _QueueOptions(ctypes.Structure):
    _fields_ = [("max_batches", ctypes.c_size_t), ("max_age_us", ctypes.c_uint64), ("policy", ctypes.c_uint32),
                ("max_inflight", ctypes.c_uint32), ("min_launch", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


TICKET_QUEUED, TICKET_LAUNCHED = 1, 2
QUEUE_EAGER, QUEUE_BATCHED = 0, 1


class Queue:
    """A submission queue (aws_crt_amd_queue_*): batches of one shape pushed one at a time are launched
    together.  policy QUEUE_EAGER (default): a push that finds fewer than max_inflight (default 1) of the
    queue's launches running launches everything queued at once (once at least min_launch are queued); QUEUE_BATCHED: only at max_batches
    queued (32 by default), once the oldest has waited max_age_us (0: no age bound), and at flush() /
    wait() / close() (which also launch under the eager policy).  push() returns the batch's ticket;
    status(ticket) / wait(ticket) give its completion (0) or the error of the launch that dropped it.
    The pushed tensors stay referenced until the engine has launched them (every ticket below
    first_pending()); thread-safe."""

    def __init__(self, alg: int, stride: int, length: int, count: int, stream=None, max_batches: int = 0,
                 max_age_us: int = 0, policy: int = QUEUE_EAGER, max_inflight: int = 0, min_launch: int = 0):
        import threading

        L = lib()
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        L.aws_crt_amd_queue_create_ex.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                                  vp, ctypes.POINTER(_QueueOptions), ctypes.POINTER(vp)]
        L.aws_crt_amd_queue_push_ex.argtypes = [vp, vp, vp, vp, ctypes.POINTER(u64)]
        L.aws_crt_amd_queue_flush.argtypes = [vp]
        L.aws_crt_amd_queue_pending.argtypes = [vp]
        L.aws_crt_amd_queue_pending.restype = ctypes.c_size_t
        L.aws_crt_amd_queue_first_pending.argtypes = [vp]
        L.aws_crt_amd_queue_first_pending.restype = u64
        L.aws_crt_amd_queue_launches.argtypes = [vp]
        L.aws_crt_amd_queue_launches.restype = u64
        L.aws_crt_amd_queue_status.argtypes = [vp, u64]
        L.aws_crt_amd_queue_wait.argtypes = [vp, u64]
        L.aws_crt_amd_queue_destroy.argtypes = [vp]
        self._L = L
        self._stream = stream
        self._keep = {}  # ticket -> tensors, until the ticket is launched
        self._lock = threading.Lock()
        h = vp()
        opt = _QueueOptions(max_batches, max_age_us, policy, max_inflight, min_launch, 0)
        _check(L.aws_crt_amd_queue_create_ex(alg, stride, length, count, _stream_handle(stream), ctypes.byref(opt),
                                             ctypes.byref(h)))
        self._h = h

    def _release_launched(self):
        """drop the references of every launched ticket (after record_stream on a side stream)"""
        first = int(self._L.aws_crt_amd_queue_first_pending(self._h)) if self._h else 1 << 64
        done = [t for t in self._keep if t < first]
        side = self._stream is not None and hasattr(self._stream, "cuda_stream")
        for t in done:
            for x in self._keep.pop(t):
                if side and getattr(x, "is_cuda", False):
                    x.record_stream(self._stream)

    def push(self, base, out, seeds=None) -> int:
        b = base.data_ptr() if hasattr(base, "data_ptr") else int(base)
        tk = ctypes.c_uint64(0)
        with self._lock:
            rc = self._L.aws_crt_amd_queue_push_ex(self._h, b, seeds.data_ptr() if seeds is not None else None,
                                                   out.data_ptr(), ctypes.byref(tk))
            if tk.value:
                self._keep[tk.value] = [t for t in (base, out, seeds) if hasattr(t, "data_ptr")]
            self._release_launched()
        _check(rc)
        return int(tk.value)

    def pending(self) -> int:
        return int(self._L.aws_crt_amd_queue_pending(self._h))

    def launches(self) -> int:
        return int(self._L.aws_crt_amd_queue_launches(self._h))

    def first_pending(self) -> int:
        return int(self._L.aws_crt_amd_queue_first_pending(self._h))

    def status(self, ticket: int) -> int:
        return int(self._L.aws_crt_amd_queue_status(self._h, ticket))

    def wait(self, ticket: int) -> int:
        """0 once the ticket's batch is complete, or the (negative) status of the launch that dropped it"""
        rc = int(self._L.aws_crt_amd_queue_wait(self._h, ticket))
        with self._lock:
            self._release_launched()
        return rc

    def flush(self) -> None:
        with self._lock:
            rc = self._L.aws_crt_amd_queue_flush(self._h)
            self._release_launched()
        _check(rc)

    def close(self) -> None:
        with self._lock:
            if not self._h:
                return
            rc = self._L.aws_crt_amd_queue_destroy(self._h)
            self._h = None
            self._release_launched()
        _check(rc)


class _IngestOptions(ctypes.Structure):
    _fields_ = [("ndevices", ctypes.c_int), ("host_threads", ctypes.c_int), ("device_bytes", ctypes.POINTER(ctypes.c_uint64))]


class HostJob:
    """A prepared host-ingest job (aws_crt_amd_host_submit_ex / aws_crt_amd_job_wait) over host buffers
    given by raw addresses: the argument arrays are built once; `run()` submits and waits (the C
    calls only); `results()` reads them back (XXH3_128: 128-bit ints).  host_threads: -1 = hybrid
    (the CPU share beside the device lanes, the default), 0 = devices only, n = n host threads.
    `device_bytes` after run(): the bytes the devices checksummed."""

    def __init__(self, alg: int, ptrs: Sequence[int], lens: Sequence[int], seeds=None, ndevices: int = 0,
                 host_threads: int = -1):
        L = lib()
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.aws_crt_amd_host_submit_ex.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(sz), sz, vp, vp,
                                                 ctypes.POINTER(_IngestOptions), ctypes.POINTER(vp)]
        L.aws_crt_amd_job_wait.argtypes = [vp]
        L.aws_crt_amd_job_last_error.restype = ctypes.c_char_p
        self.L, self.alg, self.n = L, alg, len(ptrs)
        n = self.n
        self.P = (vp * max(n, 1))(*ptrs)
        self.S = (sz * max(n, 1))(*lens)
        T = ctypes.c_uint64 if alg in WIDE else ctypes.c_uint32
        self.out = (T * max(n * (2 if alg == XXH3_128 else 1), 1))()
        self.sd = (T * max(n, 1))(*seeds) if seeds is not None else None
        self._dev_bytes = ctypes.c_uint64(0)
        self.opt = _IngestOptions(ndevices, host_threads, ctypes.pointer(self._dev_bytes))

    def run(self) -> None:
        vp = ctypes.c_void_p
        job = vp()
        rc = self.L.aws_crt_amd_host_submit_ex(self.alg, self.P, self.S, self.n,
                                               ctypes.cast(self.sd, vp) if self.sd is not None else None,
                                               ctypes.cast(self.out, vp), ctypes.byref(self.opt), ctypes.byref(job))
        if rc == 0:
            rc = self.L.aws_crt_amd_job_wait(job)
        if rc != 0:
            raise EngineError(f"host job failed ({rc}): {self.L.aws_crt_amd_job_last_error().decode()}")

    @property
    def device_bytes(self) -> int:
        return int(self._dev_bytes.value)

    def results(self) -> list:
        out, n = self.out, self.n
        if self.alg == XXH3_128:
            return [(out[2 * i] << 64) | out[2 * i + 1] for i in range(n)]
        return list(out[:n]) if n else []


def host_job(alg: int, ptrs: Sequence[int], lens: Sequence[int], seeds=None, ndevices: int = 0, host_threads: int = -1):
    """aws_crt_amd_host_submit_ex + aws_crt_amd_job_wait over host buffers given by raw addresses;
    returns the results (XXH3_128: 128-bit ints).  Synchronous from Python's point of view."""
    job = HostJob(alg, ptrs, lens, seeds, ndevices, host_threads)
    job.run()
    return job.results()


def register_host(addr: int, nbytes: int) -> None:
    L = lib()
    L.aws_crt_amd_register_host.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    _check(L.aws_crt_amd_register_host(addr, nbytes))


def unregister_host(addr: int) -> None:
    L = lib()
    L.aws_crt_amd_unregister_host.argtypes = [ctypes.c_void_p]
    _check(L.aws_crt_amd_unregister_host(addr))


def checksum_list_devices(alg: int, ptrs: Sequence[int], lens: Sequence[int], seeds=None) -> list:
    """Device buffers on any visible devices (raw addresses) -> results in caller order (host)."""
    L = lib()
    n = len(ptrs)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.aws_crt_amd_checksum_list_devices.argtypes = [ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(sz), sz, vp, vp]
    P = (vp * max(n, 1))(*ptrs)
    S = (sz * max(n, 1))(*lens)
    T = ctypes.c_uint64 if alg in WIDE else ctypes.c_uint32
    out = (T * max(n * (2 if alg == XXH3_128 else 1), 1))()
    sd = (T * max(n, 1))(*seeds) if seeds is not None else None
    _check(L.aws_crt_amd_checksum_list_devices(alg, P, S, n, ctypes.cast(sd, vp) if sd is not None else None,
                                               ctypes.cast(out, vp)))
    if alg == XXH3_128:
        return [(out[2 * i] << 64) | out[2 * i + 1] for i in range(n)]
    return [int(out[i]) for i in range(n)]


class _DeviceBatch(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("d_base", ctypes.c_void_p), ("stride", ctypes.c_size_t),
                ("len", ctypes.c_size_t), ("count", ctypes.c_size_t), ("d_seeds", ctypes.c_void_p),
                ("d_out", ctypes.c_void_p), ("hip_stream", ctypes.c_void_p)]


def checksum_devices(alg: int, entries) -> None:
    """aws_crt_amd_checksum_devices: entries of (device, base tensor/address, stride, len, count, seeds
    tensor or None, out tensor, stream or None); all devices at once, returns when all are done."""
    L = lib()
    n = len(entries)
    arr = (_DeviceBatch * max(n, 1))()
    for i, (dev, base, stride, ln, cnt, seeds, out, st) in enumerate(entries):
        arr[i].device = dev
        arr[i].d_base = base.data_ptr() if hasattr(base, "data_ptr") else int(base)
        arr[i].stride, arr[i].len, arr[i].count = stride, ln, cnt
        arr[i].d_seeds = seeds.data_ptr() if seeds is not None else None
        arr[i].d_out = out.data_ptr()
        arr[i].hip_stream = st.cuda_stream if st is not None else None
    L.aws_crt_amd_checksum_devices.argtypes = [ctypes.c_int, ctypes.POINTER(_DeviceBatch), ctypes.c_size_t]
    _check(L.aws_crt_amd_checksum_devices(alg, arr, n))


def checksum_list(alg: int, ptrs: Sequence[int], lens: Sequence[int], seeds=None, out=None, stream=None, device=None):
    """Ragged batch of device buffers given by raw device addresses and lengths (host lists)."""
    import torch

    n = len(ptrs)
    if out is None:
        out = torch.empty(n * (2 if alg == XXH3_128 else 1), dtype=_out_dtype(alg), device=device or "cuda")
    P = (ctypes.c_void_p * n)(*ptrs)
    S = (ctypes.c_size_t * n)(*lens)
    sp = seeds.data_ptr() if seeds is not None else None
    _check(lib().aws_crt_amd_checksum_list(alg, P, S, n, sp, out.data_ptr(), _stream_handle(stream)))
    return out


def combine_batch(alg: int, crc1, crc2, len2: Sequence[int], out=None, stream=None):
    import torch

    n = len(len2)
    if out is None:
        out = torch.empty(n, dtype=_out_dtype(alg), device=crc1.device)
    L2 = (ctypes.c_uint64 * n)(*len2)
    _check(lib().aws_crt_amd_crc_combine_batch(alg, crc1.data_ptr(), crc2.data_ptr(), L2, n, out.data_ptr(),
                                               _stream_handle(stream)))
    return out


def multipart_crc(alg: int, parts, stream=None):
    """S3 multipart composition (checksums_batch.h aws_crt_amd_multipart_crc): `parts` are device
    buffers in object order -- torch uint8 tensors or (address, length) pairs.  Returns
    (part checksums, full-object checksum, its base64 wire form)."""
    ptrs, lens = [], []
    for p in parts:
        if hasattr(p, "data_ptr"):
            ptrs.append(p.data_ptr())
            lens.append(p.numel() * p.element_size())
        else:
            ptrs.append(int(p[0]))
            lens.append(int(p[1]))
    n = len(ptrs)
    wide = alg == CRC64NVME
    part_out = (ctypes.c_uint64 * max(n, 1))() if wide else (ctypes.c_uint32 * max(n, 1))()
    obj = ctypes.c_uint64(0) if wide else ctypes.c_uint32(0)
    b64 = ctypes.create_string_buffer(16)
    P = (ctypes.c_void_p * max(n, 1))(*ptrs)
    Ls = (ctypes.c_size_t * max(n, 1))(*lens)
    _check(lib().aws_crt_amd_multipart_crc(alg, P, Ls, n, ctypes.addressof(part_out), ctypes.addressof(obj), b64,
                                           _stream_handle(stream)))
    return [int(part_out[i]) for i in range(n)], int(obj.value), b64.value.decode()


MULTIPART_FULL_OBJECT, MULTIPART_COMPOSITE = 0, 1


def multipart_checksum(alg: int, parts, type_: int = MULTIPART_COMPOSITE, stream=None):
    """aws_crt_amd_multipart_checksum: S3 multipart checksums for any of the six algorithms --
    FULL_OBJECT (CRCs: Combine of the parts) or COMPOSITE (the algorithm over the concatenated
    big-endian part digests, wire form base64 + "-N").  `parts` as multipart_crc.  Returns
    (part digests, object digest, wire form); XXH3-128 digests as 128-bit ints."""
    ptrs, lens = [], []
    for p in parts:
        if hasattr(p, "data_ptr"):
            ptrs.append(p.data_ptr())
            lens.append(p.numel() * p.element_size())
        else:
            ptrs.append(int(p[0]))
            lens.append(int(p[1]))
    n = len(ptrs)
    words = 4 if alg == XXH3_128 else 2  # 32-bit words per digest slot (CRC32/32C use the first)
    part_out = (ctypes.c_uint32 * max(n * words, 1))()
    obj = (ctypes.c_uint32 * 4)()
    b64 = ctypes.create_string_buffer(64)
    P = (ctypes.c_void_p * max(n, 1))(*ptrs)
    Ls = (ctypes.c_size_t * max(n, 1))(*lens)
    L = lib()
    L.aws_crt_amd_multipart_checksum.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                                 ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
    _check(L.aws_crt_amd_multipart_checksum(alg, type_, P, Ls, n, ctypes.addressof(part_out), ctypes.addressof(obj), b64,
                                            _stream_handle(stream)))

    def digest(raw, i):
        if alg in (CRC32, CRC32C):
            return raw[i]
        if alg == XXH3_128:
            hi = raw[4 * i] | (raw[4 * i + 1] << 32)
            lo = raw[4 * i + 2] | (raw[4 * i + 3] << 32)
            return (hi << 64) | lo
        return raw[2 * i] | (raw[2 * i + 1] << 32)

    return [digest(part_out, i) for i in range(n)], digest(obj, 0), b64.value.decode()


def checksum_host(alg: int, buffers: Sequence[bytes], seeds: Optional[Sequence[int]] = None):
    """Host buffers -> host results (synchronous): the host path, or pinned staging and the GPU when
    the dispatch mode is DISPATCH_GPU."""
    n = len(buffers)
    keep = [ctypes.create_string_buffer(bytes(b), len(b)) for b in buffers]
    P = (ctypes.c_void_p * n)(*[ctypes.addressof(k) for k in keep])
    S = (ctypes.c_size_t * n)(*[len(b) for b in buffers])
    T = ctypes.c_uint64 if alg in WIDE else ctypes.c_uint32
    out = (T * (2 * n if alg == XXH3_128 else n))()
    sd = (T * n)(*seeds) if seeds is not None else None
    _check(lib().aws_crt_amd_checksum_host(alg, P, S, n, ctypes.cast(sd, ctypes.c_void_p) if sd else None,
                                           ctypes.cast(out, ctypes.c_void_p)))
    if alg == XXH3_128:
        return [(out[2 * i] << 64) | out[2 * i + 1] for i in range(n)]
    return list(out)


def crc(alg_name: str, data, previous: int = 0) -> int:
    """aws_checksums_<alg>_ex on a bytes object (host) or a device tensor (in place)."""
    L = lib()
    f = getattr(L, f"aws_checksums_{alg_name}_ex")
    if hasattr(data, "data_ptr"):
        return f(data.data_ptr(), data.numel() * data.element_size(), previous)
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    return f(ctypes.addressof(buf), len(data), previous)


def combine(alg_name: str, crc1: int, crc2: int, len2: int) -> int:
    return getattr(lib(), f"aws_checksums_{alg_name}_combine")(crc1, crc2, len2)


def as_unsigned(t) -> list:
    """Result tensor (int32/int64 bit patterns) -> list of python unsigned ints."""
    bits = 64 if t.dtype.itemsize == 8 else 32
    mask = (1 << bits) - 1
    return [int(v) & mask for v in t.cpu().tolist()]
