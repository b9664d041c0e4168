// Host / device classification of the value-only ABI's input pointer (abi_single.cpp checksum_one),
// without entering the HIP runtime on the common host call.
//
// The reference's per-call shape is one small host buffer per call (aws-c-event-stream's 8-byte
// prelude CRC, headers: ComputeCRC32 / aws_checksums_crc32_ex, source/checksum/CRC.cpp:15-23).
// hipPointerGetAttributes costs ~130 ns; the CRC of 32 bytes ~20 ns.  So a thread remembers what it
// already knows to be host memory and only asks the runtime about the rest:
//   * its own stack (pthread_getattr_np, once per thread): a stack is never device memory;
//   * the last kWindows 64 KiB windows in which the runtime reported a pointer as unregistered host
//     memory (memory the HIP runtime does not know).  Device memory (hipMalloc) lives in the GPU VM
//     apertures the runtime reserves when it starts and keeps for the process's life, so a window of
//     OS-allocated host memory never turns into device memory; pinned / registered host memory
//     (runtime-known) is not cached at all.  Memory that becomes managed later is CPU-accessible, so
//     a stale window still computes the right value on the host path.
// AWS_CRT_AMD_PTR_CACHE=0 turns the windows off (every call asks the runtime).
#pragma once

#include <pthread.h>

#include <cstdint>
#include <cstdlib>

namespace amdcrc {

enum class PtrKind { Host, Device };

// Probe: PtrKind-or-unknown classification by the runtime: returns 0 = unregistered host (cacheable),
// 1 = runtime-known host (pinned / registered), 2 = device / managed / unified.
template <int (*Probe)(const void *)>
struct PtrClass {
    static constexpr int kWindows = 4;
    static constexpr unsigned kWindowShift = 16;  // 64 KiB

    struct Tls {
        uintptr_t stack_lo = 0, stack_hi = 0;
        bool stack_known = false;
        uintptr_t win[kWindows] = {~(uintptr_t)0, ~(uintptr_t)0, ~(uintptr_t)0, ~(uintptr_t)0};
        unsigned next = 0;
        uint64_t probes = 0;  // runtime calls made by this thread (tests)
    };
    static Tls &tls() {
        static thread_local Tls t;
        return t;
    }
    static bool enabled() {
        static const bool on = [] {
            const char *e = std::getenv("AWS_CRT_AMD_PTR_CACHE");
            return !(e && e[0] == '0');
        }();
        return on;
    }
    static void learn_stack(Tls &t) {
        t.stack_known = true;
        pthread_attr_t at;
        if (pthread_getattr_np(pthread_self(), &at) != 0) return;
        void *lo = nullptr;
        size_t sz = 0;
        if (pthread_attr_getstack(&at, &lo, &sz) == 0 && lo && sz) {
            t.stack_lo = (uintptr_t)lo;
            t.stack_hi = (uintptr_t)lo + sz;
        }
        pthread_attr_destroy(&at);
    }

    static PtrKind classify(const void *p) {
        const uintptr_t a = (uintptr_t)p;
        Tls &t = tls();
        if (enabled()) {
            if (!t.stack_known) learn_stack(t);
            if (a - t.stack_lo < t.stack_hi - t.stack_lo) return PtrKind::Host;
            const uintptr_t w = a >> kWindowShift;
            for (int i = 0; i < kWindows; ++i)
                if (t.win[i] == w) return PtrKind::Host;
        }
        ++t.probes;
        const int k = Probe(p);
        if (k == 2) return PtrKind::Device;
        if (k == 0 && enabled()) {
            t.win[t.next] = a >> kWindowShift;
            t.next = (t.next + 1) % kWindows;
        }
        return PtrKind::Host;
    }
};

}  // namespace amdcrc
