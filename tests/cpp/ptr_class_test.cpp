// The value-only ABI's pointer classifier (aws-crt-cpp_amd/csrc/ptr_class.h) with a stand-in for the
// runtime probe: the thread's stack and recently seen unregistered-host windows never reach the
// probe; runtime-known host memory (pinned / registered) and device memory always do; the windows are
// per thread; AWS_CRT_AMD_PTR_CACHE=0 probes every call.  Built under ASan by tests/test_abi.py.
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "ptr_class.h"

namespace {
int fails = 0;
#define CHECK(c)                                                     \
    do {                                                             \
        if (!(c)) {                                                  \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                 \
        }                                                            \
    } while (0)

// stand-in address map: [dev_lo, dev_hi) device, [pin_lo, pin_hi) pinned host, the rest unregistered
uintptr_t dev_lo, dev_hi, pin_lo, pin_hi;
int probe(const void *p) {
    const uintptr_t a = (uintptr_t)p;
    if (a >= dev_lo && a < dev_hi) return 2;
    if (a >= pin_lo && a < pin_hi) return 1;
    return 0;
}
using C = amdcrc::PtrClass<probe>;
}  // namespace

int main(int argc, char **argv) {
    const bool off = argc > 1;  // run with AWS_CRT_AMD_PTR_CACHE=0 and an argument
    std::vector<unsigned char> heap(1 << 20), dev(1 << 20), pin(1 << 20);
    dev_lo = (uintptr_t)dev.data(), dev_hi = dev_lo + dev.size();
    pin_lo = (uintptr_t)pin.data(), pin_hi = pin_lo + pin.size();
    unsigned char stack_buf[64];
    auto &t = C::tls();
    uint64_t p0 = t.probes;
    for (int i = 0; i < 1000; ++i) CHECK(C::classify(stack_buf + (i & 63)) == amdcrc::PtrKind::Host);
    CHECK(t.probes - p0 == (off ? 1000u : 0u));  // the thread's own stack: no probe
    p0 = t.probes;
    for (int i = 0; i < 1000; ++i) CHECK(C::classify(heap.data() + 8 * (i % 64)) == amdcrc::PtrKind::Host);
    CHECK(t.probes - p0 == (off ? 1000u : 1u));  // one probe, then the window
    p0 = t.probes;
    for (int i = 0; i < 100; ++i) CHECK(C::classify(dev.data() + i) == amdcrc::PtrKind::Device);
    CHECK(t.probes - p0 == 100);  // device memory is always asked about
    p0 = t.probes;
    for (int i = 0; i < 100; ++i) CHECK(C::classify(pin.data() + i) == amdcrc::PtrKind::Host);
    CHECK(t.probes - p0 == 100);  // runtime-known host memory is not cached
    // more windows than the cache holds: the oldest is asked about again
    p0 = t.probes;
    for (int w = 0; w < 6; ++w) (void)C::classify(heap.data() + (size_t)w * 65536 * 2 + 100);
    CHECK(t.probes - p0 == (off ? 6u : 5u));  // the first window (already cached above) hits
    // another thread has its own stack and windows
    std::thread th([&] {
        auto &u = C::tls();
        unsigned char mine[32];
        CHECK(C::classify(mine) == amdcrc::PtrKind::Host);
        CHECK(u.probes == (off ? 1u : 0u));
        CHECK(C::classify(stack_buf) == amdcrc::PtrKind::Host);  // main's stack: unregistered host, probed
        CHECK(u.probes == (off ? 2u : 1u));
        CHECK(C::classify(dev.data()) == amdcrc::PtrKind::Device);
    });
    th.join();
    std::printf(fails ? "[FAIL] PtrClass\n" : "[PASS] PtrClass\n");
    return fails ? 1 : 0;
}
