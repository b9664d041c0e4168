// Small-call latency of the value-only ABI, in C++ (no ctypes): the reference's
// per-call shape, Aws::Crt::Checksum::ComputeCRC32C(cursor, previous) -> aws_checksums_crc32c_ex
// (source/checksum/CRC.cpp:20-23), on 8, 12, 32 and 4096-byte host buffers (heap and stack), in AUTO
// (the pointer classified first) and forced-CPU mode, plus hipPointerGetAttributes alone on the same
// pointers, and a device pointer in AUTO (classified as device: the GPU path).
//   experiments/build/abi_latency [reps]   -> one JSON line
#include <hip/hip_runtime.h>

#include <aws/checksums/crc.h>
#include <aws_crt_amd/checksums_batch.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {
double ns_per(size_t reps, const std::chrono::steady_clock::time_point &t0) {
    return std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count() / (double)reps;
}
volatile uint32_t g_sink;

template <class F>
double best_of(int rounds, size_t reps, F &&f) {
    double best = 1e30;
    for (int r = 0; r < rounds; ++r) {
        const auto t0 = std::chrono::steady_clock::now();
        for (size_t i = 0; i < reps; ++i) f(i);
        const double v = ns_per(reps, t0);
        if (v < best) best = v;
    }
    return best;
}
}  // namespace

int main(int argc, char **argv) {
    const size_t reps = argc > 1 ? (size_t)std::atoll(argv[1]) : 200000;
    aws_crt_amd_init();
    const size_t sizes[] = {8, 12, 32, 4096};
    std::vector<unsigned char> heap(8192);
    for (size_t i = 0; i < heap.size(); ++i) heap[i] = (unsigned char)(i * 131 + 7);
    unsigned char stack[8192];
    std::memcpy(stack, heap.data(), sizeof(stack));
    std::printf("{\"reps\": %zu, \"rows\": [", reps);
    bool first = true;
    for (size_t n : sizes) {
        for (int where = 0; where < 2; ++where) {
            const uint8_t *p = where ? stack : heap.data();
            aws_crt_amd_set_dispatch(AWS_CRT_AMD_DISPATCH_AUTO);
            const double autons = best_of(5, reps, [&](size_t i) { g_sink = aws_checksums_crc32c_ex(p, n, (uint32_t)i); });
            aws_crt_amd_set_dispatch(AWS_CRT_AMD_DISPATCH_CPU);
            const double cpuns = best_of(5, reps, [&](size_t i) { g_sink = aws_checksums_crc32c_ex(p, n, (uint32_t)i); });
            aws_crt_amd_set_dispatch(AWS_CRT_AMD_DISPATCH_AUTO);
            const double probe = best_of(5, reps, [&](size_t) {
                hipPointerAttribute_t a;
                if (hipPointerGetAttributes(&a, p) != hipSuccess) (void)hipGetLastError();
                g_sink = (uint32_t)a.type;
            });
            std::printf("%s{\"bytes\": %zu, \"memory\": \"%s\", \"auto_ns\": %.1f, \"cpu_ns\": %.1f, \"ratio\": %.2f, "
                        "\"hipPointerGetAttributes_ns\": %.1f}",
                        first ? "" : ", ", n, where ? "stack" : "heap", autons, cpuns, autons / cpuns, probe);
            first = false;
        }
    }
    // a device buffer through the same call (AUTO classifies it as device: kernel + sync per call)
    void *d = nullptr;
    double devns = -1;
    if (hipMalloc(&d, 4096) == hipSuccess) {
        (void)hipMemcpy(d, heap.data(), 4096, hipMemcpyHostToDevice);
        const uint32_t want = aws_checksums_crc32c_ex(heap.data(), 4096, 0);
        const uint32_t got = aws_checksums_crc32c_ex((const uint8_t *)d, 4096, 0);
        devns = best_of(3, 2000, [&](size_t i) { g_sink = aws_checksums_crc32c_ex((const uint8_t *)d, 4096, (uint32_t)i); });
        std::printf("], \"device_4096_ns\": %.1f, \"device_parity\": %s, \"fallbacks\": %llu}\n", devns,
                    got == want ? "true" : "false", (unsigned long long)aws_crt_amd_fallback_count());
        (void)hipFree(d);
    } else {
        std::printf("], \"device_4096_ns\": null}\n");
    }
    return 0;
}
