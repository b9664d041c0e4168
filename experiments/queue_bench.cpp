// Submission-queue rate from C++ (diagnostic, not part of the product library): the driver's C2
// workload (K steps of 1024 x 64 KiB CRC32C, device-resident, K rotating batches) submitted three ways
// through the engine's C ABI, each timed on the host clock between two device synchronisations:
//   batches  aws_crt_amd_checksum_batches over all K (one launch per <= 32)
//   single   one aws_crt_amd_checksum_strided per batch, over three streams
//   queue    one aws_crt_amd_queue_push per batch, then aws_crt_amd_queue_flush
// Prints one JSON line (GiB/s, median of reps).  Build: make -C aws-crt-cpp_amd/tools queue_bench
#include <hip/hip_runtime.h>

#include <aws/checksums/crc.h>
#include <aws_crt_amd/checksums_batch.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)
#define OK(x)                                                                              \
    do {                                                                                   \
        int r_ = (x);                                                                      \
        if (r_ != 0) {                                                                     \
            std::fprintf(stderr, "%s:%d engine error %d: %s\n", __FILE__, __LINE__, r_,   \
                         aws_crt_amd_last_error());                                        \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

int main(int argc, char **argv) {
    const int K = argc > 1 ? std::atoi(argv[1]) : 20, reps = argc > 2 ? std::atoi(argv[2]) : 9;
    const size_t n = 1024, L = 65536, step = n * L;
    uint8_t *data;
    uint32_t *out;
    CK(hipMalloc(&data, step * K));
    CK(hipMalloc(&out, 4 * n * K));
    std::vector<uint8_t> h(step);
    for (size_t i = 0; i < step; ++i) h[i] = (uint8_t)(i * 2654435761u >> 13);
    for (int k = 0; k < K; ++k) CK(hipMemcpy(data + k * step, h.data(), step, hipMemcpyHostToDevice));
    hipStream_t st[3];
    for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<aws_crt_amd_batch> bs(K);
    for (int k = 0; k < K; ++k) bs[k] = {data + k * step, nullptr, out + k * n};
    auto run = [&](int how) {
        if (how == 0) {
            OK(aws_crt_amd_checksum_batches(1, bs.data(), K, L, L, n, st[0]));
        } else if (how == 1) {
            for (int k = 0; k < K; ++k) OK(aws_crt_amd_checksum_strided(1, data + k * step, L, L, n, nullptr, out + k * n, st[k % 3]));
        } else {
            aws_crt_amd_queue *q;
            OK(aws_crt_amd_queue_create(1, L, L, n, st[0], &q));
            for (int k = 0; k < K; ++k) OK(aws_crt_amd_queue_push(q, data + k * step, nullptr, out + k * n));
            OK(aws_crt_amd_queue_flush(q));
            OK(aws_crt_amd_queue_destroy(q));
        }
    };
    const char *names[3] = {"batches", "single", "queue"};
    double rate[3];
    for (int how = 0; how < 3; ++how) {
        run(how);  // warm-up: tables, workspaces, staging on every stream
        run(how);
        CK(hipDeviceSynchronize());
        std::vector<double> v;
        for (int r = 0; r < reps; ++r) {
            CK(hipDeviceSynchronize());
            const auto t0 = std::chrono::steady_clock::now();
            run(how);
            CK(hipDeviceSynchronize());
            v.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        }
        std::sort(v.begin(), v.end());
        rate[how] = (double)step * K / v[v.size() / 2] / (1u << 30);
    }
    // every path's results against the engine's host path over the same bytes (every batch holds h)
    std::vector<uint32_t> want(n);
    for (size_t i = 0; i < n; ++i) want[i] = aws_checksums_crc32c_ex(h.data() + i * L, L, 0);
    int bad[3] = {0, 0, 0};
    for (int how = 0; how < 3; ++how) {
        std::vector<uint32_t> got(n * K);
        CK(hipMemset(out, 0, 4 * n * K));
        CK(hipDeviceSynchronize());
        run(how);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), out, 4 * n * K, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n * K; ++i) bad[how] += got[i] != want[i % n];
    }
    std::printf("{\"steps\": %d, \"reps\": %d, \"gibs\": {\"%s\": %.1f, \"%s\": %.1f, \"%s\": %.1f}, "
                "\"wrong_results\": {\"%s\": %d, \"%s\": %d, \"%s\": %d}}\n",
                K, reps, names[0], rate[0], names[1], rate[1], names[2], rate[2], names[0], bad[0], names[1], bad[1], names[2], bad[2]);
    return 0;
}
