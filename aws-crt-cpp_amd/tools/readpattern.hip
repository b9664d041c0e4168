// Streaming-read rate by access ORDER (diagnostic, not part of the product library).
// Every variant reads the same bytes in 4 KiB groups (8 rows of 512 B, one global_load_dwordx2 per
// lane per row), with a ring of S groups in flight per wave, and XOR-folds them.  Only the map from
// (wave, step) to group changes:
//   C  contiguous: wave w reads groups [w*n/nw, (w+1)*n/nw)               (the scans' split)
//   I  interleaved: wave w reads groups w, w + nw, w + 2 nw, ...           (the chip sweeps together)
//   B  block-contiguous: block b owns a contiguous range; its waves interleave inside it
//   X  XCD-contiguous: the blocks of one XCD (blockIdx mod 8) own one contiguous eighth; interleaved
//   K  chunked sweep: chunks of K groups per wave-step: wave w reads chunk w, w+nw, ... (K = 4, 16)
// Prints the mean hipExtLaunchKernel-stamped duration over isolated launches (one stream).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const v2u gv2u;
constexpr uint64_t GB = 4096, ROW = 512;
constexpr int RPG = 8;

template <char P, int K>
__device__ __forceinline__ uint64_t group_of(uint64_t gw, uint64_t nw, uint64_t i, uint64_t ng, uint64_t wpb) {
    if constexpr (P == 'C') {
        return gw * ng / nw + i;
    } else if constexpr (P == 'I') {
        return gw + i * nw;
    } else if constexpr (P == 'B') {
        const uint64_t nb = nw / wpb, b = gw / wpb, w = gw % wpb;
        return b * ng / nb + w + i * wpb;
    } else if constexpr (P == 'X') {
        const uint64_t b = gw / wpb, w = gw % wpb, x = b & 7, nbx = nw / wpb / 8, bx = b >> 3;
        return x * (ng / 8) + (bx * wpb + w) + i * nbx * wpb;
    } else {  // 'K': chunks of K groups
        const uint64_t c = gw + (i / K) * nw;
        return c * K + (i % K);
    }
}

template <char P, int K, int S>
__global__ __launch_bounds__(512) void readp(const uint8_t *base, uint64_t ng, unsigned *out) {
    const int lane = threadIdx.x & 63;
    constexpr uint64_t wpb = 8;
    const uint64_t nw = (uint64_t)gridDim.x * wpb, gw = (uint64_t)blockIdx.x * wpb + (threadIdx.x >> 6);
    const uint64_t nq = ng / nw;  // groups per wave (shapes divide)
    const uint64_t lo = (uint64_t)lane * 8;
    v2u r[S][RPG];
    unsigned acc = 0;
    auto ld = [&](v2u *s, uint64_t i) {
        const uint64_t g = group_of<P, K>(gw, nw, i < nq ? i : 0, ng, wpb);
        const uint64_t a = (uint64_t)base + g * GB + lo;
#pragma unroll
        for (int k = 0; k < RPG; ++k) s[k] = __builtin_nontemporal_load((gv2u *)(a + k * ROW));
    };
#pragma unroll
    for (int j = 0; j < S - 1; ++j) ld(r[j], j);
    // as the scans: row k of the slot S-1 ahead is issued beside row k of the slot being consumed
    for (uint64_t i = 0; i < nq; i += S) {
#pragma unroll
        for (int j = 0; j < S; ++j) {
            const uint64_t ii = i + j + S - 1;
            const uint64_t g = ii < nq ? group_of<P, K>(gw, nw, ii, ng, wpb) : 0;  // past the end: one L2-resident group
            const uint64_t a = (uint64_t)base + g * GB + lo;
#pragma unroll
            for (int k = 0; k < RPG; ++k) {
                r[(j + S - 1) % S][k] = __builtin_nontemporal_load((gv2u *)(a + k * ROW));
                acc = acc * 3u ^ r[j][k].x ^ r[j][k].y;
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    if (acc == 0x12345678u) out[gw] = acc;
}

struct Variant {
    const char *name;
    void (*k)(const uint8_t *, uint64_t, unsigned *);
    int wpc;
};

int main(int argc, char **argv) {
    const uint64_t bytes = (argc > 1 ? atoll(argv[1]) : 1280) << 20;
    const int iso = argc > 2 ? atoi(argv[2]) : 16;
    const uint64_t ng = bytes / GB;
    uint8_t *buf;
    unsigned *out;
    CK(hipMalloc(&buf, bytes * 2));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(buf, 0x5a, bytes * 2));
    std::vector<Variant> vs = {
        {"C S3 x2", readp<'C', 1, 3>, 2}, {"I S3 x2", readp<'I', 1, 3>, 2}, {"B S3 x2", readp<'B', 1, 3>, 2},
        {"X S3 x2", readp<'X', 1, 3>, 2}, {"K4 S3 x2", readp<'K', 4, 3>, 2}, {"K16 S3 x2", readp<'K', 16, 3>, 2},
        {"C S3 x1", readp<'C', 1, 3>, 1}, {"I S3 x1", readp<'I', 1, 3>, 1}, {"C S4 x2", readp<'C', 1, 4>, 2},
        {"I S4 x2", readp<'I', 1, 4>, 2}, {"C S2 x2", readp<'C', 1, 2>, 2}, {"I S2 x2", readp<'I', 1, 2>, 2},
    };
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    std::vector<hipEvent_t> e0(iso), e1(iso);
    for (int i = 0; i < iso; ++i) {
        CK(hipEventCreate(&e0[i]));
        CK(hipEventCreate(&e1[i]));
    }
    std::printf("{\"bytes\": %llu, \"launches\": %d, \"variants\": {", (unsigned long long)bytes, iso);
    for (int rep = 0; rep < 2; ++rep)
        for (size_t vi = 0; vi < vs.size(); ++vi) {
            auto &v = vs[vi];
            const dim3 grid(256 * v.wpc), blk(512);
            const uint64_t nw = 256ull * v.wpc * 8;
            const uint64_t ngu = ng / (nw * 16) * (nw * 16);  // K | groups per wave
            for (int i = 0; i < 4; ++i) hipLaunchKernelGGL(v.k, grid, blk, 0, st, buf + (i & 1) * bytes, ngu, out);
            CK(hipStreamSynchronize(st));
            for (int i = 0; i < iso; ++i)
                hipExtLaunchKernelGGL(v.k, grid, blk, 0, st, e0[i], e1[i], 0, buf + (i & 1) * bytes, ngu, out);
            CK(hipStreamSynchronize(st));
            double sum = 0;
            for (int i = 0; i < iso; ++i) {
                float ms;
                CK(hipEventElapsedTime(&ms, e0[i], e1[i]));
                sum += ms;
            }
            const double us = 1e3 * sum / iso;
            std::printf("%s\"%s r%d\": [%.2f, %.1f, %llu]", (rep || vi) ? ", " : "", v.name, rep, us, ngu * GB / us * 1e-3,
                        (unsigned long long)(ngu * GB >> 20));
            std::fflush(stdout);
        }
    std::printf("}}\n");
    return 0;
}
