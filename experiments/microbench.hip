// Diagnostic microbenchmark for the scan kernel's design space (not part of the product library).
// All variants run in one process, interleaved, timed with HIP events (cdna guide 5.4 rule 24).
//
//   MODE 0  read only: lane-contiguous segments (the product layout), 64-B groups, XOR-reduce
//   MODE 1  MODE 0 + the 128 KiB LDS table build
//   MODE 2  full CRC32C slice-by-4 inner loop (replicated LDS tables, v_perm addressing)
//   MODE 3  read only, coalesced layout (lane-interleaved 16-B vectors)
//   MODE 4  CRC32C inner loop with 2 independent streams per lane (ILP 2)
//
// usage: microbench [batch_MiB=64] [seg=256] [iters=200] [rotate=8]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) {                                                                  \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u gv4u;

constexpr uint32_t POLY = 0x82F63B78u;
constexpr int kBlock = 1024, kWaves = 16;

__device__ __forceinline__ uint32_t lds32(const char *L, uint32_t a) { return *(const uint32_t *)(L + a); }

struct Ring {
    v4u v[4];
};

__device__ __forceinline__ void ld(Ring &r, uint64_t a) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r.v[i] = ((gv4u *)a)[i];
}

__device__ __forceinline__ uint32_t crcw(uint32_t s, uint32_t w, const char *L, uint32_t srcA, uint32_t srcB) {
    s ^= w;
    const uint32_t a3 = __builtin_amdgcn_perm(srcB, s, 0x0c060004u);
    const uint32_t a2 = __builtin_amdgcn_perm(srcB, s, 0x0c060104u);
    const uint32_t a1 = __builtin_amdgcn_perm(srcA, s, 0x0c060204u);
    const uint32_t a0 = __builtin_amdgcn_perm(srcA, s, 0x0c060304u);
    return lds32(L, a3 + 128) ^ lds32(L, a2) ^ lds32(L, a1 + 128) ^ lds32(L, a0);
}

template <int MODE>
__global__ __launch_bounds__(kBlock, 1) void scan(const uint8_t *base, uint64_t ntiles, uint32_t seg, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) char lds[131072];
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * kWaves;
    const uint64_t gw = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    const uint64_t t0 = gw * ntiles / nw, t1 = (gw + 1) * ntiles / nw;
    const uint32_t ng = seg / 64;
    const uint64_t tile = 64ull * seg;
    const uint64_t q0 = t0 * ng, q1 = t1 * ng;  // flattened group index range
    auto addr = [&](uint64_t q) -> uint64_t {
        const uint64_t qq = q < q1 ? q : q1 - 1;
        const uint64_t t = qq / ng, g = qq - t * ng;
        return (uint64_t)base + t * tile + (uint64_t)lane * seg + g * 64;
    };
    // MODE 3 (coalesced): group g of tile t covers 4 KiB = 64 lanes x 64 B as four 1 KiB wave loads
    auto addr3 = [&](uint64_t q, int i) -> uint64_t {
        const uint64_t qq = q < q1 ? q : q1 - 1;
        const uint64_t t = qq / ng, g = qq - t * ng;
        return (uint64_t)base + t * tile + g * 4096 + (uint64_t)i * 1024 + lane * 16;
    };
    Ring r0, r1, r2;
    auto issue = [&](Ring &r, uint64_t q) {
        if (MODE == 3) {
#pragma unroll
            for (int i = 0; i < 4; ++i) r.v[i] = *(gv4u *)addr3(q, i);
        } else {
            ld(r, addr(q));
        }
    };
    if (q0 < q1) {
        issue(r0, q0);
        issue(r1, q0 + 1);
    }
    if (MODE == 1 || MODE == 2 || MODE == 4) {
        for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) {
            const int k = (int)(i >> 8);
            const uint32_t e = i & 255u;
            uint32_t c = e;
            for (int b = 0; b < 8 * (k + 1); ++b) c = (c >> 1) ^ ((c & 1) ? POLY : 0);
            const uint32_t bse = ((uint32_t)(k >> 1) << 16) | (e << 8) | ((uint32_t)(k & 1) << 7);
            const uint4 vv = make_uint4(c, c, c, c);
#pragma unroll
            for (int j = 0; j < 8; ++j) *(uint4 *)(lds + bse + ((j + i) & 7u) * 16) = vv;
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    const uint32_t srcA = (uint32_t)(lane & 31) << 2, srcB = srcA | 0x10000u;
    uint32_t s = 0, s2 = 0, acc = 0;
    auto proc = [&](const Ring &r) {
        if (MODE == 2) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                s = crcw(s, r.v[i].x, lds, srcA, srcB);
                s = crcw(s, r.v[i].y, lds, srcA, srcB);
                s = crcw(s, r.v[i].z, lds, srcA, srcB);
                s = crcw(s, r.v[i].w, lds, srcA, srcB);
            }
        } else if (MODE == 4) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                s = crcw(s, r.v[i].x, lds, srcA, srcB);
                s2 = crcw(s2, r.v[i + 2].x, lds, srcA, srcB);
                s = crcw(s, r.v[i].y, lds, srcA, srcB);
                s2 = crcw(s2, r.v[i + 2].y, lds, srcA, srcB);
                s = crcw(s, r.v[i].z, lds, srcA, srcB);
                s2 = crcw(s2, r.v[i + 2].z, lds, srcA, srcB);
                s = crcw(s, r.v[i].w, lds, srcA, srcB);
                s2 = crcw(s2, r.v[i + 2].w, lds, srcA, srcB);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) acc ^= r.v[i].x ^ r.v[i].y ^ r.v[i].z ^ r.v[i].w;
        }
    };
    for (uint64_t q = q0; q < q1; q += 3) {
        issue(r2, q + 2);
        proc(r0);
        if (q + 1 >= q1) break;
        issue(r0, q + 3);
        proc(r1);
        if (q + 2 >= q1) break;
        issue(r1, q + 4);
        proc(r2);
    }
    out[gw * 64 + lane] = acc ^ s ^ s2;
}

template <int MODE>
float run(const uint8_t *d, uint64_t batch, int rotate, uint32_t seg, int iters, uint32_t *out, int cus) {
    const uint64_t tile = 64ull * seg, ntiles = batch / tile;
    const int blocks = (int)std::min<uint64_t>((ntiles + kWaves - 1) / kWaves, (uint64_t)cus);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(scan<MODE>, dim3(blocks), dim3(kBlock), 0, 0, d + (i % rotate) * batch, ntiles, seg, out);
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL(scan<MODE>, dim3(blocks), dim3(kBlock), 0, 0, d + (i % rotate) * batch, ntiles, seg, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / iters;
}

int main(int argc, char **argv) {
    const uint64_t mib = argc > 1 ? std::atoll(argv[1]) : 64;
    const uint32_t seg = argc > 2 ? std::atoi(argv[2]) : 256;
    const int iters = argc > 3 ? std::atoi(argv[3]) : 200;
    const int rotate = argc > 4 ? std::atoi(argv[4]) : 8;
    const uint64_t batch = mib << 20;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    uint8_t *d;
    uint32_t *out;
    CK(hipMalloc(&d, batch * rotate));
    CK(hipMalloc(&out, 64ull * 256 * kWaves * 4 * 4));
    std::vector<uint8_t> h(1 << 20);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint8_t)(i * 2654435761u >> 13);
    for (uint64_t o = 0; o < batch * rotate; o += h.size()) CK(hipMemcpy(d + o, h.data(), h.size(), hipMemcpyHostToDevice));
    const int cus = prop.multiProcessorCount;
    const char *names[] = {"read lane-contig", "read + table build", "crc32c slice4", "read coalesced", "crc32c ILP2"};
    for (int round = 0; round < 3; ++round) {
        float t[5];
        t[0] = run<0>(d, batch, rotate, seg, iters, out, cus);
        t[1] = run<1>(d, batch, rotate, seg, iters, out, cus);
        t[2] = run<2>(d, batch, rotate, seg, iters, out, cus);
        t[3] = run<3>(d, batch, rotate, seg, iters, out, cus);
        t[4] = run<4>(d, batch, rotate, seg, iters, out, cus);
        for (int m = 0; m < 5; ++m)
            std::printf("round %d batch %4llu MiB seg %4u  %-20s %8.2f us  %7.1f GB/s\n", round, (unsigned long long)mib, seg,
                        names[m], t[m] * 1e3, batch / (t[m] * 1e-3) / 1e9);
    }
    return 0;
}
