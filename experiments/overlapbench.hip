// Why do HBM streaming and LDS-table CRC work add instead of overlap?  (diagnostic)
// One persistent 1024-thread WG per CU, 128 KiB replicated slice-4 tables, 1 GiB rotated input.
//   C  compute only (CRC on register data, no loads)
//   M  memory only (XOR of loads)
//   S  split: waves 0-7 memory only, waves 8-15 compute only (same CU, independent)
//   D  decoupled: every wave loads (XOR) AND runs the CRC on register data (no dependency)
//   R  real: CRC consumes the loaded words
//   R3 real, XOR chain merged (v_bitop3 3-input XOR)
// Each variant also reports the in-kernel shader clock: d(s_memtime) / d(s_memrealtime) x 100 MHz.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t err_ = (x);                                                                  \
        if (err_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(err_)); \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u gv4u;
constexpr uint32_t POLY = 0x82F63B78u;
__device__ __forceinline__ uint32_t lds32(const char *L, uint32_t a) { return *(const uint32_t *)(L + a); }

template <bool MERGE>
__device__ __forceinline__ uint32_t crcw(uint32_t s, uint32_t w, const char *L, uint32_t srcA, uint32_t srcB) {
    s ^= w;
    const uint32_t a3 = __builtin_amdgcn_perm(srcB, s, 0x0c060004u);
    const uint32_t a2 = __builtin_amdgcn_perm(srcB, s, 0x0c060104u);
    const uint32_t a1 = __builtin_amdgcn_perm(srcA, s, 0x0c060204u);
    const uint32_t a0 = __builtin_amdgcn_perm(srcA, s, 0x0c060304u);
    uint32_t l3 = lds32(L, a3 + 128), l2 = lds32(L, a2), l1 = lds32(L, a1 + 128), l0 = lds32(L, a0);
    if (MERGE) {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(l3), "+v"(l2), "+v"(l1), "+v"(l0));
        uint32_t r, q;
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(q) : "v"(l3), "v"(l2), "v"(l1));
        return q ^ l0;
    }
    return l3 ^ l2 ^ l1 ^ l0;
}

struct Clk {
    uint64_t t, rt;
};
__device__ __forceinline__ Clk stamp() {
    Clk c;
    c.t = __builtin_amdgcn_s_memtime();
    c.rt = __builtin_amdgcn_s_memrealtime();
    return c;
}

template <int MODE, int SEGL = 64>
__global__ __launch_bounds__(1024, 4) void k(const uint8_t *base, uint64_t bytes, uint32_t *out, uint64_t *clk) {
    __shared__ __attribute__((aligned(16))) char lds[131072];
    for (uint32_t i = threadIdx.x; i < 1024; i += 1024) {
        const int kk = (int)(i >> 8);
        const uint32_t e = i & 255u;
        uint32_t c = e;
        for (int b = 0; b < 8 * (kk + 1); ++b) c = (c >> 1) ^ ((c & 1) ? POLY : 0);
        const uint32_t bse = ((uint32_t)(kk >> 1) << 16) | (e << 8) | ((uint32_t)(kk & 1) << 7);
        const uint4 vv = make_uint4(c, c, c, c);
#pragma unroll
        for (int j = 0; j < 8; ++j) *(uint4 *)(lds + bse + ((j + i) & 7u) * 16) = vv;
    }
    __syncthreads();
    const Clk c0 = stamp();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t srcA = (uint32_t)(lane & 31) << 2, srcB = srcA | 0x10000u;
    // each wave owns a contiguous slab; lane-contiguous 64-B groups, two groups in flight
    const uint64_t nw = (uint64_t)gridDim.x * 16, gw = (uint64_t)blockIdx.x * 16 + wave;
    const uint64_t slab = bytes / nw, ng = slab / 4096;
    const uint64_t b0 = (uint64_t)base + gw * slab + (uint64_t)lane * 64;
    const bool do_mem = MODE != 0 && !(MODE == 2 && wave >= 8);
    const bool do_crc = MODE != 1 && !(MODE == 2 && wave < 8);
    uint32_t s = lane, acc = 0;
    v4u r0[4], r1[4], r2[4];
    auto issue = [&](v4u (&r)[4], uint64_t g) {
        const uint64_t gg = g < ng ? g : ng - 1;
        uint64_t a;
        if (SEGL == 64) {
            a = b0 + gg * 4096;
        } else if (SEGL > 0) {  // lane l owns [l*SEGL, (l+1)*SEGL) of each 64*SEGL tile
            constexpr uint64_t gpt = SEGL / 64;
            const uint64_t t = gg / gpt, j = gg % gpt;
            a = b0 - (uint64_t)lane * 64 + t * 64 * SEGL + (uint64_t)lane * SEGL + j * 64;
        } else if (SEGL == -1) {  // braided dwords: 16 rows of 256 B, lane l reads word l of each
            const uint64_t rb = b0 - (uint64_t)lane * 64 + gg * 4096 + (uint64_t)lane * 4;
            typedef __attribute__((address_space(1))) const uint32_t gu32;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                r[i].x = *(gu32 *)(rb + 1024 * i);
                r[i].y = *(gu32 *)(rb + 1024 * i + 256);
                r[i].z = *(gu32 *)(rb + 1024 * i + 512);
                r[i].w = *(gu32 *)(rb + 1024 * i + 768);
            }
            return;
        } else {  // coalesced: 4 x 1 KiB, lane l reads 16 B of each
            a = b0 - (uint64_t)lane * 64 + gg * 4096 + (uint64_t)lane * 16;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) r[i] = *(gv4u *)(a + (SEGL > 0 ? 16 : 1024) * i);
    };
    auto proc = [&](const v4u (&r)[4], uint64_t g) {
        if (MODE == 6) asm volatile("" ::: "memory");  // burst: no load may move into the CRC steps
        if (MODE == 4 || MODE == 5 || MODE == 6) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                s = crcw<MODE == 5>(s, r[i].x, lds, srcA, srcB);
                s = crcw<MODE == 5>(s, r[i].y, lds, srcA, srcB);
                s = crcw<MODE == 5>(s, r[i].z, lds, srcA, srcB);
                s = crcw<MODE == 5>(s, r[i].w, lds, srcA, srcB);
                if (MODE == 6 && i == 3) asm volatile("" ::: "memory");
            }
            return;
        }
        if (do_mem) {
#pragma unroll
            for (int i = 0; i < 4; ++i) acc ^= r[i].x ^ r[i].y ^ r[i].z ^ r[i].w;
        }
        if (do_crc) {
#pragma unroll
            for (int i = 0; i < 16; ++i) s = crcw<false>(s, (uint32_t)(g * 16 + i), lds, srcA, srcB);
        }
    };
    if (do_mem) {
        issue(r0, 0);
        issue(r1, 1);
    }
    for (uint64_t g = 0; g < ng; g += 3) {
        if (do_mem) issue(r2, g + 2);
        proc(r0, g);
        if (g + 1 >= ng) break;
        if (do_mem) issue(r0, g + 3);
        proc(r1, g + 1);
        if (g + 2 >= ng) break;
        if (do_mem) issue(r1, g + 4);
        proc(r2, g + 2);
    }
    const Clk c1 = stamp();
    out[gw * 64 + lane] = acc ^ s;
    if (lane == 0) {
        clk[2 * gw] = c1.t - c0.t;
        clk[2 * gw + 1] = c1.rt - c0.rt;
    }
}

static hipStream_t g_st[2];
static int g_streams = 1;

template <int MODE, int SEGL = 64>
void run(const char *name, const uint8_t *d, uint64_t bytes, int rotate, uint32_t *out, uint64_t *clk, int cus) {
    // every wave's slab must hold whole tiles of the layout, or lanes would read past the allocation
    const uint64_t slab = bytes / ((uint64_t)cus * 16), unit = SEGL > 0 ? 64ull * SEGL : 4096;  // SEGL <= 0: 4 KiB groups
    if (bytes % ((uint64_t)cus * 16) != 0 || slab % unit != 0 || slab < unit) {
        std::printf("%-34s skipped (slab %llu B not a multiple of %llu)\n", name, (unsigned long long)slab, (unsigned long long)unit);
        return;
    }
    hipEvent_t a, b, j;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventCreate(&j));
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL((k<MODE, SEGL>), dim3(cus), dim3(1024), 0, 0, d + (i % rotate) * bytes, bytes, out, clk);
    CK(hipDeviceSynchronize());
    const int reps = bytes >= (512ull << 20) ? 20 : 400;
    CK(hipEventRecord(a, g_st[0]));
    CK(hipStreamWaitEvent(g_st[1], a, 0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((k<MODE, SEGL>), dim3(cus), dim3(1024), 0, g_st[i % g_streams], d + (i % rotate) * bytes, bytes,
                           out + (i % g_streams) * cus * 1024, clk);
    CK(hipEventRecord(j, g_st[1]));
    CK(hipStreamWaitEvent(g_st[0], j, 0));
    CK(hipEventRecord(b, g_st[0]));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint64_t> h(2 * (size_t)cus * 16);
    CK(hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost));
    double cyc = 0, rt = 0;
    for (size_t i = 0; i < h.size(); i += 2) cyc += h[i], rt += h[i + 1];
    const double ghz = cyc / rt * 0.1;
    const double t = ms / reps * 1e-3;
    std::printf("%-34s %8.1f us  %7.1f GB/s   clock %.2f GHz\n", name, t * 1e6, bytes / t / 1e9, ghz);
}

__global__ void fill(uint32_t *p, uint64_t n, int pattern) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t x = i * 0x9E3779B97F4A7C15ull;
        x ^= x >> 29;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 32;
        p[i] = pattern == 1 ? (uint32_t)x : pattern == 2 ? ((uint32_t)x & 0x0F0F0F0Fu) : 0x5A5A5A5Au;
    }
}

int main(int argc, char **argv) {
    const int pattern = argc > 1 ? std::atoi(argv[1]) : 1;  // 0 constant, 1 random, 2 half-entropy
    const uint64_t mib = argc > 2 ? std::atoll(argv[2]) : 1024;
    g_streams = argc > 3 ? std::atoi(argv[3]) : 1;
    CK(hipStreamCreateWithFlags(&g_st[0], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&g_st[1], hipStreamNonBlocking));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const uint64_t bytes = mib << 20;
    const int rotate = (int)std::max<uint64_t>(2, 2048 / mib);
    uint8_t *d;
    uint32_t *out;
    uint64_t *clk;
    CK(hipMalloc(&d, bytes * rotate));
    CK(hipMalloc(&out, (size_t)cus * 1024 * 4 * 2));
    CK(hipMalloc(&clk, (size_t)cus * 16 * 16));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)d, bytes * rotate / 4, pattern);
    CK(hipDeviceSynchronize());
    std::printf("data pattern %d, %llu MiB per launch, rotate %d, %d stream(s)\n", pattern, (unsigned long long)mib, rotate, g_streams);
    for (int round = 0; round < 1; ++round) {
        std::printf("-- round %d\n", round);
        run<0>("C compute only", d, bytes, rotate, out, clk, cus);
        run<1>("M memory only", d, bytes, rotate, out, clk, cus);
        run<2>("S split waves (half M, half C)", d, bytes, rotate, out, clk, cus);
        run<3>("D decoupled (M and C per wave)", d, bytes, rotate, out, clk, cus);
        run<4>("R real (CRC of loaded data)", d, bytes, rotate, out, clk, cus);
        run<5>("R3 real, merged xor3", d, bytes, rotate, out, clk, cus);
        run<1, 256>("M seg256 (product layout)", d, bytes, rotate, out, clk, cus);
        run<4, 256>("R seg256 (product layout)", d, bytes, rotate, out, clk, cus);
        run<1, 1024>("M seg1024", d, bytes, rotate, out, clk, cus);
        run<4, 1024>("R seg1024", d, bytes, rotate, out, clk, cus);
        run<1, 0>("M coalesced 1 KiB rows", d, bytes, rotate, out, clk, cus);
        run<4, 0>("R coalesced (braid timing)", d, bytes, rotate, out, clk, cus);
        run<1, -1>("M dword braid rows", d, bytes, rotate, out, clk, cus);
        run<4, -1>("R dword braid rows", d, bytes, rotate, out, clk, cus);
        run<6, -1>("R dword braid, burst issue", d, bytes, rotate, out, clk, cus);
    }
    return 0;
}
