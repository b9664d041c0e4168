// Design-space microbenchmark #2 (diagnostic; not part of the product library).
// Variants run interleaved in one process, timed with HIP events; launches alternate over S
// streams (S=1: serialised, S=2: consecutive launches may overlap).
//
// template <BLOCK, SLICE, DEPTH, SEG, NT, CRC>
//   BLOCK  threads per workgroup (1024: one WG/CU; 512 with SLICE 2: two WGs/CU fit in LDS)
//   SLICE  4 -> 128 KiB replicated tables; 2 -> 64 KiB replicated tables
//   DEPTH  groups (64 B per lane) in flight
//   SEG    bytes per lane per tile (tile = 64*SEG); a realistic per-tile combine cost is added
//   NT     non-temporal payload loads
//   CRC    0: XOR only (read ceiling), 1: CRC32C
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

__device__ __forceinline__ uint32_t lds32(const char *L, uint32_t a) { return *(const uint32_t *)(L + a); }

template <bool NT>
__device__ __forceinline__ v4u gld(uint64_t a) {
    if (NT) return __builtin_nontemporal_load((gv4u *)a);
    return *(gv4u *)a;
}

template <int SLICE>
__device__ __forceinline__ uint32_t crcw(uint32_t s, uint32_t w, const char *L, uint32_t srcA, uint32_t srcB) {
    s ^= w;
    if (SLICE == 4) {
        const uint32_t a3 = __builtin_amdgcn_perm(srcB, s, 0x0c060004u);
        const uint32_t a2 = __builtin_amdgcn_perm(srcB, s, 0x0c060104u);
        const uint32_t a1 = __builtin_amdgcn_perm(srcA, s, 0x0c060204u);
        const uint32_t a0 = __builtin_amdgcn_perm(srcA, s, 0x0c060304u);
        return lds32(L, a3 + 128) ^ lds32(L, a2) ^ lds32(L, a1 + 128) ^ lds32(L, a0);
    } else {
        // two 2-byte steps; layout e<<8 | table<<7 | copy<<2 (64 KiB)
        uint32_t b0 = __builtin_amdgcn_perm(srcA, s, 0x0c0c0004u), b1 = __builtin_amdgcn_perm(srcA, s, 0x0c0c0104u);
        s = (s >> 16) ^ lds32(L, b0 + 128) ^ lds32(L, b1);
        b0 = __builtin_amdgcn_perm(srcA, s, 0x0c0c0004u), b1 = __builtin_amdgcn_perm(srcA, s, 0x0c0c0104u);
        return (s >> 16) ^ lds32(L, b0 + 128) ^ lds32(L, b1);
    }
}

template <int BLOCK, int SLICE, int DEPTH, int SEG, bool NT, int CRC>
__global__ __launch_bounds__(BLOCK, 4) void scan(const uint8_t *base, uint64_t ntiles, uint32_t *out) {
    constexpr int WAVES = BLOCK / 64;
    constexpr uint32_t TAB = SLICE == 4 ? 131072 : 65536;
    __shared__ __attribute__((aligned(16))) char lds[TAB + 8192];
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * WAVES;
    const uint64_t gw = (uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    const uint64_t t0 = gw * ntiles / nw, t1 = (gw + 1) * ntiles / nw;
    constexpr uint32_t NG = SEG / 64;
    constexpr uint64_t TILE = 64ull * SEG;
    const uint64_t q0 = t0 * NG, q1 = t1 * NG;
    v4u ring[DEPTH + 1][4];
    auto issue = [&](int slot, uint64_t q) {
        const uint64_t qq = q < q1 ? q : q1 - 1;
        const uint64_t t = qq / NG, g = qq - t * NG;
        const uint64_t a = (uint64_t)base + t * TILE + (uint64_t)lane * SEG + g * 64;
#pragma unroll
        for (int i = 0; i < 4; ++i) ring[slot][i] = gld<NT>(a + 16 * i);
    };
    if (q0 < q1) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) issue(d, q0 + d);
    }
    if (CRC) {
        const int nent = SLICE == 4 ? 1024 : 512;
        for (int i = threadIdx.x; i < nent; i += BLOCK) {
            const int k = i >> 8;
            const uint32_t e = i & 255u;
            uint32_t c = e;
            for (int b = 0; b < 8 * (k + 1); ++b) c = (c >> 1) ^ ((c & 1) ? POLY : 0);
            const uint32_t bse = SLICE == 4 ? (((uint32_t)(k >> 1) << 16) | (e << 8) | ((uint32_t)(k & 1) << 7))
                                            : ((e << 8) | ((uint32_t)(k == 1) << 7));
            const uint4 vv = make_uint4(c, c, c, c);
#pragma unroll
            for (int j = 0; j < 8; ++j) *(uint4 *)(lds + bse + ((j + i) & 7u) * 16) = vv;
        }
        for (int i = threadIdx.x; i < 2048; i += BLOCK) ((uint32_t *)(lds + TAB))[i] = i * 2654435761u;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    const uint32_t srcA = (uint32_t)(lane & 31) << 2, srcB = srcA | 0x10000u;
    uint32_t s = 0, acc = 0, fin = 0;
    uint64_t q = q0;
    uint32_t g_in_tile = 0;
    auto proc = [&](int slot) {
        if (CRC) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                s = crcw<SLICE>(s, ring[slot][i].x, lds, srcA, srcB);
                s = crcw<SLICE>(s, ring[slot][i].y, lds, srcA, srcB);
                s = crcw<SLICE>(s, ring[slot][i].z, lds, srcA, srcB);
                s = crcw<SLICE>(s, ring[slot][i].w, lds, srcA, srcB);
            }
            if (++g_in_tile == NG) {
                // per-tile combine cost: 32-column matrix multiply from LDS + wave XOR-reduce
                uint32_t r = 0;
#pragma unroll
                for (int gg = 0; gg < 8; ++gg) {
                    const uint4 c = *(const uint4 *)(lds + TAB + (gg * 64 + lane) * 16 % 8192);
                    r ^= c.x & (uint32_t)((int32_t)(s << (4 * gg + 0)) >> 31);
                    r ^= c.y & (uint32_t)((int32_t)(s << (4 * gg + 1)) >> 31);
                    r ^= c.z & (uint32_t)((int32_t)(s << (4 * gg + 2)) >> 31);
                    r ^= c.w & (uint32_t)((int32_t)(s << (4 * gg + 3)) >> 31);
                }
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) r ^= __shfl_xor(r, off);
                fin ^= r;
                s = 0;
                g_in_tile = 0;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) acc ^= ring[slot][i].x ^ ring[slot][i].y ^ ring[slot][i].z ^ ring[slot][i].w;
        }
    };
    // ring of DEPTH+1 slots, unrolled so every slot index is a compile-time constant
    while (q < q1) {
#pragma unroll
        for (int j = 0; j <= DEPTH; ++j) {
            if (q >= q1) break;
            issue((j + DEPTH) % (DEPTH + 1), q + DEPTH);
            proc(j);
            ++q;
        }
    }
    out[gw * 64 + lane] = acc ^ s ^ fin;
}

struct Variant {
    const char *name;
    void (*kern)(const uint8_t *, uint64_t, uint32_t *);
    int block, seg;
};

#define V(name, B, S, D, G, N, C) \
    Variant { name, scan<B, S, D, G, N, C>, B, G }

float run(const Variant &v, const uint8_t *d, uint64_t batch, int rotate, int iters, uint32_t *out, int cus,
          hipStream_t *st, int nst) {
    const uint64_t ntiles = batch / (64ull * v.seg);
    const int per_cu = v.block == 512 ? 2 : 1;
    const int waves = v.block / 64;
    const int blocks = (int)std::min<uint64_t>((ntiles + waves - 1) / waves, (uint64_t)cus * per_cu);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 4; ++i)
        hipLaunchKernelGGL(v.kern, dim3(blocks), dim3(v.block), 0, st[i % nst], d + (i % rotate) * batch, ntiles, out);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, st[0]));
    for (int s = 1; s < nst; ++s) CK(hipStreamWaitEvent(st[s], a, 0));
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL(v.kern, dim3(blocks), dim3(v.block), 0, st[i % nst], d + (i % rotate) * batch, ntiles, out);
    for (int s = 1; s < nst; ++s) {
        hipEvent_t ev;
        CK(hipEventCreate(&ev));
        CK(hipEventRecord(ev, st[s]));
        CK(hipStreamWaitEvent(st[0], ev, 0));
    }
    CK(hipEventRecord(b, st[0]));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / iters;
}

int main(int argc, char **argv) {
    const uint64_t mib = argc > 1 ? std::atoll(argv[1]) : 64;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 200;
    const int rotate = argc > 3 ? std::atoi(argv[3]) : 8;
    const uint64_t batch = mib << 20;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    uint8_t *d;
    uint32_t *out;
    CK(hipMalloc(&d, batch * rotate));
    CK(hipMalloc(&out, 4 << 20));
    std::vector<uint8_t> h(1 << 20);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint8_t)(i * 2654435761u >> 13);
    for (uint64_t o = 0; o < batch * rotate; o += h.size()) CK(hipMemcpy(d + o, h.data(), h.size(), hipMemcpyHostToDevice));
    hipStream_t st[2];
    CK(hipStreamCreateWithFlags(&st[0], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&st[1], hipStreamNonBlocking));
    const int cus = prop.multiProcessorCount;
    std::vector<Variant> vs = {
        V("rd  B1024 D2 seg64", 1024, 4, 2, 64, false, 0),   V("rd  B1024 D4 seg64", 1024, 4, 4, 64, false, 0),
        V("rd  B1024 D2 seg64 nt", 1024, 4, 2, 64, true, 0), V("rd  B1024 D2 seg256", 1024, 4, 2, 256, false, 0),
        V("rd  B512  D2 seg64", 512, 2, 2, 64, false, 0),    V("rd  B512  D4 seg64", 512, 2, 4, 64, false, 0),
        V("crc B1024 s4 D2 seg256", 1024, 4, 2, 256, false, 1), V("crc B1024 s4 D4 seg256", 1024, 4, 4, 256, false, 1),
        V("crc B1024 s4 D2 seg64", 1024, 4, 2, 64, false, 1), V("crc B1024 s4 D2 seg1024", 1024, 4, 2, 1024, false, 1),
        V("crc B512  s2 D2 seg256", 512, 2, 2, 256, false, 1), V("crc B512  s2 D4 seg256", 512, 2, 4, 256, false, 1),
        V("crc B512  s2 D2 seg64", 512, 2, 2, 64, false, 1),   V("crc B512  s2 D3 seg128", 512, 2, 3, 128, false, 1),
    };
    for (int round = 0; round < 2; ++round)
        for (int nst = 1; nst <= 2; ++nst)
            for (auto &v : vs) {
                const float t = run(v, d, batch, rotate, iters, out, cus, st, nst);
                std::printf("round %d %4llu MiB streams %d  %-26s %8.2f us  %7.1f GB/s\n", round, (unsigned long long)mib, nst,
                            v.name, t * 1e3, batch / (t * 1e-3) / 1e9);
            }
    return 0;
}
