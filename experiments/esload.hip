// Event-stream load-pattern probe (round 6): the 65 MiB call's shape (131,072
// messages of 16..1024 B packed back to back, 64 consecutive messages per wave) read in several
// orders, with and without the slice-by-8 fold on the conflict-free 8-copy lane tables, so that
// the cost of the lane kernel's imbalance (a wave runs as long as its longest message) can be told
// apart from the cost of its per-lane scattered loads.
//
//   lane      one lane per message, aligned 16-byte loads, 64 bytes per block, one block ahead
//             (the product eventstream_kernel's pattern)
//   bal1/2    the wave's region [first message, last message end) cut into 64 equal chunks of whole
//             64-byte blocks, lane l the l-th chunk, one / two blocks ahead
//   balq      the same chunks, loaded by lane quads (four lanes read one lane's 64-byte block: 16
//             blocks per load instruction instead of 64) and handed to the owner through LDS
//   coal      the wave's region as 1 KiB rows (16 bytes per lane), four rows in flight
//   *+fold    the same loads, each 8-byte word folded into a running CRC32 register
//
//   build: make -C experiments build/esload    run: experiments/build/esload [launches]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 gvec;

__device__ __forceinline__ u32x4 ld16(uintptr_t a) { return *(gvec *)a; }

// the 8-copy table image (64 KiB): entry e's row at e << 8, table t at 32 t, copy c at 4 c
__device__ __forceinline__ void load_tables(char *lds, const uint32_t *img) {
    for (uint32_t i = threadIdx.x; i < 4096; i += blockDim.x) ((u32x4 *)lds)[i] = ((const u32x4 *)img)[i];
    __syncthreads();
}
struct Fold {
    const char *L;
    uint32_t cst8[8], sel8[8];
    __device__ void init(const char *lds, uint32_t lane) {
        L = lds;
        const uint32_t j = (lane >> 3) & 3u, c = lane & 7u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t q = (k + j) & 3u;
            cst8[k] = ((7u - q) << 5) | (c << 2);
            cst8[4 + k] = ((3u - q) << 5) | (c << 2);
            sel8[k] = sel8[4 + k] = 0x0c0c0004u | (q << 8);
        }
    }
    __device__ __forceinline__ uint32_t lds32(uint32_t a) const { return *(const uint32_t *)(L + a); }
    __device__ __forceinline__ uint32_t word(uint32_t s, uint32_t lo, uint32_t hi) const {
        lo ^= s;
        uint32_t x[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            x[k] = lds32(__builtin_amdgcn_perm(cst8[k], lo, sel8[k]));
            x[4 + k] = lds32(__builtin_amdgcn_perm(cst8[4 + k], hi, sel8[4 + k]));
        }
        return x[0] ^ x[1] ^ x[2] ^ x[3] ^ x[4] ^ x[5] ^ x[6] ^ x[7];
    }
    __device__ __forceinline__ uint32_t vec(uint32_t s, u32x4 v) const { return word(word(s, v.x, v.y), v.z, v.w); }
};

struct Args {
    const uint8_t *base;
    const uint64_t *offs;
    const uint32_t *lens;
    uint32_t n;
    uint32_t *sink;
    const uint32_t *img;
};

template <bool FOLD>
__global__ __launch_bounds__(256) void k_lane(Args a) {
    __shared__ __attribute__((aligned(16))) char lds[FOLD ? 65536 : 16];
    Fold f;
    if (FOLD) {
        load_tables(lds, a.img);
        f.init(lds, threadIdx.x & 63u);
    }
    const uint32_t m = blockIdx.x * 256 + threadIdx.x;
    if (m >= a.n) return;
    const uintptr_t s = (uintptr_t)(a.base + a.offs[m]);
    const uintptr_t a0 = s & ~(uintptr_t)15, a1 = (s + a.lens[m] - 4 + 15) & ~(uintptr_t)15;
    uint32_t k = (uint32_t)((a1 - a0) >> 4), u = 0;
    u32x4 acc = 0;
    auto use = [&](u32x4 v) {
        if (FOLD)
            u = f.vec(u, v);
        else
            acc ^= v;
    };
    uintptr_t p = a0;
    if (k >= 4) {
        u32x4 v0 = ld16(p), v1 = ld16(p + 16), v2 = ld16(p + 32), v3 = ld16(p + 48);
        p += 64;
        k -= 4;
        for (; k >= 4; k -= 4, p += 64) {
            const u32x4 n0 = ld16(p), n1 = ld16(p + 16), n2 = ld16(p + 32), n3 = ld16(p + 48);
            use(v0), use(v1), use(v2), use(v3);
            v0 = n0, v1 = n1, v2 = n2, v3 = n3;
        }
        use(v0), use(v1), use(v2), use(v3);
    }
    for (; k; --k, p += 16) use(ld16(p));
    const uint32_t r = acc.x ^ acc.y ^ acc.z ^ acc.w ^ u;
    if (r == 0x9E3779B9u) a.sink[m] = r;
}

// the wave's region and this lane's chunk: [rs + l C, rs + (l + 1) C) clipped to re, whole 64-byte blocks
struct Chunk {
    uintptr_t rs, re, c0;
    uint32_t C, nb;  // chunk bytes, blocks of the wave's longest chunk
};
__device__ __forceinline__ Chunk chunk_of(const Args &a, uint32_t m) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t off = a.offs[m];
    const uint32_t len = a.lens[m];
    const uint64_t o0 = __shfl(off, 0), o63 = __shfl(off, 63);
    const uint32_t l63 = __shfl(len, 63);
    Chunk c;
    c.rs = (uintptr_t)(a.base + o0) & ~(uintptr_t)63;
    c.re = ((uintptr_t)(a.base + o63 + l63) + 63) & ~(uintptr_t)63;
    const uint32_t units = (uint32_t)((c.re - c.rs) >> 6);
    c.nb = (units + 63) >> 6;
    c.C = c.nb << 6;
    c.c0 = c.rs + (uintptr_t)lane * c.C;
    return c;
}

template <bool FOLD, int AHEAD>
__global__ __launch_bounds__(256) void k_bal(Args a) {
    __shared__ __attribute__((aligned(16))) char lds[FOLD ? 65536 : 16];
    Fold f;
    if (FOLD) {
        load_tables(lds, a.img);
        f.init(lds, threadIdx.x & 63u);
    }
    const uint32_t m = blockIdx.x * 256 + threadIdx.x;
    const Chunk c = chunk_of(a, m);
    uint32_t u = 0;
    u32x4 acc = 0;
    auto use = [&](u32x4 v) {
        if (FOLD)
            u = f.vec(u, v);
        else
            acc ^= v;
    };
    // every lane runs nb blocks; blocks past the region end re-read its last block (ignored)
    auto addr = [&](uint32_t b) {
        uintptr_t p = c.c0 + ((uintptr_t)b << 6);
        return p < c.re ? p : c.re - 64;
    };
    u32x4 r[AHEAD + 1][4];
#pragma unroll
    for (int j = 0; j < AHEAD; ++j)
        if ((uint32_t)j < c.nb) {
            const uintptr_t p = addr(j);
#pragma unroll
            for (int q = 0; q < 4; ++q) r[j][q] = ld16(p + 16 * q);
        }
    for (uint32_t b = 0; b < c.nb; b += AHEAD + 1) {
#pragma unroll
        for (int j = 0; j <= AHEAD; ++j) {
            if (b + j >= c.nb) break;
            const int ls = (j + AHEAD) % (AHEAD + 1);
            if (b + j + AHEAD < c.nb) {
                const uintptr_t p = addr(b + j + AHEAD);
#pragma unroll
                for (int q = 0; q < 4; ++q) r[ls][q] = ld16(p + 16 * q);
            }
            const bool mine = c.c0 + ((uintptr_t)(b + j) << 6) < c.re;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (mine) use(r[j][q]);
        }
    }
    const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w ^ u;
    if (x == 0x9E3779B9u) a.sink[m] = x;
}

// lane quads: load j of a block step brings lanes 16 j .. 16 j + 15's blocks (lane i: 16 bytes at
// 16 (i & 3) of lane 16 j + (i >> 2)'s block); the owner reads its 64 bytes back from the wave's LDS
// rows (80-byte stride: a ds_read_b128 of 16 lanes meets 64 distinct banks).  TPB threads per
// workgroup (512: one workgroup of eight waves per CU beside the 64 KiB tables); AHEAD block steps
// in flight; SYN: no loads, synthetic words (the balanced fold alone)
template <bool FOLD, int TPB, int AHEAD, bool SYN = false>
__global__ __launch_bounds__(TPB) void k_balq(Args a) {
    constexpr uint32_t kRow = 80, kWave = 64 * kRow;
    __shared__ __attribute__((aligned(16))) char lds[(FOLD ? 65536 : 0) + (TPB / 64) * kWave];
    char *tr = lds + (FOLD ? 65536 : 0) + (threadIdx.x >> 6) * kWave;
    Fold f;
    if (FOLD) {
        load_tables(lds, a.img);
        f.init(lds, threadIdx.x & 63u);
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t m = blockIdx.x * TPB + threadIdx.x;
    const Chunk c = chunk_of(a, m);
    uint32_t u = 0;
    u32x4 acc = 0;
    auto use = [&](u32x4 v) {
        if (FOLD)
            u = f.vec(u, v);
        else
            acc ^= v;
    };
    const uintptr_t rsub = c.rs + (uintptr_t)(lane >> 2) * c.C + 16u * (lane & 3u);
    auto addr = [&](uint32_t j, uint32_t b) {
        const uintptr_t p = rsub + (uintptr_t)(16 * j) * c.C + ((uintptr_t)b << 6);
        return p < c.re ? p : c.re - 64 + 16u * (lane & 3u);
    };
    u32x4 v[AHEAD + 1][4];
    auto issue = [&](u32x4 *d, uint32_t b) {
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = SYN ? u32x4{(uint32_t)addr(j, b), b, lane, 7u} : ld16(addr(j, b));
    };
#pragma unroll
    for (int j = 0; j < AHEAD; ++j)
        if ((uint32_t)j < c.nb) issue(v[j], j);
    const bool mine_any = c.c0 < c.re;
    for (uint32_t b0 = 0; b0 < c.nb; b0 += AHEAD + 1) {
#pragma unroll
        for (int s = 0; s <= AHEAD; ++s) {
            const uint32_t b = b0 + s;
            if (b >= c.nb) break;
            if (b + AHEAD < c.nb) issue(v[(s + AHEAD) % (AHEAD + 1)], b + AHEAD);
            if (SYN) {
#pragma unroll
                for (int q = 0; q < 4; ++q) use(v[s][q]);
                continue;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) *(u32x4 *)(tr + (16 * j + (lane >> 2)) * kRow + 16 * (lane & 3)) = v[s][j];
            u32x4 w[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) w[q] = *(const u32x4 *)(tr + lane * kRow + 16 * q);
            const bool mine = mine_any && c.c0 + ((uintptr_t)b << 6) < c.re;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (mine) use(w[q]);
        }
    }
    const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w ^ u;
    if (x == 0x9E3779B9u) a.sink[m] = x;
}

// MPW messages per wave (32: twice the waves, 16 per CU in one 1024-thread workgroup beside the
// tables), the wave's region in 64 equal chunks, quad loads through LDS rows, the fold
template <int TPB, int MPW>
__global__ __launch_bounds__(TPB) void k_balq_mpw(Args a) {
    constexpr uint32_t kRow = 80, kWave = 64 * kRow;
    __shared__ __attribute__((aligned(16))) char lds[65536 + (TPB / 64) * kWave];
    char *tr = lds + 65536 + (threadIdx.x >> 6) * kWave;
    Fold f;
    load_tables(lds, a.img);
    const uint32_t lane = threadIdx.x & 63u;
    f.init(lds, lane);
    const uint32_t wave = blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
    const uint32_t m = wave * MPW + (lane < MPW ? lane : MPW - 1);
    const uint64_t off = a.offs[m];
    const uint32_t len = a.lens[m];
    const uint64_t o0 = __shfl(off, 0), ol = __shfl(off, MPW - 1);
    const uint32_t ll = __shfl(len, MPW - 1);
    const uintptr_t rs = (uintptr_t)(a.base + o0) & ~(uintptr_t)63;
    const uintptr_t re = ((uintptr_t)(a.base + ol + ll) + 63) & ~(uintptr_t)63;
    const uint32_t units = (uint32_t)((re - rs) >> 6), nb = (units + 63) >> 6, C = nb << 6;
    const uintptr_t rsub = rs + (uintptr_t)(lane >> 2) * C + 16u * (lane & 3u);
    auto addr = [&](uint32_t j, uint32_t b) {
        const uintptr_t p = rsub + (uintptr_t)(16 * j) * C + ((uintptr_t)b << 6);
        return p < re ? p : re - 64 + 16u * (lane & 3u);
    };
    u32x4 v[4], nv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = ld16(addr(j, 0));
    uint32_t u = 0;
    for (uint32_t b = 0; b < nb; ++b) {
#pragma unroll
        for (int j = 0; j < 4; ++j) nv[j] = ld16(addr(j, b + 1));
#pragma unroll
        for (int j = 0; j < 4; ++j) *(u32x4 *)(tr + (16 * j + (lane >> 2)) * kRow + 16 * (lane & 3)) = v[j];
        u32x4 w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) w[q] = *(const u32x4 *)(tr + lane * kRow + 16 * q);
#pragma unroll
        for (int q = 0; q < 4; ++q) u = f.vec(u, w[q]);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = nv[j];
    }
    if (u == 0x9E3779B9u) a.sink[m] = u;
}

// two chunks per lane (128 chunks per wave: lane l folds chunks l and l + 64 as two independent
// chains, interleaved): the same quad loads, eight per block step, through 128 LDS rows
template <int TPB>
__global__ __launch_bounds__(TPB) void k_bal2c(Args a) {
    constexpr uint32_t kRow = 80, kWave = 128 * kRow;
    __shared__ __attribute__((aligned(16))) char lds[65536 + (TPB / 64) * kWave];
    char *tr = lds + 65536 + (threadIdx.x >> 6) * kWave;
    Fold f;
    load_tables(lds, a.img);
    const uint32_t lane = threadIdx.x & 63u;
    f.init(lds, lane);
    const uint32_t m = blockIdx.x * TPB + threadIdx.x;
    const uint64_t off = a.offs[m];
    const uint32_t len = a.lens[m];
    const uint64_t o0 = __shfl(off, 0), o63 = __shfl(off, 63);
    const uint32_t l63 = __shfl(len, 63);
    const uintptr_t rs = (uintptr_t)(a.base + o0) & ~(uintptr_t)63;
    const uintptr_t re = ((uintptr_t)(a.base + o63 + l63) + 63) & ~(uintptr_t)63;
    const uint32_t units = (uint32_t)((re - rs) >> 6), nb = (units + 127) >> 7, C = nb << 6;
    const uintptr_t rsub = rs + (uintptr_t)(lane >> 2) * C + 16u * (lane & 3u);
    auto addr = [&](uint32_t j, uint32_t b) {
        const uintptr_t p = rsub + (uintptr_t)(16 * j) * C + ((uintptr_t)b << 6);
        return p < re ? p : re - 64 + 16u * (lane & 3u);
    };
    u32x4 v[8], nv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ld16(addr(j, 0));
    uint32_t ua = 0, ub = 0;
    for (uint32_t b = 0; b < nb; ++b) {
#pragma unroll
        for (int j = 0; j < 8; ++j) nv[j] = ld16(addr(j, b + 1));
#pragma unroll
        for (int j = 0; j < 8; ++j) *(u32x4 *)(tr + (16 * j + (lane >> 2)) * kRow + 16 * (lane & 3)) = v[j];
        u32x4 wa[4], wb[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            wa[q] = *(const u32x4 *)(tr + lane * kRow + 16 * q);
            wb[q] = *(const u32x4 *)(tr + (lane + 64) * kRow + 16 * q);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            ua = f.word(ua, wa[q].x, wa[q].y);
            ub = f.word(ub, wb[q].x, wb[q].y);
            ua = f.word(ua, wa[q].z, wa[q].w);
            ub = f.word(ub, wb[q].z, wb[q].w);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = nv[j];
    }
    const uint32_t x = ua ^ ub;
    if (x == 0x9E3779B9u) a.sink[m] = x;
}

// the wave's region as 1 KiB rows, D rows in flight
template <int D>
__global__ __launch_bounds__(256) void k_coal(Args a) {
    const uint32_t m = blockIdx.x * 256 + threadIdx.x;
    const Chunk c = chunk_of(a, m);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t rows = (uint32_t)((c.re - c.rs + 1023) >> 10);
    u32x4 acc = 0, r[D];
    auto addr = [&](uint32_t i) {
        const uintptr_t p = c.rs + ((uintptr_t)i << 10) + 16u * lane;
        return p < c.re ? p : c.re - 16;
    };
#pragma unroll
    for (int j = 0; j < D; ++j)
        if ((uint32_t)j < rows) r[j] = ld16(addr(j));
    for (uint32_t i = 0; i < rows; i += D) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            if (i + j >= rows) break;
            acc ^= r[j];
            if (i + j + D < rows) r[j] = ld16(addr(i + j + D));
        }
    }
    const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x9E3779B9u) a.sink[m] = x;
}

__global__ void fill(uint8_t *p, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 31)) * 0xBF58476D1CE4E5B9ull;
        ((uint64_t *)p)[i] = z ^ (z >> 29);
    }
}

static uint32_t gf2_mulx8(uint32_t v, int bytes) {  // v * x^(8 bytes), reflected CRC32 (0xEDB88320)
    for (int i = 0; i < 8 * bytes; ++i) v = (v >> 1) ^ ((v & 1u) ? 0xEDB88320u : 0u);
    return v;
}

int main(int argc, char **argv) {
    const int iso = argc > 1 ? atoi(argv[1]) : 8;
    const uint32_t n = 131072, copies = 6;
    std::vector<uint32_t> lens(n);
    std::vector<uint64_t> offs(n);
    uint64_t pos = 0, st = 0x243F6A8885A308D3ull;
    for (uint32_t i = 0; i < n; ++i) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        lens[i] = 16 + (uint32_t)((st >> 33) % 1009);
        offs[i] = pos;
        pos += lens[i];
    }
    const uint64_t span = (pos + 4095) & ~4095ull;
    uint8_t *buf;
    uint64_t *d_offs;
    uint32_t *d_lens, *sink, *img;
    CK(hipMalloc(&buf, span * copies + 4096));
    CK(hipMalloc(&d_offs, n * 8));
    CK(hipMalloc(&d_lens, n * 4));
    CK(hipMalloc(&sink, n * 4));
    CK(hipMalloc(&img, 65536));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, buf, span * copies);
    CK(hipMemcpy(d_offs, offs.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_lens, lens.data(), n * 4, hipMemcpyHostToDevice));
    {  // T_t[e] = e * x^(8 (t + 1)) with the 8 copies
        std::vector<uint32_t> h(16384);
        for (uint32_t e = 0; e < 256; ++e)
            for (int t = 0; t < 8; ++t) {
                const uint32_t v = gf2_mulx8(e, t + 1);
                for (int c = 0; c < 8; ++c) h[(e << 6) + (t << 3) + c] = v;
            }
        CK(hipMemcpy(img, h.data(), 65536, hipMemcpyHostToDevice));
    }
    struct V {
        const char *name;
        void (*k)(Args);
        int tpb;
        int mpb = 0;  // messages per workgroup (default: one per thread)
    };
    const std::vector<V> vs = {
        {"lane", k_lane<false>, 256},    {"lane+fold", k_lane<true>, 256},  {"bal1", k_bal<false, 1>, 256},
        {"bal1+fold", k_bal<true, 1>, 256},
        {"balq", k_balq<false, 256, 1>, 256},   {"balq+fold/512", k_balq<true, 512, 1>, 512},
        {"balq2+fold/512", k_balq<true, 512, 2>, 512}, {"balq/512", k_balq<false, 512, 1>, 512},
        {"balfold-only/512", k_balq<true, 512, 1, true>, 512}, {"coal4", k_coal<4>, 256},
        {"bal2c+fold/512", k_bal2c<512>, 512},
        {"balq+fold/512 mpw64", k_balq_mpw<512, 64>, 512}, {"balq+fold/1024 mpw32", k_balq_mpw<1024, 32>, 1024, 512},
    };
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<hipEvent_t> e0(iso), e1(iso);
    for (int i = 0; i < iso; ++i) {
        CK(hipEventCreate(&e0[i]));
        CK(hipEventCreate(&e1[i]));
    }
    const uint64_t crc_bytes = pos - 4ull * n;
    std::printf("{\"messages\": %u, \"region_bytes\": %llu, \"launches\": %d, \"variants\": {", n, (unsigned long long)pos, iso);
    for (int rep = 0; rep < 2; ++rep)
        for (size_t vi = 0; vi < vs.size(); ++vi) {
            const V &v = vs[vi];
            for (int i = 0; i < 4; ++i)
                hipLaunchKernelGGL(v.k, dim3(n / (v.mpb ? v.mpb : v.tpb)), dim3(v.tpb), 0, s, Args{buf + (i % copies) * span, d_offs, d_lens, n, sink, img});
            CK(hipStreamSynchronize(s));
            for (int i = 0; i < iso; ++i)
                hipExtLaunchKernelGGL(v.k, dim3(n / (v.mpb ? v.mpb : v.tpb)), dim3(v.tpb), 0, s, e0[i], e1[i], 0,
                                      Args{buf + (i % copies) * span, d_offs, d_lens, n, sink, img});
            CK(hipStreamSynchronize(s));
            double sum = 0, mn = 1e9;
            for (int i = 0; i < iso; ++i) {
                float ms;
                CK(hipEventElapsedTime(&ms, e0[i], e1[i]));
                sum += ms;
                mn = ms < mn ? ms : mn;
            }
            const double us = 1e3 * sum / iso;
            std::printf("%s\"%s r%d\": {\"us\": %.2f, \"min_us\": %.2f, \"frac\": %.3f}", (rep || vi) ? ", " : "", v.name, rep, us,
                        1e3 * mn, crc_bytes / (us * 1e-6) / 8e12);
            std::fflush(stdout);
        }
    std::printf("}}\n");
    return 0;
}
