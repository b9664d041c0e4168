// LDS lookup-throughput microbenchmark (diagnostic).  No global memory in the timed loop: every
// variant runs ITER dependent table steps per lane from register data, 16 waves per CU.
//
//   crc4 R32     slice-by-4 step, 32x replicated tables (conflict-free ds_read_b32), ILP chains
//   crc4 R1      same step, single table copy (random bank conflicts)
//   lin  b32     4 independent ds_read_b32 per step at lane-linear addresses (pure LDS rate)
//   valu only    the step's perm/xor work with the LDS reads replaced by a VALU mix
//   crc4 b64     slice-by-4 with a 64-bit table entry (two CRCs' worth per lookup)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t err_ = (x);                                                                  \
        if (err_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(err_)); \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

constexpr int ITER = 4096;
__device__ __forceinline__ uint32_t lds32(const char *L, uint32_t a) { return *(const uint32_t *)(L + a); }
__device__ __forceinline__ uint2 lds64(const char *L, uint32_t a) { return *(const uint2 *)(L + a); }

template <int MODE, int ILP>
__global__ __launch_bounds__(1024, 4) void k(uint32_t *out, uint32_t seed) {
    __shared__ __attribute__((aligned(16))) char lds[131072];
    for (int i = threadIdx.x; i < 131072 / 4; i += 1024) ((uint32_t *)lds)[i] = i * 2654435761u;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint32_t srcA = MODE == 1 ? 0u : (uint32_t)(lane & 31) << 2, srcB = srcA | 0x10000u;
    const uint32_t srcA8 = (uint32_t)(lane & 31) << 3;
    uint32_t s[ILP];
#pragma unroll
    for (int j = 0; j < ILP; ++j) s[j] = seed * (threadIdx.x + 1) * (j + 3);
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int j = 0; j < ILP; ++j) {
            uint32_t x = s[j] ^ (uint32_t)it;
            if (MODE == 0 || MODE == 1) {
                const uint32_t a3 = __builtin_amdgcn_perm(srcB, x, 0x0c060004u);
                const uint32_t a2 = __builtin_amdgcn_perm(srcB, x, 0x0c060104u);
                const uint32_t a1 = __builtin_amdgcn_perm(srcA, x, 0x0c060204u);
                const uint32_t a0 = __builtin_amdgcn_perm(srcA, x, 0x0c060304u);
                s[j] = lds32(lds, a3 + 128) ^ lds32(lds, a2) ^ lds32(lds, a1 + 128) ^ lds32(lds, a0);
            } else if (MODE == 2) {
                const uint32_t b = ((uint32_t)lane << 2) + ((it & 127u) << 8);
                s[j] ^= lds32(lds, b) ^ lds32(lds, b + 65536) ^ lds32(lds, b + 128) ^ lds32(lds, b + 65536 + 128);
            } else if (MODE == 3) {
                const uint32_t a3 = __builtin_amdgcn_perm(srcB, x, 0x0c060004u);
                const uint32_t a2 = __builtin_amdgcn_perm(srcB, x, 0x0c060104u);
                const uint32_t a1 = __builtin_amdgcn_perm(srcA, x, 0x0c060204u);
                const uint32_t a0 = __builtin_amdgcn_perm(srcA, x, 0x0c060304u);
                s[j] = (a3 * 3u) ^ (a2 + 7u) ^ (a1 >> 3) ^ a0;
            } else {
                // 64-bit entries: 32 copies x 8 B per entry row (256 B), byte -> entry<<8 | copy<<3
                const uint32_t a1 = __builtin_amdgcn_perm(srcA8 | 0x10000u, x, 0x0c060004u);
                const uint32_t a0 = __builtin_amdgcn_perm(srcA8, x, 0x0c060104u);
                const uint2 e1 = lds64(lds, a1), e0 = lds64(lds, a0);
                s[j] = (x >> 16) ^ e1.x ^ e0.x ^ e1.y ^ e0.y;
            }
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < ILP; ++j) r ^= s[j];
    out[blockIdx.x * 1024 + threadIdx.x] = r;
}

template <int MODE, int ILP>
void run(const char *name, uint32_t *out, int cus, int lookups_per_step) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((k<MODE, ILP>), dim3(cus), dim3(1024), 0, 0, out, 1u);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k<MODE, ILP>), dim3(cus), dim3(1024), 0, 0, out, (uint32_t)r + 2);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double t = ms / reps * 1e-3;
    const double steps = (double)cus * 1024 * ITER * ILP;  // per-lane steps
    const double lookups_per_cu_per_ns = steps * lookups_per_step / cus / (t * 1e9);
    std::printf("%-28s %9.1f us   %7.2f lookups/ns/CU   (%.2f per clk @2.1GHz)   bytes-equiv %.2f TB/s\n", name,
                t * 1e6, lookups_per_cu_per_ns, lookups_per_cu_per_ns / 2.1, steps * 4 / t / 1e12);
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    uint32_t *out;
    CK(hipMalloc(&out, (size_t)prop.multiProcessorCount * 1024 * 4));
    const int cus = prop.multiProcessorCount;
    for (int round = 0; round < 2; ++round) {
        std::printf("-- round %d (%d CUs)\n", round, cus);
        run<0, 1>("crc4 R32 ILP1", out, cus, 4);
        run<0, 2>("crc4 R32 ILP2", out, cus, 4);
        run<0, 4>("crc4 R32 ILP4", out, cus, 4);
        run<1, 1>("crc4 R1 ILP1", out, cus, 4);
        run<1, 4>("crc4 R1 ILP4", out, cus, 4);
        run<2, 1>("lin b32 ILP1", out, cus, 4);
        run<2, 4>("lin b32 ILP4", out, cus, 4);
        run<3, 1>("valu only ILP1", out, cus, 4);
        run<3, 4>("valu only ILP4", out, cus, 4);
        run<4, 1>("crc2 b64 ILP1", out, cus, 2);
        run<4, 4>("crc2 b64 ILP4", out, cus, 2);
    }
    return 0;
}
