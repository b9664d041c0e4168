// The CRC64NVME row step alone: crc_kernels.hip Braid64<POLY, 4>::step_x -- 8
// perms, 8 conflict-free ds_read_b64 from the 4-copy table layout, the 17-dword XOR reduction and the
// per-lane dword selects -- as a dependent chain per lane, no global memory, at the scan's occupancy
// (512-thread workgroups, two per CU: 16 waves per CU).  Reports the payload rate the chain alone
// could carry (512 bytes per wave-row step), for 1 and 2 independent chains per lane, against the
// same loop with the table reads replaced by VALU (the LDS share of the step).
//   experiments/build/crc64_rowbench [rows]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                        \
    do {                                                                                             \
        hipError_t err_ = (x);                                                                       \
        if (err_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(err_)); \
            std::exit(1);                                                                            \
        }                                                                                            \
    } while (0)

__device__ __forceinline__ uint64_t lds64(const char *L, uint32_t a) { return *(const uint64_t *)(L + a); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return a ^ b ^ c; }

// MODE 0: the row step; MODE 1: table reads replaced by a VALU mix of the addresses
template <int MODE, int ILP>
__global__ __launch_bounds__(512, 2) void rowk(uint64_t *out, uint32_t rows, uint64_t seed) {
    __shared__ __attribute__((aligned(16))) char lds[65536];
    for (uint32_t i = threadIdx.x; i < 65536 / 8; i += 512) ((uint64_t *)lds)[i] = (i + 1) * 0x9E3779B97F4A7C15ull;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t jp = (lane >> 2) & 7u, cp = lane & 3u;
    const bool lowfirst = jp < 4;
    const uint32_t lowmask = lowfirst ? ~0u : 0u;
    uint32_t cst[4], csth[4], sel[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t q = (k + jp) & 3u;
        const uint32_t t1 = lowfirst ? q : 4u + q, t2 = lowfirst ? 4u + q : q;
        cst[k] = (t1 << 5) | (cp << 3);
        csth[k] = (t2 << 5) | (cp << 3);
        sel[k] = 0x0c0c0004u | (q << 8);
    }
    uint64_t u[ILP];
#pragma unroll
    for (int c = 0; c < ILP; ++c) u[c] = seed * (threadIdx.x + 1 + 977 * c);
    for (uint32_t r = 0; r < rows; ++r) {
#pragma unroll
        for (int c = 0; c < ILP; ++c) {
            const uint64_t a = u[c] ^ ((uint64_t)r * 0x100000001b3ull);  // the row's payload word
            const uint32_t lo = (uint32_t)a, hi = (uint32_t)(a >> 32);
            const uint32_t ma = (lo & lowmask) | (hi & ~lowmask), mb = (hi & lowmask) | (lo & ~lowmask);
            uint64_t v[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t x0 = __builtin_amdgcn_perm(cst[k], ma, sel[k]), x1 = __builtin_amdgcn_perm(csth[k], mb, sel[k]);
                if (MODE == 0) {
                    v[k] = lds64(lds, x0);
                    v[4 + k] = lds64(lds, x1);
                } else {
                    v[k] = (uint64_t)x0 * 0x9E3779B1u;
                    v[4 + k] = (uint64_t)x1 * 0x85EBCA77u;
                }
            }
            uint32_t rl = xor3(xor3((uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2]), (uint32_t)v[3], (uint32_t)v[4]);
            rl = xor3(xor3(rl, (uint32_t)v[5], (uint32_t)v[6]), (uint32_t)v[7], lo);
            uint32_t rh = xor3(xor3((uint32_t)(v[0] >> 32), (uint32_t)(v[1] >> 32), (uint32_t)(v[2] >> 32)),
                               (uint32_t)(v[3] >> 32), (uint32_t)(v[4] >> 32));
            rh = xor3(xor3(rh, (uint32_t)(v[5] >> 32), (uint32_t)(v[6] >> 32)), (uint32_t)(v[7] >> 32), hi);
            u[c] = ((uint64_t)rh << 32) | rl;
        }
    }
    uint64_t acc = 0;
#pragma unroll
    for (int c = 0; c < ILP; ++c) acc ^= u[c];
    if (acc == 0x1234567) out[blockIdx.x * 512 + threadIdx.x] = acc;  // keeps the chain live
}

template <int MODE, int ILP>
void run(const char *name, int cus, uint32_t rows, uint64_t *d) {
    const int grid = 2 * cus;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((rowk<MODE, ILP>), dim3(grid), dim3(512), 0, 0, d, rows, 12345ull);  // warm
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((rowk<MODE, ILP>), dim3(grid), dim3(512), 0, 0, d, rows, 12345ull + rep);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    // payload a wave-row stands for: 64 lanes x 8 bytes, per chain
    const double wave_rows = (double)grid * 8 * rows * ILP;
    const double tbs = wave_rows * 512.0 / (best * 1e-3) / 1e12;
    std::printf("{\"variant\": \"%s\", \"ilp\": %d, \"rows\": %u, \"ms\": %.4f, \"payload_TBps\": %.2f, \"x_hbm_peak\": %.2f}\n",
                name, ILP, rows, best, tbs, tbs / 8.0);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main(int argc, char **argv) {
    const uint32_t rows = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 4096;
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    uint64_t *d;
    CK(hipMalloc(&d, (size_t)2 * p.multiProcessorCount * 512 * 8));
    std::printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", p.name, p.multiProcessorCount, p.clockRate);
    run<0, 1>("row_step", p.multiProcessorCount, rows, d);
    run<0, 2>("row_step", p.multiProcessorCount, rows, d);
    run<1, 1>("row_step_valu_only", p.multiProcessorCount, rows, d);
    run<1, 2>("row_step_valu_only", p.multiProcessorCount, rows, d);
    CK(hipFree(d));
    return 0;
}
