// Dependent-chain cost of the XXH64 round's instructions on one gfx950 wave (diagnostic, not part
// of the product library; DESIGN.md §3.4 "XXH64 dependency floor").
//
// xxh64_row_kernel's round (crc_kernels.hip xstep_y, as compiled):
//     v_alignbit_b32 rl, ul, uh, 1        \  rotl(u, 31) of the carried 64-bit state
//     v_alignbit_b32 rh, uh, ul, 1        /
//     v_mad_u64_u32  m, rl, P1lo, y       low product plus the next stripe's y = in * P2
//     v_mul_lo_u32   a, rl, P1hi          cross products
//     v_mul_lo_u32   b, rh, P1lo
//     v_add3_u32     uh, b, a, m.hi
// plus two v_mov_b32_dpp (row_newbcast) that bring y in off the chain.  Each kernel below runs one
// wave, times a loop of 256 x 16 copies of one instruction pattern with s_memtime (shader clock
// cycles) and reports cycles per copy: a dependent chain of each instruction (its latency as the
// chain sees it), four independent chains interleaved (its issue cost), and the whole round with and
// without the DPP moves.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

constexpr int kIters = 256, kUnroll = 16;

#define REP16(x) x x x x x x x x x x x x x x x x

// One pattern per kernel, the whole timed loop in one inline-asm block on fixed registers
// (v10..v17 = a..h, v[20:21] = y, v[22:23] = m, s20 = loop counter) so the compiler can neither
// reorder the pattern nor reuse its registers.  s[24:25] hold the multiplier halves P1lo, P1hi.
#define BENCH(NAME, BODY)                                                                             \
    __global__ void NAME(unsigned long long *cyc, unsigned *sink, unsigned seed) {                   \
        unsigned a = seed + threadIdx.x, r;                                                           \
        __syncthreads();                                                                              \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                   \
        asm volatile(                                                                                 \
            "v_mov_b32 v10, %1\n\tv_xor_b32 v11, 0x9E3779B9, %1\n\tv_add_u32 v12, 3, %1\n\t"         \
            "v_add_u32 v13, 7, %1\n\tv_xor_b32 v14, 1, %1\n\tv_xor_b32 v15, 2, %1\n\t"                 \
            "v_xor_b32 v16, 5, %1\n\tv_xor_b32 v17, 9, %1\n\tv_mov_b32 v20, v12\n\tv_mov_b32 v21, v13\n\t" \
            "v_mov_b32 v22, v14\n\tv_mov_b32 v23, v15\n\t"                                             \
            "s_mov_b32 s24, 0x85EBCA87\n\ts_mov_b32 s25, 0x9E3779B1\n\ts_movk_i32 s20, 0x100\n"        \
            "1:\n\t" REP16(BODY) "s_sub_u32 s20, s20, 1\n\ts_cmp_lg_u32 s20, 0\n\ts_cbranch_scc1 1b\n\t"   \
            "v_xor_b32 %0, v10, v11\n\tv_xor_b32 %0, %0, v12\n\tv_xor_b32 %0, %0, v13\n\tv_xor_b32 %0, %0, v14\n\t" \
            "v_xor_b32 %0, %0, v15\n\tv_xor_b32 %0, %0, v16\n\tv_xor_b32 %0, %0, v17\n\tv_xor_b32 %0, %0, v20\n\t" \
            "v_xor_b32 %0, %0, v21\n\tv_xor_b32 %0, %0, v22\n\tv_xor_b32 %0, %0, v23\n\t"                   \
            "s_waitcnt lgkmcnt(0)"                                                                     \
            : "=&v"(r)                                                                                \
            : "v"(a)                                                                                  \
            : "s20", "s24", "s25", "scc", "vcc", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", \
              "v20", "v21", "v22", "v23", "memory");                                                  \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                   \
        if (threadIdx.x == 0) cyc[0] = t1 - t0;                                                       \
        sink[threadIdx.x] = r;                                                                        \
    }

BENCH(dep_add, "v_add_u32 v10, v10, v11\n\t")
BENCH(dep_alignbit, "v_alignbit_b32 v10, v10, v11, 1\n\t")
BENCH(dep_mul_lo, "v_mul_lo_u32 v10, v10, s24\n\t")
BENCH(dep_mad64, "v_mad_u64_u32 v[22:23], vcc, v22, s24, v[20:21]\n\t")
BENCH(dep_add3, "v_add3_u32 v10, v10, v11, v12\n\t")
BENCH(ind_mul_lo, "v_mul_lo_u32 v10, v10, s24\n\tv_mul_lo_u32 v11, v11, s24\n\tv_mul_lo_u32 v12, v12, s24\n\tv_mul_lo_u32 v13, v13, s24\n\t")
BENCH(ind_mad64, "v_mad_u64_u32 v[20:21], vcc, v10, s24, v[20:21]\n\tv_mad_u64_u32 v[22:23], vcc, v11, s24, v[22:23]\n\t")
BENCH(ind_add, "v_add_u32 v10, v10, v14\n\tv_add_u32 v11, v11, v15\n\tv_add_u32 v12, v12, v16\n\tv_add_u32 v13, v13, v17\n\t")
// the round: (v10, v11) = (ul, uh) carried; v[20:21] = y, the next input product
BENCH(round,
      "v_alignbit_b32 v14, v10, v11, 1\n\tv_alignbit_b32 v15, v11, v10, 1\n\t"
      "v_mad_u64_u32 v[22:23], vcc, v14, s24, v[20:21]\n\t"
      "v_mul_lo_u32 v16, v14, s25\n\tv_mul_lo_u32 v17, v15, s24\n\t"
      "v_mov_b32 v10, v22\n\tv_add3_u32 v11, v17, v16, v23\n\t")
BENCH(round_dpp,
      "v_mov_b32_dpp v20, v12 row_newbcast:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_mov_b32_dpp v21, v13 row_newbcast:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_alignbit_b32 v14, v10, v11, 1\n\tv_alignbit_b32 v15, v11, v10, 1\n\t"
      "v_mad_u64_u32 v[22:23], vcc, v14, s24, v[20:21]\n\t"
      "v_mul_lo_u32 v16, v14, s25\n\tv_mul_lo_u32 v17, v15, s24\n\t"
      "v_mov_b32 v10, v22\n\tv_add3_u32 v11, v17, v16, v23\n\t")

struct K {
    const char *name;
    void (*k)(unsigned long long *, unsigned *, unsigned);
    int per;  // pattern copies counted per REP16 element (independent variants: chains per copy)
};

int main() {
    unsigned long long *cyc;
    unsigned *sink;
    CK(hipMalloc(&cyc, 8));
    CK(hipMalloc(&sink, 4096));
    const K ks[] = {{"dep v_add_u32", dep_add, 1},          {"dep v_alignbit_b32", dep_alignbit, 1},
                    {"dep v_mul_lo_u32", dep_mul_lo, 1},    {"dep v_mad_u64_u32 (64-bit result feeds the next)", dep_mad64, 1},
                    {"dep v_add3_u32", dep_add3, 1},        {"4 indep v_mul_lo_u32", ind_mul_lo, 4},
                    {"2 indep v_mad_u64_u32", ind_mad64, 2}, {"4 indep v_add_u32", ind_add, 4},
                    {"xxh64 round (no dpp)", round, 1},      {"xxh64 round (+2 dpp)", round_dpp, 1}};
    std::printf("{\"unit\": \"shader cycles per pattern copy, one wave\", \"results\": {");
    bool first = true;
    for (const K &k : ks) {
        unsigned long long best = ~0ull;
        for (int rep = 0; rep < 5; ++rep) {
            hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, cyc, sink, 12345u + rep);
            CK(hipDeviceSynchronize());
            unsigned long long c;
            CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
            if (c < best) best = c;
        }
        const double per_copy = (double)best / (kIters * kUnroll);
        std::printf("%s\"%s\": {\"per_copy\": %.2f, \"per_instruction_chain\": %.2f}", first ? "" : ", ", k.name, per_copy,
                    per_copy / k.per);
        first = false;
    }
    std::printf("}}\n");
    return 0;
}
