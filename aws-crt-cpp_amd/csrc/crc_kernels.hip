// Batched CRC32 / CRC32C / CRC64NVME scan for gfx950 (MI355X, CDNA4).
//
// Replaces the CPU loop behind aws_checksums_crc32_ex / crc32c_ex / crc64nvme_ex
// (reference call sites source/checksum/CRC.cpp:17,22,27) for batches of device-resident
// buffers.  Design notes: DESIGN.md "Kernels".  In short:
//
//  * One persistent workgroup of 1024 threads per CU.  The slice tables are built in LDS at
//    launch and replicated 32x so that lane (l mod 32) always reads bank (l mod 32): a
//    ds_read_b32 wave instruction is conflict-free whatever bytes it indexes.
//      W=32: slice-by-4, 4 tables x 256 entries x 32 copies x 4 B = 128 KiB
//      W=64: slice-by-2, 2 tables x 256 entries x 32 copies x 8 B = 128 KiB
//    LDS byte address = table-pair<<16 | entry<<8 | table-in-pair<<7 | copy<<2 (W=32), which one
//    v_perm_b32 builds from the state register (entry byte) and a per-lane constant (copy,
//    pair): one VALU op per table lookup.
//  * A wavefront owns a tile = 64 lanes x seg bytes of one buffer; lane l scans its contiguous
//    seg bytes with 16-byte loads (8 in flight per prefetch group, one group ahead).
//  * Lane partials are moved to the tile end with a per-lane GF(2) matrix (x^(8*seg*(63-l)),
//    32 columns in LDS, W=32) or bit-serial multiply (W=64), XOR-reduced across the wave, then
//    moved to the buffer end with x^(8*TILE*(T-1-k)) (column table in HBM, one column per lane)
//    and XOR-combined per buffer with device-scope atomics; the last tile to arrive finalises.
//  * No MFMA: this is a byte scan, bounded by HBM read bandwidth.
#include <hip/hip_runtime.h>

#include "engine.h"
#include "gf2.h"

using namespace amdcrc;

namespace {

constexpr uint32_t kTabBytes = 131072;
constexpr uint32_t kKmatBytes = 8192;  // W=32 only: 64 lanes x 32 columns x 4 B
constexpr uint32_t kLdsBytes = kTabBytes + kKmatBytes;

// Global-address-space loads (global_load_*, not flat_*: flat loads also count on lgkmcnt and
// would serialise against the LDS table lookups).
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;
typedef __attribute__((address_space(1))) const uint8_t gu8;
__device__ __forceinline__ uint4 gload16(uint64_t a) {
    const u32x4 v = *(gu32x4 *)a;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t gbyte(uint64_t a) { return *(gu8 *)a; }

__device__ __forceinline__ uint32_t lds32(const char *L, uint32_t a) { return *(const uint32_t *)(L + a); }
__device__ __forceinline__ uint64_t lds64(const char *L, uint32_t a) { return *(const uint64_t *)(L + a); }

__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v ^= __shfl_xor(v, off);
    return v;
}
__device__ __forceinline__ uint64_t wave_xor(uint64_t v) {
    uint32_t lo = wave_xor((uint32_t)v), hi = wave_xor((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// ------------------------------------------------------------------------------------------
// W = 32: slice-by-4
template <uint32_t POLY>
struct Eng32 {
    using T = uint32_t;
    static constexpr int W = 32;
    const char *L;
    uint32_t srcA, srcB;  // per-lane perm constants: copy<<2 (| 1<<16 for tables 2,3)

    __device__ void init(const char *lds, int lane) {
        L = lds;
        srcA = (uint32_t)(lane & 31) << 2;
        srcB = srcA | 0x10000u;
    }

    static __device__ void build(char *L, const ScanParams &p) {
        for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) {
            const int k = (int)(i >> 8);
            const uint32_t e = i & 255u;
            const uint32_t v = (uint32_t)gf2_table_entry(e, k, POLY);
            const uint32_t base = ((uint32_t)(k >> 1) << 16) | (e << 8) | ((uint32_t)(k & 1) << 7);
            const uint4 vv = make_uint4(v, v, v, v);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t m = (j + i) & 7u;  // rotate so a wave's 16-B stores spread over banks
                *(uint4 *)(L + base + m * 16) = vv;
            }
        }
        if (threadIdx.x < 64) {
            const uint32_t l = threadIdx.x;
            uint32_t col = (uint32_t)p.d_kvals[l];
            uint32_t *km = (uint32_t *)(L + kTabBytes);
            for (int j = 0; j < 32; ++j) {
                km[((j >> 2) * 64 + l) * 4 + (j & 3)] = col;
                col = (uint32_t)gf2_mulx(col, POLY);
            }
        }
    }

    // s <- (s ^ w) * x^32 mod P : four conflict-free lookups
    __device__ __forceinline__ uint32_t word(uint32_t s, uint32_t w) const {
        s ^= w;
        const uint32_t a3 = __builtin_amdgcn_perm(srcB, s, 0x0c060004u);  // byte0 -> T3
        const uint32_t a2 = __builtin_amdgcn_perm(srcB, s, 0x0c060104u);  // byte1 -> T2
        const uint32_t a1 = __builtin_amdgcn_perm(srcA, s, 0x0c060204u);  // byte2 -> T1
        const uint32_t a0 = __builtin_amdgcn_perm(srcA, s, 0x0c060304u);  // byte3 -> T0
        return lds32(L, a3 + 128) ^ lds32(L, a2) ^ lds32(L, a1 + 128) ^ lds32(L, a0);
    }
    __device__ __forceinline__ uint32_t byte(uint32_t s, uint32_t b) const {
        const uint32_t e = (s ^ b) & 0xffu;
        return (s >> 8) ^ lds32(L, (e << 8) | srcA);
    }
    // r * x^(8*seg*(63-lane)) : 32 LDS matrix columns
    __device__ __forceinline__ uint32_t mulK(uint32_t r, int lane, const ScanParams &) const {
        uint32_t acc = 0;
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            const uint4 c = *(const uint4 *)(L + kTabBytes + (g * 64 + lane) * 16);
            acc ^= c.x & (uint32_t)((int32_t)(r << (4 * g + 0)) >> 31);
            acc ^= c.y & (uint32_t)((int32_t)(r << (4 * g + 1)) >> 31);
            acc ^= c.z & (uint32_t)((int32_t)(r << (4 * g + 2)) >> 31);
            acc ^= c.w & (uint32_t)((int32_t)(r << (4 * g + 3)) >> 31);
        }
        return acc;
    }
};

// ------------------------------------------------------------------------------------------
// W = 64: slice-by-2 (two 64 KiB tables)
template <uint64_t POLY>
struct Eng64 {
    using T = uint64_t;
    static constexpr int W = 64;
    const char *L;
    uint32_t src0, src1;  // copy<<3 | table<<16

    __device__ void init(const char *lds, int lane) {
        L = lds;
        src0 = (uint32_t)(lane & 31) << 3;
        src1 = src0 | 0x10000u;
    }

    static __device__ void build(char *L, const ScanParams &) {
        for (uint32_t i = threadIdx.x; i < 512; i += blockDim.x) {
            const int k = (int)(i >> 8);
            const uint32_t e = i & 255u;
            const uint64_t v = gf2_table_entry(e, k, POLY);
            const uint32_t base = ((uint32_t)k << 16) | (e << 8);
            const uint4 vv = make_uint4((uint32_t)v, (uint32_t)(v >> 32), (uint32_t)v, (uint32_t)(v >> 32));
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t m = (j + i) & 15u;
                *(uint4 *)(L + base + m * 16) = vv;
            }
        }
    }

    __device__ __forceinline__ uint64_t half(uint64_t s, uint32_t h) const {
        s ^= h;
        const uint32_t lo = (uint32_t)s;
        const uint32_t a1 = __builtin_amdgcn_perm(src1, lo, 0x0c060004u);  // byte0 -> T1
        const uint32_t a0 = __builtin_amdgcn_perm(src0, lo, 0x0c060104u);  // byte1 -> T0
        return (s >> 16) ^ lds64(L, a1) ^ lds64(L, a0);
    }
    __device__ __forceinline__ uint64_t word(uint64_t s, uint32_t w) const {
        s = half(s, w & 0xffffu);
        return half(s, w >> 16);
    }
    __device__ __forceinline__ uint64_t byte(uint64_t s, uint32_t b) const {
        const uint32_t e = ((uint32_t)s ^ b) & 0xffu;
        return (s >> 8) ^ lds64(L, (e << 8) | src0);
    }
    __device__ __forceinline__ uint64_t mulK(uint64_t r, int lane, const ScanParams &p) const {
        uint64_t b = p.d_kvals[lane], acc = 0;
#pragma unroll 8
        for (int j = 0; j < 64; ++j) {
            acc ^= b & (uint64_t)((int64_t)(r << j) >> 63);
            b = gf2_mulx(b, POLY);
        }
        return acc;
    }
};

template <int ALG>
struct EngFor;
template <>
struct EngFor<ALG_CRC32> {
    using E = Eng32<kPoly32>;
};
template <>
struct EngFor<ALG_CRC32C> {
    using E = Eng32<kPoly32C>;
};
template <>
struct EngFor<ALG_CRC64NVME> {
    using E = Eng64<kPoly64Nvme>;
};

// ------------------------------------------------------------------------------------------
struct Tile {
    uint64_t b, k, T;
    uint64_t vbase;  // device address of this tile's virtual offset 0
    uint64_t H;      // first byte of the 16-aligned main region
    uint64_t tail;   // first tail byte
    uint64_t s_h;    // head state (tile 0 only): ~seed advanced over the head bytes
    uint32_t pad;    // virtual zero bytes in front of main (k == 0 only)
    uint32_t ngroups;
    uint32_t tail_len;
};

__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t rfl32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Tile fields are wave-uniform: keep them in SGPRs.
__device__ __forceinline__ Tile uniform(Tile d) {
    d.b = rfl64(d.b);
    d.k = rfl64(d.k);
    d.T = rfl64(d.T);
    d.vbase = rfl64(d.vbase);
    d.H = rfl64(d.H);
    d.tail = rfl64(d.tail);
    d.s_h = rfl64(d.s_h);
    d.pad = rfl32(d.pad);
    d.ngroups = rfl32(d.ngroups);
    d.tail_len = rfl32(d.tail_len);
    return d;
}

struct Walker {  // list mode: running position in the tile prefix
    uint64_t b, lo, hi;
};

template <class E>
__device__ Tile make_tile(const ScanParams &p, uint64_t t, Walker &wk, const E &eng) {
    using T = typename E::T;
    Tile d;
    uint64_t ptr, n;
    if (p.base) {
        d.T = p.tiles_per_buf;
        d.b = t / d.T;
        d.k = t - d.b * d.T;
        ptr = p.base + d.b * p.stride;
        n = p.len;
    } else {
        while (t >= wk.hi) {
            ++wk.b;
            wk.lo = wk.hi;
            wk.hi = p.d_tile_prefix[wk.b + 1];
        }
        d.b = wk.b;
        d.k = t - wk.lo;
        d.T = wk.hi - wk.lo;
        ptr = p.d_ptrs[d.b];
        n = p.d_lens[d.b];
    }
    const uint64_t end = ptr + n;
    const uint64_t H = (ptr + 15) & ~15ull;
    const uint64_t Ea = end & ~15ull;
    const uint64_t tile_bytes = (uint64_t)p.seg * kWave;
    uint64_t mainlen, headend;
    if (Ea > H) {
        mainlen = Ea - H;
        headend = H;
        d.tail = Ea;
        d.tail_len = (uint32_t)(end - Ea);
    } else {
        mainlen = 0;
        headend = end;
        d.tail = end;
        d.tail_len = 0;
    }
    const uint64_t pad = d.T * tile_bytes - mainlen;
    d.pad = d.k == 0 ? (uint32_t)pad : 0u;
    d.H = H;
    d.vbase = H - pad + d.k * tile_bytes;
    d.ngroups = mainlen ? p.seg / kGroupBytes : 0u;
    d.s_h = 0;
    if (d.k == 0) {
        uint64_t seed = p.seed_all;
        if (p.d_seeds) seed = E::W == 32 ? (uint64_t)((const uint32_t *)p.d_seeds)[d.b] : ((const uint64_t *)p.d_seeds)[d.b];
        T s = (T)~seed;
        for (uint64_t a = ptr; a < headend; ++a) s = eng.byte(s, gbyte(a));
        d.s_h = (uint64_t)s;
    }
    return d;
}

__device__ __forceinline__ void load_group(uint4 (&v)[8], const Tile &d, uint32_t g, uint32_t seg, int lane, bool masked) {
    const uint32_t vo0 = (uint32_t)lane * seg + g * kGroupBytes;
    if (!masked) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = gload16(d.vbase + vo0 + 16u * i);
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t vo = vo0 + 16u * i;
            const bool ok = vo >= d.pad;
            const uint4 x = gload16(ok ? d.vbase + vo : d.H);
            v[i] = ok ? x : make_uint4(0, 0, 0, 0);
        }
    }
}

template <class E>
__device__ __forceinline__ typename E::T proc_group(typename E::T s, const uint4 (&v)[8], const E &eng, const Tile &d,
                                                   uint32_t g, uint32_t seg, int lane, bool masked) {
    using T = typename E::T;
    if (!masked) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            s = eng.word(s, v[i].x);
            s = eng.word(s, v[i].y);
            s = eng.word(s, v[i].z);
            s = eng.word(s, v[i].w);
        }
    } else {
        const uint32_t vo0 = (uint32_t)lane * seg + g * kGroupBytes;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (vo0 + 16u * i == d.pad) s ^= (T)d.s_h;  // lane state is 0 here: inject the head state
            s = eng.word(s, v[i].x);
            s = eng.word(s, v[i].y);
            s = eng.word(s, v[i].z);
            s = eng.word(s, v[i].w);
        }
    }
    return s;
}

template <class E>
__device__ void finish_tile(const ScanParams &p, const Tile &d, typename E::T s, const E &eng, int lane) {
    using T = typename E::T;
    constexpr int W = E::W;
    T r = 0;
    if (d.ngroups) r = wave_xor(eng.mulK(s, lane, p));
    bool last;
    T fin;
    if (d.T == 1) {
        last = true;
        fin = d.ngroups ? r : (T)d.s_h;
    } else {
        const uint64_t kk = d.T - 1 - d.k;
        T v = 0;
        if (lane < W) {
            const T col = (T)p.d_pcols[kk * W + lane];
            v = ((r >> (W - 1 - lane)) & 1) ? col : (T)0;
        }
        v = wave_xor(v);
        last = false;
        fin = 0;
        if (lane == 0) {
            if (W == 32 && d.T <= 32) {
                const unsigned long long bit = 1ull << (32 + d.k);
                const unsigned long long val = (unsigned long long)(uint32_t)v | bit;
                const unsigned long long old =
                    __hip_atomic_fetch_xor(&p.d_acc[d.b], val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long now = old ^ val;
                const unsigned long long full = d.T == 32 ? 0xFFFFFFFF00000000ull : (((1ull << d.T) - 1) << 32);
                if ((now & 0xFFFFFFFF00000000ull) == full) {
                    last = true;
                    fin = (T)(uint32_t)now;
                    __hip_atomic_exchange(&p.d_acc[d.b], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            } else {
                const unsigned long long old =
                    __hip_atomic_fetch_xor(&p.d_acc[d.b], (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::"v"(old) : "memory");  // XOR performed before we count
                const unsigned int c = __hip_atomic_fetch_add(&p.d_cnt[d.b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (c == d.T - 1) {
                    last = true;
                    fin = (T)__hip_atomic_exchange(&p.d_acc[d.b], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&p.d_cnt[d.b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
    }
    if (lane == 0 && last) {
        for (uint32_t i = 0; i < d.tail_len; ++i) fin = eng.byte(fin, gbyte(d.tail + i));
        fin = ~fin;
        if (W == 32)
            ((uint32_t *)p.d_out)[d.b] = (uint32_t)fin;
        else
            ((uint64_t *)p.d_out)[d.b] = (uint64_t)fin;
    }
}

template <int ALG>
__global__ __launch_bounds__(kBlock, 1) void crc_scan_kernel(const ScanParams p) {
    using E = typename EngFor<ALG>::E;
    using T = typename E::T;
    __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
    E::build(lds, p);
    __syncthreads();

    const int lane = threadIdx.x & 63;
    E eng;
    eng.init(lds, lane);
    const uint64_t nw = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint64_t gw = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    const uint64_t t0 = gw * p.ntiles / nw, t1 = (gw + 1) * p.ntiles / nw;
    if (t0 >= t1) return;

    Walker wk{0, 0, 0};
    if (!p.base) {
        wk.b = p.d_wave_buf[gw];
        wk.lo = p.d_tile_prefix[wk.b];
        wk.hi = p.d_tile_prefix[wk.b + 1];
    }
    const uint32_t seg = p.seg;
    for (uint64_t t = t0; t < t1; ++t) {
        const Tile d = uniform(make_tile(p, t, wk, eng));
        const uint32_t ng = d.ngroups;
        T s;
        if (d.pad == 0) {
            // fast path: every vector is real; one prefetch group in flight while the other is scanned
            s = (d.k == 0 && lane == 0) ? (T)d.s_h : (T)0;
            uint4 A[8], B[8];
            if (ng) load_group(A, d, 0, seg, lane, false);
            for (uint32_t g = 0; g < ng; g += 2) {
                if (g + 1 < ng) load_group(B, d, g + 1, seg, lane, false);
                s = proc_group(s, A, eng, d, g, seg, lane, false);
                if (g + 1 >= ng) break;
                if (g + 2 < ng) load_group(A, d, g + 2, seg, lane, false);
                s = proc_group(s, B, eng, d, g + 1, seg, lane, false);
            }
        } else {
            // first tile of a buffer whose main region is not a multiple of TILE: the leading
            // `pad` virtual bytes are zeros and the head state is injected at offset `pad`
            s = 0;
            for (uint32_t g = 0; g < ng; ++g) {
                uint4 A[8];
                load_group(A, d, g, seg, lane, true);
                s = proc_group(s, A, eng, d, g, seg, lane, true);
            }
        }
        finish_tile(p, d, s, eng, lane);
    }
}

// ------------------------------------------------------------------------------------------
// xxHash64 (aws_xxhash64_compute, XXHash.cpp:17): one lane per buffer; the published
// algorithm is a serial chain per buffer, so parallelism comes only from the batch.
constexpr uint64_t XP1 = 0x9E3779B185EBCA87ull, XP2 = 0xC2B2AE3D27D4EB4Full, XP3 = 0x165667B19E3779F9ull,
                   XP4 = 0x85EBCA77C2B2AE63ull, XP5 = 0x27D4EB2F165667C5ull;
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t xround(uint64_t acc, uint64_t in) { return rotl64(acc + in * XP2, 31) * XP1; }
__device__ __forceinline__ uint64_t xmerge(uint64_t acc, uint64_t v) { return (acc ^ xround(0, v)) * XP1 + XP4; }
__device__ __forceinline__ uint64_t ld64u(const uint8_t *p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}

__global__ __launch_bounds__(256) void xxh64_kernel(const XxhParams p) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.nbuf) return;
    const uint8_t *ptr = (const uint8_t *)(p.d_ptrs ? p.d_ptrs[i] : p.base + i * p.stride);
    const uint64_t n = p.d_ptrs ? p.d_lens[i] : p.len;
    const uint64_t seed = p.d_seeds ? p.d_seeds[i] : p.seed_all;
    const uint8_t *end = ptr + n;
    uint64_t h;
    if (n >= 32) {
        uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
        if (((uintptr_t)ptr & 15) == 0) {
            while (ptr + 32 <= end) {
                const ulonglong2 a = *(const ulonglong2 *)ptr, b = *(const ulonglong2 *)(ptr + 16);
                v1 = xround(v1, a.x);
                v2 = xround(v2, a.y);
                v3 = xround(v3, b.x);
                v4 = xround(v4, b.y);
                ptr += 32;
            }
        } else {
            while (ptr + 32 <= end) {
                v1 = xround(v1, ld64u(ptr));
                v2 = xround(v2, ld64u(ptr + 8));
                v3 = xround(v3, ld64u(ptr + 16));
                v4 = xround(v4, ld64u(ptr + 24));
                ptr += 32;
            }
        }
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xmerge(h, v1);
        h = xmerge(h, v2);
        h = xmerge(h, v3);
        h = xmerge(h, v4);
    } else {
        h = seed + XP5;
    }
    h += n;
    while (ptr + 8 <= end) {
        h ^= xround(0, ld64u(ptr));
        h = rotl64(h, 27) * XP1 + XP4;
        ptr += 8;
    }
    if (ptr + 4 <= end) {
        uint32_t v;
        __builtin_memcpy(&v, ptr, 4);
        h ^= (uint64_t)v * XP1;
        h = rotl64(h, 23) * XP2 + XP3;
        ptr += 4;
    }
    while (ptr < end) {
        h ^= (*ptr++) * XP5;
        h = rotl64(h, 11) * XP1;
    }
    h ^= h >> 33;
    h *= XP2;
    h ^= h >> 29;
    h *= XP3;
    h ^= h >> 32;
    p.d_out[i] = h;
}

// ------------------------------------------------------------------------------------------
// Batched Combine (CRC.cpp:30-43 semantics): out = crc1 * x^(8*len2) ^ crc2, one lane per pair.
template <typename T, uint64_t POLY>
__global__ __launch_bounds__(256) void combine_kernel(const CombineParams p) {
    constexpr int W = sizeof(T) * 8;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.n) return;
    uint64_t len = p.d_len2[i];
    uint64_t m = 1ull << (W - 1);
    for (int bit = 0; len; ++bit, len >>= 1)
        if (len & 1) m = gf2_mulmod(m, p.d_xpow2[bit], POLY, W);
    const T a = ((const T *)p.d_crc1)[i], b = ((const T *)p.d_crc2)[i];
    ((T *)p.d_out)[i] = (T)(gf2_mulmod(a, m, POLY, W) ^ b);
}

}  // namespace

extern "C" int amdcrc_launch_combine(int alg, const CombineParams *p, void *stream) {
    const unsigned blocks = (unsigned)((p->n + 255) / 256);
    hipStream_t s = (hipStream_t)stream;
    switch (alg) {
        case ALG_CRC32: hipLaunchKernelGGL((combine_kernel<uint32_t, kPoly32>), dim3(blocks), dim3(256), 0, s, *p); break;
        case ALG_CRC32C: hipLaunchKernelGGL((combine_kernel<uint32_t, kPoly32C>), dim3(blocks), dim3(256), 0, s, *p); break;
        case ALG_CRC64NVME: hipLaunchKernelGGL((combine_kernel<uint64_t, kPoly64Nvme>), dim3(blocks), dim3(256), 0, s, *p); break;
        default: return -1;
    }
    return (int)hipGetLastError();
}

extern "C" int amdcrc_launch_scan(int alg, const ScanParams *p, int nblocks, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (alg) {
        case ALG_CRC32: hipLaunchKernelGGL(crc_scan_kernel<ALG_CRC32>, dim3(nblocks), dim3(kBlock), 0, s, *p); break;
        case ALG_CRC32C: hipLaunchKernelGGL(crc_scan_kernel<ALG_CRC32C>, dim3(nblocks), dim3(kBlock), 0, s, *p); break;
        case ALG_CRC64NVME: hipLaunchKernelGGL(crc_scan_kernel<ALG_CRC64NVME>, dim3(nblocks), dim3(kBlock), 0, s, *p); break;
        default: return -1;
    }
    return (int)hipGetLastError();
}

extern "C" int amdcrc_launch_xxh64(const XxhParams *p, void *stream) {
    const int threads = 256;
    const uint64_t blocks = (p->nbuf + threads - 1) / threads;
    if (blocks == 0) return 0;
    hipLaunchKernelGGL(xxh64_kernel, dim3((unsigned)blocks), dim3(threads), 0, (hipStream_t)stream, *p);
    return (int)hipGetLastError();
}
