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

typedef unsigned v4u __attribute__((ext_vector_type(4)));


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

    __device__ void init(const char *lds, int lane, const ScanParams &) {
        L = lds;
        srcA = (uint32_t)(lane & 31) << 2;
        srcB = srcA | 0x10000u;
    }
    uint64_t kl;  // unused (K in LDS)

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
    }
    // the host-built K-matrix image (engine.cpp get_kvals) arrives 8 bytes per thread
    static constexpr bool kKmatInLds = true;

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
    __device__ __forceinline__ uint32_t mulK(uint32_t r, int lane) const {
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
    uint64_t kl;          // K_l = x^(8*seg*(63-lane))

    static constexpr bool kKmatInLds = false;

    __device__ void init(const char *lds, int lane, const ScanParams &) {
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
    __device__ __forceinline__ uint64_t mulK(uint64_t r, int) const {
        uint64_t b = kl, acc = 0;
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
// Tile descriptor (wave-uniform, SGPRs).  Built twice per tile: by the prefetch cursor (address
// fields only) and by the scan cursor (everything); both are pure arithmetic in strided mode.
struct Tile {
    uint64_t b, k, T;
    uint64_t vbase;  // device address of this tile's virtual offset 0
    uint64_t H;      // first byte of the 16-aligned main region
    uint64_t ptr, headend, tail;
    uint32_t pad;  // virtual zero bytes in front of main (k == 0 only)
    uint32_t ngroups;
    uint32_t tail_len;
};

__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Scalar (SMEM) loads of wave-uniform descriptor words: they retire on lgkmcnt, so waiting for them
// never drains the vector-memory queue holding the prefetched payload groups.
__device__ __forceinline__ uint64_t sload64(const void *a) {
    uint64_t v;
    asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(a) : "memory");
    return v;
}
__device__ __forceinline__ uint32_t sload32(const void *a) {
    uint32_t v;
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(a) : "memory");
    return v;
}

struct Walker {  // list mode: running position in the tile prefix
    uint64_t b, lo, hi;
};

__device__ __forceinline__ Tile make_tile(const ScanParams &p, uint64_t t, Walker &wk) {
    Tile d;
    uint64_t ptr, n;
    if (!p.list_mode) {
        d.T = p.tiles_per_buf;
        d.b = t / d.T;
        d.k = t - d.b * d.T;
        ptr = p.base + d.b * p.stride;
        n = p.len;
    } else {
        while (t >= wk.hi) {
            ++wk.b;
            wk.lo = wk.hi;
            wk.hi = sload64(p.d_tile_prefix + wk.b + 1);
        }
        d.b = wk.b;
        d.k = t - wk.lo;
        d.T = wk.hi - wk.lo;
        ptr = sload64(p.d_ptrs + d.b);
        n = sload64(p.d_lens + d.b);
    }
    const uint64_t end = ptr + n;
    const uint64_t H = (ptr + 15) & ~15ull;
    const uint64_t Ea = end & ~15ull;
    const uint64_t tile_bytes = (uint64_t)p.seg * kWave;
    uint64_t mainlen;
    if (Ea > H) {
        mainlen = Ea - H;
        d.headend = H;
        d.tail = Ea;
        d.tail_len = (uint32_t)(end - Ea);
    } else {
        mainlen = 0;
        d.headend = end;
        d.tail = end;
        d.tail_len = 0;
    }
    const uint64_t pad = d.T * tile_bytes - mainlen;
    d.ptr = ptr;
    d.pad = d.k == 0 ? (uint32_t)pad : 0u;
    d.H = H;
    d.vbase = H - pad + d.k * tile_bytes;
    d.ngroups = mainlen ? p.seg / kGroupBytes : 0u;
    return d;
}

// Payload groups are plain global loads (address space 1) into registers.  Everything else the
// loop reads -- descriptors, seeds, head/tail bytes, the P columns -- is a scalar (SMEM) load that
// retires on lgkmcnt, so the compiler's vmcnt accounting sees only the ring loads (and the combine
// atomic) and can keep two groups in flight across tile boundaries.
struct Group {
    v4u v[kVecPerGroup];
};
typedef __attribute__((address_space(1))) const v4u gv4u;

__device__ __forceinline__ void issue_group(Group &g, uint64_t a) {
#pragma unroll
    for (int i = 0; i < kVecPerGroup; ++i) g.v[i] = ((gv4u *)a)[i];
}
__device__ __forceinline__ void issue_group4(Group &g, uint64_t a0, uint64_t a1, uint64_t a2, uint64_t a3) {
    g.v[0] = *(gv4u *)a0;
    g.v[1] = *(gv4u *)a1;
    g.v[2] = *(gv4u *)a2;
    g.v[3] = *(gv4u *)a3;
}
template <int N>
__device__ __forceinline__ void wait_group(Group &) {}

__device__ __forceinline__ void load_group(Group &grp, const Tile &d, uint32_t g, uint32_t seg, int lane) {
    const uint32_t vo0 = (uint32_t)lane * seg + g * kGroupBytes;
    if (d.pad == 0) {
        issue_group(grp, d.vbase + vo0);
    } else {
        // virtual zero bytes [0, pad): read a valid address (the main start) and zero in proc_group
        uint64_t a[kVecPerGroup];
#pragma unroll
        for (int i = 0; i < kVecPerGroup; ++i) {
            const uint32_t vo = vo0 + 16u * i;
            a[i] = vo >= d.pad ? d.vbase + vo : d.H;
        }
        issue_group4(grp, a[0], a[1], a[2], a[3]);
    }
}

template <class E>
__device__ __forceinline__ typename E::T proc_group(typename E::T s, const Group &grp, const E &eng, const Tile &d,
                                                   uint32_t g, uint32_t seg, int lane, typename E::T s_h) {
    if (d.pad == 0) {
#pragma unroll
        for (int i = 0; i < kVecPerGroup; ++i) {
            s = eng.word(s, grp.v[i].x);
            s = eng.word(s, grp.v[i].y);
            s = eng.word(s, grp.v[i].z);
            s = eng.word(s, grp.v[i].w);
        }
    } else {
        const uint32_t vo0 = (uint32_t)lane * seg + g * kGroupBytes;
#pragma unroll
        for (int i = 0; i < kVecPerGroup; ++i) {
            const uint32_t vo = vo0 + 16u * i;
            const uint32_t keep = vo >= d.pad ? ~0u : 0u;
            if (vo == d.pad) s ^= s_h;  // lane state is 0 here: inject the head state
            s = eng.word(s, grp.v[i].x & keep);
            s = eng.word(s, grp.v[i].y & keep);
            s = eng.word(s, grp.v[i].z & keep);
            s = eng.word(s, grp.v[i].w & keep);
        }
    }
    return s;
}

// bytes [a, end) folded into state s (a < end, both inside 16-aligned blocks read by SMEM)
template <class E>
__device__ __forceinline__ typename E::T fold_bytes(typename E::T s, uint64_t a, uint64_t end, const E &eng) {
    for (uint64_t blk = a & ~15ull; blk < end; blk += 16) {
        v4u w;
        asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(w) : "s"(blk) : "memory");
        const uint32_t wv[4] = {w.x, w.y, w.z, w.w};
        const uint64_t lo = a > blk ? a : blk, hi = end < blk + 16 ? end : blk + 16;
        for (uint64_t x = lo; x < hi; ++x) {
            const uint32_t o = (uint32_t)(x - blk);
            const uint32_t word = o < 4 ? wv[0] : o < 8 ? wv[1] : o < 12 ? wv[2] : wv[3];
            s = eng.byte(s, (word >> (8 * (o & 3))) & 0xffu);
        }
    }
    return s;
}

// head state of a buffer: ~seed advanced over the unaligned head bytes [ptr, headend)
template <class E>
__device__ __forceinline__ typename E::T head_state(const ScanParams &p, const Tile &d, const E &eng) {
    using T = typename E::T;
    uint64_t seed = p.seed_all;
    if (p.d_seeds)
        seed = E::W == 32 ? (uint64_t)sload32((const uint32_t *)p.d_seeds + d.b) : sload64((const uint64_t *)p.d_seeds + d.b);
    T s = (T)~seed;
    if (d.headend > d.ptr) s = fold_bytes(s, d.ptr, d.headend, eng);
    return s;
}

// r * x^(8*TILE*kk) for a wave-uniform r: the 32/64 columns come in by SMEM, eight at a time
template <class T, int W>
__device__ __forceinline__ T mul_pcols(T r, const uint64_t *cols) {
    T acc = 0;
#pragma unroll
    for (int c = 0; c < W; c += 8) {
        uint64_t k0, k1, k2, k3, k4, k5, k6, k7;
        asm volatile(
            "s_load_dwordx2 %0, %8, 0x0\n\ts_load_dwordx2 %1, %8, 0x8\n\t"
            "s_load_dwordx2 %2, %8, 0x10\n\ts_load_dwordx2 %3, %8, 0x18\n\t"
            "s_load_dwordx2 %4, %8, 0x20\n\ts_load_dwordx2 %5, %8, 0x28\n\t"
            "s_load_dwordx2 %6, %8, 0x30\n\ts_load_dwordx2 %7, %8, 0x38\n\t"
            "s_waitcnt lgkmcnt(0)"
            // early-clobber: a returning load must never overwrite the shared address operand
            : "=&s"(k0), "=&s"(k1), "=&s"(k2), "=&s"(k3), "=&s"(k4), "=&s"(k5), "=&s"(k6), "=&s"(k7)
            : "s"(cols + c)
            : "memory");
        const uint64_t k[8] = {k0, k1, k2, k3, k4, k5, k6, k7};
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if ((r >> (W - 1 - (c + j))) & 1) acc ^= (T)k[j];
    }
    return acc;
}

// A tile's contribution to the per-buffer accumulator is published with one device-scope atomic;
// its returned value (who arrived last) is examined at the next tile boundary, by which time at
// least one more payload group (4 loads) has been issued behind it: vmcnt(4) then covers it.
struct Pending {
    bool valid;
    unsigned long long val, old;
    uint64_t b, T_, tail;
    uint32_t tail_len;
};

__device__ __forceinline__ unsigned long long atomic_xor_ret(unsigned long long *a, unsigned long long v) {
    return __hip_atomic_fetch_xor(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <class E>
__device__ void finalize(const ScanParams &p, uint64_t b, typename E::T fin, uint64_t tail, uint32_t tail_len, const E &eng) {
    if (tail_len) fin = fold_bytes(fin, tail, tail + tail_len, eng);
    fin = ~fin;
    if (E::W == 32)
        ((uint32_t *)p.d_out)[b] = (uint32_t)fin;
    else
        ((uint64_t *)p.d_out)[b] = (uint64_t)fin;
}

template <class E>
__device__ void resolve(const ScanParams &p, Pending &pd, const E &eng, int lane) {
    using T = typename E::T;
    if (!pd.valid) return;
    pd.valid = false;
    const unsigned long long old = rfl64(pd.old);  // lane 0 issued the atomic
    const unsigned long long now = old ^ pd.val;
    const unsigned long long full = pd.T_ == 32 ? 0xFFFFFFFF00000000ull : (((1ull << pd.T_) - 1) << 32);
    if ((now & 0xFFFFFFFF00000000ull) == full) {
        if (lane == 0) __hip_atomic_exchange(&p.d_acc[pd.b], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const T fin = (T)(uint32_t)now;
        if (lane == 0) finalize(p, pd.b, fin, pd.tail, pd.tail_len, eng);
    }
}

template <class E>
__device__ void finish_tile(const ScanParams &p, const Tile &d, typename E::T s, typename E::T s_h, const E &eng,
                            int lane, Pending &pd) {
    using T = typename E::T;
    constexpr int W = E::W;
    T r = 0;
    if (d.ngroups) r = wave_xor(eng.mulK(s, lane));
    if (d.T == 1) {
        const T fin = d.ngroups ? r : s_h;
        if (lane == 0) finalize(p, d.b, fin, d.tail, d.tail_len, eng);
        return;
    }
    // move the (wave-uniform) tile partial to the buffer end: r * x^(8*TILE*(T-1-k))
    const T v = mul_pcols<T, W>((T)rfl64((uint64_t)r), p.d_pcols + (d.T - 1 - d.k) * W);
    resolve(p, pd, eng, lane);
    if (W == 32 && d.T <= 32) {
        // one 64-bit word per buffer: {arrival bit of each tile | XOR of the tile partials}
        const unsigned long long val = (unsigned long long)(uint32_t)v | (1ull << (32 + d.k));
        unsigned long long old = 0;
        if (lane == 0) old = atomic_xor_ret(&p.d_acc[d.b], val);
        pd.valid = true;
        pd.val = val;
        pd.old = old;
        pd.b = d.b;
        pd.T_ = d.T;
        pd.tail = d.tail;
        pd.tail_len = d.tail_len;
    } else if (lane == 0) {
        // wide state or more than 32 tiles: XOR, wait for it to be performed, then count arrivals
        const unsigned long long old =
            __hip_atomic_fetch_xor(&p.d_acc[d.b], (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::"v"(old) : "memory");
        const unsigned int c = __hip_atomic_fetch_add(&p.d_cnt[d.b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (c == d.T - 1) {
            const T fin = (T)__hip_atomic_exchange(&p.d_acc[d.b], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&p.d_cnt[d.b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            finalize(p, d.b, fin, d.tail, d.tail_len, eng);
        }
    }
}

template <int ALG>
__global__ __launch_bounds__(kBlock, 1) void crc_scan_kernel(const ScanParams p) {
    using E = typename EngFor<ALG>::E;
    using T = typename E::T;
    __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];

    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint64_t gw = rfl64((uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
    const uint64_t t0 = gw * p.ntiles / nw, t1 = (gw + 1) * p.ntiles / nw;
    const uint32_t seg = p.seg;

    Walker w0{0, 0, 0};
    if (p.list_mode && t0 < t1) {
        w0.b = sload64(p.d_wave_buf + gw);
        w0.lo = sload64(p.d_tile_prefix + w0.b);
        w0.hi = sload64(p.d_tile_prefix + w0.b + 1);
    }
    // ---- prefetch cursor: the next (tile, group) to load; parks on the last group when exhausted
    Walker wf = w0;
    uint64_t tf = t0;
    uint32_t gf = 0;
    Tile df{};
    bool any = false;
    for (; tf < t1; ++tf) {
        df = make_tile(p, tf, wf);
        if (df.ngroups) {
            any = true;
            break;
        }
    }
    bool pf_done = !any;
    auto pf_advance = [&]() {
        if (gf + 1 < df.ngroups) {
            ++gf;
            return;
        }
        if (pf_done) return;
        Walker w2 = wf;
        for (uint64_t t = tf + 1; t < t1; ++t) {
            Tile d2 = make_tile(p, t, w2);
            if (d2.ngroups) {
                df = d2;
                wf = w2;
                tf = t;
                gf = 0;
                return;
            }
        }
        pf_done = true;
    };
    // K data first (W=32: 8 bytes of the LDS K-matrix image per thread; W=64: this lane's K_l),
    // then the first two payload groups, all before the LDS table build so their latency overlaps it
    const uint64_t kq = *(const __attribute__((address_space(1))) uint64_t *)(E::kKmatInLds ? p.d_kvals + threadIdx.x
                                                                                        : p.d_kvals + lane);
    Group r0, r1, r2;
    if (any) {
        load_group(r0, df, gf, seg, lane);
        pf_advance();
        load_group(r1, df, gf, seg, lane);
        pf_advance();
    }

    E::build(lds, p);
    if (E::kKmatInLds) *(uint64_t *)(lds + kTabBytes + 8 * threadIdx.x) = kq;
    // LDS-only barrier: __syncthreads()'s fence would also wait vmcnt(0) for the prefetched groups
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    E eng;
    eng.init(lds, lane, p);
    eng.kl = kq;
    if (t0 >= t1) return;

    // ---- scan cursor
    Walker wp = w0;
    uint64_t tp = t0;
    uint32_t gp = 0;
    Tile dp = make_tile(p, tp, wp);
    T s_h = dp.k == 0 ? head_state(p, dp, eng) : (T)0;
    T s = (dp.k == 0 && dp.pad == 0 && lane == 0) ? s_h : (T)0;
    Pending pd{};
    pd.valid = false;

    // finish tiles whose groups are all scanned (and empty tiles); false once the wave is done
    auto settle = [&]() -> bool {
        while (gp >= dp.ngroups) {
            finish_tile(p, dp, s, s_h, eng, lane, pd);
            if (++tp >= t1) return false;
            dp = make_tile(p, tp, wp);
            gp = 0;
            s_h = dp.k == 0 ? head_state(p, dp, eng) : (T)0;
            s = (dp.k == 0 && dp.pad == 0 && lane == 0) ? s_h : (T)0;
        }
        return true;
    };

    if (any) {
        // three-slot ring, prefetch distance two groups; each step issues 4 loads, then waits
        // for the oldest group with 8 younger loads allowed in flight
        for (;;) {
            load_group(r2, df, gf, seg, lane);
            pf_advance();
            if (!settle()) break;
            wait_group<8>(r0);
            s = proc_group(s, r0, eng, dp, gp++, seg, lane, s_h);

            load_group(r0, df, gf, seg, lane);
            pf_advance();
            if (!settle()) break;
            wait_group<8>(r1);
            s = proc_group(s, r1, eng, dp, gp++, seg, lane, s_h);

            load_group(r1, df, gf, seg, lane);
            pf_advance();
            if (!settle()) break;
            wait_group<8>(r2);
            s = proc_group(s, r2, eng, dp, gp++, seg, lane, s_h);
        }
    } else {
        settle();
    }
    resolve(p, pd, eng, lane);
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
