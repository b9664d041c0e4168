// Batched CRC32 / CRC32C / CRC64NVME scans for gfx950 (MI355X, CDNA4).
//
// Replaces the CPU loop behind aws_checksums_crc32_ex / crc32c_ex / crc64nvme_ex
// (reference call sites source/checksum/CRC.cpp:17,22,27) for batches of device-resident
// buffers.  Design notes: DESIGN.md "Kernels".  In short:
//
//  * Braided scans.  A buffer's 16-aligned main region is cut into tiles; a wavefront scans a tile
//    row by row, lane l owning the 8-byte word l of every 512-byte row (one fully coalesced
//    global_load_dwordx2 per row).  Each lane's state is one "braid" of the CRC:
//    u <- (u ^ w) * x^(8*512), one slice-by-8 step whose byte tables fold in the skip over the other
//    63 lanes' words (for W=32 the word's high half does not meet u: its lookups run a row ahead).
//    4-byte words / 256-byte rows remain as the AMDCRC_STREAM_W8=0 build.
//  * Byte tables live in LDS in several copies laid out so that every ds_read of a half-wave
//    touches distinct banks whatever bytes it indexes (W=32: 8 copies, 64 KiB + constants; W=64
//    streaming scan: 4 copies, 64 KiB + nibble tables; W=64 braided scan: 8 copies, 128 KiB).
//  * A lane's state times x^(-w*l) is its share of the tile register (K_l); the wave XOR-reduces
//    the shares, moves the tile register to its 32-tile group's end and then to the buffer end with
//    column tables, and device-scope atomics combine the tiles of a buffer; the last arrival
//    finalises (tail bytes, complement, store).
//  * No MFMA: this is a byte scan, bounded by HBM read bandwidth.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <type_traits>

#include "variant_guard.h"

#ifndef AMDCRC_R16_XCD  // compile-time only: crc64_rows16_kernel's sets in XCD-window order (1) or contiguous (0)
#define AMDCRC_R16_XCD 1
#endif
#ifndef AMDCRC_ES_FLAT  // compile-time only: event-stream frames on the balanced flat kernel (1) or one lane per message (0)
#define AMDCRC_ES_FLAT 1
#endif
#ifndef AMDCRC_STREAM_W8  // compile-time only: the W=32 streaming scan on 8-byte words (1) or 4-byte words (0)
#define AMDCRC_STREAM_W8 1
#endif

#include "engine.h"
#include "gf2.h"

using namespace amdcrc;

namespace {

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const v4u gv4u;
typedef __attribute__((address_space(1))) const uint32_t gu32;
typedef __attribute__((address_space(1))) const uint64_t gu64;

// floor(n / d) for wave-uniform n and d >= 1.  The compiler's 64-bit integer division is ~150 scalar
// instructions (issued at most one per 4 cycles per SIMD); the W=32 streaming scan's prologue had nine
// of them and took 3.2-6.5 us from entry to its first barrier (per-wave stamps, profiles/r05/stamps).
// Here: the correctly rounded double quotient, which for n < 2^52 is floor(n / d) or one more (an
// exact quotient k is representable and stays k; a larger one cannot round below its floor), and one
// correction.  About a dozen vector instructions on uniform values.
__device__ __forceinline__ uint64_t udiv_u(uint64_t n, uint64_t d) {
    if (d == 1) return n;
    if ((n | d) >> 52) {  // never on a real launch (2^52 tiles); compact shift-subtract, not 150 inlined ops
        uint64_t q = 0, r = 0;
#pragma unroll 1
        for (int i = 63; i >= 0; --i) {
            r = (r << 1) | ((n >> i) & 1u);
            if (r >= d) r -= d, q |= 1ull << i;
        }
        return q;
    }
    uint64_t q = (uint64_t)((double)n / (double)d);
    if (q * d > n) --q;
    return q;
}

__device__ __forceinline__ uint32_t lds32(const char *L, uint32_t a) { return *(const uint32_t *)(L + a); }
__device__ __forceinline__ uint64_t lds64(const char *L, uint32_t a) { return *(const uint64_t *)(L + a); }

__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Scalar (SMEM) loads of wave-uniform descriptor words: they retire on lgkmcnt, so waiting for them
// never drains the vector-memory queue holding the prefetched payload groups.
// The address is wave-uniform by construction; readfirstlane keeps it in SGPRs even where the
// compiler cannot prove uniformity (an "s" operand in a VGPR does not assemble).
__device__ __forceinline__ uint64_t sload64(const void *a) {
    uint64_t v;
    const uint64_t sa = rfl64((uint64_t)a);
    asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(sa) : "memory");
    return v;
}
__device__ __forceinline__ uint32_t sload32(const void *a) {
    uint32_t v;
    const uint64_t sa = rfl64((uint64_t)a);
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(sa) : "memory");
    return v;
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t xor_and(uint32_t acc, uint32_t c, uint32_t m) {  // acc ^ (c & m)
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x78" : "=v"(r) : "v"(acc), "v"(c), "v"(m));
    return r;
}

// XOR over the 64 lanes, returned wave-uniform: two quad_perm and two row_ror DPP steps leave each
// 16-lane row's XOR in all its lanes; four readlanes finish in scalar registers.
__device__ __forceinline__ uint32_t wave_xor_s(uint32_t v) {
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    return (uint32_t)(__builtin_amdgcn_readlane((int)v, 0) ^ __builtin_amdgcn_readlane((int)v, 16) ^
                      __builtin_amdgcn_readlane((int)v, 32) ^ __builtin_amdgcn_readlane((int)v, 48));
}
__device__ __forceinline__ uint64_t wave_xor64_s(uint64_t v) {
    const uint32_t lo = wave_xor_s((uint32_t)v), hi = wave_xor_s((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// ------------------------------------------------------------------------------------------
// Work decomposition (engine.h): buffer b = [ptr, end) is head [ptr, H) (H = ptr rounded up to 16),
// main [H, Ea) (Ea = end rounded down to 16) and tail [Ea, end).  Main is front-padded virtually
// with zeros to T tiles of TILE = 64 * seg bytes (free for a raw CRC); tile k starts at virtual
// offset k * TILE.  LIST = ragged batch (descriptors by SMEM), else uniform (pure arithmetic).
struct Tile {        // wave-uniform (SGPRs): everything the scan needs per tile
    uint64_t b, k, T;
    uint64_t tbase;  // global index of the buffer's first tile
    uint64_t vbase;  // device address of this tile's virtual offset 0; main starts at vbase + pad
    uint32_t pad;    // virtual zero bytes in front of main (k == 0 only)
    uint32_t ngroups;
};
struct Edges {       // head / tail of a buffer, recomputed where needed instead of kept in SGPRs
    uint64_t ptr, headend, tail, end;
};
struct Walker {  // list mode: running position in the tile prefix
    uint64_t b, lo, hi;
};

// strided launches: batch j and index i of buffer b (wave-uniform; the division runs on the scalar
// unit, once per buffer at its head and at its finish)
struct BatchPos {
    uint64_t j, i;
};
__device__ __forceinline__ BatchPos batch_pos(const ScanParams &p, uint64_t b) {
    if (p.nbatch <= 1) return {0, b};
    // (no power-of-two shortcut here: one more branch in this per-set helper made the compiler copy the
    // whole ScanParams to scratch in crc64_rows16_kernel -- 0.53 of peak instead of 0.79, round 5)
    const uint64_t j = udiv_u(b, p.bcount);
    return {j, b - j * p.bcount};
}
// the kernel-argument arrays, indexed with a wave-uniform j (ordinary reads of the kernarg segment:
// the compiler emits scalar loads; the build checks that no kernel uses scratch)
__device__ __forceinline__ uint64_t karg64(const uint64_t *a, uint64_t j) { return a[j]; }

__device__ __forceinline__ Edges edges_of(uint64_t ptr, uint64_t n) {
    const uint64_t end = ptr + n, H = (ptr + 15) & ~15ull, Ea = end & ~15ull;
    return Ea > H ? Edges{ptr, H, Ea, end} : Edges{ptr, end, end, end};
}
// a list buffer's address and length: both scalar loads in flight together, one wait
__device__ __forceinline__ void list_desc(const ScanParams &p, uint64_t b, uint64_t &ptr, uint64_t &n) {
    const uint64_t pa = rfl64((uint64_t)(p.d_ptrs + b)), la = rfl64((uint64_t)(p.d_lens + b));
    asm volatile("s_load_dwordx2 %0, %2, 0x0\n\ts_load_dwordx2 %1, %3, 0x0\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(ptr), "=&s"(n)
                 : "s"(pa), "s"(la)
                 : "memory");
}

template <bool LIST>
__device__ __forceinline__ Edges buffer_edges(const ScanParams &p, uint64_t b) {
    uint64_t ptr, n;
    if (LIST) {
        list_desc(p, b, ptr, n);
    } else {
        const BatchPos bp = batch_pos(p, b);
        ptr = karg64(p.bbase, bp.j) + bp.i * p.stride;
        n = p.len;
    }
    return edges_of(ptr, n);
}

template <bool LIST>
__device__ __forceinline__ Tile make_tile(const ScanParams &p, uint64_t t, Walker &wk) {
    Tile d;
    if (!LIST) {
        d.T = p.tiles_per_buf;
        d.b = udiv_u(t, d.T);
        d.k = t - d.b * d.T;
        d.tbase = t - d.k;
    } else {
        while (t >= wk.hi) {
            ++wk.b;
            wk.lo = wk.hi;
            wk.hi = sload64(p.d_tile_prefix + wk.b + 1);
        }
        d.b = wk.b;
        d.k = t - wk.lo;
        d.T = wk.hi - wk.lo;
        d.tbase = wk.lo;
    }
    const Edges e = buffer_edges<LIST>(p, d.b);
    const uint64_t mainlen = e.tail - e.headend;  // 0 when there is no 16-aligned main region
    const uint64_t tile_bytes = (uint64_t)p.seg * kWave;
    const uint64_t pad = d.T * tile_bytes - mainlen;
    d.pad = d.k == 0 ? (uint32_t)pad : 0u;
    d.vbase = e.headend - pad + d.k * tile_bytes;
    d.ngroups = mainlen ? p.seg / kGroupBytes : 0u;
    return d;
}

// Front pad of a buffer's first tile: the braids stay zero through the virtual zero rows (u starts
// at 0 and T'(0) = 0), so the scans start at the group holding the pad's end, and a group is
// "clean" (no zeroed rows, no head-state injection: the fused load-and-scan path) once it starts
// past the pad.  A wave group is 4 KiB for both widths (16 rows of 256 B, 8 of 512 B).
constexpr uint32_t kWaveGroupBytes = 4096;
__device__ __forceinline__ uint32_t first_group(uint32_t pad) { return pad / kWaveGroupBytes; }
__device__ __forceinline__ bool group_clean(uint32_t pad, uint32_t g) { return pad == 0 || pad < g * kWaveGroupBytes; }

// bytes [a, end) folded into state s (a < end, both inside 16-aligned blocks read by SMEM)
template <class E>
__device__ __forceinline__ typename E::T fold_bytes(typename E::T s, uint64_t a, uint64_t end, const E &eng) {
    for (uint64_t blk = a & ~15ull; blk < end; blk += 16) {
        v4u w;
        const uint64_t sblk = rfl64(blk);
        asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(w) : "s"(sblk) : "memory");
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

// head state of buffer b with edges e: ~seed advanced over the unaligned head bytes [ptr, headend)
template <bool LIST, class E>
__device__ __forceinline__ typename E::T head_state_e(const ScanParams &p, uint64_t b, const Edges &e, const E &eng) {
    using T = typename E::T;
    uint64_t seed = p.seed_all;
    const void *seeds = p.d_seeds;
    uint64_t si = b;
    if (!LIST) {
        const BatchPos bp = batch_pos(p, b);
        seeds = (const void *)karg64(p.bseed, bp.j);
        si = bp.i;
    }
    if (seeds)
        seed = E::W == 32 ? (uint64_t)sload32((const uint32_t *)seeds + si) : sload64((const uint64_t *)seeds + si);
    T s = (T)~seed;
    if (e.headend > e.ptr) s = fold_bytes(s, e.ptr, e.headend, eng);
    return s;
}
// head state of buffer b: ~seed advanced over the unaligned head bytes [ptr, headend)
template <bool LIST, class E>
__device__ __forceinline__ typename E::T head_state(const ScanParams &p, uint64_t b, const E &eng) {
    using T = typename E::T;
    uint64_t seed = p.seed_all;
    const void *seeds = p.d_seeds;
    uint64_t si = b;
    if (!LIST) {
        const BatchPos bp = batch_pos(p, b);
        seeds = (const void *)karg64(p.bseed, bp.j);
        si = bp.i;
    }
    if (seeds)
        seed = E::W == 32 ? (uint64_t)sload32((const uint32_t *)seeds + si) : sload64((const uint64_t *)seeds + si);
    T s = (T)~seed;
    const Edges e = buffer_edges<LIST>(p, b);
    if (e.headend > e.ptr) s = fold_bytes(s, e.ptr, e.headend, eng);
    return s;
}

// buffer b's register after its main region -> tail bytes, complement, store
template <bool LIST, class E>
__device__ __forceinline__ void finalize_e(const ScanParams &p, uint64_t b, const Edges &e, typename E::T fin, const E &eng);
template <bool LIST, class E>
__device__ __forceinline__ void finalize(const ScanParams &p, uint64_t b, typename E::T fin, const E &eng) {
    finalize_e<LIST>(p, b, buffer_edges<LIST>(p, b), fin, eng);
}
template <bool LIST, class E>
__device__ __forceinline__ void finalize_e(const ScanParams &p, uint64_t b, const Edges &e, typename E::T fin, const E &eng) {
    if (e.end > e.tail) fin = fold_bytes(fin, e.tail, e.end, eng);
    fin = ~fin;
    void *out = p.d_out;
    uint64_t oi = b;
    if (!LIST) {
        const BatchPos bp = batch_pos(p, b);
        out = (void *)karg64(p.bout, bp.j);
        oi = bp.i;
    }
    // result stores are inline asm: a compiler-visible store inside a scan loop makes the loop-header
    // merge of the compiler's wait counts pessimistic (it then drains the payload ring early)
    if (E::W == 32)
        asm volatile("global_store_dword %0, %1, off" : : "v"((uint32_t *)out + oi), "v"((uint32_t)fin) : "memory");
    else
        asm volatile("global_store_dwordx2 %0, %1, off" : : "v"((uint64_t *)out + oi), "v"((uint64_t)fin) : "memory");
}

// r * x^(8*TILE*kk) for a wave-uniform r: the 32/64 columns come in by SMEM, eight at a time (sixteen
// per round trip, 32 SGPRs live, made the compiler spill 100-2000 SGPRs in the scans: round 4)
template <class T, int W>
__device__ __forceinline__ T mul_pcols(T r, const uint64_t *cols) {
    T acc = 0;
#pragma unroll
    for (int c = 0; c < W; c += 8) {
        uint64_t k0, k1, k2, k3, k4, k5, k6, k7;
        const uint64_t a = rfl64((uint64_t)(cols + c));  // the table address must live in SGPRs
        asm volatile(
            "s_load_dwordx2 %0, %8, 0x0\n\ts_load_dwordx2 %1, %8, 0x8\n\t"
            "s_load_dwordx2 %2, %8, 0x10\n\ts_load_dwordx2 %3, %8, 0x18\n\t"
            "s_load_dwordx2 %4, %8, 0x20\n\ts_load_dwordx2 %5, %8, 0x28\n\t"
            "s_load_dwordx2 %6, %8, 0x30\n\ts_load_dwordx2 %7, %8, 0x38\n\t"
            "s_waitcnt lgkmcnt(0)"
            // early-clobber: a returning load must never overwrite the shared address operand
            : "=&s"(k0), "=&s"(k1), "=&s"(k2), "=&s"(k3), "=&s"(k4), "=&s"(k5), "=&s"(k6), "=&s"(k7)
            : "s"(a)
            : "memory");
        const uint64_t k[8] = {k0, k1, k2, k3, k4, k5, k6, k7};
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if ((r >> (W - 1 - (c + j))) & 1) acc ^= (T)k[j];
    }
    return acc;
}

// r * M for a wave-uniform r from M's nibble image (engine.cpp nib_image: entry 16 i + v = the product
// of nibble i's value v): one scalar load per nibble at a data-dependent offset, all issued before one
// wait -- one round trip for W = 32, two for W = 64 (sixteen 64-bit results at once would hold ~50
// SGPRs), against mul_pcols' W / 8 dependent rounds (round 5: the list scans' head entries and part
// shifts, the CRC64 part shifts)
__device__ __forceinline__ uint32_t mul_nib32(uint32_t r, const uint32_t *img) {
    const uint64_t a = rfl64((uint64_t)img);
    r = __builtin_amdgcn_readfirstlane(r);
    uint32_t o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = 64u * i + 4u * ((r >> (28 - 4 * i)) & 15u);
    uint32_t k0, k1, k2, k3, k4, k5, k6, k7;
    asm volatile(
        "s_load_dword %0, %8, %9\n\ts_load_dword %1, %8, %10\n\ts_load_dword %2, %8, %11\n\ts_load_dword %3, %8, %12\n\t"
        "s_load_dword %4, %8, %13\n\ts_load_dword %5, %8, %14\n\ts_load_dword %6, %8, %15\n\ts_load_dword %7, %8, %16\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(k0), "=&s"(k1), "=&s"(k2), "=&s"(k3), "=&s"(k4), "=&s"(k5), "=&s"(k6), "=&s"(k7)
        : "s"(a), "s"(o[0]), "s"(o[1]), "s"(o[2]), "s"(o[3]), "s"(o[4]), "s"(o[5]), "s"(o[6]), "s"(o[7])
        : "memory");
    return k0 ^ k1 ^ k2 ^ k3 ^ k4 ^ k5 ^ k6 ^ k7;
}
__device__ __forceinline__ uint64_t mul_nib64(uint64_t r, const uint64_t *img) {
    const uint64_t a = rfl64((uint64_t)img);
    r = rfl64(r);
    uint64_t acc = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        uint32_t o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = 128u * (8 * h + i) + 8u * (uint32_t)((r >> (60 - 4 * (8 * h + i))) & 15u);
        uint64_t k0, k1, k2, k3, k4, k5, k6, k7;
        asm volatile(
            "s_load_dwordx2 %0, %8, %9\n\ts_load_dwordx2 %1, %8, %10\n\ts_load_dwordx2 %2, %8, %11\n\ts_load_dwordx2 %3, %8, %12\n\t"
            "s_load_dwordx2 %4, %8, %13\n\ts_load_dwordx2 %5, %8, %14\n\ts_load_dwordx2 %6, %8, %15\n\ts_load_dwordx2 %7, %8, %16\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&s"(k0), "=&s"(k1), "=&s"(k2), "=&s"(k3), "=&s"(k4), "=&s"(k5), "=&s"(k6), "=&s"(k7)
            : "s"(a), "s"(o[0]), "s"(o[1]), "s"(o[2]), "s"(o[3]), "s"(o[4]), "s"(o[5]), "s"(o[6]), "s"(o[7])
            : "memory");
        acc ^= k0 ^ k1 ^ k2 ^ k3 ^ k4 ^ k5 ^ k6 ^ k7;
    }
    return acc;
}

__device__ __forceinline__ unsigned long long atomic_xor_ret(unsigned long long *a, unsigned long long v) {
    return __hip_atomic_fetch_xor(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------
// W = 32 braided scan (CRC32 / CRC32C).
//
// A tile of TILE bytes is R = TILE/256 rows of 256 bytes; lane l owns the 4-byte word at 4l of
// every row, so each wave-wide load reads 256 contiguous bytes.  Lane l's state u is one braid:
//     u <- (u ^ w_row) * x^(8*256)       (four lookups in T', whose entries fold in the skip over
//                                          the other 63 lanes' words of the row)
// After the R rows u = sum_c w_c * x^(8*256(R-c)), while word (c, l) belongs at x^(8(TILE-256c-4l))
// relative to the tile end.  So u * x^(-32 l) is lane l's exact share (x is invertible mod P since
// P(0) = 1): K_l = x^(-32 l), and the tile register is XOR_l u_l * K_l.
//
// LDS (77 KiB, so two 512-thread workgroups share a CU and a launch's prologue overlaps the previous
// launch's scan on the same CU):
//   T' tables, 8 copies, quarter-rotated: the 256-byte row of entry e holds the four tables in
//   quarters of 32 bytes (quarter q = the table indexed by byte q of a, i.e. T'_(3-q)), 8 copies
//   of 4 bytes each; bytes [128, 256) of every row are unused (v_perm can place the entry byte at
//   bit 8, not bit 7).  In table slot k, lane quarter j = (lane >> 3) & 3 reads quarter (k + j) & 3
//   with copy lane & 7, so a ds_read_b32 half-wave touches its 32 banks (bank = 8q + copy) once.
constexpr uint32_t kBTabBytes = 65536;
constexpr uint32_t kBKOff = kBTabBytes;               // K image, [j/4][lane][j%4] (8 KiB)
constexpr uint32_t kPcolOff = kBKOff + 8192;          // [m < 32][column j] of x^(8*TILE*m) (4 KiB)
constexpr uint32_t kT0Off = kPcolOff + 4096;          // plain byte table (1 KiB; wave-uniform reads)
constexpr uint32_t kConstFlagOff = kT0Off + 1024;     // waves that have published their K / P words
constexpr uint32_t kPoolOff = kConstFlagOff + 4;      // workgroup tile pool: tiles claimed so far
constexpr uint32_t kBraidLds = kConstFlagOff + 16;
// streaming scans: workgroup-local buffer slots (tile registers of buffers whose tiles all lie in one
// workgroup's range are combined with LDS atomics instead of device-scope ones)
#ifndef AMDCRC_STREAM_PRIO  // compile-time only (A/B builds): crc32_stream_kernel issue priority by work left
#define AMDCRC_STREAM_PRIO 1
#endif
#ifndef AMDCRC_R16_PRIO  // compile-time only (A/B builds): the same in crc64_rows16_kernel
#define AMDCRC_R16_PRIO 1
#endif
#ifndef AMDCRC_PRIO_ALL  // compile-time only (A/B builds): the same in the CRC64 and list scans
#define AMDCRC_PRIO_ALL 0
#endif
// Issue priority by the work a wave has left (round 5).  Two workgroups share a CU and the one
// dispatched first is served first (oldest-first issue): its waves finished a 20-batch C2 launch at
// ~144 us, the second workgroup's at ~190 us of ~200 (per-wave stamps), the launch's last 25 % running
// on half the waves.  Every fourth group a wave sets s_setprio to min(3, groups left * 6 / groups),
// so the waves behind are issued first and the waves of a CU finish together (A/B: 0.845 -> 0.862;
// scale 6 against 4: +0.3 %, within the noise of two sessions).
#ifndef AMDCRC_PRIO_EVERY  // compile-time only (A/B builds): groups between priority updates (power of two)
#define AMDCRC_PRIO_EVERY 4
#endif
#ifndef AMDCRC_PRIO_SCALE  // compile-time only (A/B builds): priority = groups left * SCALE / groups, capped at 3
#define AMDCRC_PRIO_SCALE 6
#endif
__device__ __forceinline__ void prio_by_work_left(uint32_t q, uint32_t nq) {
    if (q & (AMDCRC_PRIO_EVERY - 1u)) return;
    const uint32_t pr = (uint32_t)(((uint64_t)(nq - q) * AMDCRC_PRIO_SCALE) / ((uint64_t)nq + 1u));
    if (pr >= 3) __builtin_amdgcn_s_setprio(3);
    else if (pr == 2) __builtin_amdgcn_s_setprio(2);
    else if (pr == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}
constexpr uint32_t kLocalSlots = 128;
static_assert(kLocalSlots == kStreamLocalSlots, "engine.cpp stream_local_only mirrors the slot count");
constexpr uint32_t kLocalOff = kBraidLds;
constexpr uint32_t kStreamLds = kLocalOff + 8 * kLocalSlots;
constexpr int kBraidBlock = 512;                      // 8 waves; two workgroups per CU
constexpr int kBraidWaves = kBraidBlock / kWave;

// Compile-time GF(2) bases of the braided scan's byte tables: entry e of a table is the XOR of the
// basis values of e's set bits (the tables are linear in e), so the tables are built from
// immediates with no memory traffic.
//   b[k][i] = T'_k[1 << i] = (1 << i) * x^(8(k+1)) * x^(8*252)     (k < 4)
//   b[4][i] = T_0[1 << i]  = (1 << i) * x^8
template <uint32_t POLY>
struct BraidBasis {
    uint32_t b[5][8];
    constexpr BraidBasis() : b() {
        const uint64_t skip = gf2_xpow8n(kBraidRow - 4, POLY, 32);
        for (int i = 0; i < 8; ++i) {
            for (int k = 0; k < 4; ++k) b[k][i] = (uint32_t)gf2_mulmod(gf2_table_entry(1u << i, k, POLY), skip, POLY, 32);
            b[4][i] = (uint32_t)gf2_table_entry(1u << i, 0, POLY);
        }
    }
};

// basis value b[k][bit] for a per-lane (runtime) table index k < 4: four compile-time candidates
// (masks made opaque: a select chain over constants becomes a per-lane global load from a constant
// table, which the table build would then wait for behind the payload loads already in flight)
template <uint32_t POLY>
__device__ __forceinline__ uint32_t basis_bit(uint32_t k, int bit) {
    constexpr BraidBasis<POLY> B{};
    uint32_t m0 = k == 0 ? ~0u : 0u, m1 = k == 1 ? ~0u : 0u, m2 = k == 2 ? ~0u : 0u, m3 = k == 3 ? ~0u : 0u;
    asm("" : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3));
    return (B.b[0][bit] & m0) | (B.b[1][bit] & m1) | (B.b[2][bit] & m2) | (B.b[3][bit] & m3);
}

template <uint32_t POLY, int K>
__device__ __forceinline__ uint32_t basis_entry(uint32_t e) {
    constexpr BraidBasis<POLY> B{};
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) v ^= ((e >> i) & 1u) ? B.b[K][i] : 0u;
    return v;
}

template <uint32_t POLY>
struct Braid32 {
    using T = uint32_t;
    static constexpr int W = 32;
    const char *L;
    const char *C;  // the constants region (K image, P columns, byte table, flags, local slots)
    uint32_t cst[4], sel[4];  // per lane and table slot k: quarter<<5 | copy<<2, and the v_perm selector

    __device__ void init(const char *lds, int lane) {
        L = lds;
        C = lds + kBKOff;
        const uint32_t j = ((uint32_t)lane >> 3) & 3u, cp = (uint32_t)lane & 7u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t q = (k + j) & 3u;
            cst[k] = (q << 5) | (cp << 2);
            sel[k] = 0x0c0c0004u | (q << 8);  // byte0 <- cst, byte1 <- byte q of a, bytes 2-3 <- 0
        }
    }
    // the four T' lookups of a = u ^ w: slot k reads the table of byte (k + j) & 3 (any order: XORed)
    __device__ __forceinline__ void look(uint32_t a, uint32_t &l3, uint32_t &l2, uint32_t &l1, uint32_t &l0) const {
        l3 = lds32(L, __builtin_amdgcn_perm(cst[0], a, sel[0]));
        l2 = lds32(L, __builtin_amdgcn_perm(cst[1], a, sel[1]));
        l1 = lds32(L, __builtin_amdgcn_perm(cst[2], a, sel[2]));
        l0 = lds32(L, __builtin_amdgcn_perm(cst[3], a, sel[3]));
    }
    // a * x^(8*256)
    __device__ __forceinline__ uint32_t step(uint32_t a) const {
        uint32_t l3, l2, l1, l0;
        look(a, l3, l2, l1, l0);
        return l3 ^ l2 ^ l1 ^ l0;
    }
    // a * x^(8*256) ^ wn  (two 3-input XORs)
    __device__ __forceinline__ uint32_t step_x(uint32_t a, uint32_t wn) const {
        uint32_t l3, l2, l1, l0;
        look(a, l3, l2, l1, l0);
        return xor3(xor3(l3, l2, wn), l1, l0);
    }
    // plain byte step for head / tail bytes (s is wave-uniform: broadcast reads)
    __device__ __forceinline__ uint32_t byte(uint32_t s, uint32_t b) const {
        return (s >> 8) ^ lds32(C, (kT0Off - kBKOff) + 4 * ((s ^ b) & 0xffu));
    }
    // the constants region: after the tables (kBKOff for the 4- and 8-byte-word tables)
    __device__ __forceinline__ const char *cbase() const { return C; }
    // r * K_lane : 32 LDS matrix columns
    __device__ __forceinline__ uint32_t mulK(uint32_t r, int lane) const {
        uint32_t acc = 0;
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            const uint4 c = *(const uint4 *)(C + (g * 64 + lane) * 16);
            acc = xor_and(acc, c.x, (uint32_t)__builtin_amdgcn_sbfe((int)r, 31 - (4 * g + 0), 1));
            acc = xor_and(acc, c.y, (uint32_t)__builtin_amdgcn_sbfe((int)r, 31 - (4 * g + 1), 1));
            acc = xor_and(acc, c.z, (uint32_t)__builtin_amdgcn_sbfe((int)r, 31 - (4 * g + 2), 1));
            acc = xor_and(acc, c.w, (uint32_t)__builtin_amdgcn_sbfe((int)r, 31 - (4 * g + 3), 1));
        }
        return acc;
    }
};

struct BGroup {
    uint32_t w[kBraidRowsPerGroup];
};

// ---- the W=32 streaming scan on 8-byte words (crc32_stream_kernel<POLY, true>).  A row is 512
// bytes, lane l owning the 8-byte word at 8l (one global_load_dwordx2 per lane: half the load
// instructions of 4-byte words for the same bytes).  The row step is slice-by-8 for the 32-bit
// register: a = (u ^ lo(w), hi(w)), u' = XOR_t T'_t[byte (7-t) of a] with
// T'_t[e] = e * x^(8(t+1)) * x^(8*504), so the four lookups of hi(w) do not depend on u and only
// half of a row's lookups sit on the braid's dependency chain.  Lane l's share is u * x^(-64 l).
// LDS: the eight tables in 8 copies, one 256-byte row per entry e (table t at 32 t, copy c at 4 c:
// the row is fully used, the constants region at kBKOff is unchanged).  In slot k < 4 a lane reads
// byte q = (k + j) & 3 of lo (table 7 - q), in slot 4 + k the same byte of hi (table 3 - q), with
// j = (lane >> 3) & 3 and copy lane & 7: a ds_read_b32 half-wave meets 32 distinct dword columns.
constexpr uint32_t kW8Row = 512;
constexpr int kW8RowsPerGroup = 8;  // 4 KiB per wave per ring slot, as the 4-byte rows
static_assert(kW8Row * kW8RowsPerGroup == kBraidRow * kBraidRowsPerGroup, "ring slot size");

template <uint32_t POLY>
struct BraidW8Basis {
    uint32_t b[9][8];  // b[t][i] = T'_t[1 << i] (t < 8); b[8][i] = T_0[1 << i]
    constexpr BraidW8Basis() : b() {
        const uint64_t skip = gf2_xpow8n(kW8Row - 8, POLY, 32);
        for (int i = 0; i < 8; ++i) {
            for (int t = 0; t < 8; ++t) b[t][i] = (uint32_t)gf2_mulmod(gf2_table_entry(1u << i, t, POLY), skip, POLY, 32);
            b[8][i] = (uint32_t)gf2_table_entry(1u << i, 0, POLY);
        }
    }
};
template <uint32_t POLY, int K>
__device__ __forceinline__ uint32_t basis_w8(uint32_t e) {
    constexpr BraidW8Basis<POLY> B{};
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) v ^= ((e >> i) & 1u) ? B.b[K][i] : 0u;
    return v;
}
// bt[i] = T'_t[1 << i] for a per-lane t < 8: one AND-OR per candidate through opaque masks (a select
// chain over constants would become a per-lane load from a constant table, waited for behind the
// payload loads already in flight)
template <uint32_t POLY>
__device__ __forceinline__ void basis_w8_lane(uint32_t t, uint32_t (&bt)[8]) {
    constexpr BraidW8Basis<POLY> B{};
    uint32_t m[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        m[k] = t == (uint32_t)k ? ~0u : 0u;
        asm("" : "+v"(m[k]));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) v |= B.b[k][i] & m[k];
        bt[i] = v;
    }
}
// The eight slice-by-8 tables in 8 copies (64 KiB: one 256-byte row per entry e, table t at 32 t,
// copies 0-3 then 4-7) from a 512-thread workgroup, as 4096 chunks of 16 bytes: chunk k = tid + 512 m
// holds copies 4 (k & 1) .. + 3 of T'_t[e], t = (k & 15) >> 1, e = k >> 4 = (tid >> 4) + 32 m.
// Consecutive lanes store consecutive chunks, so every ds_write_b128 is conflict-free.  Round 4 built
// table t in wave t: the 64 lanes of each store met one 32-byte bank group, and the per-wave stamps
// put ~4 us between a wave's entry and its barrier (tools/stamp_probe.py).
template <uint32_t POLY>
__device__ __forceinline__ void build_w8_tables(char *lds, uint32_t tid) {
    uint32_t bt[8];
    basis_w8_lane<POLY>((tid & 15u) >> 1, bt);
    const uint32_t e0 = tid >> 4;  // bits 0-4 of e; bits 5-7 are m
    uint32_t t0v = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) t0v ^= ((e0 >> i) & 1u) ? bt[i] : 0u;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const uint32_t te = t0v ^ (m & 1 ? bt[5] : 0u) ^ (m & 2 ? bt[6] : 0u) ^ (m & 4 ? bt[7] : 0u);
        *(uint4 *)(lds + 16u * (tid + 512u * m)) = make_uint4(te, te, te, te);
    }
}
template <uint32_t POLY>
__device__ __forceinline__ uint32_t basis_w8_rt(uint32_t t, uint32_t e) {  // t wave-uniform
    switch (t) {
        case 0: return basis_w8<POLY, 0>(e);
        case 1: return basis_w8<POLY, 1>(e);
        case 2: return basis_w8<POLY, 2>(e);
        case 3: return basis_w8<POLY, 3>(e);
        case 4: return basis_w8<POLY, 4>(e);
        case 5: return basis_w8<POLY, 5>(e);
        case 6: return basis_w8<POLY, 6>(e);
        default: return basis_w8<POLY, 7>(e);
    }
}

template <uint32_t POLY>
struct Braid32W8 : Braid32<POLY> {
    uint32_t cst8[8], sel8[8];
    __device__ void init(const char *lds, int lane) {
        this->L = lds;
        this->C = lds + kBKOff;
        const uint32_t j = ((uint32_t)lane >> 3) & 3u, c = (uint32_t)lane & 7u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t q = (k + j) & 3u;
            cst8[k] = ((7u - q) << 5) | (c << 2);
            cst8[4 + k] = ((3u - q) << 5) | (c << 2);
            sel8[k] = sel8[4 + k] = 0x0c0c0004u | (q << 8);  // byte0 <- cst, byte1 <- byte q of the dword
        }
    }
    // the row step in two parts: the lo word's four lookups (on the braid's chain) and the hi word's
    // four (independent of u), which are looked up one row ahead, while the previous row's chain runs
    struct Hi {
        uint32_t v[4];
    };
    __device__ __forceinline__ uint32_t look_lo(uint32_t lo, const Hi &h, uint32_t wn) const {
        uint32_t v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = lds32(this->L, __builtin_amdgcn_perm(cst8[k], lo, sel8[k]));
        return xor3(xor3(xor3(h.v[0], h.v[1], h.v[2]), h.v[3], wn), xor3(v[0], v[1], v[2]), v[3]);
    }
    __device__ __forceinline__ Hi look_hi(uint32_t hi) const {
        Hi h;
#pragma unroll
        for (int k = 0; k < 4; ++k) h.v[k] = lds32(this->L, __builtin_amdgcn_perm(cst8[4 + k], hi, sel8[4 + k]));
        return h;
    }
};

struct W8Group {
    uint64_t w[kW8RowsPerGroup];
};

// ---- the W=32 streaming scan on 16-byte words (crc32_stream_kernel<POLY, 16>, large launches).  A row
// is 1024 bytes, lane l owning the 16-byte word at 16l (one global_load_dwordx4 per lane per row: half
// the load instructions and half the row steps of 8-byte words for the same bytes).  The row step is
// slice-by-16 on a = (u ^ d0, d1, d2, d3): u' = XOR_i T'_(15-i)[byte i of a] with
// T'_t[e] = e * x^(8(t+1)) * x^(8*1008), so only d0's four lookups sit on the braid's dependency
// chain; d1..d3's twelve are looked up one row ahead.  Lane l's share is u * x^(-128 l).
// LDS: two regions shaped like the 8-byte-word tables, A = T'_15..T'_8 (bytes 0..7) at 0 and
// B = T'_7..T'_0 (bytes 8..15) at 64 KiB; table t at (t & 7) * 32 of entry e's 256-byte row, 8 copies
// of 4 bytes.  In slot k a lane reads byte q = (k + j) & 3 of dword d (table 15 - 4d - q), copy
// lane & 7, j = (lane >> 3) & 3: bank 8 (3 - q) + copy, so every ds_read_b32 half-wave meets 32
// distinct banks (tests/test_braid_model.py::test_w16_lds_schedule_conflict_free_and_complete).  The
// 128 KiB of tables take one 1024-thread workgroup (16 waves) per CU.
constexpr uint32_t kW16Row = 1024;
constexpr int kW16RowsPerGroup = 4;  // 4 KiB per wave per ring slot, as the other widths
constexpr uint32_t kW16TabBytes = 131072;
constexpr int kW16Block = 1024;
static_assert(kW16Row * kW16RowsPerGroup == kBraidRow * kBraidRowsPerGroup, "ring slot size");

template <uint32_t POLY>
struct BraidW16Basis {
    uint32_t b[17][8];  // b[t][i] = T'_t[1 << i] (t < 16); b[16][i] = T_0[1 << i]
    constexpr BraidW16Basis() : b() {
        const uint64_t skip = gf2_xpow8n(kW16Row - 16, POLY, 32);
        for (int i = 0; i < 8; ++i) {
            for (int t = 0; t < 16; ++t) b[t][i] = (uint32_t)gf2_mulmod(gf2_table_entry(1u << i, t, POLY), skip, POLY, 32);
            b[16][i] = (uint32_t)gf2_table_entry(1u << i, 0, POLY);
        }
    }
};
template <uint32_t POLY, int K>
__device__ __forceinline__ uint32_t basis_w16(uint32_t e) {
    constexpr BraidW16Basis<POLY> B{};
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) v ^= ((e >> i) & 1u) ? B.b[K][i] : 0u;
    return v;
}
template <uint32_t POLY, int K = 0>
__device__ __forceinline__ uint32_t basis_w16_rt(uint32_t t, uint32_t e) {  // t wave-uniform
    if constexpr (K < 15) {
        if (t == K) return basis_w16<POLY, K>(e);
        return basis_w16_rt<POLY, K + 1>(t, e);
    } else {
        return basis_w16<POLY, 15>(e);
    }
}

template <uint32_t POLY>
struct Braid32W16 : Braid32<POLY> {
    uint32_t cst16[4][4];  // [dword d][slot k]: region B << 16 | (t & 7) << 5 | copy << 2, t = 15 - 4d - q
    uint32_t sel16[4];     // [slot k]: byte0 <- cst, byte1 <- byte q of the dword, byte2 <- cst (region)
    __device__ void init(const char *lds, int lane) {
        this->L = lds;
        this->C = lds + kW16TabBytes;
        const uint32_t j = ((uint32_t)lane >> 3) & 3u, c = (uint32_t)lane & 7u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t q = (k + j) & 3u;
            sel16[k] = 0x0c060004u | (q << 8);
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const uint32_t t = 15u - 4u * d - q;
                cst16[d][k] = (t < 8 ? 0x10000u : 0u) | ((t & 7u) << 5) | (c << 2);
            }
        }
    }
    __device__ __forceinline__ uint32_t look(int d, int k, uint32_t v) const {
        return lds32(this->L, __builtin_amdgcn_perm(cst16[d][k], v, sel16[k]));
    }
    // d1..d3's twelve lookups of a row (independent of u), XORed in at the next row's chain step
    struct Hi {
        uint32_t v[12];
    };
    __device__ __forceinline__ Hi look_hi(const v4u &w) const {
        Hi h;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            h.v[k] = look(1, k, w.y);
            h.v[4 + k] = look(2, k, w.z);
            h.v[8 + k] = look(3, k, w.w);
        }
        return h;
    }
    // the chain step in two parts: the four lookups of x = u ^ d0 (issued first), then the row's
    // u' ^ wn once they return, with the row's other twelve lookups h
    struct Lo {
        uint32_t v[4];
    };
    __device__ __forceinline__ Lo lo_issue(uint32_t x) const {
        Lo l;
#pragma unroll
        for (int k = 0; k < 4; ++k) l.v[k] = look(0, k, x);
        return l;
    }
    __device__ __forceinline__ uint32_t lo_finish(const Lo &l, const Hi &h, uint32_t wn) const {
        const uint32_t o = xor3(xor3(xor3(h.v[0], h.v[1], h.v[2]), xor3(h.v[3], h.v[4], h.v[5]), xor3(h.v[6], h.v[7], h.v[8])),
                                xor3(h.v[9], h.v[10], h.v[11]), wn);
        return xor3(xor3(o, l.v[0], l.v[1]), l.v[2], l.v[3]);
    }
    __device__ __forceinline__ uint32_t look_lo(uint32_t x, const Hi &h, uint32_t wn) const { return lo_finish(lo_issue(x), h, wn); }
};

struct W16Group {
    v4u w[kW16RowsPerGroup];
};

// one payload word; NT: non-temporal (streamed once, not kept in the caches)
template <bool NT>
__device__ __forceinline__ uint32_t ldpay(uint64_t a) {
    if (NT) return __builtin_nontemporal_load((gu32 *)a);
    return *(gu32 *)a;
}

// group gi of a tile: rows [16 gi, 16 gi + 16), this lane's word of each (virtual offset
// gi*4096 + 256 r + 4 lane).  Words in the virtual front pad read a valid address (the main start)
// and are zeroed by braid_proc.  Rows go out in order on every path (scheduling barriers): the
// compiler's vmcnt bookkeeping merges paths, and one path with row 0 issued late would make every
// wait for row 0 drain the whole group.
template <bool NT>
__device__ __forceinline__ void braid_load(BGroup &g, uint64_t vbase, uint32_t pad, uint32_t gi, int lane) {
    const uint32_t vo0 = gi * (kBraidRow * kBraidRowsPerGroup) + 4u * lane;
#pragma unroll
    for (int r = 0; r < kBraidRowsPerGroup; ++r) {
        const uint32_t vo = vo0 + kBraidRow * r;
        g.w[r] = ldpay<NT>(vbase + (vo >= pad ? vo : pad));
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <class B>
__device__ __forceinline__ uint32_t braid_proc(uint32_t u, const BGroup &g, const B &eng, const Tile &d, uint32_t gi,
                                               int lane, uint32_t s_h) {
    if (group_clean(d.pad, gi)) {
        uint32_t a = u ^ g.w[0];
#pragma unroll
        for (int r = 0; r + 1 < kBraidRowsPerGroup; ++r) a = eng.step_x(a, g.w[r + 1]);
        return eng.step(a);
    }
    const uint32_t vo0 = gi * (kBraidRow * kBraidRowsPerGroup) + 4u * lane;
#pragma unroll
    for (int r = 0; r < kBraidRowsPerGroup; ++r) {
        const uint32_t vo = vo0 + kBraidRow * r;
        uint32_t w = vo >= d.pad ? g.w[r] : 0u;
        if (vo == d.pad) w ^= s_h;  // this braid is still zero here: the head state enters with the word
        u = eng.step(u ^ w);
    }
    return u;
}

// Steady state (neither the scanned nor the prefetched group in a front-padded tile): scan group g
// while issuing group g+1's loads, RATE per table step.  Issue and scan share one basic block and a
// scheduling barrier after every step, so the loads stream out between the table steps instead of in
// a 16-load burst per wave (measured: a burst-issue loop is 20 % slower at the same work).  With two
// ring slots the other slot's loads are always the youngest in flight at every loop point, which
// keeps the compiler's vmcnt bookkeeping exact across the loop.
template <int RATE, bool NT, class B>
__device__ __forceinline__ uint32_t braid_fused(uint32_t u, const BGroup &g, BGroup &dst, uint64_t a, const B &eng) {
    uint32_t x = u ^ g.w[0];
#pragma unroll
    for (int st = 0; st < kBraidRowsPerGroup; ++st) {
#pragma unroll
        for (int q = 0; q < RATE; ++q) {
            const int r = RATE * st + q;
            if (r < kBraidRowsPerGroup) dst.w[r] = ldpay<NT>(a + kBraidRow * r);
        }
        x = st + 1 < kBraidRowsPerGroup ? eng.step_x(x, g.w[st + 1]) : eng.step(x);
        __builtin_amdgcn_sched_barrier(0);
    }
    return x;
}

// The same three steps on 8-byte words (crc32_braid_kernel<POLY, LIST, NT, true>): group gi is rows
// [8 gi, 8 gi + 8) of 512 bytes, this lane's word at virtual offset gi*4096 + 512 r + 8 lane; the row
// step splits into the lo word's lookups (the chain) and the hi word's, looked up one row ahead.
template <bool NT>
__device__ __forceinline__ uint64_t ldpay8(uint64_t a) {
    if (NT) return __builtin_nontemporal_load((gu64 *)a);
    return *(gu64 *)a;
}
template <bool NT>
__device__ __forceinline__ void braid_load(W8Group &g, uint64_t vbase, uint32_t pad, uint32_t gi, int lane) {
    const uint32_t vo0 = gi * (kW8Row * kW8RowsPerGroup) + 8u * lane;
#pragma unroll
    for (int r = 0; r < kW8RowsPerGroup; ++r) {
        const uint32_t vo = vo0 + kW8Row * r;
        g.w[r] = ldpay8<NT>(vbase + (vo >= pad ? vo : pad));
        __builtin_amdgcn_sched_barrier(0);
    }
}
template <class B>
__device__ __forceinline__ uint32_t braid_proc(uint32_t u, const W8Group &g, const B &eng, const Tile &d, uint32_t gi,
                                               int lane, uint32_t s_h) {
    if (group_clean(d.pad, gi)) {
        uint32_t x = u ^ (uint32_t)g.w[0];
        typename B::Hi h = eng.look_hi((uint32_t)(g.w[0] >> 32));
#pragma unroll
        for (int r = 1; r < kW8RowsPerGroup; ++r) {
            x = eng.look_lo(x, h, (uint32_t)g.w[r]);
            h = eng.look_hi((uint32_t)(g.w[r] >> 32));
        }
        return eng.look_lo(x, h, 0u);
    }
    const uint32_t vo0 = gi * (kW8Row * kW8RowsPerGroup) + 8u * lane;
#pragma unroll
    for (int r = 0; r < kW8RowsPerGroup; ++r) {
        const uint32_t vo = vo0 + kW8Row * r;
        uint64_t w = vo >= d.pad ? g.w[r] : 0ull;
        if (vo == d.pad) w ^= s_h;  // this braid is still zero here: the head state enters with the word
        u = eng.look_lo(u ^ (uint32_t)w, eng.look_hi((uint32_t)(w >> 32)), 0u);
    }
    return u;
}
template <int RATE, bool NT, class B>
__device__ __forceinline__ uint32_t braid_fused(uint32_t u, const W8Group &g, W8Group &dst, uint64_t a, const B &eng) {
    static_assert(RATE == 1, "one load per row step");
    uint32_t x = u ^ (uint32_t)g.w[0];
    typename B::Hi h{};
#pragma unroll
    for (int r = 0; r < kW8RowsPerGroup; ++r) {
        dst.w[r] = ldpay8<NT>(a + kW8Row * r);
        if (r > 0) x = eng.look_lo(x, h, (uint32_t)g.w[r]);
        h = eng.look_hi((uint32_t)(g.w[r] >> 32));
        __builtin_amdgcn_sched_barrier(0);
    }
    return eng.look_lo(x, h, 0u);
}

// Cross-tile combine.  Tiles form groups of 32; tile k's register is moved to its group's end
// (r * x^(8*TILE*m), m < 32: columns in LDS, one per lane).  A wave merges the shares of its own
// tiles of one group in registers {arrival bits | XOR} and publishes them with one 64-bit atomic XOR
// into the group's slot when it moves to another group or runs out of tiles.  Whoever completes the
// slot's arrival bits finishes the buffer (T <= 32), or moves the group value to the buffer end
// (scalar column table, once per group) and XORs it into the buffer word, counting groups (T > 32).
// At most 32 atomics meet on one address, and a wave waits for a returned value only when it
// publishes its next group (rare) or at its end.
struct BGroupAcc {
    uint64_t slot;  // ~0: no open group
    unsigned long long val;
    uint64_t b, T;
    uint32_t g0;  // first tile of the group within its buffer
};
struct BPending {
    bool valid;
    unsigned long long val, old;
    BGroupAcc g;
};

template <bool LIST, class B>
__device__ __forceinline__ void braid_resolve(const ScanParams &p, BPending &pd, const B &eng, int lane) {
    if (!pd.valid) return;
    pd.valid = false;
    const unsigned long long now = rfl64(pd.old) ^ pd.val;
    const BGroupAcc &g = pd.g;
    const uint64_t n = g.T - g.g0 < 32 ? g.T - g.g0 : 32, G = (g.T + 31) / 32, shift = g.T - g.g0 - n;
    const unsigned long long full = n >= 32 ? 0xFFFFFFFF00000000ull : (((1ull << n) - 1) << 32);
    if ((now & 0xFFFFFFFF00000000ull) != full) return;
    uint32_t grp = (uint32_t)now;
    if (G > 1 && shift) grp = mul_pcols<uint32_t, 32>(grp, p.d_pcols + shift * 32);
    if (lane != 0) return;
    __hip_atomic_exchange(&p.d_acc1[g.slot], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (G == 1) {
        finalize<LIST>(p, g.b, grp, eng);
        return;
    }
    const unsigned long long o =
        __hip_atomic_fetch_xor(&p.d_acc[g.b], (unsigned long long)grp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(o) : "memory");  // performed before it is counted
    const unsigned int c = __hip_atomic_fetch_add(&p.d_cnt[g.b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (c == G - 1) {
        const uint32_t fin = (uint32_t)__hip_atomic_exchange(&p.d_acc[g.b], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&p.d_cnt[g.b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        finalize<LIST>(p, g.b, fin, eng);
    }
}

template <bool LIST, class B>
__device__ __forceinline__ void braid_publish(const ScanParams &p, BGroupAcc &acc, BPending &pd, const B &eng, int lane) {
    if (acc.slot == ~0ull) return;
    braid_resolve<LIST>(p, pd, eng, lane);
    unsigned long long old = 0;
    if (lane == 0) old = atomic_xor_ret(&p.d_acc1[acc.slot], acc.val);
    pd.valid = true;
    pd.val = acc.val;
    pd.old = old;
    pd.g = acc;
    acc.slot = ~0ull;
}

template <bool LIST, class B>
__device__ __forceinline__ void braid_finish(const ScanParams &p, const Tile &d, uint32_t u, uint32_t s_h, const B &eng, int lane,
                                             BGroupAcc &acc, BPending &pd) {
    const uint32_t r = d.ngroups ? wave_xor_s(eng.mulK(u, lane)) : 0u;
    if (d.T == 1) {
        if (lane == 0) finalize<LIST>(p, d.b, d.ngroups ? r : s_h, eng);
        return;
    }
    // r * x^(8*TILE*m) to the group end: lane j < 32 takes column j if bit (31 - j) of r is set
    const uint64_t g0 = d.k & ~31ull, gend = d.T - g0 < 32 ? d.T : g0 + 32;
    const uint32_t m = (uint32_t)(gend - 1 - d.k);
    const uint32_t colv = lds32(eng.L, kPcolOff + 4 * (m * 32 + (lane & 31)));
    const uint32_t sel = lane < 32 ? (uint32_t)__builtin_amdgcn_sbfe((int)r, 31 - lane, 1) : 0u;
    const uint32_t v = wave_xor_s(colv & sel);
    const uint64_t slot = d.tbase + g0;
    if (slot != acc.slot) {
        braid_publish<LIST>(p, acc, pd, eng, lane);
        acc.slot = slot;
        acc.val = 0;
        acc.b = d.b;
        acc.T = d.T;
        acc.g0 = (uint32_t)g0;
    }
    acc.val ^= (unsigned long long)v | (1ull << (32 + (d.k & 31)));
}

template <uint32_t POLY, bool LIST, bool NT = true, bool W8 = AMDCRC_STREAM_W8>
__global__ __launch_bounds__(kBraidBlock, 4) void crc32_braid_kernel(const ScanParams p) {
    using B = typename std::conditional<W8, Braid32W8<POLY>, Braid32<POLY>>::type;
    using Grp = typename std::conditional<W8, W8Group, BGroup>::type;
    __shared__ __attribute__((aligned(16))) char lds[kBraidLds];

    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * kBraidWaves;
    const uint64_t gw = rfl64((uint64_t)blockIdx.x * kBraidWaves + (threadIdx.x >> 6));
    // Tiles.  Static: an even split of [0, ntiles) over the waves.  Workgroup pool (p.nstatic != 0,
    // uniform batches): the workgroup's even share [wb0, wb1) is split into one static tile per wave
    // and a pool the waves claim from an LDS counter as they run dry, so a wave the memory system
    // serves late scans less of its workgroup's share.
    const bool dyn = !LIST && p.nstatic != 0;
    uint64_t t0, t1, pool_base = 0, pool_size = 0;
    if (dyn) {
        const uint64_t wb0 = udiv_u((uint64_t)blockIdx.x * p.ntiles, gridDim.x), wb1 = udiv_u(((uint64_t)blockIdx.x + 1) * p.ntiles, gridDim.x);
        const uint64_t wv = (uint64_t)(threadIdx.x >> 6);
        t0 = wb0 + wv < wb1 ? wb0 + wv : wb1;
        t1 = wb0 + wv < wb1 ? t0 + 1 : wb1;
        pool_base = wb0 + kBraidWaves;
        pool_size = pool_base < wb1 ? wb1 - pool_base : 0;
    } else {
        t0 = udiv_u(gw * p.ntiles, nw);
        t1 = udiv_u((gw + 1) * p.ntiles, nw);
    }
    t0 = rfl64(t0), t1 = rfl64(t1);
    // tiles entered by the prefetch cursor from the pool, in order, for the scan cursor
    uint64_t fifo0 = 0, fifo1 = 0;
    uint32_t fifo_n = 0;

    Walker w0{0, 0, 0};
    if (LIST && t0 < t1) {
        w0.b = sload64(p.d_wave_buf + gw);
        w0.lo = sload64(p.d_tile_prefix + w0.b);
        w0.hi = sload64(p.d_tile_prefix + w0.b + 1);
    }
    // ---- prefetch cursor: the next (tile, group) to load; pf_done once every group is in flight
    Walker wf = w0;
    uint64_t tf = t0;
    uint32_t gf = 0;
    uint64_t fvb = 0;  // the cursor tile's vbase, pad and group count
    uint32_t fpad = 0, fng = 0;
    bool any = false;
    for (; tf < t1; ++tf) {
        const Tile d = make_tile<LIST>(p, tf, wf);
        if (d.ngroups) {
            fvb = d.vbase, fpad = d.pad, fng = d.ngroups;
            gf = first_group(d.pad);
            any = true;
            break;
        }
    }
    bool pf_done = !any;
    auto pf_advance = [&]() {
        if (gf + 1 < fng) {
            ++gf;
            return;
        }
        if (pf_done) return;
        Walker w2 = wf;
        for (uint64_t t = tf + 1; t < t1; ++t) {
            const Tile d = make_tile<LIST>(p, t, w2);
            if (d.ngroups) {
                fvb = d.vbase, fpad = d.pad, fng = d.ngroups;
                wf = w2;
                tf = t;
                gf = first_group(d.pad);
                return;
            }
        }
        if (pool_size) {
            uint32_t v = 0;
            if (lane == 0) v = __hip_atomic_fetch_add((uint32_t *)(lds + kPoolOff), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            v = __builtin_amdgcn_readfirstlane(v);
            if (v < pool_size) {
                const uint64_t t = pool_base + v;
                const Tile d = make_tile<LIST>(p, t, w2);
                fvb = d.vbase, fpad = d.pad, fng = d.ngroups;
                tf = t;
                gf = first_group(d.pad);
                if (fifo_n == 0) fifo0 = t; else fifo1 = t;
                ++fifo_n;
                return;
            }
        }
        pf_done = true;
    };
    // K-image word and P column of this thread: needed only when a tile finishes, so they are
    // published to LDS after the first group is scanned (see publish_consts), not before the scan
    const v4u kq = *(gv4u *)((const uint32_t *)p.d_kvals + (W8 ? kBraidK64Word : 0) + 4 * threadIdx.x);  // 16 B of the 8 KiB image
    const uint64_t *pcs = p.d_pcols ? p.d_pcols : p.d_kvals;
    const uint32_t pce0 = *(gu32 *)(pcs + threadIdx.x), pce1 = *(gu32 *)(pcs + threadIdx.x + kBraidBlock);
    // prime the first group unconditionally (a wave without payload reads the 13 KiB constant block).
    // Only one group is primed, before the table build: issuing a load stalls the wave while the
    // memory system is saturated (every CU primes at once), so priming two groups kept the first scan
    // waiting for 8 KiB per wave to be accepted.  The ring scans group 0 while group 1's loads go out
    // between its table steps.
    Grp r0, r1;
    braid_load<NT>(r0, any ? fvb : (uint64_t)p.d_kvals, any ? fpad : 0u, any ? gf : 0u, lane);
    if (any && !dyn) pf_advance();  // pool mode: after the barrier, where the pool counter is set up
    if constexpr (W8) {
        // the eight slice-by-8 tables, 8 copies (as crc32_stream_kernel<POLY, true>)
        static_assert(kBraidBlock == 512, "build_w8_tables: 512 threads");
        build_w8_tables<POLY>(lds, threadIdx.x);
        if (threadIdx.x < 256) *(uint32_t *)(lds + kT0Off + 4 * threadIdx.x) = basis_w8<POLY, 8>(threadIdx.x);
        if (threadIdx.x == 0) *(uint32_t *)(lds + kConstFlagOff) = 0u;
        if (threadIdx.x == 0) *(uint32_t *)(lds + kPoolOff) = 0u;
    } else {
        // T' (4 tables x 256 entries, 8 copies each) and T0 from the compile-time bases.  One 16-byte
        // store = 4 copies of one (table, entry); the 8 lanes of a ds_write_b128 group take the 8
        // (quarter, half) slots of a row, so each group fills 128 distinct bytes (no bank conflict).
        const uint32_t i = threadIdx.x;
        const uint32_t q = (i >> 1) & 3u, h = i & 1u;
        uint32_t bq[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) bq[b] = basis_bit<POLY>(3 - q, b);  // quarter q holds T'_(3-q)
#pragma unroll
        for (int pass = 0; pass < 4; ++pass) {
            const uint32_t e = (i >> 3) + 64u * pass;
            uint32_t te = 0;
#pragma unroll
            for (int b = 0; b < 8; ++b) te ^= ((e >> b) & 1u) ? bq[b] : 0u;
            *(uint4 *)(lds + (e << 8) + (q << 5) + (h << 4)) = make_uint4(te, te, te, te);
        }
        if (i < 256) *(uint32_t *)(lds + kT0Off + 4 * i) = basis_entry<POLY, 4>(i);
        if (i == 0) *(uint32_t *)(lds + kConstFlagOff) = 0u;
        if (i == 0) *(uint32_t *)(lds + kPoolOff) = 0u;
    }
    // LDS-only barrier: __syncthreads()'s fence would also wait vmcnt(0) for the prefetched group
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    B eng;
    eng.init(lds, lane);
    // pool mode: the prefetch cursor may reach the pool only now (the host gives every wave of a
    // pooled launch a static tile with payload, so a wave's pool tiles always follow it)
    if (dyn && any) pf_advance();
    // Every wave publishes its 1/8 of the K image and P columns once its constants have arrived
    // (after its first group, by which time they have: loads retire in order) and counts itself in
    // LDS; a wave spins on the count only before its first tile finish.  A wave without work
    // publishes before leaving, so the count always completes.
    bool consts_ready = false, published = false;
    auto publish_consts = [&]() {
        if (published) return;
        published = true;
        *(v4u *)(lds + kBKOff + 16 * threadIdx.x) = kq;
        *(uint32_t *)(lds + kPcolOff + 4 * threadIdx.x) = pce0;
        *(uint32_t *)(lds + kPcolOff + 4 * (threadIdx.x + kBraidBlock)) = pce1;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_add((uint32_t *)(lds + kConstFlagOff), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto await_consts = [&]() {
        if (consts_ready) return;
        while (__hip_atomic_load((uint32_t *)(lds + kConstFlagOff), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <
               (uint32_t)kBraidWaves)
            __builtin_amdgcn_s_sleep(1);
        consts_ready = true;
    };
    if (t0 >= t1) {
        publish_consts();
        return;
    }

    // ---- scan cursor
    Walker wp = w0;
    uint64_t tp = t0;
    uint32_t gp = 0;
    Tile dp = make_tile<LIST>(p, tp, wp);
    gp = first_group(dp.pad);
    uint32_t s_h = dp.k == 0 ? head_state<LIST>(p, dp.b, eng) : 0u;
    uint32_t u = (dp.k == 0 && dp.pad == 0 && lane == 0) ? s_h : 0u;
    BPending pd{};
    pd.valid = false;
    BGroupAcc acc{};
    acc.slot = ~0ull;

    // the scan cursor's next tile: the static range, then the pool tiles the prefetch cursor entered
    bool scan_pool = false;
    auto next_scan = [&]() -> bool {
        if (!scan_pool) {
            if (++tp < t1) {
                dp = make_tile<LIST>(p, tp, wp);
                return true;
            }
            scan_pool = true;
        }
        if (fifo_n == 0) return false;
        tp = fifo0;
        fifo0 = fifo1;
        --fifo_n;
        dp = make_tile<LIST>(p, tp, wp);
        return true;
    };
    auto settle = [&]() -> bool {
        while (gp >= dp.ngroups) {
            await_consts();
            braid_finish<LIST>(p, dp, u, s_h, eng, lane, acc, pd);
            if (!next_scan()) return false;
            gp = first_group(dp.pad);
            s_h = dp.k == 0 ? head_state<LIST>(p, dp.b, eng) : 0u;
            u = (dp.k == 0 && dp.pad == 0 && lane == 0) ? s_h : 0u;
        }
        return true;
    };

    // one ring step: scan `cur` (group gp of tile dp) and load `dst` with the prefetch cursor's group
    // (once the prefetch cursor is parked on the wave's last group that group is already in flight:
    // a second load of it would be pure extra traffic -- non-temporal loads do not leave it in L2)
    auto ring_step = [&](const Grp &cur, Grp &dst) {
        if (pf_done) {
            u = braid_proc(u, cur, eng, dp, gp, lane, s_h);
        } else if (group_clean(dp.pad, gp) && group_clean(fpad, gf)) {
            u = braid_fused<1, NT>(u, cur, dst, fvb + gf * (kBraidRow * kBraidRowsPerGroup) + (W8 ? 8u : 4u) * lane, eng);
        } else {
            braid_load<NT>(dst, fvb, fpad, gf, lane);
            u = braid_proc(u, cur, eng, dp, gp, lane, s_h);
        }
        ++gp;
        pf_advance();
    };
    if (any) {
        // two-slot ring: group g+1's loads stream out while group g is scanned
        // leading tiles without payload finish before the primed group is reached: publish first then
        if (dp.ngroups == 0) publish_consts();
        if (settle()) {
            ring_step(r0, r1);
            publish_consts();
            for (;;) {
                if (!settle()) break;
                ring_step(r1, r0);
                if (!settle()) break;
                ring_step(r0, r1);
            }
        }
    } else {
        publish_consts();
        settle();
    }
    publish_consts();
    braid_publish<LIST>(p, acc, pd, eng, lane);
    braid_resolve<LIST>(p, pd, eng, lane);
}

// ------------------------------------------------------------------------------------------
// W = 32 streaming scan for uniform batches whose main region is a whole number of tiles (no
// virtual front pad): 1024 x 64 KiB, 16 x 256 MiB, 131072 x 8 KiB.  The same braided rows, tables
// and tile combine as crc32_braid_kernel, restructured so the compiler's wait counts stay precise:
//
//  * A three-slot register ring on one code path: while group g is scanned, group g+1 is in flight
//    and group g+2 streams out between the table steps (8-12 KiB per wave in flight).  Past a wave's
//    last group the placeholder rows read the L2-resident constant block, so every step issues the
//    same 16 loads.  The generic kernel's merged paths left the compiler a full vmcnt(0) drain per
//    group, so a wave waited one whole HBM latency for every 4 KiB.
//  * Nothing else in the loop is a compiler-visible vector-memory operation: the combine atomics and
//    result stores are inline asm (rare, self-waiting) and the tables' basis constants immediates.
//    A returning atomic left pending across the loop made the compiler's loop-header merge drain
//    the ring.
//  * The row loads themselves stay compiler-visible.  Inline-asm loads with hand-counted waits were
//    tried: the compiler may move or reuse the destination register of an in-flight asm load, and
//    the returning data then overwrote live values (device faults).
template <int R>
__device__ __forceinline__ uint32_t gld_row(uint32_t voff, uint64_t sbase) {
    return __builtin_nontemporal_load((gu32 *)(sbase + voff + R * kBraidRow));
}

template <int R, class B>
__device__ __forceinline__ uint32_t stream_rows(uint32_t x, BGroup &cur, BGroup &nxt, uint32_t voff, uint64_t snext, const B &eng) {
    if constexpr (R < kBraidRowsPerGroup) {
        nxt.w[R] = gld_row<R>(voff, snext);
        x = R == 0 ? x ^ cur.w[0] : eng.step_x(x, cur.w[R]);
        __builtin_amdgcn_sched_barrier(0);
        return stream_rows<R + 1, B>(x, cur, nxt, voff, snext, eng);
    } else {
        return eng.step(x);
    }
}

template <int R>
__device__ __forceinline__ uint64_t gld_w8(uint32_t voff, uint64_t sbase) {
    return __builtin_nontemporal_load((gu64 *)(sbase + voff + R * kW8Row));
}

// 8-byte rows: x = u ^ lo(w_r) is the chained value; the hi lookups of row r are issued with row
// r - 1's chain step and XORed in at row r (h = row r - 1's hi part).  One row ahead measured 0.4-1 %
// shorter launches than all eight lookups per step (profiles/r02/w8_ab/split.jsonl).
template <int R, class B>
__device__ __forceinline__ uint32_t stream_rows_w8(uint32_t x, typename B::Hi h, W8Group &cur, W8Group &nxt, uint32_t voff,
                                                   uint64_t snext, const B &eng) {
    if constexpr (R < kW8RowsPerGroup) {
        nxt.w[R] = gld_w8<R>(voff, snext);
        typename B::Hi hn;
        if constexpr (R == 0) {
            x ^= (uint32_t)cur.w[0];
            hn = eng.look_hi((uint32_t)(cur.w[0] >> 32));
        } else {
            x = eng.look_lo(x, h, (uint32_t)cur.w[R]);
            hn = eng.look_hi((uint32_t)(cur.w[R] >> 32));
        }
        __builtin_amdgcn_sched_barrier(0);
        return stream_rows_w8<R + 1, B>(x, hn, cur, nxt, voff, snext, eng);
    } else {
        return eng.look_lo(x, h, 0u);
    }
}
template <int R, class B>
__device__ __forceinline__ uint32_t stream_rows(uint32_t x, W8Group &cur, W8Group &nxt, uint32_t voff, uint64_t snext, const B &eng) {
    static_assert(R == 0, "the 8-byte row walk starts at row 0");
    return stream_rows_w8<0, B>(x, typename B::Hi{}, cur, nxt, voff, snext, eng);
}

// 16-byte rows: the same walk as stream_rows_w8 (x = u ^ d0(w_r); d1..d3 of row r looked up with
// row r - 1's chain step)
template <int R>
__device__ __forceinline__ v4u gld_w16(uint32_t voff, uint64_t sbase) {
    return __builtin_nontemporal_load((gv4u *)(sbase + voff + R * kW16Row));
}
template <int R, class B>
__device__ __forceinline__ uint32_t stream_rows_w16(uint32_t x, const typename B::Hi &h, W16Group &cur, W16Group &nxt,
                                                    uint32_t voff, uint64_t snext, const B &eng) {
    if constexpr (R < kW16RowsPerGroup) {
        // issue order: this row's load, the chain's four lookups, the row's twelve off-chain lookups;
        // only then the XORs (a scheduling barrier keeps the compiler from reducing the previous row's
        // twelve, and waiting for them, ahead of the chain's lookups)
        nxt.w[R] = gld_w16<R>(voff, snext);
        typename B::Lo lo{};
        if constexpr (R > 0) lo = eng.lo_issue(x);
        const typename B::Hi hn = eng.look_hi(cur.w[R]);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (R == 0)
            x ^= cur.w[0].x;
        else
            x = eng.lo_finish(lo, h, cur.w[R].x);
        __builtin_amdgcn_sched_barrier(0);
        return stream_rows_w16<R + 1, B>(x, hn, cur, nxt, voff, snext, eng);
    } else {
        return eng.look_lo(x, h, 0u);
    }
}
template <int R, class B>
__device__ __forceinline__ uint32_t stream_rows(uint32_t x, W16Group &cur, W16Group &nxt, uint32_t voff, uint64_t snext,
                                                const B &eng) {
    static_assert(R == 0, "the 16-byte row walk starts at row 0");
    return stream_rows_w16<0, B>(x, typename B::Hi{}, cur, nxt, voff, snext, eng);
}
template <int R>
__device__ __forceinline__ void stream_issue(W16Group &g, uint32_t voff, uint64_t s) {
    if constexpr (R < kW16RowsPerGroup) {
        g.w[R] = gld_w16<R>(voff, s);
        stream_issue<R + 1>(g, voff, s);
    }
}
#define AMDCRC_R4V(g) "+v"(g.w[0]), "+v"(g.w[1]), "+v"(g.w[2]), "+v"(g.w[3])
[[maybe_unused]] __device__ __forceinline__ void ring_drain(W16Group &a, W16Group &b, W16Group &c) {
    asm volatile("s_waitcnt vmcnt(0)" : AMDCRC_R4V(a)::"memory");
    asm volatile("" : AMDCRC_R4V(b));
    asm volatile("" : AMDCRC_R4V(c));
}

template <int R>
__device__ __forceinline__ void stream_issue(W8Group &g, uint32_t voff, uint64_t s) {
    if constexpr (R < kW8RowsPerGroup) {
        g.w[R] = gld_w8<R>(voff, s);
        stream_issue<R + 1>(g, voff, s);
    }
}

#define AMDCRC_R8W(g) "+v"(g.w[0]), "+v"(g.w[1]), "+v"(g.w[2]), "+v"(g.w[3]), "+v"(g.w[4]), "+v"(g.w[5]), "+v"(g.w[6]), \
    "+v"(g.w[7])
__device__ __forceinline__ void ring_drain(W8Group &a, W8Group &b, W8Group &c) {
    asm volatile("s_waitcnt vmcnt(0)" : AMDCRC_R8W(a)::"memory");
    asm volatile("" : AMDCRC_R8W(b));
    asm volatile("" : AMDCRC_R8W(c));
}

// Keep a ring slot's registers live up to this point.  A row load whose value is never read (the
// placeholder rows past a wave's last group) would otherwise leave its destination registers "free"
// to the compiler while the load is still in flight, and the returning data would overwrite whatever
// the compiler placed there (tile-finish temporaries, addresses).  Used after the final vmcnt(0).
#define AMDCRC_R16(g) "+v"(g.w[0]), "+v"(g.w[1]), "+v"(g.w[2]), "+v"(g.w[3]), "+v"(g.w[4]), "+v"(g.w[5]), "+v"(g.w[6]), \
    "+v"(g.w[7]), "+v"(g.w[8]), "+v"(g.w[9]), "+v"(g.w[10]), "+v"(g.w[11]), "+v"(g.w[12]), "+v"(g.w[13]),          \
    "+v"(g.w[14]), "+v"(g.w[15])
[[maybe_unused]] __device__ __forceinline__ void ring_drain(BGroup &a, BGroup &b, BGroup &c) {
    asm volatile("s_waitcnt vmcnt(0)" : AMDCRC_R16(a)::"memory");
    asm volatile("" : AMDCRC_R16(b));
    asm volatile("" : AMDCRC_R16(c));
}

template <int R>
__device__ __forceinline__ void stream_issue(BGroup &g, uint32_t voff, uint64_t s) {
    if constexpr (R < kBraidRowsPerGroup) {
        g.w[R] = gld_row<R>(voff, s);
        stream_issue<R + 1>(g, voff, s);
    }
}

#ifdef AMDCRC_GUARD
// Debug builds only (-DAMDCRC_GUARD): every global address the streaming scan forms is range-checked;
// a bad one is recorded here and replaced, so a cursor bug reports instead of faulting the device.
__device__ unsigned long long g_amdcrc_guard[4];
__device__ __forceinline__ bool guard_ok(bool ok, int what, unsigned long long v) {
    if (!ok) {
        __hip_atomic_fetch_or(&g_amdcrc_guard[0], 1ull << what, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        g_amdcrc_guard[1 + (what & 1)] = v;
    }
    return ok;
}
#define AMDCRC_GUARD_OK(c, w, v) guard_ok((c), (w), (unsigned long long)(v))
#else
#define AMDCRC_GUARD_OK(c, w, v) true
#endif

// Cross-tile combine for the streaming scan: the same group slots as braid_finish / braid_publish /
// braid_resolve, with every global atomic in inline asm that waits for its own completion.  These
// run once per 32-tile group at most; a compiler-visible returning atomic would instead leave its
// destination registers "pending" across the scan loop and the compiler would guard later writes of
// them with a full vmcnt(0) drain of the payload ring on every scan step.
__device__ __forceinline__ unsigned long long sx_xor64_ret(unsigned long long *a, unsigned long long v) {
    unsigned long long r;
    asm volatile("global_atomic_xor_x2 %0, %1, %2, off sc0\n\ts_waitcnt vmcnt(0)" : "=&v"(r) : "v"(a), "v"(v) : "memory");
    return r;
}
__device__ __forceinline__ unsigned long long sx_swap64_ret(unsigned long long *a, unsigned long long v) {
    unsigned long long r;
    asm volatile("global_atomic_swap_x2 %0, %1, %2, off sc0\n\ts_waitcnt vmcnt(0)" : "=&v"(r) : "v"(a), "v"(v) : "memory");
    return r;
}
__device__ __forceinline__ unsigned int sx_add32_ret(unsigned int *a, unsigned int v) {
    unsigned int r;
    asm volatile("global_atomic_add %0, %1, %2, off sc0\n\ts_waitcnt vmcnt(0)" : "=&v"(r) : "v"(a), "v"(v) : "memory");
    return r;
}
__device__ __forceinline__ void sx_store32(unsigned int *a, unsigned int v) {  // agent-scope atomic store
    asm volatile("global_store_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : : "v"(a), "v"(v) : "memory");
}

// publish the wave's merged tiles of one group and, if they complete it, finish the group at once
template <class B, bool LIST = false>
__device__ __forceinline__ void stream_publish(const ScanParams &p, BGroupAcc &g, const B &eng, int lane) {
    if (g.slot == ~0ull) return;
    if (!AMDCRC_GUARD_OK(g.slot < p.ntiles && g.b < p.nbuf, 4, g.slot)) return;
    unsigned long long old = 0;
    if (lane == 0) old = sx_xor64_ret(&p.d_acc1[g.slot], g.val);
    const unsigned long long now = rfl64(old) ^ g.val;
    const uint64_t slot = g.slot;
    g.slot = ~0ull;
    const uint64_t n = g.T - g.g0 < 32 ? g.T - g.g0 : 32, G = (g.T + 31) / 32, shift = g.T - g.g0 - n;
    const unsigned long long full = n >= 32 ? 0xFFFFFFFF00000000ull : (((1ull << n) - 1) << 32);
    if ((now & 0xFFFFFFFF00000000ull) != full) return;
    uint32_t grp = (uint32_t)now;
    if (G > 1 && shift) grp = mul_pcols<uint32_t, 32>(grp, p.d_pcols + shift * 32);
    if (lane != 0) return;
    (void)sx_swap64_ret(&p.d_acc1[slot], 0ull);
    if (G == 1) {
        finalize<LIST>(p, g.b, grp, eng);
        return;
    }
    (void)sx_xor64_ret(&p.d_acc[g.b], (unsigned long long)grp);  // performed before it is counted
    const unsigned int c = sx_add32_ret(&p.d_cnt[g.b], 1u);
    if (c == G - 1) {
        const uint32_t fin = (uint32_t)sx_swap64_ret(&p.d_acc[g.b], 0ull);
        sx_store32(&p.d_cnt[g.b], 0u);
        finalize<LIST>(p, g.b, fin, eng);
    }
}

// Buffers [b0, b1) lie wholly inside this workgroup's tiles (T <= 32): combined in LDS slots
struct LocalBufs {
    uint64_t b0, b1;
};

template <class B, bool LIST = false>
__device__ __forceinline__ void stream_finish(const ScanParams &p, const Tile &d, uint32_t u, const B &eng, int lane, BGroupAcc &acc,
                                              const LocalBufs &lb) {
    const uint32_t r = wave_xor_s(eng.mulK(u, lane));
    if (!AMDCRC_GUARD_OK(d.b < p.nbuf && d.k < d.T, 2, d.b)) return;
    if (d.T == 1) {
        if (lane == 0) finalize<LIST>(p, d.b, r, eng);
        return;
    }
    const uint64_t g0 = d.k & ~31ull, gend = d.T - g0 < 32 ? d.T : g0 + 32;
    const uint32_t m = (uint32_t)(gend - 1 - d.k);
    const uint32_t colv = lds32(eng.cbase(), (kPcolOff - kBKOff) + 4 * (m * 32 + (lane & 31)));
    const uint32_t sel = lane < 32 ? (uint32_t)__builtin_amdgcn_sbfe((int)r, 31 - lane, 1) : 0u;
    const uint32_t v = wave_xor_s(colv & sel);
    if (d.b >= lb.b0 && d.b < lb.b1) {  // T <= 32 here: the group end is the buffer end
        if (lane == 0) {
            const unsigned long long add = (unsigned long long)v | (1ull << (32 + d.k));
            unsigned long long *slot = (unsigned long long *)(eng.cbase() + (kLocalOff - kBKOff)) + (d.b - lb.b0);
            const unsigned long long now =
                __hip_atomic_fetch_xor(slot, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) ^ add;
            const unsigned long long full = d.T >= 32 ? 0xFFFFFFFF00000000ull : (((1ull << d.T) - 1) << 32);
            if ((now & 0xFFFFFFFF00000000ull) == full) finalize<LIST>(p, d.b, (uint32_t)now, eng);
        }
        return;
    }
    const uint64_t slot = d.tbase + g0;
    if (slot != acc.slot) {
        stream_publish<B, LIST>(p, acc, eng, lane);
        acc.slot = slot;
        acc.val = 0;
        acc.b = d.b;
        acc.T = d.T;
        acc.g0 = (uint32_t)g0;
    }
    acc.val ^= (unsigned long long)v | (1ull << (32 + (d.k & 31)));
}

// XCD-window order (ScanParams::xcd_order): tile d of a buffer of T <= WAVES tiles, all scanned at the
// same step by consecutive waves of this workgroup; its share moved to the buffer end joins LDS slot
// `slot` (value XOR, one arrival bit per tile), and the tile completing the slot finishes the buffer.
template <class B>
__device__ __forceinline__ void stream_finish_xcd(const ScanParams &p, const Tile &d, uint32_t u, const B &eng, int lane,
                                                  uint32_t slot) {
    uint32_t r = wave_xor_s(eng.mulK(u, lane));
    if (d.T == 1) {
        if (lane == 0) finalize<false>(p, d.b, r, eng);
        return;
    }
    const uint32_t m = (uint32_t)(d.T - 1 - d.k);
    if (m) {
        const uint32_t colv = lds32(eng.cbase(), (kPcolOff - kBKOff) + 4 * (m * 32 + (lane & 31)));
        const uint32_t sel = lane < 32 ? (uint32_t)__builtin_amdgcn_sbfe((int)r, 31 - lane, 1) : 0u;
        r = wave_xor_s(colv & sel);
    }
    if (lane == 0) {
        const unsigned long long add = (unsigned long long)r | (1ull << (32 + d.k));
        unsigned long long *sl = (unsigned long long *)(eng.cbase() + (kLocalOff - kBKOff)) + slot;
        const unsigned long long now = __hip_atomic_fetch_xor(sl, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) ^ add;
        if ((now & 0xFFFFFFFF00000000ull) == (((1ull << d.T) - 1) << 32)) finalize<false>(p, d.b, (uint32_t)now, eng);
    }
}

#if AWS_CRT_AMD_DIAG
// Diagnostic library only: per-wave timeline of crc32_stream_kernel (aws_crt_amd_debug_scan_stamps),
// kStampWords words per wave at (blockIdx * waves + wave): entry, tables built (after the barrier),
// first group scanned, loop end, exit (s_memrealtime, 100 MHz), hardware id (HW_ID | XCC_ID << 32),
// groups scanned, tile finishes.  Null: no stamps.  Stamps are taken outside the scan loop only.
__device__ uint64_t *g_scan_stamps;
constexpr int kStampWords = 16;  // [8..11]: kernel arguments in, first group issued, second group issued, tables stored
__device__ __forceinline__ uint64_t stamp_now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ uint64_t stamp_hwid() {
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    return (uint64_t)hw | ((uint64_t)(xcc & 0xF) << 32);
}
#endif

// Tiles: an even static split over the waves (a workgroup-local pool was tried: see DESIGN.md).
// WB = bytes per lane word: 8 (512-thread workgroups, 64 KiB of tables, two per CU) or 16 (one
// 1024-thread workgroup per CU, 128 KiB of tables); 4 remains as the AMDCRC_STREAM_W8=0 build.
template <int WB>
struct StreamShape {
    static constexpr int kBlock = WB == 16 ? kW16Block : kBraidBlock;
    static constexpr int kWaves = kBlock / kWave;
    static constexpr uint32_t kTab = WB == 16 ? kW16TabBytes : kBTabBytes;  // the constants region follows
    static constexpr uint32_t kLds = kTab + (kStreamLds - kBKOff);
    static constexpr int kKWord = WB == 16 ? kBraidK128Word : WB == 8 ? kBraidK64Word : 0;
};

template <uint32_t POLY, int WB, bool XO = false>
__global__ __launch_bounds__(StreamShape<WB>::kBlock, 4) void crc32_stream_kernel(const ScanParams p) {
    using SS = StreamShape<WB>;
    using B = typename std::conditional<WB == 16, Braid32W16<POLY>,
                                        typename std::conditional<WB == 8, Braid32W8<POLY>, Braid32<POLY>>::type>::type;
    using Grp = typename std::conditional<WB == 16, W16Group, typename std::conditional<WB == 8, W8Group, BGroup>::type>::type;
    constexpr int WAVES = SS::kWaves;
    __shared__ __attribute__((aligned(16))) char lds[SS::kLds];
    char *const cb = lds + SS::kTab;  // constants region (K image, P columns, byte table, flag, local slots)
#if AWS_CRT_AMD_DIAG
    uint64_t *const stamps = g_scan_stamps;
    const uint64_t t_entry = stamp_now();
    uint64_t t_tab = 0, t_first = 0, t_loop = 0, t_karg = 0, t_ra = 0, t_rb = 0, t_built = 0;
#endif

    const int lane = threadIdx.x & 63;
    // Prologue (round 5): the kernel arguments that the first group's address needs come in as one
    // batch of scalar loads with one wait.  The compiler had spread them over five dependent round
    // trips between branches, and the per-wave stamps put ~4 us between a wave's entry and its
    // barrier in a 16 us one-batch launch (tools/stamp_probe.py).  The wave's first two groups are
    // then issued before the tables are built, so HBM streams through the table build.
    const uint64_t a_ntiles = p.ntiles, a_T = p.tiles_per_buf, a_base = p.base, a_stride = p.stride, a_len = p.len,
                   a_bcount = p.bcount, a_kv = (uint64_t)p.d_kvals, a_pc = (uint64_t)p.d_pcols, a_bb0 = p.bbase[0];
    const uint32_t a_seg = p.seg, a_nbatch = p.nbatch, a_grid = gridDim.x, a_r = p.split_r;
    const uint64_t a_q = p.split_q;
    const uint32_t a_sh = p.shifts1;
    asm volatile("" ::"s"(a_ntiles), "s"(a_T), "s"(a_base), "s"(a_stride), "s"(a_len), "s"(a_bcount), "s"(a_kv), "s"(a_pc),
                 "s"(a_bb0), "s"(a_seg), "s"(a_nbatch), "s"(a_grid), "s"(a_r), "s"(a_q), "s"(a_sh));
    const uint32_t a_tsh1 = a_sh & 0xFFu, a_bsh1 = a_sh >> 8;
#if AWS_CRT_AMD_DIAG
    t_karg = stamp_now();
#endif
    const uint64_t wv = (uint64_t)(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)a_grid * WAVES;
    const uint64_t gw = rfl64((uint64_t)blockIdx.x * WAVES + wv);
    // the static split (ScanParams::split_q): wave w's first tile, no division
    auto split_at = [&](uint64_t w) -> uint64_t { return w * a_q + (w < a_r ? w : (uint64_t)a_r); };
    // geometry: G groups of 4 KiB per tile, T tiles per buffer, main region at hoff of every buffer
    const uint32_t G = a_seg / kGroupBytes;
    const uint64_t T = a_T, tile_bytes = (uint64_t)a_seg * kWave;
    const uint64_t hoff = edges_of(a_bb0, a_len).headend - a_base;  // buffer 0 of batch 0
    const uint32_t voff = (uint32_t)WB * (uint32_t)lane;
    const uint64_t dummy = rfl64(a_kv);
    // the wave's tiles: t0, t0 + tstep, ... (ntw of them).  XCD windows (p.xcd_order): the waves of XCD
    // x = blockIdx mod 8 take tiles j, j + nwx, ... of the x-th eighth, so at every step an XCD's waves
    // read one compact window (DESIGN.md "Read order"); a buffer's T tiles go to T consecutive waves of
    // one workgroup at the same step, combined in the workgroup's LDS slots (slot = step * WAVES / T +
    // wave / T).  Otherwise each wave takes a contiguous range.
    constexpr bool xo = WB == 8 && XO;  // a separate instantiation: the contiguous split's loop is unchanged
    uint64_t t0, tstep = 1, ntw;
    if constexpr (xo) {
        const uint64_t nwx = nw / 8, xcd = blockIdx.x & 7u, xlo = xcd * a_ntiles / 8, xhi = (xcd + 1) * a_ntiles / 8;
        t0 = rfl64(xlo + (uint64_t)(blockIdx.x >> 3) * WAVES + wv);
        tstep = nwx;
        ntw = rfl64(t0 < xhi ? udiv_u(xhi - t0 + nwx - 1, nwx) : 0);
    } else {
        t0 = rfl64(split_at(gw));
        ntw = rfl64(a_q + (gw < a_r ? 1u : 0u));
    }
    const uint32_t gsh = __builtin_ctz(G);
    const uint32_t nq = (uint32_t)(ntw << gsh);  // groups of this wave
    const bool work = ntw > 0;
    // prefetch cursor: the next group to issue, as (buffer, tile, group); fbuf is the main-region
    // address of buffer fb, which walks batch by batch (fj, fi)
    uint32_t fq = 0;  // groups issued
    uint64_t fb = a_tsh1 ? t0 >> (a_tsh1 - 1) : udiv_u(t0, T), fk = t0 - fb * T;
    const uint64_t b_first = fb, k_first = fk;  // the scan cursor starts here too
    uint32_t fg = 0;
    BatchPos fpos{0, fb};
    if (a_nbatch > 1) {
        fpos.j = a_bsh1 ? fb >> (a_bsh1 - 1) : udiv_u(fb, a_bcount);
        fpos.i = fb - fpos.j * a_bcount;
    }
    // (a wave starting in batch 0 needs no second round trip for its base)
    uint64_t fbuf = work ? (fpos.j == 0 ? a_bb0 : karg64(p.bbase, fpos.j)) + fpos.i * a_stride + hoff : 0;
    uint64_t ft = t0;  // XCD windows: the tile being issued
    auto f_addr = [&]() -> uint64_t {
        uint64_t a = fq < nq ? fbuf + fk * tile_bytes + (uint64_t)fg * (kBraidRow * kBraidRowsPerGroup) : dummy;
        if (!AMDCRC_GUARD_OK(fq >= nq || p.nbatch > 1 || (a >= p.base + hoff && a + kBraidRow * kBraidRowsPerGroup <=
                                                                 p.base + (p.nbuf - 1) * p.stride + hoff + T * tile_bytes),
                             1, a))
            a = dummy;
        return rfl64(a);
    };
    auto f_next = [&]() {
        ++fq;
        if (++fg == G) {
            fg = 0;
            if constexpr (xo) {  // the wave's next tile is tstep tiles on
                ft += tstep;
                if (fq < nq) {
                    fb = udiv_u(ft, T), fk = ft - fb * T;
                    fpos = batch_pos(p, fb);
                    fbuf = karg64(p.bbase, fpos.j) + fpos.i * p.stride + hoff;
                }
            } else if (++fk == T) {
                fk = 0, ++fb;
                if (++fpos.i == p.bcount && fq < nq) {
                    fpos.i = 0, ++fpos.j;
                    fbuf = karg64(p.bbase, fpos.j) + hoff;
                } else {
                    fbuf += p.stride;
                }
            }
        }
    };
    Grp ra, rb, rc;
    if (work) {
        stream_issue<0>(ra, voff, f_addr());
        f_next();
    }
#if AWS_CRT_AMD_DIAG
    t_ra = stamp_now();
#endif
    // K-image words and P columns of this thread, published to LDS after the first scan step (ordinary
    // loads between the first and the second group, so the compiler's wait for them in the peeled first
    // step is the exact count of the row loads issued after them).  The K image is 8 KiB (512 x 16 B)
    // and the P columns 4 KiB (1024 words) whatever the workgroup size.
    const uint64_t *pcs = (const uint64_t *)(a_pc ? a_pc : a_kv);
    const uint32_t kti = (uint32_t)threadIdx.x & 511u;
    const v4u kq = *(gv4u *)((const uint32_t *)a_kv + SS::kKWord + 4 * kti);
    const uint32_t pce0 = *(gu32 *)(pcs + threadIdx.x);
    const uint32_t pce1 = SS::kBlock < 1024 ? *(gu32 *)(pcs + threadIdx.x + SS::kBlock) : 0u;
    if (work) {
        stream_issue<0>(rb, voff, f_addr());
        f_next();
    }
#if AWS_CRT_AMD_DIAG
    t_rb = stamp_now();
#endif
    // buffers wholly inside this workgroup's tile range (T <= 32, slots permitting): LDS combine
    LocalBufs lb{0, 0};
    if (!xo && T > 1 && T <= 32) {
        const uint64_t wt0 = split_at((uint64_t)blockIdx.x * WAVES), wt1 = split_at(((uint64_t)blockIdx.x + 1) * WAVES);
        const uint64_t b0 = udiv_u(wt0 + T - 1, T), b1 = udiv_u(wt1, T);
        if (b1 > b0 && b1 - b0 <= kLocalSlots) lb = LocalBufs{b0, b1};
    }
    if constexpr (WB == 16) {
        // wave t builds table T'_t (t wave-uniform): entries lane + 64 n, 8 copies (two 16-byte stores)
        const uint32_t t = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        char *region = lds + (t < 8 ? 65536u : 0u) + ((t & 7u) << 5);
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const uint32_t e = (uint32_t)lane + 64u * n;
            const uint32_t te = basis_w16_rt<POLY>(t, e);
            char *row = region + (e << 8);
            *(uint4 *)row = make_uint4(te, te, te, te);
            *(uint4 *)(row + 16) = make_uint4(te, te, te, te);
        }
        if (threadIdx.x < 256) *(uint32_t *)(cb + (kT0Off - kBKOff) + 4 * threadIdx.x) = basis_w16<POLY, 16>(threadIdx.x);
    } else if constexpr (WB == 8) {
        static_assert(SS::kBlock == 512, "build_w8_tables: 512 threads");
        const uint32_t tid = threadIdx.x;
        build_w8_tables<POLY>(lds, tid);
        if (tid < 256) *(uint32_t *)(cb + (kT0Off - kBKOff) + 4 * tid) = basis_w8<POLY, 8>(tid);
    } else {
        const uint32_t i = threadIdx.x;
        const uint32_t q = (i >> 1) & 3u, h = i & 1u;
        uint32_t bq[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) bq[b] = basis_bit<POLY>(3 - q, b);
#pragma unroll
        for (int pass = 0; pass < 4; ++pass) {
            const uint32_t e = (i >> 3) + 64u * pass;
            uint32_t te = 0;
#pragma unroll
            for (int b = 0; b < 8; ++b) te ^= ((e >> b) & 1u) ? bq[b] : 0u;
            *(uint4 *)(lds + (e << 8) + (q << 5) + (h << 4)) = make_uint4(te, te, te, te);
        }
        if (i < 256) *(uint32_t *)(cb + (kT0Off - kBKOff) + 4 * i) = basis_entry<POLY, 4>(i);
    }
    if (threadIdx.x == 0) *(uint32_t *)(cb + (kConstFlagOff - kBKOff)) = 0u;
    if (threadIdx.x < kLocalSlots) ((unsigned long long *)(cb + (kLocalOff - kBKOff)))[threadIdx.x] = 0ull;
#if AWS_CRT_AMD_DIAG
    t_built = stamp_now();
#endif
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#if AWS_CRT_AMD_DIAG
    t_tab = stamp_now();
#endif
    B eng;
    eng.init(lds, lane);
    bool consts_ready = false;
    // every wave publishes its share of the K image and P columns once and counts itself in LDS; a
    // wave spins on the count only before its first tile finish
    auto publish_consts = [&]() {
        if (threadIdx.x < 512) *(v4u *)(cb + 16 * threadIdx.x) = kq;
        *(uint32_t *)(cb + (kPcolOff - kBKOff) + 4 * threadIdx.x) = pce0;
        if (SS::kBlock < 1024) *(uint32_t *)(cb + (kPcolOff - kBKOff) + 4 * (threadIdx.x + SS::kBlock)) = pce1;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_add((uint32_t *)(cb + (kConstFlagOff - kBKOff)), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto await_consts = [&]() {
        if (consts_ready) return;
        while (__hip_atomic_load((uint32_t *)(cb + (kConstFlagOff - kBKOff)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <
               (uint32_t)WAVES)
            __builtin_amdgcn_s_sleep(1);
        consts_ready = true;
    };
#if AWS_CRT_AMD_DIAG
    auto put_stamps = [&](uint64_t groups) {
        if (stamps && lane == 0) {
            uint64_t *w = stamps + kStampWords * ((uint64_t)blockIdx.x * WAVES + wv);
            w[0] = t_entry, w[1] = t_tab, w[2] = t_first, w[3] = t_loop, w[4] = stamp_now(), w[5] = stamp_hwid();
            w[6] = groups, w[7] = groups >> gsh;
            w[8] = t_karg, w[9] = t_ra, w[10] = t_rb, w[11] = t_built;
        }
    };
#endif
    if (!work) {
        publish_consts();
#if AWS_CRT_AMD_DIAG
        put_stamps(0);
#endif
        return;
    }

    // scan cursor: tile d (buffer, index in buffer), group g, global group q
    Tile d;
    d.T = T;
    d.b = b_first;
    d.k = k_first;
    d.tbase = d.b * T;
    d.vbase = 0;
    d.pad = 0;
    d.ngroups = G;
    uint32_t g = 0, u = 0;
    uint32_t q = 0;  // groups scanned
    uint64_t st_t = t0, st_n = 0;  // XCD windows: the tile being scanned, tiles finished
    BGroupAcc acc{};
    acc.slot = ~0ull;
    auto step = [&](Grp &cur, Grp &nxt, bool first) {
        if (g == 0) u = d.k == 0 && lane == 0 ? head_state<false>(p, d.b, eng) : 0u;
#if AMDCRC_STREAM_PRIO
        prio_by_work_left(q, nq);
#endif
        const uint64_t sn = f_addr();
        f_next();
        u = stream_rows<0, B>(u, cur, nxt, voff, sn, eng);
        if (first) publish_consts();
        ++q;
        if (++g == G) {
            g = 0;
            await_consts();
            if constexpr (xo) {
                stream_finish_xcd(p, d, u, eng, lane, (uint32_t)(st_n * (WAVES / T) + wv / T));
                ++st_n;
                st_t += tstep;
                d.b = udiv_u(st_t, T), d.k = st_t - d.b * T, d.tbase = d.b * T;
            } else {
                stream_finish(p, d, u, eng, lane, acc, lb);
                if (++d.k == T) d.k = 0, ++d.b, d.tbase += T;
            }
        }
    };
    // the first step is peeled (it publishes the constants, whose loads are then out of the loop),
    // so the loop header sees the same two ring slots in flight from the prologue and the back edge
    // The loop body runs whole rotations of three steps with no exit between them, and the last one
    // or two steps follow it.  With a break after each step (the round-2 loop) the compiler's wait-count
    // pass reached the loop header with a merged state in which the slot about to be loaded still had
    // loads in flight, and drained most of the ring at the top of every rotation (vmcnt 7..2 before the
    // first step's row loads); without the breaks every row waits exactly vmcnt(16).
    step(ra, rc, true);
#if AWS_CRT_AMD_DIAG
    t_first = stamp_now();
#endif
    while (q + 3 <= nq) {
        step(rb, ra, false);
        step(rc, rb, false);
        step(ra, rc, false);
    }
    if (q < nq) {
        step(rb, ra, false);
        if (q < nq) step(rc, rb, false);
    }
#if AWS_CRT_AMD_DIAG
    t_loop = stamp_now();
#endif
    ring_drain(ra, rb, rc);  // the trailing placeholder rows
    stream_publish(p, acc, eng, lane);
#if AWS_CRT_AMD_DIAG
    put_stamps(nq);
#endif
}

// ------------------------------------------------------------------------------------------
// Ragged lists on the streaming scan (crc32_list_stream_kernel, round 3).  crc32_braid_kernel<POLY,
// true> runs lists on a two-slot ring whose merged code paths (front-padded groups, tile walks) leave
// the compiler inexact wait counts.  This kernel is crc32_stream_kernel's one-path three-slot ring on
// 8-byte words, with no tiles at all:
//  * A buffer's main region is front-padded to whole 4 KiB groups (pad < 4096) and the list is one
//    sequence of groups.  Wave w scans groups [wq[w], wq[w+1]) of it -- an even split, cut anywhere,
//    so every wave scans the same bytes (+-1 group) whatever the buffer lengths.
//  * Group g of a buffer reads through a raw buffer resource based at its first real byte, with the
//    group's real bytes as records (4096, or 4096 - pad for group 0).  A lane's row offset is its
//    offset in the virtual group minus the pad (group 0), clamped to the record count: the pad's rows
//    come out negative (wrapped), clamp to the limit, and the range check returns zeros -- the virtual
//    zeros the braid needs, with no masking and no traffic.  Past the wave's last group the
//    placeholder rows go through a zero-record resource.
//  * The part of a buffer one wave scans ends with its share XOR_l u_l K_l (relative to the part's
//    end) moved to the buffer's end: times x^(8*4096*m) for the m groups after the part, one scalar
//    column product per set bit of m (columns of x^(8*4096*2^i) follow the braid constants).  A
//    buffer inside one wave finishes at once; otherwise every part XORs its share into the buffer's
//    accumulator and adds its group count, and the part that completes the count finishes it.
//  * The head state enters lane l0 = (pad mod 512) / 8 at the start of group 0 divided by X^j
//    (X = x^(8*512), the row step; j = the pad's row): the lane's words before the pad are zero, so
//    its j row steps bring it to exactly s_h where the first real word joins (X^(-j) columns).
//  * Buffers without a main region (under 16 aligned bytes) are folded whole by the wave whose range
//    holds their place in the sequence.
// Host side: engine.cpp list_stream (d_wave_buf = start buffer per wave, nw + 1; d_tile_prefix = start
// group within it, nw + 1; then the group prefix wq, nw + 1; ntiles = groups in the list).
// A part of a buffer cut between waves joins the buffer's other parts in this workgroup in an LDS
// slot (engine.cpp list_stream's join descriptor d: slot d & 15, d >> 4 & 15 parts expected):
// value XOR, then parts and groups counted in one add; the part completing the count gets the
// slot's value and group count (lane 0).  LDS atomics: no device round trip and no wait on the
// payload ring (round 4: returning device atomics for every cut part cost ragged lists ~6 us).
constexpr uint32_t kListJoinSlots = 9;
static_assert(kLocalOff + 16 * kListJoinSlots <= kStreamLds, "list join slots");
template <class T, class F>
__device__ __forceinline__ void list_join(uint64_t *slot, uint32_t d, T r, uint32_t groups, F &&done) {
    __hip_atomic_fetch_xor(slot, (uint64_t)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint64_t add = (1ull << 32) | groups;
    const uint64_t now = __hip_atomic_fetch_add(slot + 1, add, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP) + add;
    if ((uint32_t)(now >> 32) != ((d >> 4) & 15u)) return;
    done(__hip_atomic_load(slot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP), (uint32_t)now);
}

// The list streaming scans' buffers (round 5): a buffer of at least kListMainMin bytes is scanned as the
// 8-byte words [ptr & ~7, end & ~7) -- no serial head fold.  The o = ptr & 7 bytes in front of it in its
// first word are not the buffer's: the scan clears them in the registers (list_mask_edges) and the head
// state enters divided by x^(8 o), so it reaches ~seed exactly at ptr.  The tail (< 8 bytes) is folded.
// (Masking the last word too -- [ptr & ~7, (end + 7) & ~7), the register leaving times x^(-8 k) -- made
// unaligned 64 KiB buffers one 4 KiB group longer, 2 us per 256 MiB list slower; that path is gone,
// ADVICE r05.)  A shorter buffer has no main region and is folded whole (engine.cpp main_len_list).
constexpr uint64_t kListMainMin = 16;
struct LBuf {        // the cursor's buffer (wave-uniform)
    uint64_t b;      // buffer index
    uint64_t vb;     // virtual start of group 0 (main start - pad)
    uint32_t vg;     // groups (0: no main region)
    uint32_t pad;    // virtual zero bytes in front of main (< 4096)
    uint64_t ptr, n; // the buffer
    uint32_t o;      // bytes of the first main word in front of the buffer
    __device__ __forceinline__ Edges edges() const {  // the tail (< 8 bytes), or a whole short buffer, is folded
        return vg ? Edges{ptr, ptr, (ptr + n) & ~7ull, ptr + n} : Edges{ptr, ptr + n, ptr + n, ptr + n};
    }
};
__device__ __forceinline__ LBuf lbuf_at(const ScanParams &p, uint64_t b) {
    uint64_t ptr, n;
    list_desc(p, b, ptr, n);
    if (n < kListMainMin) return LBuf{b, 0, 0, 0, ptr, n, 0};
    const uint64_t m0 = ptr & ~7ull, m1 = (ptr + n) & ~7ull, m = m1 - m0;
    const uint64_t vg = (m + kWaveGroupBytes - 1) / kWaveGroupBytes;
    const uint32_t pad = (uint32_t)(vg * kWaveGroupBytes - m);
    return LBuf{b, m0 - pad, (uint32_t)vg, pad, ptr, n, (uint32_t)(ptr - m0)};
}
// clears the bytes in front of the buffer in its first word (group 0, row pad / 512, lane (pad mod 512)
// / 8); only in that group (wave-uniform test)
template <class G>
__device__ __forceinline__ void list_mask_edges(G &cur, uint32_t g, const LBuf &sc, int lane) {
    if (g != 0 || !sc.o) return;
    const uint32_t jh = (sc.pad >> 9) & 7u, lh = (sc.pad & 511u) >> 3;
    const uint64_t mh = (uint32_t)lane == lh ? ~0ull << (8 * sc.o) : ~0ull;
#pragma unroll
    for (int R = 0; R < 8; ++R) cur.w[R] &= (uint32_t)R == jh ? mh : ~0ull;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t list_rsrc(uint64_t base, uint32_t nrec) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)rfl64(base), (short)0, (int)__builtin_amdgcn_readfirstlane(nrec),
                                             0x00020000);
}

template <int R>
__device__ __forceinline__ uint64_t bld_w8(__amdgpu_buffer_rsrc_t rs, uint32_t o0, uint32_t lim) {
    const uint32_t o = __builtin_elementwise_min(o0 + (uint32_t)(R * kW8Row), lim);
    const v2u v = __builtin_amdgcn_raw_buffer_load_b64(rs, o, 0, 2);  // aux 2: non-temporal
    return ((uint64_t)v.y << 32) | v.x;
}

// stream_rows_w8 with the next group's rows read through a buffer resource
template <int R, class B>
__device__ __forceinline__ uint32_t list_rows_w8(uint32_t x, typename B::Hi h, W8Group &cur, W8Group &nxt,
                                                 __amdgpu_buffer_rsrc_t rs, uint32_t o0, uint32_t lim, const B &eng) {
    if constexpr (R < kW8RowsPerGroup) {
        nxt.w[R] = bld_w8<R>(rs, o0, lim);
        typename B::Hi hn;
        if constexpr (R == 0) {
            x ^= (uint32_t)cur.w[0];
            hn = eng.look_hi((uint32_t)(cur.w[0] >> 32));
        } else {
            x = eng.look_lo(x, h, (uint32_t)cur.w[R]);
            hn = eng.look_hi((uint32_t)(cur.w[R] >> 32));
        }
        __builtin_amdgcn_sched_barrier(0);
        return list_rows_w8<R + 1, B>(x, hn, cur, nxt, rs, o0, lim, eng);
    } else {
        return eng.look_lo(x, h, 0u);
    }
}
template <int R>
__device__ __forceinline__ void list_issue(W8Group &g, __amdgpu_buffer_rsrc_t rs, uint32_t o0, uint32_t lim) {
    if constexpr (R < kW8RowsPerGroup) {
        g.w[R] = bld_w8<R>(rs, o0, lim);
        list_issue<R + 1>(g, rs, o0, lim);
    }
}

template <uint32_t POLY>
__global__ __launch_bounds__(kBraidBlock, 4) void crc32_list_stream_kernel(const ScanParams p) {
    using SS = StreamShape<8>;
    using B = Braid32W8<POLY>;
    constexpr int WAVES = SS::kWaves;
    __shared__ __attribute__((aligned(16))) char lds[SS::kLds];
    char *const cb = lds + SS::kTab;

    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * WAVES;
    const uint64_t gw = rfl64((uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6));
    const uint64_t *wbuf = p.d_wave_buf, *woff = p.d_tile_prefix, *wq = p.d_tile_prefix + nw + 1;
    const uint64_t b0 = sload64(wbuf + gw), b_end = sload64(wbuf + gw + 1);
    const uint32_t g0 = (uint32_t)sload64(woff + gw);
    const uint32_t nq = (uint32_t)(sload64(wq + gw + 1) - sload64(wq + gw));  // groups of this wave
    const uint32_t lo8 = 8u * (uint32_t)lane;
    const uint64_t dummy = rfl64((uint64_t)p.d_kvals);
    const uint32_t *xinv = (const uint32_t *)p.d_kvals + kBraidNibXinvWord;  // nibble images (mul_nib32)
    const uint32_t *gsh = (const uint32_t *)p.d_kvals + kBraidNibGshiftWord;
    const uint32_t *gmc = (const uint32_t *)p.d_kvals + kBraidNibGmWord;
    const uint32_t *xneg = (const uint32_t *)p.d_kvals + kBraidNibXneg8Word;  // x^(-8 t), t < 8
    const uint64_t jd = sload64(wq + (nw + 1) + gw);  // join descriptors of the first and last parts
    uint64_t *const jslots = (uint64_t *)(cb + (kLocalOff - kBKOff));  // 9 x {value, parts << 32 | groups}
    if (threadIdx.x < 2 * kListJoinSlots) jslots[threadIdx.x] = 0;

    // prefetch cursor: buffer fc, group fg; it skips buffers without a main region (nq groups ahead)
    const bool owns = b0 < b_end || nq;  // b0 < nbuf then (the host's wbuf is nbuf only past the groups)
    LBuf fc = owns ? lbuf_at(p, b0) : LBuf{};
    uint32_t fq = 0, fg = g0;
    if (nq)
        while (fc.vg == 0) fc = lbuf_at(p, fc.b + 1), fg = 0;
    auto f_adj = [&]() -> uint32_t { return fg == 0 ? fc.pad : 0u; };
    auto f_rsrc = [&]() {
        return fq < nq ? list_rsrc(fc.vb + (uint64_t)fg * kWaveGroupBytes + f_adj(), kWaveGroupBytes - f_adj())
                       : list_rsrc(dummy, 0u);
    };
    auto f_off = [&]() { return fq < nq ? lo8 - f_adj() : lo8; };
    auto f_lim = [&]() { return fq < nq ? kWaveGroupBytes - f_adj() : 0u; };
    auto f_next = [&]() {
        if (++fq >= nq) return;
        if (++fg == fc.vg) {
            do fc = lbuf_at(p, fc.b + 1);
            while (fc.vg == 0);
            fg = 0;
        }
    };
    const v4u kq = *(gv4u *)((const uint32_t *)p.d_kvals + SS::kKWord + 4 * threadIdx.x);
    // the two primed slots are issued unconditionally (a wave without groups issues zero-record
    // placeholders), so the compiler's wait-count pass sees one prologue shape
    W8Group ra, rb, rc;
    list_issue<0>(ra, f_rsrc(), f_off(), f_lim());
    f_next();
    {
        static_assert(kBraidBlock == 512, "build_w8_tables: 512 threads");
        build_w8_tables<POLY>(lds, threadIdx.x);
        if (threadIdx.x < 256) *(uint32_t *)(cb + (kT0Off - kBKOff) + 4 * threadIdx.x) = basis_w8<POLY, 8>(threadIdx.x);
    }
    if (threadIdx.x == 0) *(uint32_t *)(cb + (kConstFlagOff - kBKOff)) = 0u;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    B eng;
    eng.init(lds, lane);
    list_issue<0>(rb, f_rsrc(), f_off(), f_lim());
    f_next();
    bool consts_ready = false;
    auto publish_consts = [&]() {  // the K image only (no tile columns)
        *(v4u *)(cb + 16 * threadIdx.x) = kq;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_add((uint32_t *)(cb + (kConstFlagOff - kBKOff)), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto await_consts = [&]() {
        if (consts_ready) return;
        while (__hip_atomic_load((uint32_t *)(cb + (kConstFlagOff - kBKOff)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <
               (uint32_t)WAVES)
            __builtin_amdgcn_s_sleep(1);
        consts_ready = true;
    };
    // scan cursor: buffer sc, group g, the part's first group ga
    LBuf sc = fc;
    if (owns) sc = lbuf_at(p, b0);
    // a buffer without a main region: its head fold is the whole CRC
    auto finish_empty = [&]() {
        const uint32_t s_h = head_state_e<true>(p, sc.b, sc.edges(), eng);
        if (lane == 0) finalize_e<true>(p, sc.b, sc.edges(), s_h, eng);
    };
    // leading buffers without a main region (with groups to scan, the first buffer that has some may
    // lie past b_end: the next wave then starts inside it)
    if (owns)
        while (sc.vg == 0) {
            finish_empty();
            if (!nq && sc.b + 1 >= b_end) break;
            sc = lbuf_at(p, sc.b + 1);
        }
    if (!nq) {
        publish_consts();
        ring_drain(ra, rb, rb);
        return;
    }
    uint32_t g = g0, ga = g0, u = 0, q = 0;
    // a part's first group: the head state (group 0) enters its lane, divided by x^(8 o) and X^j
    auto part_begin = [&]() {
        ga = g;
        u = 0;
        if (g == 0) {
            uint32_t s_h = head_state_e<true>(p, sc.b, sc.edges(), eng);
            if (sc.o) s_h = mul_nib32(s_h, xneg + 128 * sc.o);
            const uint32_t j = (sc.pad >> 9) & 7u;
            if (j) s_h = mul_nib32(s_h, xinv + 128 * j);
            if ((uint32_t)lane == ((sc.pad & 511u) >> 3)) u = s_h;
        }
    };
    // the buffer's register at the end of its main words -> its tail folded -> stored (lane 0)
    auto finish = [&](uint32_t r) { finalize_e<true>(p, sc.b, sc.edges(), r, eng); };
    // value r of n groups of a buffer of vg groups into its accumulator; the part completing the count
    // finishes it (lane 0)
    auto publish = [&](uint64_t b, uint32_t r, uint32_t n, uint32_t vg) {
        (void)sx_xor64_ret(&p.d_acc[b], (unsigned long long)r);  // performed before it is counted
        const uint32_t c = sx_add32_ret(&p.d_cnt[b], n);
        if (c + n == vg) {
            const uint32_t fin = (uint32_t)sx_swap64_ret(&p.d_acc[b], 0ull);
            sx_store32(&p.d_cnt[b], 0u);
            finish(fin);  // (b is sc.b at every call)
        }
    };
    uint32_t nparts = 0;  // parts this wave has finished
    // the part [ga, g) ends: its share, moved to the buffer's end, finishes the buffer or joins it
    auto part_finish = [&]() {
        uint32_t r = wave_xor_s(eng.mulK(u, lane));
        const uint32_t mg = sc.vg - g;  // groups after the part
        if (mg && mg < (uint32_t)kBraidGmCount) {
            r = mul_nib32(r, gmc + 128 * mg);
        } else {
            for (uint32_t m = mg, i = 0; m; m >>= 1, ++i)
                if (m & 1u) r = mul_nib32(r, gsh + 128 * i);
        }
        const uint32_t d = (uint32_t)(nparts == 0 ? jd : jd >> 16) & 0xffffu;
        ++nparts;
        if (ga == 0 && g == sc.vg) {
            if (lane == 0) finish(r);
            return;
        }
        if (lane != 0) return;
        if (!(d & 0x8000u)) {  // (no descriptor: the device accumulator directly)
            publish(sc.b, r, g - ga, sc.vg);
            return;
        }
        list_join(jslots + 2 * (d & 15u), d, r, g - ga, [&](uint64_t v, uint32_t groups) {
            if (d & 0x100u)
                publish(sc.b, (uint32_t)v, groups, sc.vg);
            else
                finish((uint32_t)v);
        });
    };
    part_begin();
    auto step = [&](W8Group &cur, W8Group &nxt, bool first) {
#if AMDCRC_PRIO_ALL
        prio_by_work_left(q, nq);
#endif
        const __amdgpu_buffer_rsrc_t rs = f_rsrc();
        const uint32_t fo = f_off(), fl = f_lim();
        f_next();
        list_mask_edges(cur, g, sc, lane);
        u = list_rows_w8<0, B>(u, typename B::Hi{}, cur, nxt, rs, fo, fl, eng);
        if (first) publish_consts();
        ++q;
        if (++g == sc.vg || q == nq) {
            await_consts();
            part_finish();
            if (q < nq) {
                // the next buffer with a main region, finishing the empty ones on the way
                for (;;) {
                    sc = lbuf_at(p, sc.b + 1);
                    if (sc.vg) break;
                    finish_empty();
                }
                g = 0;
                part_begin();
            }
        }
    };
    step(ra, rc, true);
    while (q + 3 <= nq) {  // whole rotations, then the rest (see crc32_stream_kernel)
        step(rb, ra, false);
        step(rc, rb, false);
        step(ra, rc, false);
    }
    if (q < nq) {
        step(rb, ra, false);
        if (q < nq) step(rc, rb, false);
    }
    ring_drain(ra, rb, rc);  // the trailing placeholder rows
    // trailing buffers without a main region
    while (sc.b + 1 < b_end) {
        sc = lbuf_at(p, sc.b + 1);
        finish_empty();
    }
}

// ------------------------------------------------------------------------------------------
// W = 64 braided scan (CRC64NVME).
//
// The W=32 braid with 8-byte words: a row is 512 bytes, lane l owns the word at 8l (one
// global_load_dwordx2 per row, 512 contiguous bytes per wave instruction), and
//     u <- (u ^ w_row) * x^(8*512)
// is one slice-by-8 step whose tables T'_t[e] = e * x^(8(t+1)) * x^(8*504) fold in the skip over the
// other 63 words (byte i of a = u ^ w indexes T'_(7-i)): eight lookups per 8-byte word, one per byte.
// Lane l's share of the tile register is u * x^(-64 l).
//
// LDS: the eight 64-bit tables in 8 copies, quarter-rotated (128 KiB; 32 copies would need 512 KiB).
// Region r (= dword r of a) holds, in the 256-byte row of entry e, the four tables indexed by the
// bytes of that dword: quarter q (64 bytes) = byte q, 8 copies x 8 bytes.  In table slot k, lane
// quarter j = (lane >> 3) & 3 reads quarter (k + j) & 3 with copy lane & 7, so the 32 lanes of a
// ds_read_b64 half-wave cover the 32 bank pairs of the row exactly once (tests/test_braid64_model.py
// checks the schedule).  Tiles are combined in groups of 32 (slot value + arrival count per group),
// then per buffer, so at most 32 atomics meet on one address.
constexpr uint32_t kB64Row = 512;
constexpr int kB64RowsPerGroup = 8;                 // 4 KiB per wave per ring slot (= 64 B per lane)
constexpr uint32_t kB64TabBytes = 131072;
constexpr uint32_t kB64T0Off = kB64TabBytes;        // plain byte table, 256 x u64 (head / tail)
constexpr uint32_t kB64Lds = kB64T0Off + 2048;

template <uint64_t POLY, uint32_t ROW = kB64Row>
struct Braid64Basis {
    uint64_t b[9][8];  // b[t][i] = T'_t[1 << i] (t < 8) for rows of ROW bytes; b[8][i] = T_0[1 << i]
    constexpr Braid64Basis() : b() {
        const uint64_t skip = gf2_xpow8n(ROW - 8, POLY, 64);
        for (int i = 0; i < 8; ++i) {
            for (int t = 0; t < 8; ++t) b[t][i] = gf2_mulmod(gf2_table_entry(1u << i, t, POLY), skip, POLY, 64);
            b[8][i] = gf2_table_entry(1u << i, 0, POLY);
        }
    }
};

template <uint64_t POLY, int K, uint32_t ROW = kB64Row>
__device__ __forceinline__ uint64_t basis64(uint32_t e) {
    constexpr Braid64Basis<POLY, ROW> B{};
    uint64_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) v ^= ((e >> i) & 1u) ? B.b[K][i] : 0ull;
    return v;
}

template <uint64_t POLY, uint32_t ROW = kB64Row>
__device__ __forceinline__ uint64_t basis64_rt(uint32_t t, uint32_t e) {  // t wave-uniform
    switch (t) {
        case 0: return basis64<POLY, 0, ROW>(e);
        case 1: return basis64<POLY, 1, ROW>(e);
        case 2: return basis64<POLY, 2, ROW>(e);
        case 3: return basis64<POLY, 3, ROW>(e);
        case 4: return basis64<POLY, 4, ROW>(e);
        case 5: return basis64<POLY, 5, ROW>(e);
        case 6: return basis64<POLY, 6, ROW>(e);
        default: return basis64<POLY, 7, ROW>(e);
    }
}

// COPIES = 8: the layout above (two 64 KiB regions).  COPIES = 4 (crc64_stream4_kernel): one
// 64 KiB region in which the 256-byte row of entry e holds the table of byte t of a (T'_(7-t)) at
// bytes [32 t, 32 t + 32), 4 copies x 8 bytes.  A ds_read_b64 half-wave is conflict-free when its 32
// lanes use 32 distinct 8-byte columns (bank pair = column, whatever the row): lane group
// jp = (lane >> 2) & 7 reads, in table slot k < 4, byte q = (k + jp) & 3 of one dword -- the low one
// for jp < 4, the high one for jp >= 4 -- with copy lane & 3, so the half-wave covers 8 tables x 4
// copies; slots 4..7 read the other dword.  (A layout with 4 tables per instruction met 16 columns:
// 2-way conflicts.)  tests/test_braid64_model.py::test_four_copy_layout checks the schedule.
constexpr uint32_t kB64x4T0Off = 65536;
// the tile finish's per-lane nibble multiples NT_l[v] = sum_(i<4) bit(3-i) of v * K_l x^i (64 lanes x
// 16 x u64) and R4[u] = u * x^4 (16 x u64): see Braid64::mulK
constexpr uint32_t kB64x4NibOff = kB64x4T0Off + 2048;
constexpr uint32_t kB64x4R4Off = kB64x4NibOff + 64 * 16 * 8;
constexpr uint32_t kB64x4Lds = kB64x4R4Off + 16 * 8;
static_assert(2 * kB64x4Lds <= 160 * 1024, "two crc64_stream4_kernel workgroups per CU");

template <uint64_t POLY, int COPIES = 8>
struct Braid64 {
    using T = uint64_t;
    static constexpr int W = 64;
    const char *L;
    uint32_t cst[4], csth[4], sel[4];
    uint32_t lowmask;  // COPIES = 4: ~0 for lanes whose slots 0..3 read the low dword
    uint64_t kl;       // K_l = x^(-64 l)
    const char *nib;   // COPIES = 4: this lane's nibble multiples NT_l

    __device__ void init(const char *lds, int lane) {
        L = lds;
        nib = lds + kB64x4NibOff + 128u * (uint32_t)lane;
        if (COPIES == 8) {
            const uint32_t j = ((uint32_t)lane >> 3) & 3u, cp = (uint32_t)lane & 7u;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t q = (k + j) & 3u;
                cst[k] = (q << 6) | (cp << 3);
                csth[k] = cst[k] | 0x10000u;
                sel[k] = 0x0c060004u | (q << 8);  // byte0 <- cst, byte1 <- byte q of a, byte2 <- region
            }
            lowmask = ~0u;
        } else {
            const uint32_t jp = ((uint32_t)lane >> 2) & 7u, cp = (uint32_t)lane & 3u;
            const bool lowfirst = jp < 4;
            lowmask = lowfirst ? ~0u : 0u;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t q = (k + jp) & 3u;
                const uint32_t t1 = lowfirst ? q : 4u + q, t2 = lowfirst ? 4u + q : q;  // byte t of a
                cst[k] = (t1 << 5) | (cp << 3);
                csth[k] = (t2 << 5) | (cp << 3);
                sel[k] = 0x0c0c0004u | (q << 8);  // byte0 <- cst, byte1 <- byte q of the dword
            }
        }
    }
    // a * x^(8*512) ^ wn
    __device__ __forceinline__ uint64_t step_x(uint64_t a, uint64_t wn) const {
        const uint32_t lo = (uint32_t)a, hi = (uint32_t)(a >> 32);
        // COPIES = 4: slots 0..3 read dword ma, slots 4..7 dword mb (per lane half, see the layout)
        const uint32_t ma = COPIES == 8 ? lo : (lo & lowmask) | (hi & ~lowmask);
        const uint32_t mb = COPIES == 8 ? hi : (hi & lowmask) | (lo & ~lowmask);
        uint64_t v[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[k] = lds64(L, __builtin_amdgcn_perm(cst[k], ma, sel[k]));
            v[4 + k] = lds64(L, __builtin_amdgcn_perm(csth[k], mb, sel[k]));
        }
        uint32_t rl = xor3(xor3((uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2]), (uint32_t)v[3], (uint32_t)v[4]);
        rl = xor3(xor3(rl, (uint32_t)v[5], (uint32_t)v[6]), (uint32_t)v[7], (uint32_t)wn);
        uint32_t rh = xor3(xor3((uint32_t)(v[0] >> 32), (uint32_t)(v[1] >> 32), (uint32_t)(v[2] >> 32)),
                           (uint32_t)(v[3] >> 32), (uint32_t)(v[4] >> 32));
        rh = xor3(xor3(rh, (uint32_t)(v[5] >> 32), (uint32_t)(v[6] >> 32)), (uint32_t)(v[7] >> 32), (uint32_t)(wn >> 32));
        return ((uint64_t)rh << 32) | rl;
    }
    __device__ __forceinline__ uint64_t step(uint64_t a) const { return step_x(a, 0); }
    // plain byte step for head / tail bytes (s wave-uniform: broadcast reads)
    __device__ __forceinline__ uint64_t byte(uint64_t s, uint32_t b) const {
        return (s >> 8) ^ lds64(L, (COPIES == 8 ? kB64T0Off : kB64x4T0Off) + 8 * (((uint32_t)s ^ b) & 0xffu));
    }
    // r * K_l with the nibble multiples in LDS (COPIES = 4): the byte-Horner form below with each
    // B_m = NT_l[high nibble] ^ NT_l[low nibble] * x^4, and a * x^4 = (a >> 4) ^ R4[a & 15].  24 LDS
    // reads and ~60 VALU for the bytes of r instead of ~190 VALU of masked column XORs.
    // tests/test_braid64_model.py::test_mulk_nibble_tables models it.
    __device__ __forceinline__ uint64_t mulK_nib(uint64_t r) const {
        uint64_t acc = 0;
#pragma unroll
        for (int m = 7; m >= 0; --m) {
            const uint32_t word = (7 - m) < 4 ? (uint32_t)r : (uint32_t)(r >> 32);
            const int sh = 8 * ((7 - m) & 3);
            const uint64_t nh = lds64(nib, 8u * ((word >> (sh + 4)) & 15u));
            const uint64_t nl = lds64(nib, 8u * ((word >> sh) & 15u));
            const uint64_t b = nh ^ (nl >> 4) ^ lds64(L, kB64x4R4Off + 8u * ((uint32_t)nl & 15u));
            acc = m == 7 ? b : (acc >> 8) ^ lds64(L, kB64x4T0Off + 8u * ((uint32_t)acc & 0xffu)) ^ b;
        }
        return acc;
    }
    // r * K_l (once per tile), Horner over the bytes of r: bit 63-j of r pairs with K_l * x^j, so
    // with B_m = sum_i bit(63-8m-i) * K_l x^i (byte 7-m of r against the eight columns K_l x^i),
    // r * K_l = sum_m B_m x^(8m) = (((B_7 x^8 ^ B_6) x^8 ^ ...) ^ B_0, and a * x^8 is one plain
    // byte step, (a >> 8) ^ T0[a & 0xff].  About 230 VALU and 7 LDS reads instead of a 64-step
    // bit-serial product (~950 VALU).  tests/test_braid64_model.py::test_mulk_byte_horner models it.
    __device__ __forceinline__ uint64_t mulK(uint64_t r) const {
        if constexpr (COPIES == 4) return mulK_nib(r);
        uint32_t cl[8], ch[8];
        uint64_t b = kl;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            cl[i] = (uint32_t)b, ch[i] = (uint32_t)(b >> 32);
            b = gf2_mulx(b, POLY);
        }
        const uint32_t rl = (uint32_t)r, rh = (uint32_t)(r >> 32);
        auto bm = [&](int m) -> uint64_t {
            const uint32_t word = m < 4 ? rh : rl;
            const int sh = 8 * ((7 - m) & 3);
            uint32_t al = 0, ah = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t mask = (uint32_t)((int32_t)(word << (31 - (sh + 7 - i))) >> 31);
                al = xor_and(al, cl[i], mask);
                ah = xor_and(ah, ch[i], mask);
            }
            return ((uint64_t)ah << 32) | al;
        };
        constexpr uint32_t t0 = COPIES == 8 ? kB64T0Off : kB64x4T0Off;
        uint64_t acc = bm(7);
#pragma unroll
        for (int m = 6; m >= 0; --m) acc = (acc >> 8) ^ lds64(L, t0 + 8u * ((uint32_t)acc & 0xffu)) ^ bm(m);
        return acc;
    }
};

struct B64Group {
    uint64_t w[kB64RowsPerGroup];
};

template <bool NT>
__device__ __forceinline__ uint64_t ldpay64(uint64_t a) {
    if (NT) return __builtin_nontemporal_load((gu64 *)a);
    return *(gu64 *)a;
}

// group gi of a tile: rows [8 gi, 8 gi + 8), this lane's word of each (virtual offset
// gi*4096 + 512 r + 8 lane); words in the virtual front pad read the main start and are zeroed later
template <bool NT>
__device__ __forceinline__ void b64_load(B64Group &g, uint64_t vbase, uint32_t pad, uint32_t gi, int lane) {
    const uint32_t vo0 = gi * (kB64Row * kB64RowsPerGroup) + 8u * lane;
#pragma unroll
    for (int r = 0; r < kB64RowsPerGroup; ++r) {
        const uint32_t vo = vo0 + kB64Row * r;
        g.w[r] = ldpay64<NT>(vbase + (vo >= pad ? vo : pad));
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <class B>
__device__ __forceinline__ uint64_t b64_proc(uint64_t u, const B64Group &g, const B &eng, const Tile &d, uint32_t gi,
                                             int lane, uint64_t s_h) {
    if (group_clean(d.pad, gi)) {
        uint64_t a = u ^ g.w[0];
#pragma unroll
        for (int r = 0; r + 1 < kB64RowsPerGroup; ++r) a = eng.step_x(a, g.w[r + 1]);
        return eng.step(a);
    }
    const uint32_t vo0 = gi * (kB64Row * kB64RowsPerGroup) + 8u * lane;
#pragma unroll
    for (int r = 0; r < kB64RowsPerGroup; ++r) {
        const uint32_t vo = vo0 + kB64Row * r;
        uint64_t w = vo >= d.pad ? g.w[r] : 0ull;
        if (vo == d.pad) w ^= s_h;  // this braid is still zero here: the head state enters with the word
        u = eng.step(u ^ w);
    }
    return u;
}

// steady state: scan group g while issuing group g+1's loads, one per table step
template <bool NT, class B>
__device__ __forceinline__ uint64_t b64_fused(uint64_t u, const B64Group &g, B64Group &dst, uint64_t a, const B &eng) {
    uint64_t x = u ^ g.w[0];
#pragma unroll
    for (int st = 0; st < kB64RowsPerGroup; ++st) {
        dst.w[st] = ldpay64<NT>(a + kB64Row * st);
        x = st + 1 < kB64RowsPerGroup ? eng.step_x(x, g.w[st + 1]) : eng.step(x);
        __builtin_amdgcn_sched_barrier(0);
    }
    return x;
}

// Tile finish: lane shares -> tile register -> its 32-tile group slot (value XOR, then arrival
// count); the group's last arrival moves the group value to the buffer end and XORs it into the
// buffer word (count of groups); the buffer's last group finalises.
template <bool LIST, class B>
__device__ __forceinline__ void b64_finish(const ScanParams &p, const Tile &d, uint64_t u, uint64_t s_h, const B &eng, int lane) {
    const uint64_t r = d.ngroups ? wave_xor64_s(eng.mulK(u)) : 0ull;
    if (d.T == 1) {
        if (lane == 0) finalize<LIST>(p, d.b, d.ngroups ? r : s_h, eng);
        return;
    }
    const uint64_t g0 = d.k & ~31ull, gend = d.T - g0 < 32 ? d.T : g0 + 32;
    const uint64_t v = mul_pcols<uint64_t, 64>(r, p.d_pcols + (gend - 1 - d.k) * 64);
    const uint64_t slot = d.tbase + g0;
    unsigned int c = 0;
    if (lane == 0) {
        const unsigned long long o =
            __hip_atomic_fetch_xor(&p.d_acc1[slot], (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::"v"(o) : "memory");  // performed before it is counted
        c = __hip_atomic_fetch_add(&p.d_cnt1[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    c = __builtin_amdgcn_readfirstlane(c);
    if (c != (unsigned int)(gend - g0 - 1)) return;
    unsigned long long gv = 0;
    if (lane == 0) {
        gv = __hip_atomic_exchange(&p.d_acc1[slot], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&p.d_cnt1[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    gv = rfl64(gv);
    const uint64_t G = (d.T + 31) / 32;
    if (G == 1) {
        if (lane == 0) finalize<LIST>(p, d.b, (uint64_t)gv, eng);
        return;
    }
    const uint64_t gs = d.T > gend ? mul_pcols<uint64_t, 64>((uint64_t)gv, p.d_pcols + (d.T - gend) * 64) : (uint64_t)gv;
    if (lane == 0) {
        const unsigned long long o =
            __hip_atomic_fetch_xor(&p.d_acc[d.b], (unsigned long long)gs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::"v"(o) : "memory");
        const unsigned int c2 = __hip_atomic_fetch_add(&p.d_cnt[d.b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (c2 == (unsigned int)(G - 1)) {
            const uint64_t fin = __hip_atomic_exchange(&p.d_acc[d.b], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&p.d_cnt[d.b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            finalize<LIST>(p, d.b, fin, eng);
        }
    }
}

// T'_t: two waves per table (t wave-uniform), each thread two entries x 8 copies; T0 (1024 threads)
template <uint64_t POLY>
__device__ __forceinline__ void b64_build_tables(char *lds) {
    const uint32_t i = threadIdx.x, wv = i >> 6;
    const uint32_t t = __builtin_amdgcn_readfirstlane(wv >> 1);
    const uint32_t reg = t >= 4 ? 0u : 1u, q = t >= 4 ? 7u - t : 3u - t;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const uint32_t e = ((wv & 1u) << 7) | ((uint32_t)n << 6) | (i & 63u);
        const uint64_t v = basis64_rt<POLY>(t, e);
        const v4u vv = {(uint32_t)v, (uint32_t)(v >> 32), (uint32_t)v, (uint32_t)(v >> 32)};
        char *row = lds + (reg << 16) + (e << 8) + (q << 6);
#pragma unroll
        for (int h = 0; h < 4; ++h) *(v4u *)(row + (((h + i) & 3u) << 4)) = vv;  // rotated: spread banks
    }
    if (i < 256) *(uint64_t *)(lds + kB64T0Off + 8 * i) = basis64<POLY, 8>(i);
}

// the 4-copy layout (Braid64<POLY, 4>: row e of 256 bytes, slot t at 32 t holding T'_(7-t)[e] in 4
// copies) from 512 threads, as 4096 chunks of 16 bytes: chunk k = i + 512 m holds copies 2 (k & 1),
// +1 of slot t = (k & 15) >> 1 of entry e = k >> 4 = (i >> 4) + 32 m; consecutive lanes store
// consecutive chunks (conflict-free, as build_w8_tables; round 4 built slot t in wave t, one 32-byte
// bank group per store); then T0
template <uint64_t POLY, uint32_t ROW = kB64Row>
__device__ __forceinline__ void b64x4_build_tables(char *lds) {
    constexpr Braid64Basis<POLY, ROW> B{};
    const uint32_t i = threadIdx.x;
    if (i >= 512) return;
    const uint32_t t = (i & 15u) >> 1;
    uint32_t mk[8];  // opaque per-lane masks: table 7 - t (a select chain over constants would load them)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        mk[k] = t == 7u - (uint32_t)k ? ~0u : 0u;
        asm("" : "+v"(mk[k]));
    }
    uint64_t bt[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) lo |= (uint32_t)B.b[k][b] & mk[k], hi |= (uint32_t)(B.b[k][b] >> 32) & mk[k];
        bt[b] = ((uint64_t)hi << 32) | lo;
    }
    const uint32_t e0 = i >> 4;
    uint64_t v0 = 0;
#pragma unroll
    for (int b = 0; b < 5; ++b) v0 ^= ((e0 >> b) & 1u) ? bt[b] : 0ull;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const uint64_t v = v0 ^ (m & 1 ? bt[5] : 0ull) ^ (m & 2 ? bt[6] : 0ull) ^ (m & 4 ? bt[7] : 0ull);
        *(v4u *)(lds + 16u * (i + 512u * m)) = v4u{(uint32_t)v, (uint32_t)(v >> 32), (uint32_t)v, (uint32_t)(v >> 32)};
    }
    if (i < 256) *(uint64_t *)(lds + kB64x4T0Off + 8 * i) = basis64<POLY, 8>(i);
}

// the tile finish's nibble tables (Braid64<POLY, 4>::mulK_nib): thread i fills NT_l[v] of lane
// l = i & 63 (its own K_l) for v = i >> 6 and v + 8; threads below 16 fill R4
template <uint64_t POLY>
__device__ __forceinline__ void b64x4_build_nib(char *lds, uint64_t kl) {
    const uint32_t i = threadIdx.x;
    if (i >= 512) return;
    uint64_t c[4];
    c[0] = kl;
#pragma unroll
    for (int k = 1; k < 4; ++k) c[k] = gf2_mulx(c[k - 1], POLY);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t v = (i >> 6) + 8u * h;
        uint64_t a = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) a ^= ((v >> (3 - k)) & 1u) ? c[k] : 0ull;
        *(uint64_t *)(lds + kB64x4NibOff + 128u * (i & 63u) + 8u * v) = a;
    }
    if (i < 16) {
        uint64_t u = i;
#pragma unroll
        for (int k = 0; k < 4; ++k) u = gf2_mulx(u, POLY);
        *(uint64_t *)(lds + kB64x4R4Off + 8u * i) = u;
    }
}

template <uint64_t POLY, bool LIST, bool NT = true>
__global__ __launch_bounds__(kBlock, 1) void crc64_braid_kernel(const ScanParams p) {
    using B = Braid64<POLY>;
    __shared__ __attribute__((aligned(16))) char lds[kB64Lds];

    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint64_t gw = rfl64((uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
    const uint64_t t0 = udiv_u(gw * p.ntiles, nw), t1 = udiv_u((gw + 1) * p.ntiles, nw);

    Walker w0{0, 0, 0};
    if (LIST && t0 < t1) {
        w0.b = sload64(p.d_wave_buf + gw);
        w0.lo = sload64(p.d_tile_prefix + w0.b);
        w0.hi = sload64(p.d_tile_prefix + w0.b + 1);
    }
    // ---- prefetch cursor: the next (tile, group) to load; pf_done once every group is in flight
    Walker wf = w0;
    uint64_t tf = t0;
    uint32_t gf = 0;
    uint64_t fvb = 0;
    uint32_t fpad = 0, fng = 0;
    bool any = false;
    for (; tf < t1; ++tf) {
        const Tile d = make_tile<LIST>(p, tf, wf);
        if (d.ngroups) {
            fvb = d.vbase, fpad = d.pad, fng = d.ngroups;
            gf = first_group(d.pad);
            any = true;
            break;
        }
    }
    bool pf_done = !any;
    auto pf_advance = [&]() {
        if (gf + 1 < fng) {
            ++gf;
            return;
        }
        if (pf_done) return;
        Walker w2 = wf;
        for (uint64_t t = tf + 1; t < t1; ++t) {
            const Tile d = make_tile<LIST>(p, t, w2);
            if (d.ngroups) {
                fvb = d.vbase, fpad = d.pad, fng = d.ngroups;
                wf = w2;
                tf = t;
                gf = first_group(d.pad);
                return;
            }
        }
        pf_done = true;
    };
    const uint64_t kl = *(gu64 *)(p.d_kvals + lane);
    // prime the first group (a wave without payload reads the 16 KiB constant block)
    B64Group r0, r1;
    b64_load<NT>(r0, any ? fvb : (uint64_t)p.d_kvals, any ? fpad : 0u, any ? gf : 0u, lane);
    if (any) pf_advance();
    b64_build_tables<POLY>(lds);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    B eng;
    eng.init(lds, lane);
    eng.kl = kl;
    if (t0 >= t1) return;

    // ---- scan cursor
    Walker wp = w0;
    uint64_t tp = t0;
    uint32_t gp = 0;
    Tile dp = make_tile<LIST>(p, tp, wp);
    gp = first_group(dp.pad);
    uint64_t s_h = dp.k == 0 ? head_state<LIST>(p, dp.b, eng) : 0ull;
    uint64_t u = (dp.k == 0 && dp.pad == 0 && lane == 0) ? s_h : 0ull;

    auto settle = [&]() -> bool {
        while (gp >= dp.ngroups) {
            b64_finish<LIST>(p, dp, u, s_h, eng, lane);
            if (++tp >= t1) return false;
            dp = make_tile<LIST>(p, tp, wp);
            gp = first_group(dp.pad);
            s_h = dp.k == 0 ? head_state<LIST>(p, dp.b, eng) : 0ull;
            u = (dp.k == 0 && dp.pad == 0 && lane == 0) ? s_h : 0ull;
        }
        return true;
    };
    auto ring_step = [&](const B64Group &cur, B64Group &dst) {
        if (pf_done) {
            u = b64_proc(u, cur, eng, dp, gp, lane, s_h);
        } else if (group_clean(dp.pad, gp) && group_clean(fpad, gf)) {
            u = b64_fused<NT>(u, cur, dst, fvb + gf * (kB64Row * kB64RowsPerGroup) + 8u * lane, eng);
        } else {
            b64_load<NT>(dst, fvb, fpad, gf, lane);
            u = b64_proc(u, cur, eng, dp, gp, lane, s_h);
        }
        ++gp;
        pf_advance();
    };
    if (any) {
        for (;;) {
            if (!settle()) break;
            ring_step(r0, r1);
            if (!settle()) break;
            ring_step(r1, r0);
        }
    } else {
        settle();
    }
}

// ------------------------------------------------------------------------------------------
// W = 64 streaming scan (CRC64NVME) for uniform batches whose main region is a whole number of
// tiles: crc32_stream_kernel's structure on crc64_braid_kernel's 512-byte rows.  A three-slot ring
// of 8-row groups (4 KiB per wave per slot, 48 VGPRs) on one code path, placeholder rows past the
// wave's last group, one static tile per wave slot, and the tile combine with self-waiting asm
// atomics, so the compiler's wait counts for the row loads stay exact.
template <int R>
__device__ __forceinline__ uint64_t gld_row64(uint32_t voff, uint64_t sbase) {
    return __builtin_nontemporal_load((gu64 *)(sbase + voff + R * kB64Row));
}

template <int R, class B>
__device__ __forceinline__ uint64_t stream64_rows(uint64_t x, B64Group &cur, B64Group &nxt, uint32_t voff, uint64_t snext,
                                                  const B &eng) {
    if constexpr (R < kB64RowsPerGroup) {
        nxt.w[R] = gld_row64<R>(voff, snext);
        x = R == 0 ? x ^ cur.w[0] : eng.step_x(x, cur.w[R]);
        __builtin_amdgcn_sched_barrier(0);
        return stream64_rows<R + 1>(x, cur, nxt, voff, snext, eng);
    } else {
        return eng.step(x);
    }
}

template <int R>
__device__ __forceinline__ void stream64_issue(B64Group &g, uint32_t voff, uint64_t s) {
    if constexpr (R < kB64RowsPerGroup) {
        g.w[R] = gld_row64<R>(voff, s);
        stream64_issue<R + 1>(g, voff, s);
    }
}

// b64_finish with self-waiting asm atomics: the tile register into its 32-tile group slot (value,
// then arrival count); the group's last arrival moves the group to the buffer end and counts groups
// per buffer; the buffer's last group finalises.
template <class B>
__device__ __forceinline__ void stream64_finish(const ScanParams &p, const Tile &d, uint64_t u, const B &eng, int lane) {
    const uint64_t r = wave_xor64_s(eng.mulK(u));
    if (d.T == 1) {
        if (lane == 0) finalize<false>(p, d.b, r, eng);
        return;
    }
    const uint64_t g0 = d.k & ~31ull, gend = d.T - g0 < 32 ? d.T : g0 + 32;
    const uint64_t v = mul_pcols<uint64_t, 64>(r, p.d_pcols + (gend - 1 - d.k) * 64);
    const uint64_t slot = d.tbase + g0;
    unsigned int c = 0;
    if (lane == 0) {
        (void)sx_xor64_ret(&p.d_acc1[slot], (unsigned long long)v);  // performed before it is counted
        c = sx_add32_ret(&p.d_cnt1[slot], 1u);
    }
    c = __builtin_amdgcn_readfirstlane(c);
    if (c != (unsigned int)(gend - g0 - 1)) return;
    unsigned long long gv = 0;
    if (lane == 0) {
        gv = sx_swap64_ret(&p.d_acc1[slot], 0ull);
        sx_store32(&p.d_cnt1[slot], 0u);
    }
    gv = rfl64(gv);
    const uint64_t G = (d.T + 31) / 32;
    if (G == 1) {
        if (lane == 0) finalize<false>(p, d.b, (uint64_t)gv, eng);
        return;
    }
    const uint64_t gs = d.T > gend ? mul_pcols<uint64_t, 64>((uint64_t)gv, p.d_pcols + (d.T - gend) * 64) : (uint64_t)gv;
    if (lane == 0) {
        (void)sx_xor64_ret(&p.d_acc[d.b], (unsigned long long)gs);
        const unsigned int c2 = sx_add32_ret(&p.d_cnt[d.b], 1u);
        if (c2 == (unsigned int)(G - 1)) {
            const uint64_t fin = sx_swap64_ret(&p.d_acc[d.b], 0ull);
            sx_store32(&p.d_cnt[d.b], 0u);
            finalize<false>(p, d.b, fin, eng);
        }
    }
}

// The same scan on the 4-copy table layout (66 KiB of LDS) in 512-thread workgroups, two per CU, so
// a launch queued on another stream co-resides with the running one.  The default W=64 streaming
// scan: C5 pipelined 5500-5558 vs 5138-5143 GiB/s for an 8-copy kernel with one workgroup per CU, at a
// 4 % slower isolated launch (2-way bank conflicts on the lookups).
template <uint64_t POLY, int BLOCK>
__global__ __launch_bounds__(BLOCK, 4) void crc64_stream4_kernel(const ScanParams p) {
    using B = Braid64<POLY, 4>;
    __shared__ __attribute__((aligned(16))) char lds[kB64x4Lds];
    constexpr int kBraidWaves = BLOCK / 64;

    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * kBraidWaves;
    const uint64_t gw = rfl64((uint64_t)blockIdx.x * kBraidWaves + (threadIdx.x >> 6));
    const uint64_t t0 = rfl64(udiv_u(gw * p.ntiles, nw)), t1 = rfl64(udiv_u((gw + 1) * p.ntiles, nw));
    // geometry: G groups of 4 KiB per tile, T tiles per buffer, main region at hoff of every buffer
    const uint32_t G = p.seg / kGroupBytes;
    const uint32_t gsh = __builtin_ctz(G);
    const uint64_t T = p.tiles_per_buf, tile_bytes = (uint64_t)p.seg * kWave;
    const uint64_t hoff = buffer_edges<false>(p, 0).headend - p.base;
    const uint32_t voff = 8u * (uint32_t)lane;
    const uint64_t dummy = rfl64((uint64_t)p.d_kvals);  // 16 KiB constant block (placeholder rows)
    const uint32_t nq = (uint32_t)((t1 - t0) << gsh);  // groups of this wave
    const bool work = t0 < t1;
    uint32_t fq = 0;  // groups issued
    uint64_t fb = udiv_u(t0, T), fk = t0 - fb * T;
    uint32_t fg = 0;
    BatchPos fpos = work ? batch_pos(p, fb) : BatchPos{0, 0};
    uint64_t fbuf = work ? karg64(p.bbase, fpos.j) + fpos.i * p.stride + hoff : 0;
    auto f_addr = [&]() -> uint64_t {
        return rfl64(fq < nq ? fbuf + fk * tile_bytes + (uint64_t)fg * (kB64Row * kB64RowsPerGroup) : dummy);
    };
    auto f_next = [&]() {
        ++fq;
        if (++fg == G) {
            fg = 0;
            if (++fk == T) {
                fk = 0, ++fb;
                if (++fpos.i == p.bcount && fq < nq) {
                    fpos.i = 0, ++fpos.j;
                    fbuf = karg64(p.bbase, fpos.j) + hoff;
                } else {
                    fbuf += p.stride;
                }
            }
        }
    };
    const uint64_t kl = *(gu64 *)(p.d_kvals + lane);
    B64Group ra, rb, rc;
    if (work) {
        stream64_issue<0>(ra, voff, f_addr());
        f_next();
    }
    b64x4_build_tables<POLY>(lds);
    b64x4_build_nib<POLY>(lds, kl);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    B eng;
    eng.init(lds, lane);
    eng.kl = kl;
    if (!work) return;
    stream64_issue<0>(rb, voff, f_addr());
    f_next();

    Tile d;
    d.T = T;
    d.b = udiv_u(t0, T);
    d.k = t0 - d.b * T;
    d.tbase = d.b * T;
    d.vbase = 0;
    d.pad = 0;
    d.ngroups = G;
    uint32_t g = 0;
    uint64_t u = 0;
    uint32_t q = 0;  // groups scanned
    auto step = [&](B64Group &cur, B64Group &nxt) {
#if AMDCRC_PRIO_ALL
        prio_by_work_left(q, nq);
#endif
        if (g == 0) u = d.k == 0 && lane == 0 ? head_state<false>(p, d.b, eng) : 0ull;
        const uint64_t sn = f_addr();
        f_next();
        u = stream64_rows<0>(u, cur, nxt, voff, sn, eng);
        ++q;
        if (++g == G) {
            g = 0;
            stream64_finish(p, d, u, eng, lane);
            if (++d.k == T) d.k = 0, ++d.b, d.tbase += T;
        }
    };
    // whole rotations of three steps, then the rest (the breaks drained the ring at every loop
    // header: see crc32_stream_kernel)
    while (q + 3 <= nq) {
        step(ra, rc);
        step(rb, ra);
        step(rc, rb);
    }
    if (q < nq) {
        step(ra, rc);
        if (q < nq) step(rb, ra);
    }
}


// ------------------------------------------------------------------------------------------
// W = 64 scan of long uniform buffers in XCD windows (crc64_xcd_kernel, round 3).  Streaming reads
// ran 4-10 % faster when the waves of one XCD read neighbouring 4-16 KiB pieces of one window than
// when every wave streams its own contiguous range (experiments/readpattern.hip; with the
// CRC64 scan's slower waves the gap was 6 %: profiles/r03/order).  So the launch's main bytes, all
// buffers' main regions in order, are cut into chunks of kXcdChunkGroups 4 KiB groups; XCD x
// (blockIdx mod 8 under round-robin dispatch) takes the x-th eighth of the chunks, and its nwx waves
// take chunks j, j + nwx, j + 2 nwx, ... of that eighth (j = the wave's index in the XCD).
//  * Inside a chunk a wave runs crc64_stream4_kernel's rows (8-byte lane words, 512-byte rows, the
//    4-copy tables, the three-slot ring).
//  * A wave's next chunk in the same buffer starts (nwx - 1) chunks past the end of the last one; every
//    lane's braid jumps there with u <- u * J, J = x^(8 * chunk * (nwx - 1)), from nibble tables of J in
//    LDS (16 broadcast-friendly reads; ScanParams::d_pcols holds them and the shift columns).
//  * A part (the wave's chunks of one buffer) ends with the stream kernel's tile finish (lane shares
//    K_l, wave XOR), moved to the buffer end by x^(8 * chunk * m), m = chunks after its last one (one
//    column product per set bit of m), then XORed into the workgroup's part table in LDS (one entry per
//    buffer: value, chunk count).  After the scan wave 0 publishes the table, one entry per lane, into
//    the buffers' accumulators and counts; the entry completing a buffer's count finalises it.
// Taken by strided CRC64NVME launches whose main regions are whole chunks of at least kXcdMinChunks.
constexpr int kXcdChunkGroups = AMDCRC_XCD_CHUNK_GROUPS;
constexpr uint32_t kXcdChunk = kXcdChunkGroups * kB64Row * kB64RowsPerGroup;
constexpr uint32_t kXcdJumpOff = kB64x4Lds;               // 16 nibbles x 16 x u64: v << 4n times J
constexpr uint32_t kXcdSlotOff = kXcdJumpOff + 16 * 16 * 8;  // part table: buffer, value, chunks
constexpr uint32_t kXcdSlots = 64;
constexpr uint32_t kXcdLds = kXcdSlotOff + kXcdSlots * (8 + 8 + 4);
static_assert(2 * kXcdLds <= 160 * 1024, "two crc64_xcd_kernel workgroups per CU");

__device__ __forceinline__ uint64_t xcd_jump(const char *lds, uint64_t u) {
    const uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
    uint64_t v[16];
#pragma unroll
    for (int n = 0; n < 8; ++n) {
        v[n] = lds64(lds, kXcdJumpOff + 128u * n + 8u * ((lo >> (4 * n)) & 15u));
        v[8 + n] = lds64(lds, kXcdJumpOff + 128u * (8 + n) + 8u * ((hi >> (4 * n)) & 15u));
    }
    uint32_t rl = 0, rh = 0;
#pragma unroll
    for (int n = 0; n < 16; n += 2) {
        rl = xor3(rl, (uint32_t)v[n], (uint32_t)v[n + 1]);
        rh = xor3(rh, (uint32_t)(v[n] >> 32), (uint32_t)(v[n + 1] >> 32));
    }
    return ((uint64_t)rh << 32) | rl;
}

// a wave-uniform walk over the chunks j, j + nwx, ... of [lo, hi): chunk k of buffer b
struct XcdCursor {
    uint64_t b, k;      // buffer, chunk in buffer
    uint64_t main;      // virtual start of buffer b's chunk 0 (main-region start - front pad)
};

// rows through a raw buffer resource (crc32_list_stream_kernel's loads): offsets at or past `lim`
// read zeros, so a chunk's front pad costs no masking and no traffic
template <int R>
__device__ __forceinline__ uint64_t xcd_bld(__amdgpu_buffer_rsrc_t rs, uint32_t o0, uint32_t lim) {
    const uint32_t o = __builtin_elementwise_min(o0 + (uint32_t)(R * kB64Row), lim);
    const v2u v = __builtin_amdgcn_raw_buffer_load_b64(rs, o, 0, 2);  // aux 2: non-temporal
    return ((uint64_t)v.y << 32) | v.x;
}
template <int R, class B>
__device__ __forceinline__ uint64_t xcd_rows(uint64_t x, B64Group &cur, B64Group &nxt, __amdgpu_buffer_rsrc_t rs, uint32_t o0,
                                             uint32_t lim, const B &eng) {
    if constexpr (R < kB64RowsPerGroup) {
        nxt.w[R] = xcd_bld<R>(rs, o0, lim);
        x = R == 0 ? x ^ cur.w[0] : eng.step_x(x, cur.w[R]);
        __builtin_amdgcn_sched_barrier(0);
        return xcd_rows<R + 1>(x, cur, nxt, rs, o0, lim, eng);
    } else {
        return eng.step(x);
    }
}
template <int R>
__device__ __forceinline__ void xcd_issue(B64Group &g, __amdgpu_buffer_rsrc_t rs, uint32_t o0, uint32_t lim) {
    if constexpr (R < kB64RowsPerGroup) {
        g.w[R] = xcd_bld<R>(rs, o0, lim);
        xcd_issue<R + 1>(g, rs, o0, lim);
    }
}

// PADDED: some main regions hold no whole number of chunks (ScanParams::xcd_pad != 0): every group
// reads through a buffer resource.  Otherwise plain global loads (1-2 % shorter C5 launches).
template <uint64_t POLY, int BLOCK, bool PADDED, bool PRIO = false>
__global__ __launch_bounds__(BLOCK, AMDCRC_XCD_WPE) void crc64_xcd_kernel(const ScanParams p) {
    using B = Braid64<POLY, 4>;
    __shared__ __attribute__((aligned(16))) char lds[kXcdLds];
    constexpr int kWaves = BLOCK / 64;
    const int lane = threadIdx.x & 63;
    // the kernel arguments the first group's address needs, in one batch of scalar loads with one wait
    // (crc32_stream_kernel's round-5 prologue: the compiler had spread them over dependent round trips)
    {
        const uint64_t a0 = p.ntiles, a1 = p.tiles_per_buf, a2 = p.base, a3 = p.stride, a4 = p.len, a5 = p.bcount,
                       a6 = (uint64_t)p.d_kvals, a7 = (uint64_t)p.d_pcols, a8 = p.bbase[0];
        const uint32_t a9 = p.nbatch, a10 = p.xcd_pad, a11 = gridDim.x;
        asm volatile("" ::"s"(a0), "s"(a1), "s"(a2), "s"(a3), "s"(a4), "s"(a5), "s"(a6), "s"(a7), "s"(a8), "s"(a9), "s"(a10),
                     "s"(a11));
    }
    const uint64_t nwx = (uint64_t)gridDim.x * kWaves / 8;  // waves per XCD (gridDim % 8 == 0)
    const uint64_t xcd = blockIdx.x & 7u;
    const uint64_t j = rfl64((uint64_t)(blockIdx.x >> 3) * kWaves + (threadIdx.x >> 6));
    const uint64_t NC = p.ntiles, CPB = p.tiles_per_buf;
    const uint64_t xlo = xcd * NC / 8, xhi = (xcd + 1) * NC / 8;
    const uint64_t c0 = xlo + j;
    const uint32_t nchunks = c0 < xhi ? (uint32_t)udiv_u(xhi - c0 + nwx - 1, nwx) : 0u;
    const uint32_t nq = nchunks * kXcdChunkGroups;  // groups of this wave
    const uint64_t hoff = buffer_edges<false>(p, 0).headend - p.base;
    const uint32_t voff = 8u * (uint32_t)lane;
    const uint64_t dummy = rfl64((uint64_t)p.d_kvals);  // 16 KiB constant block (placeholder rows)
    const uint64_t dq = udiv_u(nwx, CPB), dr = nwx - dq * CPB;   // chunk step as (buffers, chunks)
    // every buffer's main region is front-padded with virtual zeros to CPB whole chunks (pad < chunk)
    const uint32_t pad = p.xcd_pad;
    auto cur_at = [&](uint64_t c) -> XcdCursor {
        const uint64_t b = udiv_u(c, CPB);
        const BatchPos bp = batch_pos(p, b);
        return XcdCursor{b, c - b * CPB, karg64(p.bbase, bp.j) + bp.i * p.stride + hoff - pad};
    };
    auto cur_next = [&](XcdCursor &x) {
        uint64_t b = x.b + dq, k = x.k + dr;
        if (k >= CPB) k -= CPB, ++b;
        if (b != x.b) {
            const BatchPos bp = batch_pos(p, b);
            x.main = karg64(p.bbase, bp.j) + bp.i * p.stride + hoff - pad;
        }
        x.b = b, x.k = k;
    };
    // prefetch cursor: chunk fc, group fg; fq groups issued.  A group reads through a buffer resource
    // based at its first real byte with its real bytes as records; a lane's offset into the pad comes
    // out negative (wrapped), is clamped to the record count and reads zero.
    XcdCursor fc = nq ? cur_at(c0) : XcdCursor{0, 0, 0};
    uint32_t fq = 0, fg = 0;
    constexpr uint32_t kGB = kB64Row * kB64RowsPerGroup;
    auto f_adj = [&]() -> uint32_t {  // pad bytes at the front of group fg of chunk fc.k
        if (fc.k != 0 || pad <= fg * kGB) return 0u;
        const uint32_t a = pad - fg * kGB;
        return a < kGB ? a : kGB;
    };
    auto f_rsrc = [&]() {
        return fq < nq ? list_rsrc(fc.main + fc.k * kXcdChunk + (uint64_t)fg * kGB + f_adj(), kGB - f_adj())
                       : list_rsrc(dummy, 0u);
    };
    auto f_off = [&]() { return fq < nq ? voff - f_adj() : voff; };
    auto f_lim = [&]() { return fq < nq ? kGB - f_adj() : 0u; };
    auto f_addr = [&]() -> uint64_t { return rfl64(fq < nq ? fc.main + fc.k * kXcdChunk + (uint64_t)fg * kGB : dummy); };
    auto issue = [&](B64Group &g) {
        if constexpr (PADDED)
            xcd_issue<0>(g, f_rsrc(), f_off(), f_lim());
        else
            stream64_issue<0>(g, voff, f_addr());
    };
    auto f_next = [&]() {
        ++fq;
        if (++fg == (uint32_t)kXcdChunkGroups) {
            fg = 0;
            if (fq < nq) cur_next(fc);
        }
    };
    // the tile-finish constants (needed before the barrier), then the wave's first two groups, issued
    // unconditionally (placeholder rows past a wave's last group), so that the wait for the constants
    // is one exact count on every path and both groups stream while the tables are built (round 5; the
    // conditional issue had left the compiler a vmcnt(0) before the barrier)
    // (PADDED keeps the round-4 order -- the first group only, the second after the barrier: its
    // buffer resources then push the kernel to 128 VGPRs and spill)
    const uint64_t kl = *(gu64 *)(p.d_kvals + lane);
    const uint64_t jt = threadIdx.x < 256 ? *(gu64 *)(p.d_pcols + threadIdx.x) : 0ull;
    B64Group ra, rb, rc;
    if (!PADDED || nq) {
        issue(ra);
        f_next();
    }
    if constexpr (!PADDED) {
        issue(rb);
        f_next();
    }
    b64x4_build_tables<POLY>(lds);
    b64x4_build_nib<POLY>(lds, kl);
    if (threadIdx.x < 256) *(uint64_t *)(lds + kXcdJumpOff + 8u * threadIdx.x) = jt;
    uint64_t *const ptag = (uint64_t *)(lds + kXcdSlotOff);  // the part table (empty tag ~0)
    uint64_t *const pval = ptag + kXcdSlots;
    uint32_t *const pcnt = (uint32_t *)(pval + kXcdSlots);
    if (threadIdx.x < kXcdSlots) ptag[threadIdx.x] = ~0ull, pval[threadIdx.x] = 0ull, pcnt[threadIdx.x] = 0u;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    B eng;
    eng.init(lds, lane);
    eng.kl = kl;
    const uint64_t *bytecols = p.d_pcols + 256 + 40 * 64;  // [level][v][j]: x^(8 * chunk * v * 256^level) * x^j
    uint64_t pb = ~0ull, pk = 0;  // the open part: buffer, last chunk
    uint32_t pn = 0;              // chunks in the part
    uint64_t u = 0;
    // the open part's register (lane shares joined), at the end of its last chunk
    auto part_raw = [&]() -> uint64_t { return wave_xor64_s(eng.mulK(u)); };
    // r * x^(8 * chunk * m): one 64-column product per nonzero byte of m, the columns spread over the
    // lanes (lane c holds column c, a coalesced 512-byte load; the four loads issue together) and the
    // selected columns XORed across the wave.  Only where the payload ring is drained.
    auto shift_lanes = [&](uint64_t r, uint64_t m) -> uint64_t {
        uint64_t col[4];
#pragma unroll
        for (int L = 0; L < 4; ++L) {
            const uint64_t v = (m >> (8 * L)) & 255u;
            col[L] = v ? *(gu64 *)(bytecols + (256u * L + v) * 64 + lane) : 0ull;
        }
#pragma unroll
        for (int L = 0; L < 4; ++L) {
            if (((m >> (8 * L)) & 255u) == 0) continue;
            const uint64_t sel = (r >> (63 - lane)) & 1u;
            r = wave_xor64_s(sel ? col[L] : 0ull);
        }
        return r;
    };
    // the same product on the scalar unit (columns by SMEM): a part ending inside the scan (one per
    // buffer a wave leaves: multi-batch launches cross many).  One product per nonzero byte of m --
    // m < nwx, so one or two -- not one per set bit (round 4: up to twelve products of eight L2 round
    // trips each made a 20-batch C5 launch 0.63 of the HBM peak).  (Round 5: the nibble-image product,
    // two round trips, measured 0.5 % slower here -- 1,024 images of 2 KiB against 512-byte column
    // sets, each product touching sixteen lines -- and is kept for the list scans.)
    auto shift_scalar = [&](uint64_t r, uint64_t m) -> uint64_t {
        for (int L = 0; m; ++L, m >>= 8)
            if (m & 255u) r = mul_pcols<uint64_t, 64>(r, bytecols + (256u * L + (m & 255u)) * 64);
        return r;
    };
    // value r of n chunks of buffer b into the buffer's accumulator; the part completing the count
    // finalises the buffer (lane 0)
    auto publish = [&](uint64_t b, uint64_t r, uint32_t n) {
        (void)sx_xor64_ret(&p.d_acc[b], (unsigned long long)r);  // performed before it is counted
        const unsigned int c = sx_add32_ret(&p.d_cnt[b], n);
        if (c + n == (unsigned int)CPB) {
            const uint64_t fin = sx_swap64_ret(&p.d_acc[b], 0ull);
            sx_store32(&p.d_cnt[b], 0u);
            finalize<false>(p, b, fin, eng);
        }
    };
    // a part into the workgroup's table (lane 0; LDS atomics, open addressing from b): no global atomic
    // and so no drained payload ring inside the scan (round 4's held parts published one part per buffer
    // crossing with three returning atomics, each a vmcnt(0): 20-batch C5 launches at 0.66 against 0.77
    // for one batch).  A full table -- more than kXcdSlots buffers in one workgroup -- publishes directly.
    auto part_put = [&](uint64_t b, uint64_t v, uint32_t n) {
#pragma unroll 1
        for (uint32_t i = 0; i < kXcdSlots; ++i) {
            const uint32_t e = ((uint32_t)b + i) & (kXcdSlots - 1);
            uint64_t t = ~0ull;
            __hip_atomic_compare_exchange_strong(&ptag[e], &t, b, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (t == ~0ull || t == b) {
                __hip_atomic_fetch_xor(&pval[e], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&pcnt[e], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                return;
            }
        }
        publish(b, v, n);
    };
    auto part_finish = [&]() {
        const uint64_t v = shift_scalar(part_raw(), CPB - 1 - pk);
        if (lane == 0) part_put(pb, v, pn);
    };
    // the wave's last part, then wave 0 publishes the table: entry e in lane e, all accumulators in one
    // round trip and all counts in a second; the buffers completed finalise one at a time
    auto final_parts = [&](bool have) {
        if (have) {
            const uint64_t v = shift_lanes(part_raw(), CPB - 1 - pk);
            if (lane == 0) part_put(pb, v, pn);
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (threadIdx.x >= 64) return;
        static_assert(kXcdSlots == 64, "one table entry per lane of wave 0");
        const uint64_t eb = ptag[lane];
        bool done = false;
        if (eb != ~0ull) {
            const uint32_t en = pcnt[lane];
            (void)sx_xor64_ret(&p.d_acc[eb], (unsigned long long)pval[lane]);  // every value lands first
            done = sx_add32_ret(&p.d_cnt[eb], en) + en == (unsigned int)CPB;
        }
        uint64_t fm = __builtin_amdgcn_ballot_w64(done);
        while (fm) {
            const int e = __builtin_ctzll(fm);
            fm &= fm - 1;
            const uint64_t b = rfl64((uint64_t)__builtin_amdgcn_readlane((int)(uint32_t)eb, e) |
                                     ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(eb >> 32), e) << 32));
            if (lane == 0) {
                const uint64_t fin = sx_swap64_ret(&p.d_acc[b], 0ull);
                sx_store32(&p.d_cnt[b], 0u);
                finalize<false>(p, b, fin, eng);
            }
        }
    };
    if (!nq) {
        if constexpr (!PADDED)  // the placeholder groups land before the wave ends
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(ra.w[0]), "+v"(ra.w[1]), "+v"(ra.w[2]), "+v"(ra.w[3]), "+v"(ra.w[4]),
                         "+v"(ra.w[5]), "+v"(ra.w[6]), "+v"(ra.w[7]), "+v"(rb.w[0]), "+v"(rb.w[1]), "+v"(rb.w[2]), "+v"(rb.w[3]),
                         "+v"(rb.w[4]), "+v"(rb.w[5]), "+v"(rb.w[6]), "+v"(rb.w[7])::"memory");
        final_parts(false);
        return;
    }
    if constexpr (PADDED) {
        issue(rb);
        f_next();
    }

    // the head state enters lane (pad mod 512) / 8 at the start of chunk 0 divided by X^jr (X = x^(8*512),
    // jr = the pad's row): that lane's words before the pad are zero, so jr row steps bring it to the head
    // state exactly where the first real word joins (crc32_list_stream_kernel's head entry)
    const uint32_t jr = pad / kB64Row, l0 = (pad % kB64Row) / 8u;
    XcdCursor sc = cur_at(c0);
    uint32_t g = 0, q = 0;
    // PRIO (multi-batch launches): issue priority by the work left, crc32_stream_kernel's.  Measured
    // here in round 5: 20-batch C5 0.70 -> 0.72-0.73, but one-batch launches overlapping over three
    // streams lost 8 % with it and a run-time switch cost the single launch 12 % (profiles/r05/ab/
    // r05ad_*, r05ae_*), hence a separate instantiation chosen at launch by batch count
    auto step = [&](B64Group &cur, B64Group &nxt) {
        if constexpr (PRIO || AMDCRC_PRIO_ALL) prio_by_work_left(q, nq);
        if (g == 0) {
            if (pn && sc.b == pb) {
                u = xcd_jump(lds, u);
            } else {
                if (pn) part_finish();
                pb = sc.b, pn = 0;
                u = 0ull;
                if (sc.k == 0) {
                    uint64_t s_h = head_state<false>(p, sc.b, eng);
                    if (jr) s_h = mul_nib64(s_h, p.d_pcols + kXcdNibXinvU64 + 256 * jr);
                    if ((uint32_t)lane == l0) u = s_h;
                }
            }
            ++pn, pk = sc.k;
        }
        if constexpr (PADDED) {
            const __amdgpu_buffer_rsrc_t rs = f_rsrc();
            const uint32_t fo = f_off(), fl = f_lim();
            f_next();
            u = xcd_rows<0>(u, cur, nxt, rs, fo, fl, eng);
        } else {
            const uint64_t sn = f_addr();
            f_next();
            u = stream64_rows<0>(u, cur, nxt, voff, sn, eng);
        }
        ++q;
        if (++g == (uint32_t)kXcdChunkGroups) {
            g = 0;
            if (q < nq) cur_next(sc);
        }
    };
    // whole rotations of three steps, then the rest (see crc32_stream_kernel)
    while (q + 3 <= nq) {
        step(ra, rc);
        step(rb, ra);
        step(rc, rb);
    }
    if (q < nq) {
        step(ra, rc);
        if (q < nq) step(rb, ra);
    }
    // the trailing placeholder rows land before the finish reuses registers
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(ra.w[0]), "+v"(ra.w[1]), "+v"(ra.w[2]), "+v"(ra.w[3]), "+v"(ra.w[4]), "+v"(ra.w[5]),
                 "+v"(ra.w[6]), "+v"(ra.w[7])::"memory");
    asm volatile("" : "+v"(rb.w[0]), "+v"(rb.w[1]), "+v"(rb.w[2]), "+v"(rb.w[3]), "+v"(rb.w[4]), "+v"(rb.w[5]), "+v"(rb.w[6]), "+v"(rb.w[7]));
    asm volatile("" : "+v"(rc.w[0]), "+v"(rc.w[1]), "+v"(rc.w[2]), "+v"(rc.w[3]), "+v"(rc.w[4]), "+v"(rc.w[5]), "+v"(rc.w[6]), "+v"(rc.w[7]));
    final_parts(true);
}

// ------------------------------------------------------------------------------------------
// Ragged CRC64NVME lists on the streaming scan (crc64_list_stream_kernel, round 3):
// crc32_list_stream_kernel's walk at W = 64.  Every buffer's main region is front-padded to whole
// 4 KiB groups and the list is one sequence of groups, split evenly over the waves (cut anywhere, also
// inside buffers); groups read through buffer resources whose range check supplies the pad's zeros; the
// head state enters lane (pad mod 512)/8 of group 0 divided by X^j (X = x^(8*512), j = the pad's row);
// a part of a buffer ends with the lane shares (nibble-table K_l product, wave XOR), is moved to the
// buffer end by x^(8*4096*m) for the m groups after it, and finishes the buffer or joins it through the
// per-buffer accumulator and group count.  The tables, the nibble-table finish and the row step are
// crc64_stream4_kernel's (4 copies, two 512-thread workgroups per CU).  Constants: ScanParams::d_pcols
// = engine.cpp get_xcd_consts (the nibble images of X^(-j), x^(8*4096*2^i) and x^(8*4096*m): engine.h
// kXcdNib*).

template <uint64_t POLY>
__global__ __launch_bounds__(512, 4) void crc64_list_stream_kernel(const ScanParams p) {
    using B = Braid64<POLY, 4>;
    __shared__ __attribute__((aligned(16))) char lds[kB64x4Lds];
    constexpr int WAVES = 8;
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * WAVES;
    const uint64_t gw = rfl64((uint64_t)blockIdx.x * WAVES + (threadIdx.x >> 6));
    const uint64_t *wbuf = p.d_wave_buf, *woff = p.d_tile_prefix, *wq = p.d_tile_prefix + nw + 1;
    const uint64_t b0 = sload64(wbuf + gw), b_end = sload64(wbuf + gw + 1);
    const uint32_t g0 = (uint32_t)sload64(woff + gw);
    const uint32_t nq = (uint32_t)(sload64(wq + gw + 1) - sload64(wq + gw));  // groups of this wave
    const uint32_t lo8 = 8u * (uint32_t)lane;
    const uint64_t dummy = rfl64((uint64_t)p.d_kvals);
    const uint64_t *xinv = p.d_pcols + kXcdNibXinvU64;  // nibble images (mul_nib64)
    const uint64_t *gsh = p.d_pcols + kXcdNibGshiftU64;
    const uint64_t *gmc = p.d_pcols + kXcdNibGmU64;
    const uint64_t *xneg = p.d_pcols + kXcdNibXneg8U64;  // x^(-8 t), t < 8
    const uint64_t jd = sload64(wq + (nw + 1) + gw);  // join descriptors of the first and last parts
    __shared__ uint64_t jslots[2 * kListJoinSlots];   // {value, parts << 32 | groups}
    if (threadIdx.x < 2 * kListJoinSlots) jslots[threadIdx.x] = 0;

    // prefetch cursor: buffer fc, group fg; it skips buffers without a main region (nq groups ahead)
    const bool owns = b0 < b_end || nq;
    LBuf fc = owns ? lbuf_at(p, b0) : LBuf{};
    uint32_t fq = 0, fg = g0;
    if (nq)
        while (fc.vg == 0) fc = lbuf_at(p, fc.b + 1), fg = 0;
    auto f_adj = [&]() -> uint32_t { return fg == 0 ? fc.pad : 0u; };
    auto f_rsrc = [&]() {
        return fq < nq ? list_rsrc(fc.vb + (uint64_t)fg * kWaveGroupBytes + f_adj(), kWaveGroupBytes - f_adj())
                       : list_rsrc(dummy, 0u);
    };
    auto f_off = [&]() { return fq < nq ? lo8 - f_adj() : lo8; };
    auto f_lim = [&]() { return fq < nq ? kWaveGroupBytes - f_adj() : 0u; };
    auto f_next = [&]() {
        if (++fq >= nq) return;
        if (++fg == fc.vg) {
            do fc = lbuf_at(p, fc.b + 1);
            while (fc.vg == 0);
            fg = 0;
        }
    };
    const uint64_t kl = *(gu64 *)(p.d_kvals + lane);
    // the two primed slots are issued unconditionally (zero-record placeholders for a wave without
    // groups), so the compiler's wait-count pass sees one prologue shape
    B64Group ra, rb, rc;
    xcd_issue<0>(ra, f_rsrc(), f_off(), f_lim());
    f_next();
    b64x4_build_tables<POLY>(lds);
    b64x4_build_nib<POLY>(lds, kl);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    B eng;
    eng.init(lds, lane);
    eng.kl = kl;
    xcd_issue<0>(rb, f_rsrc(), f_off(), f_lim());
    f_next();
    auto drain = [&]() {  // the placeholder rows land before anything reuses their registers
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(ra.w[0]), "+v"(ra.w[1]), "+v"(ra.w[2]), "+v"(ra.w[3]), "+v"(ra.w[4]),
                     "+v"(ra.w[5]), "+v"(ra.w[6]), "+v"(ra.w[7])::"memory");
        asm volatile("" : "+v"(rb.w[0]), "+v"(rb.w[1]), "+v"(rb.w[2]), "+v"(rb.w[3]), "+v"(rb.w[4]), "+v"(rb.w[5]), "+v"(rb.w[6]),
                     "+v"(rb.w[7]));
        asm volatile("" : "+v"(rc.w[0]), "+v"(rc.w[1]), "+v"(rc.w[2]), "+v"(rc.w[3]), "+v"(rc.w[4]), "+v"(rc.w[5]), "+v"(rc.w[6]),
                     "+v"(rc.w[7]));
    };
    // scan cursor: buffer sc, group g, the part's first group ga
    LBuf sc = fc;
    if (owns) sc = lbuf_at(p, b0);
    auto finish_empty = [&]() {  // a buffer without a main region: its head fold is the whole CRC
        const uint64_t s_h = head_state_e<true>(p, sc.b, sc.edges(), eng);
        if (lane == 0) finalize_e<true>(p, sc.b, sc.edges(), s_h, eng);
    };
    if (owns)
        while (sc.vg == 0) {
            finish_empty();
            if (!nq && sc.b + 1 >= b_end) break;
            sc = lbuf_at(p, sc.b + 1);
        }
    if (!nq) {
        drain();
        return;
    }
    uint32_t g = g0, ga = g0, q = 0;
    uint64_t u = 0;
    auto part_begin = [&]() {
        ga = g;
        u = 0;
        if (g == 0) {
            uint64_t s_h = head_state_e<true>(p, sc.b, sc.edges(), eng);
            if (sc.o) s_h = mul_nib64(s_h, xneg + 256 * sc.o);
            const uint32_t j = (sc.pad >> 9) & 7u;
            if (j) s_h = mul_nib64(s_h, xinv + 256 * j);
            if ((uint32_t)lane == ((sc.pad & 511u) >> 3)) u = s_h;
        }
    };
    auto finish = [&](uint64_t r) {  // at the end of the main words -> its tail folded -> stored
        finalize_e<true>(p, sc.b, sc.edges(), r, eng);
    };
    auto publish = [&](uint64_t b, uint64_t r, uint32_t n, uint32_t vg) {  // lane 0
        (void)sx_xor64_ret(&p.d_acc[b], (unsigned long long)r);  // performed before it is counted
        const uint32_t c = sx_add32_ret(&p.d_cnt[b], n);
        if (c + n == vg) {
            const uint64_t fin = sx_swap64_ret(&p.d_acc[b], 0ull);
            sx_store32(&p.d_cnt[b], 0u);
            finish(fin);  // (b is sc.b at every call)
        }
    };
    uint32_t nparts = 0;  // parts this wave has finished
    auto part_finish = [&]() {
        uint64_t r = wave_xor64_s(eng.mulK(u));
        const uint32_t mg = sc.vg - g;  // groups after the part
        if (mg && mg < (uint32_t)kBraidGmCount) {
            r = mul_nib64(r, gmc + 256 * mg);
        } else {
            for (uint32_t m = mg, i = 0; m; m >>= 1, ++i)
                if (m & 1u) r = mul_nib64(r, gsh + 256 * i);
        }
        const uint32_t d = (uint32_t)(nparts == 0 ? jd : jd >> 16) & 0xffffu;
        ++nparts;
        if (ga == 0 && g == sc.vg) {
            if (lane == 0) finish(r);
            return;
        }
        if (lane != 0) return;
        if (!(d & 0x8000u)) {  // (no descriptor: the device accumulator directly)
            publish(sc.b, r, g - ga, sc.vg);
            return;
        }
        // a buffer cut between waves: its parts in this workgroup join in LDS (list_join)
        list_join(jslots + 2 * (d & 15u), d, r, g - ga, [&](uint64_t v, uint32_t groups) {
            if (d & 0x100u)
                publish(sc.b, v, groups, sc.vg);
            else
                finish(v);
        });
    };
    part_begin();
    auto step = [&](B64Group &cur, B64Group &nxt) {
#if AMDCRC_PRIO_ALL
        prio_by_work_left(q, nq);
#endif
        const __amdgpu_buffer_rsrc_t rs = f_rsrc();
        const uint32_t fo = f_off(), fl = f_lim();
        f_next();
        list_mask_edges(cur, g, sc, lane);
        u = xcd_rows<0>(u, cur, nxt, rs, fo, fl, eng);
        ++q;
        if (++g == sc.vg || q == nq) {
            part_finish();
            if (q < nq) {
                for (;;) {  // the next buffer with a main region, finishing the empty ones on the way
                    sc = lbuf_at(p, sc.b + 1);
                    if (sc.vg) break;
                    finish_empty();
                }
                g = 0;
                part_begin();
            }
        }
    };
    step(ra, rc);
    while (q + 3 <= nq) {  // whole rotations, then the rest (see crc32_stream_kernel)
        step(rb, ra);
        step(rc, rb);
        step(ra, rc);
    }
    if (q < nq) {
        step(rb, ra);
        if (q < nq) step(rc, rb);
    }
    drain();
    while (sc.b + 1 < b_end) {  // trailing buffers without a main region
        sc = lbuf_at(p, sc.b + 1);
        finish_empty();
    }
}

// ------------------------------------------------------------------------------------------
// W = 64 scan of many short uniform buffers (the C4 per-GPU shard: 131,072 x 8 KiB), 16 lanes per
// buffer.  A wave scans four buffers at once, one per 16-lane row: lane t of row r owns the 8-byte
// word at 8t of every 128-byte row of buffer 4s + r, so the braid step's tables fold in the skip over
// the row's other 15 words (T'_t[e] = e * x^(8(t+1)) * x^(8*120)), and lane t's share of its buffer's
// register is u * x^(-64 t).  One tile finish -- the nibble-table product (31 LDS reads) and a 16-lane
// reduction -- then covers four buffers instead of one: at 8 KiB per buffer the per-buffer finish of
// crc64_stream4_kernel took an eighth of the launch (profiles/r03/crc64_xp).  The table layout (4
// copies, conflict-free for any data) and the three-slot ring are crc64_stream4_kernel's; each lane
// streams its own buffer, so the ring's addresses are per lane.
constexpr uint32_t kR16Row = 128;                           // bytes per buffer row (16 lanes x 8 B)
constexpr uint32_t kR16Group = kR16Row * kB64RowsPerGroup;  // 1 KiB of each buffer per ring slot
constexpr int kR16Block = 512;

template <int R>
__device__ __forceinline__ uint64_t gld_r16(uint64_t a) {
    return __builtin_nontemporal_load((gu64 *)(a + R * kR16Row));
}
template <int R>
__device__ __forceinline__ void r16_issue(B64Group &g, uint64_t a) {
    if constexpr (R < kB64RowsPerGroup) {
        g.w[R] = gld_r16<R>(a);
        r16_issue<R + 1>(g, a);
    }
}
template <int R, class B>
__device__ __forceinline__ uint64_t r16_rows(uint64_t x, B64Group &cur, B64Group &nxt, uint64_t anext, const B &eng) {
    if constexpr (R < kB64RowsPerGroup) {
        nxt.w[R] = gld_r16<R>(anext);
        x = R == 0 ? x ^ cur.w[0] : eng.step_x(x, cur.w[R]);
        __builtin_amdgcn_sched_barrier(0);
        return r16_rows<R + 1>(x, cur, nxt, anext, eng);
    } else {
        return eng.step(x);
    }
}
// XOR over the 16 lanes of each row, left in every lane of the row
__device__ __forceinline__ uint32_t row16_xor(uint32_t v) {
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    return v;
}

template <uint64_t POLY>
__global__ __launch_bounds__(kR16Block, 4) void crc64_rows16_kernel(const ScanParams p) {
    using B = Braid64<POLY, 4>;
    __shared__ __attribute__((aligned(16))) char lds[kB64x4Lds];
    constexpr int kWaves = kR16Block / 64;

    const int lane = threadIdx.x & 63;
    const uint32_t row = (uint32_t)lane >> 4, t = (uint32_t)lane & 15u;
    const uint64_t nsets = (p.nbuf + 3) / 4;
    const uint64_t nw = (uint64_t)gridDim.x * kWaves;
    const uint64_t gw = rfl64((uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6));
    // the wave's sets: s0, s0 + sstep, ... (nsw of them).  With a grid of whole XCD rows (gridDim % 8
    // == 0) the waves of XCD x = blockIdx mod 8 take sets j, j + nwx, ... of the x-th eighth
    // (neighbouring sets at every step: crc64_xcd_kernel's read order); otherwise contiguous ranges.
    uint64_t s0, sstep, nsw;
#if AMDCRC_R16_XCD
    if ((gridDim.x & 7u) == 0) {
        const uint64_t nwx = nw / 8, xcd = blockIdx.x & 7u, xlo = xcd * nsets / 8, xhi = (xcd + 1) * nsets / 8;
        const uint64_t j = rfl64((uint64_t)(blockIdx.x >> 3) * kWaves + (threadIdx.x >> 6));
        s0 = xlo + j, sstep = nwx, nsw = s0 < xhi ? udiv_u(xhi - s0 + nwx - 1, nwx) : 0;
    } else
#endif
    {
        s0 = rfl64(udiv_u(gw * nsets, nw)), sstep = 1, nsw = rfl64(udiv_u((gw + 1) * nsets, nw)) - s0;
    }
    const Edges e0 = buffer_edges<false>(p, 0);
    const uint64_t hoff = e0.headend - p.base, ml = e0.tail - e0.headend;
    const uint32_t G = (uint32_t)(ml / kR16Group);  // groups per buffer (the host checks ml % kR16Group == 0)
    const uint32_t nq = (uint32_t)(nsw * G);  // groups of this wave
    const bool work = nsw > 0;
    const uint64_t dummy = (uint64_t)p.d_kvals + 8u * t;  // placeholder rows: the 16 KiB constant block
    // this lane's buffer of set s: main-region address + 8 t (rows past the batch read the constants)
    // (the four row bases are wave-uniform: computed on the scalar unit, so a multi-batch launch reads
    // its batch bases with scalar loads -- a per-lane kernarg load is a vector load whose wait drained
    // the payload ring once per set)
    auto lane_base = [&](uint64_t s) -> uint64_t {
        uint64_t a[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint64_t b = rfl64(4 * s + (uint64_t)r);
            if (b < p.nbuf) {
                const BatchPos bp = batch_pos(p, b);
                a[r] = rfl64(karg64(p.bbase, bp.j) + bp.i * p.stride + hoff);
            } else {
                a[r] = rfl64((uint64_t)p.d_kvals);
            }
        }
        return (row == 0 ? a[0] : row == 1 ? a[1] : row == 2 ? a[2] : a[3]) + 8u * t;
    };
    uint32_t fq = 0, fg = 0;  // prefetch cursor: groups issued, group within the set
    uint64_t fs = s0;
    uint64_t fbase = work ? lane_base(fs) : dummy;
    auto f_addr = [&]() -> uint64_t { return fq < nq ? fbase + (uint64_t)fg * kR16Group : dummy; };
    auto f_next = [&]() {
        ++fq;
        if (++fg == G) {
            fg = 0;
            fs += sstep;
            if (fq < nq) fbase = lane_base(fs);
        }
    };
    const uint64_t kl = *(gu64 *)(p.d_kvals + t);  // K_t = x^(-64 t)
    B64Group ra, rb, rc;
    if (work) {
        r16_issue<0>(ra, f_addr());
        f_next();
    }
    b64x4_build_tables<POLY, kR16Row>(lds);
    b64x4_build_nib<POLY>(lds, kl);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    B eng;
    eng.init(lds, lane);
    eng.kl = kl;
    if (!work) return;
    r16_issue<0>(rb, f_addr());
    f_next();

    uint64_t s = s0;  // scan cursor: set s, group g
    uint32_t g = 0, q = 0;
    uint64_t u = 0;
    auto step = [&](B64Group &cur, B64Group &nxt) {
#if AMDCRC_R16_PRIO || AMDCRC_PRIO_ALL
        prio_by_work_left(q, nq);  // (A/B on one box: C4 shard 0.786-0.795 -> 0.829-0.843)
#endif
        if (g == 0) {
            // head states of the set's four buffers (wave-uniform), each entering its row's lane 0
            uint64_t h[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) h[r] = 4 * s + (uint64_t)r < p.nbuf ? head_state<false>(p, 4 * s + r, eng) : 0ull;
            const uint64_t hr = row == 0 ? h[0] : row == 1 ? h[1] : row == 2 ? h[2] : h[3];
            u = t == 0 ? hr : 0ull;
        }
        const uint64_t an = f_addr();
        f_next();
        u = r16_rows<0>(u, cur, nxt, an, eng);
        ++q;
        if (++g == G) {
            g = 0;
            const uint64_t v = eng.mulK(u);
            const uint32_t lo = row16_xor((uint32_t)v), hi = row16_xor((uint32_t)(v >> 32));
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint64_t b = 4 * s + (uint64_t)r;
                const uint64_t fin = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, 16 * r) << 32) |
                                     (uint32_t)__builtin_amdgcn_readlane((int)lo, 16 * r);
                if (b < p.nbuf && lane == 0) finalize<false>(p, b, fin, eng);
            }
            s += sstep;
        }
    };
    // whole rotations of three steps, then the rest (the breaks drained the ring at every loop
    // header: see crc32_stream_kernel)
    while (q + 3 <= nq) {
        step(ra, rc);
        step(rb, ra);
        step(rc, rb);
    }
    if (q < nq) {
        step(ra, rc);
        if (q < nq) step(rb, ra);
    }
    // the trailing placeholder rows: their registers stay live until the loads have landed
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(ra.w[0]), "+v"(ra.w[1]), "+v"(ra.w[2]), "+v"(ra.w[3]), "+v"(ra.w[4]), "+v"(ra.w[5]),
                 "+v"(ra.w[6]), "+v"(ra.w[7])::"memory");
    asm volatile("" : "+v"(rb.w[0]), "+v"(rb.w[1]), "+v"(rb.w[2]), "+v"(rb.w[3]), "+v"(rb.w[4]), "+v"(rb.w[5]), "+v"(rb.w[6]),
                 "+v"(rb.w[7]));
    asm volatile("" : "+v"(rc.w[0]), "+v"(rc.w[1]), "+v"(rc.w[2]), "+v"(rc.w[3]), "+v"(rc.w[4]), "+v"(rc.w[5]), "+v"(rc.w[6]),
                 "+v"(rc.w[7]));
}

// ------------------------------------------------------------------------------------------
// xxHash64 (aws_xxhash64_compute, XXHash.cpp:17).  The published algorithm is four serial chains
// per buffer (nonlinear: add, rotate, multiply mod 2^64), so a buffer has at most four lanes of
// parallelism; the batch supplies the rest.
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

// XXH64 with one quad (4 lanes) per buffer: lane j owns accumulator v_(j+1), i.e. word j of every
// 32-byte stripe, so a buffer's four independent serial chains run on four lanes instead of
// interleaving in one (the per-lane chain, not issue, then bounds a buffer: 8 B per round latency).
// Each lane loads its words of four stripes per iteration, the next four in flight while these are
// mixed in.  Lane 0 of the quad finishes (merge, remaining < 32 bytes, avalanche).
// one global_load_dwordx2 whatever the alignment (the loads issue without a per-lane branch, so
// the waits before the rounds count only the oldest slot)
typedef uint64_t u64_any_align __attribute__((aligned(1)));
__device__ __forceinline__ uint64_t ldw(const uint8_t *p) { return *(const __attribute__((address_space(1))) u64_any_align *)p; }

// One round with the input product taken off the chain: the carried state is u = v + in * P2; the
// round computes v' = rotl(u, 31) * P1 and returns u' = v' + y where y = next_in * P2 is computed
// beforehand.  Dependent depth per round: two alignbits, then mad_u64_u32 (low product plus y) beside
// two mul_lo (cross products), then one add3.
__device__ __forceinline__ void xstep_y(uint32_t &ul, uint32_t &uh, uint64_t y) {
    const uint32_t rl = __builtin_amdgcn_alignbit(ul, uh, 1), rh = __builtin_amdgcn_alignbit(uh, ul, 1);
    const uint64_t m = (uint64_t)rl * (uint32_t)XP1 + y;
    ul = (uint32_t)m;
    uh = (uint32_t)(m >> 32) + rl * (uint32_t)(XP1 >> 32) + rh * (uint32_t)XP1;
}
// the same with y computed in this lane: the empty asm keeps the input product opaque, otherwise it
// is re-associated into the chain's mad (a second dependent mad per round)
__device__ __forceinline__ void xstep(uint32_t &ul, uint32_t &uh, uint64_t y) {
    asm volatile("" : "+v"(y));
    xstep_y(ul, uh, y);
}

// lane k of each quad, broadcast to the quad (DPP quad_perm [k,k,k,k])
template <int K>
__device__ __forceinline__ uint64_t quad_bcast(uint64_t v) {
    constexpr int sel = K | (K << 2) | (K << 4) | (K << 6);
    const uint32_t l = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, sel, 0xF, 0xF, false);
    const uint32_t h = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), sel, 0xF, 0xF, false);
    return ((uint64_t)h << 32) | l;
}

// merge of the four lanes (n >= 32), the < 32-byte tail and the avalanche (XXH64 digest)
__device__ __noinline__ uint64_t xxh64_finish(uint64_t v1, uint64_t v2, uint64_t v3, uint64_t v4, const uint8_t *ptr,
                                              uint64_t n, uint64_t seed) {
    uint64_t h;
    if (n >= 32) {
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xmerge(h, v1);
        h = xmerge(h, v2);
        h = xmerge(h, v3);
        h = xmerge(h, v4);
    } else {
        h = seed + XP5;
    }
    h += n;
    const uint8_t *t = ptr + (n & ~31ull), *end = ptr + n;
    while (t + 8 <= end) {
        h ^= xround(0, ld64u(t));
        h = rotl64(h, 27) * XP1 + XP4;
        t += 8;
    }
    if (t + 4 <= end) {
        uint32_t w;
        __builtin_memcpy(&w, t, 4);
        h ^= (uint64_t)w * XP1;
        h = rotl64(h, 23) * XP2 + XP3;
        t += 4;
    }
    while (t < end) {
        h ^= (*t++) * XP5;
        h = rotl64(h, 11) * XP1;
    }
    h ^= h >> 33;
    h *= XP2;
    h ^= h >> 29;
    h *= XP3;
    h ^= h >> 32;
    return h;
}

// One wave per block, bpw buffers per wave (quads 0..bpw-1; the rest of the wave idles), bpw sized
// on the host so that the launch spreads over the SIMDs.
__global__ __launch_bounds__(64) void xxh64_quad_kernel(const XxhParams p, uint32_t bpw) {
    const uint32_t quad = threadIdx.x >> 2;
    const uint64_t i = (uint64_t)blockIdx.x * bpw + quad;
    const int j = (int)(threadIdx.x & 3);
    const bool valid = quad < bpw && i < p.nbuf;
    const uint8_t *ptr = nullptr;
    uint64_t n = 0, seed = 0;
    if (valid) {
        ptr = (const uint8_t *)(p.d_ptrs ? p.d_ptrs[i] : p.base + i * p.stride);
        n = p.d_ptrs ? p.d_lens[i] : p.len;
        seed = p.d_seeds ? p.d_seeds[i] : p.seed_all;
    }
    const uint64_t ns = n >= 32 ? n / 32 : 0;
    uint64_t v = seed + (j == 0 ? XP1 + XP2 : j == 1 ? XP2 : j == 2 ? 0ull : 0ull - XP1);
    const uint8_t *q = ptr + 8 * j;
    // kXxSlots x 4 stripes in flight per lane: an HBM load takes ~2 us, a round a few dependent
    // integer ops; the kernel runs a few waves per CU, so registers are plentiful
    constexpr int kXxSlots = 12;
    if (ns > 0) {
        uint64_t u = v + ldw(q) * XP2;  // stripe 0 entered; stripes 1..ns-1 follow as y
        uint32_t ul = (uint32_t)u, uh = (uint32_t)(u >> 32);
        const uint8_t *q1 = q + 32;
        const uint64_t nr = ns - 1;
        uint64_t s = 0;
        if (nr >= 4 * kXxSlots) {
            uint64_t w[kXxSlots][4];
#pragma unroll
            for (int k = 0; k < kXxSlots; ++k)
#pragma unroll
                for (int m = 0; m < 4; ++m) w[k][m] = ldw(q1 + 32 * (4 * k + m));
            for (s = 4 * kXxSlots; s + 4 * kXxSlots <= nr; s += 4 * kXxSlots) {
#pragma unroll
                for (int k = 0; k < kXxSlots; ++k) {
#pragma unroll
                    for (int m = 0; m < 4; ++m) xstep(ul, uh, w[k][m] * XP2);
#pragma unroll
                    for (int m = 0; m < 4; ++m) w[k][m] = ldw(q1 + 32 * (s + 4 * k + m));
                }
            }
#pragma unroll
            for (int k = 0; k < kXxSlots; ++k)
#pragma unroll
                for (int m = 0; m < 4; ++m) xstep(ul, uh, w[k][m] * XP2);
        }
        for (; s < nr; ++s) xstep(ul, uh, ldw(q1 + 32 * s) * XP2);
        xstep(ul, uh, 0);  // the last stripe's round
        v = ((uint64_t)uh << 32) | ul;
    }
    // lane 0 of the quad gathers v1..v4 (quad_perm DPP broadcasts of lanes 1..3)
    const uint64_t v1 = quad_bcast<0>(v), v2 = quad_bcast<1>(v), v3 = quad_bcast<2>(v), v4 = quad_bcast<3>(v);
    if (!valid || j != 0) return;
    p.d_out[i] = xxh64_finish(v1, v2, v3, v4, ptr, n, seed);
}

// XXH64 over strided batches (equal lengths), B buffers per wave: lane l = 4 (B t + b) + j loads
// word j of stripe s0 + t of buffer b, so one load instruction brings T = 16 / B stripes of every
// buffer of the wave and their input products y = w * P2 are formed lane-parallel (off the chains);
// the chain lanes then take y of stripe s0 + t from lane l + 4 B t by ds_bpermute (LDS pipe) and
// spend only the six-op round on the VALU.  Every t group runs the same chains redundantly.  B is
// chosen on the host so that the launch has about one wave per SIMD (a round issues from one wave).
constexpr uint64_t inv_odd64(uint64_t a) {  // a^-1 mod 2^64 for odd a (Newton: 6 doublings of precision)
    uint64_t x = a;
    for (int k = 0; k < 6; ++k) x *= 2 - a * x;
    return x;
}
constexpr uint64_t kXP1Inv = inv_odd64(XP1);
static_assert(kXP1Inv * XP1 == 1, "P1 inverse");
__device__ __forceinline__ uint64_t bperm64(uint64_t v, int src_lane) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

template <int B>
__global__ __launch_bounds__(64) void xxh64_wave_kernel(const XxhParams p) {
    constexpr int T = 16 / B, DS = 12;  // stripes per load; loads in flight
    const int lane = threadIdx.x, j = lane & 3, b = (lane >> 2) % B, t = lane / (4 * B);
    const uint64_t i = (uint64_t)blockIdx.x * B + b;
    const bool valid = i < p.nbuf;
    const uint64_t ic = valid ? i : p.nbuf - 1;  // loads stay inside the batch
    const uint8_t *ptr = (const uint8_t *)(p.base + ic * p.stride);
    const uint64_t n = p.len, seed = p.d_seeds ? p.d_seeds[ic] : p.seed_all;
    const uint64_t ns = n / 32, nslot = (ns + T - 1) / T;
    uint64_t v = seed + (j == 0 ? XP1 + XP2 : j == 1 ? XP2 : j == 2 ? 0ull : 0ull - XP1);
    const int src0 = lane & (4 * B - 1);
    const uint8_t *q = ptr + 8 * j;
    auto ld = [&](uint64_t slot) -> uint64_t {
        uint64_t st = slot * T + (uint64_t)t;
        st = st < ns ? st : ns - 1;  // the last slot's spare lanes re-read the last stripe
        return ldw(q + 32 * st);
    };
    if (ns > 0) {
        uint64_t x[DS];
#pragma unroll
        for (int d = 0; d < DS; ++d) x[d] = ld(d);
        // every stripe's product is added by the round before it; the chain starts from the state
        // whose round yields v: rotl(u0, 31) * P1 = v, so stripe 0 needs no special case
        const uint64_t u0 = rotl64(v * kXP1Inv, 33);
        uint32_t ul = (uint32_t)u0, uh = (uint32_t)(u0 >> 32);
        // software pipeline: the next slot's products and bpermutes issue before this slot's T
        // rounds (sched_barrier keeps the scheduler from sinking them to their uses; interleaving
        // them two per round measured 11 % slower)
        uint64_t ya[T], yb[T];
        auto perm = [&](uint64_t xv, uint64_t (&yt)[T]) {
            const uint64_t y = xv * XP2;
#pragma unroll
            for (int tt = 0; tt < T; ++tt) yt[tt] = bperm64(y, src0 + 4 * B * tt);
        };
        auto rounds = [&](const uint64_t (&yt)[T], uint64_t slot, bool full) {
#pragma unroll
            for (int tt = 0; tt < T; ++tt)
                if (full || slot * T + tt < ns) xstep_y(ul, uh, yt[tt]);  // yt is a bpermute result: opaque
        };
        perm(x[0], ya);
        const uint64_t nfull = ns / T;  // slots whose T stripes all exist
        uint64_t slot = 0;
        for (; slot + DS <= nfull; slot += DS) {
#pragma unroll
            for (int d = 0; d < DS; ++d) {
                uint64_t (&cur)[T] = (d & 1) ? yb : ya;
                uint64_t (&nxt)[T] = (d & 1) ? ya : yb;
                perm(x[(d + 1) % DS], nxt);  // slot + d + 1 (x[0] already holds slot + DS)
                x[d] = ld(slot + DS + d);
                __builtin_amdgcn_sched_barrier(0);
                rounds(cur, slot + d, true);
                __builtin_amdgcn_sched_barrier(0);
            }
            if (DS & 1) {  // keep the next slot's products in ya
#pragma unroll
                for (int tt = 0; tt < T; ++tt) ya[tt] = yb[tt];
            }
        }
        // at most DS slots remain (the last may be partial); their words are already in the ring
#pragma unroll
        for (int d = 0; d < DS; ++d) {
            if (slot + d < nslot) {
                uint64_t (&cur)[T] = (d & 1) ? yb : ya;
                uint64_t (&nxt)[T] = (d & 1) ? ya : yb;
                if (d + 1 < DS && slot + d + 1 < nslot) perm(x[d + 1], nxt);
                rounds(cur, slot + d, false);
            }
        }
        xstep_y(ul, uh, 0);  // the last stripe's round
        v = ((uint64_t)uh << 32) | ul;
    }
    const uint64_t v1 = quad_bcast<0>(v), v2 = quad_bcast<1>(v), v3 = quad_bcast<2>(v), v4 = quad_bcast<3>(v);
    if (!valid || t != 0 || j != 0) return;
    p.d_out[i] = xxh64_finish(v1, v2, v3, v4, ptr, n, seed);
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

// ------------------------------------------------------------------------------------------
// Lane-per-buffer scan for lists of short buffers (event-stream framing CRCs: an 8-byte prelude and
// a message body per message).  The wave-per-tile scans fold a short
// buffer's unaligned head and tail with serial scalar loads and spend a tile pass on a few hundred
// bytes; here each lane owns one buffer: bytes up to 8-byte alignment, then slice-by-8 steps
// (eight independent table lookups per aligned 8-byte word, one dependent XOR chain per word),
// then the tail bytes.  Tables: eight 256-entry tables in LDS (8 KiB for W=32, 16 KiB for W=64),
// T_0 = the bytewise table, T_k[e] = T_(k-1)[e] advanced over one zero byte.  Lanes of a wave read
// neighbouring buffers, so packed messages share cache lines across lanes.
template <class T, T POLY>
__device__ __forceinline__ void lane_tables(T (*tab)[256]) {
    const uint32_t i = threadIdx.x;
    T c = (T)i;
#pragma unroll
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1) ? POLY : (T)0);
    tab[0][i] = c;
    __syncthreads();
#pragma unroll
    for (int t = 1; t < 8; ++t) {
        c = (c >> 8) ^ tab[0][c & 0xff];
        tab[t][i] = c;
    }
    __syncthreads();
}

// The lane scans' folds.  TabFold: eight plain 256-entry tables (lane_tables; any width): a lane's
// eight lookups of a word meet random banks, about 3.5-way conflicted per half-wave.  LaneW8 (W = 32,
// round 4): the same tables T_t[e] = e * x^(8(t+1)) in crc32_stream_kernel's 8-copy layout (64 KiB,
// one 256-byte row per entry: table t at 32 t, copy c at 4 c), looked up with its per-lane byte
// rotation, so each ds_read_b32 half-wave meets 32 distinct banks whatever the data.
template <class T>
struct TabFold {
    const T (*tab)[256];
    __device__ __forceinline__ T word(T s, uint64_t v) const {
        if (sizeof(T) == 4) {
            const uint32_t lo = (uint32_t)v ^ (uint32_t)s, hi = (uint32_t)(v >> 32);
            return tab[7][lo & 0xff] ^ tab[6][(lo >> 8) & 0xff] ^ tab[5][(lo >> 16) & 0xff] ^ tab[4][lo >> 24] ^
                   tab[3][hi & 0xff] ^ tab[2][(hi >> 8) & 0xff] ^ tab[1][(hi >> 16) & 0xff] ^ tab[0][hi >> 24];
        } else {
            const uint64_t x = v ^ (uint64_t)s;
            return tab[7][x & 0xff] ^ tab[6][(x >> 8) & 0xff] ^ tab[5][(x >> 16) & 0xff] ^ tab[4][(x >> 24) & 0xff] ^
                   tab[3][(x >> 32) & 0xff] ^ tab[2][(x >> 40) & 0xff] ^ tab[1][(x >> 48) & 0xff] ^ tab[0][x >> 56];
        }
    }
    __device__ __forceinline__ T bytes(T s, uint64_t v, uint32_t nb) const {
        for (uint32_t j = 0; j < nb; ++j, v >>= 8) s = (s >> 8) ^ tab[0][(s ^ (T)v) & 0xff];
        return s;
    }
};

constexpr uint32_t kLaneW8Lds = 65536;
template <uint32_t POLY>
struct LaneW8Basis {
    uint32_t b[8][8];  // b[t][i] = T_t[1 << i]
    constexpr LaneW8Basis() : b() {
        for (int t = 0; t < 8; ++t)
            for (int i = 0; i < 8; ++i) b[t][i] = (uint32_t)gf2_table_entry(1u << i, t, POLY);
    }
};
// the bases of T_tl and T_(tl + 4) for a per-lane tl < 4, in registers: the selects are made over
// register copies of the constants (the compiler had turned B.b[tl][b] into indexed loads from a
// constant array in global memory -- a dependent memory round trip before every table build)
template <uint32_t POLY>
__device__ __forceinline__ void lane_w8_basis(uint32_t tl, uint32_t (&bl)[8], uint32_t (&bh)[8]) {
    constexpr LaneW8Basis<POLY> B{};
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        uint32_t c[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            c[t] = B.b[t][b];
            asm volatile("" : "+v"(c[t]));  // opaque: a register, not a table entry
        }
        bl[b] = tl == 0 ? c[0] : tl == 1 ? c[1] : tl == 2 ? c[2] : c[3];
        bh[b] = tl == 0 ? c[4] : tl == 1 ? c[5] : tl == 2 ? c[6] : c[7];
    }
}
// the 64 KiB table image from a 256-thread workgroup, 16 ds_write_b128 per thread.  Store k of thread
// i writes entry e = (i >> 3) + 32 (k >> 1), table t = ((i & 7) >> 1) + 4 (k & 1), copies 4 (i & 1)..+3,
// so the eight lanes of each ds_write_b128 lane group cover the 128 bytes of all 32 banks once (16
// bytes at (2 t + (i & 1)) mod 8 of a 128-byte line).  Round 4: thread e writing its own row made
// every group 8-way conflicted -- 8,000 conflict cycles per CU before the first message.
template <uint32_t POLY>
__device__ __forceinline__ void lane_w8_tables(char *lds) {
    const uint32_t i = threadIdx.x, tl = (i & 7u) >> 1, half = i & 1u;
    uint32_t bl[8], bh[8];  // the bases of T_tl and T_(tl + 4)
    lane_w8_basis<POLY>(tl, bl, bh);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t e = (i >> 3) + 32u * (uint32_t)(k >> 1), t = tl + 4u * (uint32_t)(k & 1);
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 8; ++b) v ^= ((e >> b) & 1u) ? ((k & 1) ? bh[b] : bl[b]) : 0u;
        *(uint4 *)(lds + (e << 8) + (t << 5) + (half << 4)) = make_uint4(v, v, v, v);
    }
    __syncthreads();
}
struct LaneW8 {
    const char *L;
    uint32_t cst8[8], sel8[8], c4;
    __device__ void init(const char *lds, uint32_t lane) {  // Braid32W8::init's schedule
        L = lds;
        const uint32_t j = (lane >> 3) & 3u, c = lane & 7u;
        c4 = c << 2;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t q = (k + j) & 3u;
            cst8[k] = ((7u - q) << 5) | (c << 2);
            cst8[4 + k] = ((3u - q) << 5) | (c << 2);
            sel8[k] = sel8[4 + k] = 0x0c0c0004u | (q << 8);  // byte0 <- cst, byte1 <- byte q of the dword
        }
    }
    __device__ __forceinline__ uint32_t word(uint32_t s, uint64_t v) const {
        const uint32_t lo = (uint32_t)v ^ s, hi = (uint32_t)(v >> 32);
        uint32_t x[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            x[k] = lds32(L, __builtin_amdgcn_perm(cst8[k], lo, sel8[k]));
            x[4 + k] = lds32(L, __builtin_amdgcn_perm(cst8[4 + k], hi, sel8[4 + k]));
        }
        return xor3(xor3(x[0], x[1], x[2]), xor3(x[3], x[4], x[5]), x[6] ^ x[7]);
    }
    __device__ __forceinline__ uint32_t bytes(uint32_t s, uint64_t v, uint32_t nb) const {  // T_0, copy c
        for (uint32_t j = 0; j < nb; ++j, v >>= 8) s = (s >> 8) ^ lds32(L, ((((s ^ (uint32_t)v) & 0xffu)) << 8) | c4);
        return s;
    }
};

// register s advanced over [ptr, ptr + n).  All loads are aligned 8-byte words: the unaligned head
// and the tail come from the aligned words that contain them (never past their page), so a short
// buffer costs a few independent loads, not a serial chain of byte loads; whole words go eight loads
// at a time before their slice-by-8 steps.
template <class T, class F>
__device__ __forceinline__ T lane_scan(T s, const uint8_t *ptr, uint64_t n, const F &f) {
    if (n == 0) return s;
    const uintptr_t a = (uintptr_t)ptr;
    const uint64_t *w = (const uint64_t *)(a & ~(uintptr_t)7);
    const uint32_t o = (uint32_t)(a & 7);
    if (o) {
        const uint32_t hb = n < 8 - o ? (uint32_t)n : 8 - o;
        s = f.bytes(s, *w++ >> (8 * o), hb);
        n -= hb;
    }
    uint64_t k = n >> 3;
    // 16 bytes per lane per load instruction: the lanes of a wave read 64 different buffers, so the
    // instruction count per byte (one cache-line request per lane), not bandwidth, bounds the loads.
    // Software-pipelined (round 4): the next 64 bytes' loads are in flight while the current 64 are
    // folded.  (Deeper rings -- 2, 4, 8 steps in flight -- measured slower: profiles/r04/f.)
    typedef uint64_t u64x2 __attribute__((ext_vector_type(2), aligned(8)));
    auto load8 = [](const uint64_t *p, uint64_t *v) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u64x2 x = *(const __attribute__((address_space(1))) u64x2 *)(p + 2 * j);
            v[2 * j] = x.x;
            v[2 * j + 1] = x.y;
        }
    };
    if (k >= 8) {
        uint64_t v[8], nv[8];
        load8(w, v);
        w += 8;
        k -= 8;
        auto fold8 = [&](const uint64_t *x) {
#pragma unroll
            for (int j = 0; j < 8; ++j) s = f.word(s, x[j]);
        };
        for (; k >= 8; k -= 8, w += 8) {
            load8(w, nv);
            fold8(v);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = nv[j];
        }
        fold8(v);
    }
    if (k >= 4) {
        const uint64_t v0 = w[0], v1 = w[1], v2 = w[2], v3 = w[3];
        s = f.word(s, v0);
        s = f.word(s, v1);
        s = f.word(s, v2);
        s = f.word(s, v3);
        k -= 4;
        w += 4;
    }
    for (; k; --k) s = f.word(s, *w++);
    if (n & 7) s = f.bytes(s, *w, (uint32_t)(n & 7));
    return s;
}

// one lane per buffer: W = 32 on the conflict-free 8-copy tables, W = 64 on plain tables
template <class T, T POLY>
__global__ __launch_bounds__(256) void crc_lanes_kernel(const LaneParams p) {
    constexpr bool w8 = sizeof(T) == 4;
    __shared__ __attribute__((aligned(16))) char lds[w8 ? kLaneW8Lds : 8 * 256 * sizeof(T)];
    TabFold<T> tf{(const T (*)[256])lds};
    LaneW8 lw;
    if constexpr (w8) {
        lane_w8_tables<(uint32_t)POLY>(lds);
        lw.init(lds, threadIdx.x & 63u);
    } else {
        lane_tables<T, POLY>((T (*)[256])lds);
    }
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.nbuf) return;
    const uint8_t *ptr;
    uint64_t n, ix = b;
    const void *seeds = p.d_seeds;
    void *out = p.d_out;
    if (p.d_ptrs) {
        ptr = (const uint8_t *)p.d_ptrs[b];
        n = p.d_lens[b];
    } else {  // strided batches
        // the batch index differs between lanes: read the descriptors through the kernarg segment
        // (an indexed read of the by-value parameter would copy the whole block to scratch)
        const LaneParams *kp = (const LaneParams *)__builtin_amdgcn_kernarg_segment_ptr();
        const uint64_t j = udiv_u(b, p.bcount);
        ix = b - j * p.bcount;
        ptr = (const uint8_t *)(kp->bbase[j] + ix * p.stride);
        n = p.len;
        seeds = (const void *)kp->bseed[j];
        out = (void *)kp->bout[j];
    }
    uint64_t seed = p.seed_all;
    if (seeds) seed = sizeof(T) == 4 ? (uint64_t)((const uint32_t *)seeds)[ix] : ((const uint64_t *)seeds)[ix];
    T s;
    if constexpr (w8)
        s = (T)lane_scan<uint32_t>((uint32_t)~seed, ptr, n, lw);
    else
        s = lane_scan<T>((T)~seed, ptr, n, tf);
    ((T *)out)[ix] = (T)~s;
}

// Event-stream framing check, one lane per message (aws_crt_amd_eventstream_crcs): the lane reads
// total_length and headers_length from the message's prelude (big-endian), refuses lengths outside
// [16, limit - offset] and headers longer than total - 16 before touching the body, then folds the
// prelude (-> prelude CRC) and continues over the headers and payload (-> message CRC, the running
// form of CRC32 over [0, total - 4)), and compares both with the big-endian values stored at offset 8
// and total - 4.  Folds on the conflict-free tables (LaneW8).  Measured and dropped in round 4
// (profiles/r04/f-s; the code is in git history, commit baaa268): deeper load rings
// (37-39 us against 28-29), four lanes per message on a quad braid (52-54 us), a lane pair per message
// (42 us; 35 us with 512-thread workgroups), slice-by-16 (30 us), whole 128-byte line batches (35 us).
__device__ __forceinline__ uint32_t be32(const uint8_t *q) {
    return ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
}

__global__ __launch_bounds__(256) void eventstream_kernel(const EventStreamParams p) {
    __shared__ __attribute__((aligned(16))) char lds[kLaneW8Lds];
    lane_w8_tables<kPoly32>(lds);
    LaneW8 f;
    f.init(lds, threadIdx.x & 63u);
    const uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= p.count) return;
    const uint64_t off = p.d_offsets[m];
    uint32_t pre = 0, msg = 0, st = 4u;  // bit 2: malformed
    if (off <= p.limit && p.limit - off >= 16) {
        const uint8_t *q = p.base + off;
        const uint64_t total = be32(q), headers = be32(q + 4);
        // aws-c-event-stream's decoder refuses a prelude whose headers do not fit the message
        // (headers_length > total_length - 16): malformed, whatever the CRCs say
        if (total >= 16 && total <= p.limit - off && headers <= total - 16) {
            uint32_t s = lane_scan<uint32_t>(~0u, q, 8, f);
            pre = ~s;
            s = lane_scan<uint32_t>(s, q + 8, total - 12, f);
            msg = ~s;
            st = (be32(q + 8) == pre ? 1u : 0u) | (be32(q + total - 4) == msg ? 2u : 0u);
        }
    }
    p.d_prelude_crc[m] = pre;
    p.d_message_crc[m] = msg;
    p.d_status[m] = st;
}

// ------------------------------------------------------------------------------------------
// Balanced event-stream framing check (round 6).  A wave takes 64
// consecutive messages.  When they are well formed and packed back to back (a stream of frames), the
// wave's region -- the messages' bytes widened to 64-byte alignment -- is cut into 64 equal chunks
// (C bytes, a multiple of 16) and lane l folds chunk l as ONE flat loop of 8-byte words from register
// 0: no masks, no resets, the stored CRCs and each next message's first bytes folded along.  At a
// message's end word the lane records the fold's two halves (lo4: the lookups of bytes 0..3, which
// carry the register; hi4: bytes 4..7); after the loop, message i's CRC is assembled from its record,
// the previous message's record, the lanes' chunk-end registers and a few corrections, all linear
// (tests/test_eventstream_flat_model.py restates the algebra against zlib):
//
//   rec_i = lo4 (a_i <= 4) or lo4 ^ hi4, a_i = e_i - P_i, e_i the span end, P_i its end word
//   Y_i   = word(rec_(i-1) ^ word(0, V1), V2)   V1, V2: the words at B_i = P_(i-1) and B_i + 8 with the
//           previous stored-CRC bytes outside rec_(i-1) and 0xFF over message i's first four bytes
//   Z_i   = rec_i ^ word(0, stored-CRC bytes inside rec_i) ^ Y_i x^(8 (P_i - B_i - 8))
//           ^ sum over the chunks k between: end_k x^(8 (P_i + 8 - c0_(k+1)))
//   CRC_i = ~(Z_i x^(-8 (8 - a_i)))
//
// Products are nibble images of x^(64 v 16^d) (digits 0, 1 and x^(-8 t) in LDS, digits 2, 3 read from
// the image buffer).  The chunks are loaded by lane quads (four lanes read one chunk's 64-byte block:
// 16 blocks per load instruction, not 64) and handed to their owners through the wave's LDS rows.
// Waves whose messages are malformed, not packed back to back, or span more than kEsMaxRegion take the
// one-lane-per-message path of eventstream_kernel.  Probe: experiments/esload.hip.
constexpr uint32_t kEsBlock = 512;                     // one workgroup of 8 waves per CU
constexpr uint32_t kEsRow = 80;                        // transposition row: 64 B + 16 (bank spread)
constexpr uint32_t kEsMaxRegion = 256u << 10;          // word distances < 32768: four hex digits
constexpr uint32_t kEsLdsImgs = 37;                    // images 0..29 (digits 0, 1), then x^(-8 t)
struct EsWave {
    char rows[64 * kEsRow];
    uint32_t rec[64];           // message i's register at its end word
    uint32_t P[68], endst[64];  // P[64..67]: sentinels
};
constexpr uint32_t kEsLds = kLaneW8Lds + kEsLdsImgs * 512 + (kEsBlock / 64) * sizeof(EsWave);
static_assert(kEsLds <= 160 * 1024, "event-stream LDS");

// r * K for a per-lane K from its nibble image in LDS (entry 16 i + v: nibble i's value v times K)
__device__ __forceinline__ uint32_t es_mul(uint32_t r, const uint32_t *img) {
    uint32_t x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = img[16 * i + ((r >> (28 - 4 * i)) & 15u)];
    return xor3(xor3(x[0], x[1], x[2]), xor3(x[3], x[4], x[5]), x[6] ^ x[7]);
}
__device__ __forceinline__ uint32_t es_mul_g(uint32_t r, gu32 *img) {
    uint32_t x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = img[16 * i + ((r >> (28 - 4 * i)) & 15u)];
    return xor3(xor3(x[0], x[1], x[2]), xor3(x[3], x[4], x[5]), x[6] ^ x[7]);
}
// r * x^(64 m), m < 65536
__device__ __forceinline__ uint32_t es_shift_words(uint32_t r, uint32_t m, const uint32_t *limg, gu32 *gimg) {
    if (m & 15u) r = es_mul(r, limg + 128 * ((m & 15u) - 1));
    if ((m >> 4) & 15u) r = es_mul(r, limg + 128 * (14 + ((m >> 4) & 15u)));
    if ((m >> 8) & 15u) r = es_mul_g(r, gimg + 128 * (29 + ((m >> 8) & 15u)));
    if ((m >> 12) & 15u) r = es_mul_g(r, gimg + 128 * (44 + ((m >> 12) & 15u)));
    return r;
}
__device__ __forceinline__ uint32_t es_word(const LaneW8 &f, uint32_t s, uint64_t v) { return f.word(s, v); }

__global__ __launch_bounds__(kEsBlock) void eventstream_flat_kernel(const EventStreamParams p) {
    __shared__ __attribute__((aligned(16))) char lds[kEsLds];
    // the offsets first: their round trip overlaps the table build below
    const uint64_t m = (uint64_t)blockIdx.x * kEsBlock + threadIdx.x;
    const bool in = m < p.count, has_next = m + 1 < p.count;
    const uint64_t off = in ? p.d_offsets[m] : 0, off_next = has_next ? p.d_offsets[m + 1] : 0;
    {  // tables (the 256-thread build's stores, split over the two halves) and images
        const uint32_t i = threadIdx.x & 255u, tl = (i & 7u) >> 1, half = i & 1u, k0 = 8u * (threadIdx.x >> 8);
        uint32_t bl[8], bh[8];
        lane_w8_basis<kPoly32>(tl, bl, bh);
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
            const uint32_t k = k0 + kk, e = (i >> 3) + 32u * (k >> 1), t = tl + 4u * (k & 1);
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 8; ++b) v ^= ((e >> b) & 1u) ? ((k & 1) ? bh[b] : bl[b]) : 0u;
            *(uint4 *)(lds + (e << 8) + (t << 5) + (half << 4)) = make_uint4(v, v, v, v);
        }
        v4u *li = (v4u *)(lds + kLaneW8Lds);
        for (uint32_t j = threadIdx.x; j < kEsLdsImgs * 32; j += kEsBlock)
            li[j] = ((gv4u *)p.d_imgs)[j < 30 * 32 ? j : j + 30 * 32];
    }
    __syncthreads();
    LaneW8 f;
    const uint32_t lane = threadIdx.x & 63u;
    f.init(lds, lane);
    const uint32_t *limg = (const uint32_t *)(lds + kLaneW8Lds);
    EsWave &W = ((EsWave *)(lds + kLaneW8Lds + kEsLdsImgs * 512))[threadIdx.x >> 6];

    const uint8_t *q = p.base + off;
    // the prelude's first 12 bytes from the four aligned dwords holding them (issued now, used after
    // the scan on the flat path)
    const bool readable = in && off <= p.limit && p.limit - off >= 16;
    // and the 4 bytes in front of it (a packed stream's previous stored CRC): 20 bytes from the aligned
    // dword at q - 4 in one 16-byte and one 4-byte load (round 6: six dword loads here, each one 64
    // scattered lines per wave, cost ~2 us of the 26 us call)
    typedef v4u v4u_a4 __attribute__((aligned(4)));
    uint32_t pd[4] = {0, 0, 0, 0}, prevraw = 0;
    const uint32_t qo = (uint32_t)((uintptr_t)q & 3u);
    const bool back = off >= 4;
    uint32_t px[5] = {0, 0, 0, 0, 0};
    if (readable) {
        const uintptr_t ea = ((uintptr_t)q - (back ? 4 : 0)) & ~(uintptr_t)3;
        const v4u x = *(const __attribute__((address_space(1))) v4u_a4 *)ea;
        px[0] = x.x, px[1] = x.y, px[2] = x.z, px[3] = x.w;
        px[4] = *(gu32 *)(ea + (back ? 16 : 12));  // (without the 4 bytes in front: never past the 16 bytes)
    }
    auto prelude_words = [&]() {  // the prelude's dwords (pd) and the 4 bytes in front of the message
#pragma unroll
        for (int j = 0; j < 4; ++j) pd[j] = back ? px[j + 1] : px[j];
        prevraw = back ? __builtin_amdgcn_alignbyte(px[1], px[0], qo) : 0u;
    };
    // the lane path: lengths from the preludes, one lane per message (eventstream_kernel's walk)
    auto lane_path = [&]() {
        if (!in) return;
        prelude_words();
        uint32_t pre = 0, msg = 0, st = 4u;
        if (readable) {
            const uint32_t b0 = __builtin_amdgcn_alignbyte(pd[1], pd[0], qo), b1 = __builtin_amdgcn_alignbyte(pd[2], pd[1], qo);
            const uint32_t b2 = __builtin_amdgcn_alignbyte(pd[3], pd[2], qo);
            const uint32_t total = __builtin_bswap32(b0), headers = __builtin_bswap32(b1);
            if (total >= 16 && total <= p.limit - off && headers <= total - 16) {
                const uint32_t s8 = f.word(~0u, (uint64_t)b0 | (uint64_t)b1 << 32);
                pre = ~s8;
                msg = ~lane_scan<uint32_t>(s8, q + 8, total - 12, f);
                const uintptr_t x = (uintptr_t)(q + total - 4), xa = x & ~(uintptr_t)3;
                const uint32_t stored = __builtin_bswap32(__builtin_amdgcn_alignbyte(*(gu32 *)(xa + ((x & 3u) ? 4 : 0)), *(gu32 *)xa, (uint32_t)(x & 3u)));
                st = (__builtin_bswap32(b2) == pre ? 1u : 0u) | (stored == msg ? 2u : 0u);
            }
        }
        p.d_prelude_crc[m] = pre;
        p.d_message_crc[m] = msg;
        p.d_status[m] = st;
    };
    // The flat path is taken on the offsets alone (the preludes are still in flight): every message
    // of the wave followed by the next one's offset, at least 16 bytes apart, the region bounded and
    // readable.  Message i's length is then off_(i+1) - off_i; once the first block's loads are issued the preludes must agree
    // (total_length equal to it, headers within it), or the wave is redone on the lane path.
    const uint64_t off0 = __shfl(off, 0), end63 = __shfl(off_next, 63);
    const bool flat = __all(in && has_next && off_next >= off + 16 && off_next - off <= 0xffffffffull && end63 <= p.limit &&
                            end63 - off0 <= kEsMaxRegion);
    if (!flat) {
        lane_path();
        return;
    }
    const uint32_t total = (uint32_t)(off_next - off);
    // wave-uniform values in SGPRs (the shuffles' results are VGPRs to the compiler)
    const uintptr_t rs = rfl64((uintptr_t)(p.base + off0) & ~(uintptr_t)15);  // 16-aligned: message 0 starts < 16 in
    const uint32_t s_i = (uint32_t)((uintptr_t)q - rs), e_i = s_i + total - 4;
    const uint32_t P_i = (e_i - 1) & ~7u, a_i = e_i - P_i;
    // region end relative to rs, 16-aligned (so never past the page of the last message's last byte)
    const uint32_t re = __builtin_amdgcn_readfirstlane((__shfl(e_i, 63) + 4 + 15) & ~15u);
    const uint32_t C = (((re + 63) >> 6) + 15) & ~15u;  // 64 C >= re, C a multiple of 16
    const uint32_t nb = (C + 63) >> 6, wl = (C & 63u) ? (C & 63u) >> 3 : 8u;
    const uint32_t c0 = lane * C;
    // the ends, ascending: P in bits 0..23, a in bits 24..31; sentinels past the last
    W.P[lane] = P_i | a_i << 24;
    if (lane < 4) W.P[64 + lane] = 0x00ffffffu;
    constexpr uint32_t kPMask = 0x00ffffffu;
    // the lane's first end at or after its chunk start
    uint32_t i0 = (W.P[63] & kPMask) < c0 ? 64u : 0u;
    if (i0 == 0)
#pragma unroll
        for (uint32_t sp = 32; sp; sp >>= 1)
            if ((W.P[i0 + sp - 1] & kPMask) < c0) i0 += sp;
    // the next four ends (a 64-byte block holds at most four: spans of >= 12 bytes, 4-byte gaps)
    uint32_t pw[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) pw[j] = W.P[i0 + j];

    // the stored message CRC: in front of the next message (its lane loaded those 4 bytes); lane 63's
    // own load
    const uintptr_t crc_a = (uintptr_t)(q + total - 4);
    uint32_t crc_lo = 0, crc_hi = 0;
    if (lane == 63) {
        crc_lo = *(gu32 *)(crc_a & ~(uintptr_t)3);
        crc_hi = *(gu32 *)((crc_a & ~(uintptr_t)3) + ((crc_a & 3u) ? 4 : 0));
    }
    const uintptr_t rea = rs + re;
    const uintptr_t qbase = rs + (uintptr_t)(lane >> 2) * C + 16u * (lane & 3u);
    // quad load j of a block step reads chunk 16 j + lane / 4; past the region's last 16 bytes it
    // re-reads the chunk's last readable block (folded as garbage after the last message: harmless)
    uintptr_t qb[4];
    uint32_t qlast[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uintptr_t b0 = qbase + (uintptr_t)(16u * j) * C;
        qb[j] = b0 + 16 <= rea ? b0 : rs + 16u * (lane & 3u);
        qlast[j] = b0 + 16 <= rea ? (uint32_t)((rea - 16 - b0) >> 6) : 0u;
    }
    auto qaddr = [&](uint32_t j, uint32_t b) { return qb[j] + ((uintptr_t)min(b, qlast[j]) << 6); };
    v4u v[4], nv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = *(gv4u *)qaddr(j, 0);
    prelude_words();
    {  // the preludes (issued before these loads, so they land first) must agree with the offsets
        const uint32_t b0 = __builtin_amdgcn_alignbyte(pd[1], pd[0], qo), b1 = __builtin_amdgcn_alignbyte(pd[2], pd[1], qo);
        if (!__all(__builtin_bswap32(b0) == total && __builtin_bswap32(b1) <= total - 16)) {
            lane_path();
            return;
        }
    }
    const uint32_t nraw = __shfl_down(prevraw, 1);
    const uint32_t raw = lane == 63 ? __builtin_amdgcn_alignbyte(crc_hi, crc_lo, (uint32_t)(crc_a & 3u)) : nraw;  // in memory order

    // This message's end patch: the stored CRC's four bytes at [e_i, e_i + 4) XORed with themselves
    // (cleared) and the next message's first four bytes XORed with 0xFF (CRC32's ~0 start), so that
    // with the register reset at each end word every record is its message's own register.  The three
    // dwords are XORed into their owners' LDS rows (ds_xor) in the block step that holds them.
    uint32_t pt_b[3], pt_a[3], pt_x[3];
    {
        const uint64_t pat = (uint64_t)raw | 0xffffffff00000000ull;  // bytes e_i .. e_i + 7
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const uint32_t y = (e_i & ~3u) + 4u * d;
            const int rel = (int)y - (int)e_i;
            pt_x[d] = rel >= 8 ? 0u : rel >= 0 ? (uint32_t)(pat >> (8 * rel)) : (uint32_t)(pat << (-8 * rel));
            const uint32_t o = y / C, yo = y - o * C;
            pt_b[d] = rel < 8 && o < 64 ? yo >> 6 : ~0u;  // the block step, or never
            pt_a[d] = (uint32_t)(o * kEsRow + (yo & 63u)) >> 2;  // a dword of the owner's row
        }
    }


    char *wrow = W.rows + (lane >> 2) * kEsRow + 16 * (lane & 3);
    const char *rrow = W.rows + lane * kEsRow;
    uint32_t *rows32 = (uint32_t *)W.rows;
    const uint32_t s0 = __builtin_amdgcn_readfirstlane(__shfl(s_i, 0));  // message 0's start (< 16)
    uint32_t u = 0;
    // one block's words.  Bit k of `ends`: word k is an end word; its record (lo4 for a <= 4, which
    // leaves the next message's head in hi4, else lo4 ^ hi4) goes to message r0 + (the ends before
    // it) and the register restarts with hi4 or 0.  FEW: no lane has two ends in the block (two need
    // a message of < 64 bytes): the end word is handled by selects and the record stored after the
    // block, so the fold is straight-line code.
    auto fold_words = [&](auto few_c, const v4u(&w)[4], uint32_t ends, uint32_t r0, auto nw) {
        constexpr bool few = decltype(few_c)::value;
        const uint32_t kend = ends ? (uint32_t)__builtin_ctz(ends) : 8u;
        const uint32_t m5 = (pw[0] >> 24) >= 5 ? ~0u : 0u;  // FEW: the block's end (window entry 0)
        uint32_t rv = 0;
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
            if (k < nw) {
                const uint32_t lo = w[k >> 1][2 * (k & 1)] ^ u, hi = w[k >> 1][2 * (k & 1) + 1];
                uint32_t x[8];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    x[t] = lds32(f.L, __builtin_amdgcn_perm(f.cst8[t], lo, f.sel8[t]));
                    x[4 + t] = lds32(f.L, __builtin_amdgcn_perm(f.cst8[4 + t], hi, f.sel8[4 + t]));
                }
                const uint32_t lo4 = xor3(x[0], x[1], x[2]) ^ x[3], hi4 = xor3(x[4], x[5], x[6]) ^ x[7];
                if constexpr (few) {  // selects only (no asm: the compiler would branch around it)
                    const bool hit = k == kend;
                    const uint32_t rec = lo4 ^ (hi4 & m5), nxt = hi4 & ~m5, run = lo4 ^ hi4;
                    rv = hit ? rec : rv;
                    u = hit ? nxt : run;
                } else {
                    if ((ends >> k) & 1u) {
                        const uint32_t j = __builtin_popcount(ends & ((1u << k) - 1u));
                        const uint32_t pj = j == 0 ? pw[0] : j == 1 ? pw[1] : j == 2 ? pw[2] : pw[3];
                        const bool a5 = (pj >> 24) >= 5;
                        W.rec[r0 + j] = a5 ? lo4 ^ hi4 : lo4;
                        u = a5 ? 0u : hi4;
                    } else {
                        u = lo4 ^ hi4;
                    }
                }
            }
        }
        if constexpr (few) {
            if (ends) W.rec[r0] = rv;
        }
    };
    using few_t = std::integral_constant<bool, true>;
    using many_t = std::integral_constant<bool, false>;
    for (uint32_t b = 0; b < nb; ++b) {
#pragma unroll
        for (int j = 0; j < 4; ++j) nv[j] = *(gv4u *)qaddr(j, b + 1);  // unconditional: exact vmcnt waits
#pragma unroll
        for (int j = 0; j < 4; ++j) *(v4u *)(wrow + j * 16 * kEsRow) = v[j];
#pragma unroll
        for (int d = 0; d < 3; ++d)
            if (pt_b[d] == b) __hip_atomic_fetch_xor(rows32 + pt_a[d], pt_x[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        v4u w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = *(const v4u *)(rrow + 16 * j);
        if (b == 0) {  // the bytes in front of message 0 (< 16) cleared, its first four flipped (~0 start)
#pragma unroll
            for (int d = 0; d < 5; ++d) {
                const int rel = (int)(c0 + 4 * d) - (int)s0;
                const uint32_t keep = rel >= 0 ? ~0u : rel <= -4 ? 0u : ~0u << (-8 * rel);
                const uint32_t flip = rel >= 4 || rel <= -4 ? 0u : rel >= 0 ? 0xffffffffu >> (8 * rel) : 0xffffffffu << (-8 * rel);
                w[d >> 2][d & 3] = (w[d >> 2][d & 3] & keep) ^ flip;
            }
        }
        const uint32_t bs = c0 + 64 * b, be = min(bs + 64, c0 + C);
        uint32_t ends = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t pj = pw[j] & kPMask;
            ends |= pj < be ? 1u << ((pj - bs) >> 3) : 0u;
        }
        const uint32_t r0 = i0;
        const uint32_t nw = b + 1 < nb ? 8u : wl;
        if (__any(ends & (ends - 1)))
            fold_words(many_t(), w, ends, r0, nw);
        else if (nw == 8)
            fold_words(few_t(), w, ends, r0, std::integral_constant<uint32_t, 8>());
        else
            fold_words(few_t(), w, ends, r0, nw);
        i0 += __builtin_popcount(ends);
#pragma unroll
        for (int j = 0; j < 4; ++j) pw[j] = W.P[i0 + j];  // the next block's window
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = nv[j];
    }
    W.endst[lane] = u;
    __builtin_amdgcn_wave_barrier();

    // message `lane`: its record, plus the pieces of the chunks it began in (chunks lane(B) ..
    // lane(P_i) - 1, B = the previous end word or message 0's first word), moved to its end word;
    // then the end word's overshoot past e_i taken off
    const uint32_t b0 = __builtin_amdgcn_alignbyte(pd[1], pd[0], qo), b1 = __builtin_amdgcn_alignbyte(pd[2], pd[1], qo);
    const uint32_t b2 = __builtin_amdgcn_alignbyte(pd[3], pd[2], qo);
    const uint32_t pre = ~f.word(~0u, (uint64_t)b0 | (uint64_t)b1 << 32);
    uint32_t st = __builtin_bswap32(b2) == pre ? 1u : 0u;
    uint32_t z = (uint32_t)W.rec[lane];
    const uint32_t B = lane ? (W.P[lane - 1] & kPMask) : 0u;
    gu32 *gimg = (gu32 *)p.d_imgs;
    for (uint32_t k = B / C, kp = P_i / C; k < kp; ++k) z ^= es_shift_words(W.endst[k], (P_i + 8 - (k + 1) * C) >> 3, limg, gimg);
    if (a_i < 8) z = es_mul(z, limg + 128 * (30 + (7 - a_i)));  // x^(-8 (8 - a_i))
    const uint32_t msg = ~z;
    st |= __builtin_bswap32(raw) == msg ? 2u : 0u;
    p.d_prelude_crc[m] = pre;
    p.d_message_crc[m] = msg;
    p.d_status[m] = st;
}

}  // namespace

#if AWS_CRT_AMD_DIAG  // diagnostic library only (lib/libaws-crt-cpp-amd-diag.so)
// ------------------------------------------------------------------------------------------
// Streaming-read ceiling (diagnostics; SURVEY.md §8(d) "secondary denominator"): the W=32 streaming
// scan's launch shape with the CRC removed -- 512-thread workgroups, one per CU, each wave a
// contiguous slab read as 256-byte non-temporal rows, two 16-row groups in flight, XOR-reduced.
// What an HBM-bound kernel of this shape can reach for the same bytes per launch.
__global__ __launch_bounds__(kBraidBlock) void read_ceiling_kernel(const uint8_t *base, uint64_t bytes, uint32_t *sink) {
    constexpr int D = kBraidRowsPerGroup;
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * kBraidWaves, gw = (uint64_t)blockIdx.x * kBraidWaves + (threadIdx.x >> 6);
    const uint64_t rows = bytes / kBraidRow, r0 = udiv_u(gw * rows, nw), r1 = udiv_u((gw + 1) * rows, nw);
    const uint64_t a0 = (uint64_t)base + r0 * kBraidRow + 4u * lane;
    const uint64_t ng = (r1 - r0) / D;
    uint32_t s0[D], s1[D], acc = 0;
    auto ld = [&](uint32_t *s, uint64_t g) {
#pragma unroll
        for (int i = 0; i < D; ++i) s[i] = __builtin_nontemporal_load((gu32 *)(a0 + (g * D + i) * kBraidRow));
    };
    auto use = [&](const uint32_t *s) {
#pragma unroll
        for (int i = 0; i < D; ++i) acc = acc * 3u ^ s[i];
    };
    if (ng) ld(s0, 0);
    for (uint64_t g = 0; g < ng;) {
        if (g + 1 < ng) ld(s1, g + 1);
        use(s0);
        if (++g >= ng) break;
        if (g + 1 < ng) ld(s0, g + 1);
        use(s1);
        ++g;
    }
    if (acc == 0x9E3779B9u) sink[gw] = acc;  // keeps the loads live; practically never stored
}

extern "C" int amdcrc_launch_read_ceiling(const void *base, uint64_t bytes, uint32_t *sink, int nblocks, void *stream,
                                          void *const *ev) {
    struct Args {
        const uint8_t *b;
        uint64_t n;
        uint32_t *s;
    } a{(const uint8_t *)base, bytes, sink};
    hipStream_t s = (hipStream_t)stream;
    if (ev && (ev[0] || ev[1]))
        hipExtLaunchKernelGGL(read_ceiling_kernel, dim3(nblocks), dim3(kBraidBlock), 0, s, (hipEvent_t)ev[0], (hipEvent_t)ev[1], 0,
                              a.b, a.n, a.s);
    else
        hipLaunchKernelGGL(read_ceiling_kernel, dim3(nblocks), dim3(kBraidBlock), 0, s, a.b, a.n, a.s);
    return (int)hipGetLastError();
}

#if AWS_CRT_AMD_DIAG
// Diagnostic library only: crc32_stream_kernel writes its per-wave timeline to d_buf (kStampWords words
// per wave; null turns the stamps off).  Returns 0 on success.
extern "C" __attribute__((visibility("default"))) int aws_crt_amd_debug_scan_stamps(void *d_buf) {
    uint64_t *p = (uint64_t *)d_buf;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_scan_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
// Debug builds (-DAMDCRC_GUARD): read and clear the streaming scan's guard record
extern "C" __attribute__((visibility("default"))) int amdcrc_debug_guard(unsigned long long *out4) {
#ifdef AMDCRC_GUARD
    if (hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_amdcrc_guard), sizeof(unsigned long long) * 4) != hipSuccess) return -1;
    unsigned long long z[4] = {0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_amdcrc_guard), z, sizeof(z)) == hipSuccess ? 1 : -1;
#else
    (void)out4;
    return 0;
#endif
}
#endif
#endif  // AWS_CRT_AMD_DIAG

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

// Scan launch.  ev[0] / ev[1] (diagnostics, may be null): HIP events stamped with the dispatch's own
// start / end time (hipExtLaunchKernel), i.e. the interval a kernel-trace profiler reports.
template <typename K, typename P, typename... A>
static void launch(K kernel, int nblocks, int threads, hipStream_t s, const P *p, void *const *ev, A... extra) {
    if (ev && (ev[0] || ev[1]))
        hipExtLaunchKernelGGL(kernel, dim3(nblocks), dim3(threads), 0, s, (hipEvent_t)ev[0], (hipEvent_t)ev[1], 0, *p,
                              extra...);
    else
        hipLaunchKernelGGL(kernel, dim3(nblocks), dim3(threads), 0, s, *p, extra...);
}

extern "C" int amdcrc_launch_scan(int alg, const ScanParams *p, int nblocks, void *stream, void *const *ev) {
    hipStream_t s = (hipStream_t)stream;
    const bool list = p->list_mode != 0;
    switch (alg) {
        case ALG_CRC32:
#if AMDCRC_STREAM_W16
            if (p->stream == 2 && !list)
                launch(crc32_stream_kernel<kPoly32, 16>, nblocks, kW16Block, s, p, ev);
            else
#endif
            if (p->stream && !list)
                p->xcd_order ? launch(crc32_stream_kernel<kPoly32, 8, true>, nblocks, kBraidBlock, s, p, ev)
                             : launch(crc32_stream_kernel<kPoly32, AMDCRC_STREAM_W8 ? 8 : 4>, nblocks, kBraidBlock, s, p, ev);
            else if (list && p->stream == 4)
                launch(crc32_list_stream_kernel<kPoly32>, nblocks, kBraidBlock, s, p, ev);
            else if (list)
                launch(crc32_braid_kernel<kPoly32, true>, nblocks, kBraidBlock, s, p, ev);
            else
                launch(crc32_braid_kernel<kPoly32, false>, nblocks, kBraidBlock, s, p, ev);
            break;
        case ALG_CRC32C:
#if AMDCRC_STREAM_W16
            if (p->stream == 2 && !list)
                launch(crc32_stream_kernel<kPoly32C, 16>, nblocks, kW16Block, s, p, ev);
            else
#endif
            if (p->stream && !list)
                p->xcd_order ? launch(crc32_stream_kernel<kPoly32C, 8, true>, nblocks, kBraidBlock, s, p, ev)
                             : launch(crc32_stream_kernel<kPoly32C, AMDCRC_STREAM_W8 ? 8 : 4>, nblocks, kBraidBlock, s, p, ev);
            else if (list && p->stream == 4)
                launch(crc32_list_stream_kernel<kPoly32C>, nblocks, kBraidBlock, s, p, ev);
            else if (list)
                launch(crc32_braid_kernel<kPoly32C, true>, nblocks, kBraidBlock, s, p, ev);
            else
                launch(crc32_braid_kernel<kPoly32C, false>, nblocks, kBraidBlock, s, p, ev);
            break;
        case ALG_CRC64NVME:
            if (p->stream == 3 && !list)  // many short buffers: 16 lanes per buffer
                launch(crc64_rows16_kernel<kPoly64Nvme>, nblocks, kR16Block, s, p, ev);
            else if (p->stream == 5 && !list && p->xcd_pad)  // long buffers: XCD-window chunks, front pads
                launch(crc64_xcd_kernel<kPoly64Nvme, kXcdBlock, true>, nblocks, kXcdBlock, s, p, ev);
            else if (p->stream == 5 && !list)  // long buffers of whole chunks
                p->nbatch > 1 ? launch(crc64_xcd_kernel<kPoly64Nvme, kXcdBlock, false, true>, nblocks, kXcdBlock, s, p, ev)
                              : launch(crc64_xcd_kernel<kPoly64Nvme, kXcdBlock, false>, nblocks, kXcdBlock, s, p, ev);
            else if (p->stream && !list)  // 4-copy tables
                launch(crc64_stream4_kernel<kPoly64Nvme, kW64StreamBlock>, nblocks, kW64StreamBlock, s, p, ev);
            else if (list && p->stream == 4)  // ragged lists: the list streaming scan
                launch(crc64_list_stream_kernel<kPoly64Nvme>, nblocks, 512, s, p, ev);
            else if (list)
                launch(crc64_braid_kernel<kPoly64Nvme, true>, nblocks, kBlock, s, p, ev);
            else
                launch(crc64_braid_kernel<kPoly64Nvme, false>, nblocks, kBlock, s, p, ev);
            break;
        default: return -1;
    }
    return (int)hipGetLastError();
}

extern "C" int amdcrc_launch_lanes(int alg, const LaneParams *p, void *stream, void *const *ev) {
    const uint64_t blocks = (p->nbuf + 255) / 256;
    if (blocks == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    switch (alg) {
        case ALG_CRC32: launch(crc_lanes_kernel<uint32_t, kPoly32>, (int)blocks, 256, s, p, ev); break;
        case ALG_CRC32C: launch(crc_lanes_kernel<uint32_t, kPoly32C>, (int)blocks, 256, s, p, ev); break;
        case ALG_CRC64NVME: launch(crc_lanes_kernel<uint64_t, kPoly64Nvme>, (int)blocks, 256, s, p, ev); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

extern "C" int amdcrc_launch_eventstream(const EventStreamParams *p, void *stream, void *const *ev) {
    if (p->count == 0) return 0;
    if (AMDCRC_ES_FLAT && p->d_imgs) {
        launch(eventstream_flat_kernel, (int)((p->count + kEsBlock - 1) / kEsBlock), kEsBlock, (hipStream_t)stream, p, ev);
    } else {
        const uint64_t blocks = (p->count + 255) / 256;
        launch(eventstream_kernel, (int)blocks, 256, (hipStream_t)stream, p, ev);
    }
    return (int)hipGetLastError();
}

// XXH64, one buffer per wave (strided batches of at most one buffer per SIMD): row r of the wave
// (lanes 16 r .. 16 r + 15) runs chain r (accumulator v_(r+1)), replicated over the row; lane t of the
// row loads word r of stripe s0 + t, so one load instruction brings 16 stripes (512 contiguous
// bytes) and their input products form lane-parallel.  Stripe t's product reaches its row by two DPP
// row_newbcast:t moves (VALU, no LDS round trip); the round is xstep_y.
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {  // lane l's value (l wave-uniform)
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}
template <int T>
__device__ __forceinline__ uint64_t row_bcast64(uint64_t v) {
    // bound_ctrl set and every row and bank enabled: every lane reads a live lane, no "old" operand
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, 0x150 + T, 0xF, 0xF, true);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), 0x150 + T, 0xF, 0xF, true);
    return ((uint64_t)hi << 32) | lo;
}
template <int T>
__device__ __forceinline__ void row_rounds(uint32_t &ul, uint32_t &uh, uint64_t y, uint64_t first, uint64_t ns, bool full) {
    if constexpr (T < 16) {
        const uint64_t yt = row_bcast64<T>(y);
        if (full || first + T < ns) xstep_y(ul, uh, yt);  // yt comes through DPP: opaque to re-association
        row_rounds<T + 1>(ul, uh, y, first, ns, full);
    }
}
__global__ __launch_bounds__(64) void xxh64_row_kernel(const XxhParams p) {
    constexpr int DS = 12;  // loads in flight
    const int lane = threadIdx.x, r = lane >> 4, t = lane & 15;
    const uint64_t i = blockIdx.x;
    const uint8_t *ptr = (const uint8_t *)(p.base + i * p.stride);
    const uint64_t n = p.len, seed = p.d_seeds ? p.d_seeds[i] : p.seed_all;
    const uint64_t ns = n / 32, nslot = (ns + 15) / 16;
    uint64_t v = seed + (r == 0 ? XP1 + XP2 : r == 1 ? XP2 : r == 2 ? 0ull : 0ull - XP1);
    const uint8_t *q = ptr + 8 * r;
    auto ld = [&](uint64_t slot) -> uint64_t {
        uint64_t st = slot * 16 + (uint64_t)t;
        st = st < ns ? st : ns - 1;  // the last slot's spare lanes re-read the last stripe
        return ldw(q + 32 * st);
    };
    if (ns > 0) {
        uint64_t x[DS];
#pragma unroll
        for (int d = 0; d < DS; ++d) x[d] = ld(d);
        const uint64_t u0 = rotl64(v * kXP1Inv, 33);  // its round yields v (stripe 0 needs no special case)
        uint32_t ul = (uint32_t)u0, uh = (uint32_t)(u0 >> 32);
        const uint64_t nfull = ns / 16;
        uint64_t slot = 0;
        for (; slot + DS <= nfull; slot += DS) {
#pragma unroll
            for (int d = 0; d < DS; ++d) {
                const uint64_t y = x[d] * XP2;
                x[d] = ld(slot + DS + d);
                row_rounds<0>(ul, uh, y, 0, 0, true);
            }
        }
#pragma unroll
        for (int d = 0; d < DS; ++d)
            if (slot + d < nslot) row_rounds<0>(ul, uh, x[d] * XP2, (slot + d) * 16, ns, false);
        xstep_y(ul, uh, 0);  // the last stripe's round
        v = ((uint64_t)uh << 32) | ul;
    }
    const uint64_t v1 = rl64(v, 0), v2 = rl64(v, 16), v3 = rl64(v, 32), v4 = rl64(v, 48);
    if (lane != 0) return;
    p.d_out[i] = xxh64_finish(v1, v2, v3, v4, ptr, n, seed);
}

extern "C" int amdcrc_launch_xxh64(const XxhParams *p, void *stream, void *const *ev) {
    if (p->nbuf == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    if (!p->d_ptrs) {
        // strided: B buffers per wave, the fewest that keep the launch near one wave per SIMD
        constexpr uint64_t kSimds = 1024;
        auto go = [&](auto kern, uint64_t bper) { launch(kern, (int)((p->nbuf + bper - 1) / bper), 64, s, p, ev); };
        if (p->nbuf <= kSimds) go(xxh64_row_kernel, 1);
        else if (p->nbuf <= 2 * kSimds) go(xxh64_wave_kernel<2>, 2);
        else if (p->nbuf <= 4 * kSimds) go(xxh64_wave_kernel<4>, 4);
        else if (p->nbuf <= 8 * kSimds) go(xxh64_wave_kernel<8>, 8);
        else go(xxh64_wave_kernel<16>, 16);
        return (int)hipGetLastError();
    }
    // lists (ragged lengths): a quad per buffer, the fewest buffers per wave that keep about one
    // wave per SIMD
    const uint64_t bpw = std::min<uint64_t>(16, std::max<uint64_t>(1, (p->nbuf + 1023) / 1024));
    launch(xxh64_quad_kernel, (int)((p->nbuf + bpw - 1) / bpw), 64, s, p, ev, (uint32_t)bpw);
    return (int)hipGetLastError();
}
