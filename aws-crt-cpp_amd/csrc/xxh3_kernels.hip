// XXH3-64 / XXH3-128 (xxHash 0.8 algorithm) on gfx950: one wavefront per buffer, stripe-parallel.
//
// Drop-in for aws_xxhash3_64_compute / aws_xxhash3_128_compute (reference call sites
// source/checksum/XXHash.cpp:22,27; known answers tests/XXHashTest.cpp:44, :73-74).  Every length
// class of the published algorithm is implemented.  Inputs up to 240 bytes are a short serial
// computation (lane 0 of the buffer's wave); longer ones run the stripe-parallel wave loop below
// (SURVEY.md 8(f) rank 3).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include "engine.h"

using namespace amdcrc;

namespace {

__constant__ uint8_t kSecret[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
    0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
    0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
    0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
    0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
    0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
    0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
    0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
    0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
};

constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ull, P64_2 = 0xC2B2AE3D27D4EB4Full, P64_3 = 0x165667B19E3779F9ull,
                   P64_4 = 0x85EBCA77C2B2AE63ull, P64_5 = 0x27D4EB2F165667C5ull;
constexpr uint64_t P32_1 = 0x9E3779B1u, P32_2 = 0x85EBCA77u, P32_3 = 0xC2B2AE3Du;
constexpr uint64_t MX1 = 0x165667919E3779F9ull, MX2 = 0x9FB21C651E98DF25ull;

struct U128 {
    uint64_t lo, hi;
};
typedef uint64_t v2u64 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint64_t rd64(const uint8_t *p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}
__device__ __forceinline__ uint32_t rd32(const uint8_t *p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ U128 mul128(uint64_t a, uint64_t b) { return {a * b, __umul64hi(a, b)}; }
__device__ __forceinline__ uint64_t fold64(uint64_t a, uint64_t b) {
    const U128 m = mul128(a, b);
    return m.lo ^ m.hi;
}
__device__ __forceinline__ uint64_t avalanche3(uint64_t h) {
    h ^= h >> 37;
    h *= MX1;
    return h ^ (h >> 32);
}
__device__ __forceinline__ uint64_t avalanche64(uint64_t h) {
    h ^= h >> 33;
    h *= P64_2;
    h ^= h >> 29;
    h *= P64_3;
    return h ^ (h >> 32);
}
__device__ __forceinline__ uint64_t rrmxmx(uint64_t h, uint64_t len) {
    h ^= rotl64(h, 49) ^ rotl64(h, 24);
    h *= MX2;
    h ^= (h >> 35) + len;
    h *= MX2;
    return h ^ (h >> 28);
}
__device__ __forceinline__ uint64_t mix16(const uint8_t *in, const uint8_t *sec, uint64_t seed) {
    return fold64(rd64(in) ^ (rd64(sec) + seed), rd64(in + 8) ^ (rd64(sec + 8) - seed));
}
__device__ __forceinline__ void mix32(U128 &acc, const uint8_t *a, const uint8_t *b, const uint8_t *sec, uint64_t seed) {
    acc.lo += mix16(a, sec, seed);
    acc.lo ^= rd64(b) + rd64(b + 8);
    acc.hi += mix16(b, sec + 16, seed);
    acc.hi ^= rd64(a) + rd64(a + 8);
}

// long inputs (> 240 bytes): 8 accumulators over 64-byte stripes, scrambled every 1 KiB block
__device__ void long_acc(uint64_t acc[8], const uint8_t *in, uint64_t len, const uint8_t *sec) {
    acc[0] = P32_3, acc[1] = P64_1, acc[2] = P64_2, acc[3] = P64_3;
    acc[4] = P64_4, acc[5] = P32_2, acc[6] = P64_5, acc[7] = P32_1;
    const uint64_t stripes = (192 - 64) / 8, block = 64 * stripes;
    const uint64_t nb = (len - 1) / block;
    auto stripe = [&](const uint8_t *p, const uint8_t *s) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint64_t v = rd64(p + 8 * i), k = v ^ rd64(s + 8 * i);
            acc[i ^ 1] += v;
            acc[i] += (k & 0xFFFFFFFFull) * (k >> 32);
        }
    };
    for (uint64_t n = 0; n < nb; ++n) {
        for (uint64_t s = 0; s < stripes; ++s) stripe(in + n * block + 64 * s, sec + 8 * s);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            uint64_t a = acc[i];
            a ^= a >> 47;
            a ^= rd64(sec + 192 - 64 + 8 * i);
            acc[i] = a * P32_1;
        }
    }
    const uint64_t ns = ((len - 1) - block * nb) / 64;
    for (uint64_t s = 0; s < ns; ++s) stripe(in + nb * block + 64 * s, sec + 8 * s);
    stripe(in + len - 64, sec + 192 - 64 - 7);
}
__device__ uint64_t merge(const uint64_t acc[8], const uint8_t *sec, uint64_t start) {
    uint64_t r = start;
#pragma unroll
    for (int i = 0; i < 4; ++i) r += fold64(acc[2 * i] ^ rd64(sec + 16 * i), acc[2 * i + 1] ^ rd64(sec + 16 * i + 8));
    return avalanche3(r);
}

__device__ void secret_for(uint8_t *out, uint64_t seed) {
    for (int i = 0; i < 12; ++i) {
        const uint64_t lo = rd64(kSecret + 16 * i) + seed, hi = rd64(kSecret + 16 * i + 8) - seed;
        __builtin_memcpy(out + 16 * i, &lo, 8);
        __builtin_memcpy(out + 16 * i + 8, &hi, 8);
    }
}

__device__ uint64_t xxh3_64(const uint8_t *p, uint64_t n, uint64_t seed) {
    const uint8_t *s = kSecret;
    if (n <= 16) {
        if (n > 8) {
            const uint64_t lo = rd64(p) ^ ((rd64(s + 24) ^ rd64(s + 32)) + seed);
            const uint64_t hi = rd64(p + n - 8) ^ ((rd64(s + 40) ^ rd64(s + 48)) - seed);
            return avalanche3(n + __builtin_bswap64(lo) + hi + fold64(lo, hi));
        }
        if (n >= 4) {
            const uint64_t sd = seed ^ ((uint64_t)__builtin_bswap32((uint32_t)seed) << 32);
            const uint64_t in64 = rd32(p + n - 4) + ((uint64_t)rd32(p) << 32);
            return rrmxmx(in64 ^ ((rd64(s + 8) ^ rd64(s + 16)) - sd), n);
        }
        if (n > 0) {
            const uint32_t c = ((uint32_t)p[0] << 16) | ((uint32_t)p[n >> 1] << 24) | p[n - 1] | ((uint32_t)n << 8);
            return avalanche64((uint64_t)c ^ ((uint64_t)(rd32(s) ^ rd32(s + 4)) + seed));
        }
        return avalanche64(seed ^ (rd64(s + 56) ^ rd64(s + 64)));
    }
    if (n <= 128) {
        uint64_t acc = n * P64_1;
        if (n > 32) {
            if (n > 64) {
                if (n > 96) {
                    acc += mix16(p + 48, s + 96, seed);
                    acc += mix16(p + n - 64, s + 112, seed);
                }
                acc += mix16(p + 32, s + 64, seed);
                acc += mix16(p + n - 48, s + 80, seed);
            }
            acc += mix16(p + 16, s + 32, seed);
            acc += mix16(p + n - 32, s + 48, seed);
        }
        acc += mix16(p, s, seed);
        acc += mix16(p + n - 16, s + 16, seed);
        return avalanche3(acc);
    }
    if (n <= 240) {
        uint64_t acc = n * P64_1;
        for (int i = 0; i < 8; ++i) acc += mix16(p + 16 * i, s + 16 * i, seed);
        acc = avalanche3(acc);
        for (int i = 8; i < (int)(n / 16); ++i) acc += mix16(p + 16 * i, s + 16 * (i - 8) + 3, seed);
        acc += mix16(p + n - 16, s + 136 - 17, seed);
        return avalanche3(acc);
    }
    uint8_t custom[192];
    const uint8_t *sec = kSecret;
    if (seed) {
        secret_for(custom, seed);
        sec = custom;
    }
    uint64_t acc[8];
    long_acc(acc, p, n, sec);
    return merge(acc, sec + 11, n * P64_1);
}

__device__ U128 xxh3_128(const uint8_t *p, uint64_t n, uint64_t seed) {
    const uint8_t *s = kSecret;
    if (n <= 16) {
        if (n > 8) {
            const uint64_t bfl = (rd64(s + 32) ^ rd64(s + 40)) - seed, bfh = (rd64(s + 48) ^ rd64(s + 56)) + seed;
            uint64_t ilo = rd64(p), ihi = rd64(p + n - 8);
            U128 m = mul128(ilo ^ ihi ^ bfl, P64_1);
            m.lo += (n - 1) << 54;
            ihi ^= bfh;
            m.hi += ihi + (uint64_t)(uint32_t)ihi * (P32_2 - 1);
            m.lo ^= __builtin_bswap64(m.hi);
            U128 h = mul128(m.lo, P64_2);
            h.hi += m.hi * P64_2;
            return {avalanche3(h.lo), avalanche3(h.hi)};
        }
        if (n >= 4) {
            const uint64_t sd = seed ^ ((uint64_t)__builtin_bswap32((uint32_t)seed) << 32);
            const uint64_t in64 = rd32(p) + ((uint64_t)rd32(p + n - 4) << 32);
            U128 m = mul128(in64 ^ ((rd64(s + 16) ^ rd64(s + 24)) + sd), P64_1 + (n << 2));
            m.hi += m.lo << 1;
            m.lo ^= m.hi >> 3;
            m.lo ^= m.lo >> 35;
            m.lo *= MX2;
            m.lo ^= m.lo >> 28;
            return {m.lo, avalanche3(m.hi)};
        }
        if (n > 0) {
            const uint32_t cl = ((uint32_t)p[0] << 16) | ((uint32_t)p[n >> 1] << 24) | p[n - 1] | ((uint32_t)n << 8);
            const uint32_t sw = __builtin_bswap32(cl);
            const uint32_t ch = (sw << 13) | (sw >> 19);
            return {avalanche64((uint64_t)cl ^ ((uint64_t)(rd32(s) ^ rd32(s + 4)) + seed)),
                    avalanche64((uint64_t)ch ^ ((uint64_t)(rd32(s + 8) ^ rd32(s + 12)) - seed))};
        }
        return {avalanche64(seed ^ (rd64(s + 64) ^ rd64(s + 72))), avalanche64(seed ^ (rd64(s + 80) ^ rd64(s + 88)))};
    }
    U128 acc{n * P64_1, 0};
    if (n <= 128) {
        if (n > 32) {
            if (n > 64) {
                if (n > 96) mix32(acc, p + 48, p + n - 64, s + 96, seed);
                mix32(acc, p + 32, p + n - 48, s + 64, seed);
            }
            mix32(acc, p + 16, p + n - 32, s + 32, seed);
        }
        mix32(acc, p, p + n - 16, s, seed);
    } else if (n <= 240) {
        for (int i = 0; i < 4; ++i) mix32(acc, p + 32 * i, p + 32 * i + 16, s + 32 * i, seed);
        acc.lo = avalanche3(acc.lo);
        acc.hi = avalanche3(acc.hi);
        for (int i = 4; i < (int)(n / 32); ++i) mix32(acc, p + 32 * i, p + 32 * i + 16, s + 3 + 32 * (i - 4), seed);
        mix32(acc, p + n - 16, p + n - 32, s + 136 - 17 - 16, 0ull - seed);
    } else {
        uint8_t custom[192];
        const uint8_t *sec = kSecret;
        if (seed) {
            secret_for(custom, seed);
            sec = custom;
        }
        uint64_t a[8];
        long_acc(a, p, n, sec);
        return {merge(a, sec + 11, n * P64_1), merge(a, sec + 192 - 64 - 11, ~(n * P64_2))};
    }
    const uint64_t rl = acc.lo + acc.hi;
    const uint64_t rh = acc.lo * P64_1 + acc.hi * P64_4 + (n - seed) * P64_2;
    return {avalanche3(rl), 0ull - avalanche3(rh)};
}

// ------------------------------------------------------------------------------------------
// Stripe-parallel XXH3 for long inputs (> 240 bytes): one wavefront per buffer.
//
// The long loop's accumulators only ever add within a 1 KiB block (16 stripes of 64 bytes); the
// nonlinear scramble runs once per block.  So a block is one coalesced wave load (lane l: 16 bytes
// at 16 l = words 2(l&3), 2(l&3)+1 of stripe l>>2), each lane computes its two accumulator
// contributions, the 16 lanes of each residue class mod 4 sum them (64-bit adds over lane
// shuffles), and every lane then updates and scrambles the two accumulators of its class
// (replicated, so the next block needs no broadcast).  The serial part per block is the reduction
// and the scramble; the loads run several blocks ahead.
__device__ __forceinline__ uint64_t cw(int w, uint64_t seed) {  // word w of the (seeded) secret
    return rd64(kSecret + 8 * w) + ((w & 1) ? 0ull - seed : seed);
}
__device__ __forceinline__ uint64_t sec64(int off, uint64_t seed) {  // 8 secret bytes at byte offset off
    const int w = off >> 3, b = off & 7;
    const uint64_t lo = cw(w, seed);
    if (!b) return lo;
    return (lo >> (8 * b)) | (cw(w + 1, seed) << (64 - 8 * b));
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t class_sum(uint64_t v) {  // sum over the 16 lanes with equal lane & 3
    v += shfl_xor64(v, 4);
    v += shfl_xor64(v, 8);
    v += shfl_xor64(v, 16);
    v += shfl_xor64(v, 32);
    return v;
}
__device__ __forceinline__ uint64_t mul32x32(uint64_t k) { return (k & 0xFFFFFFFFull) * (k >> 32); }
constexpr uint64_t inv_odd64(uint64_t a) {  // a^-1 mod 2^64 for odd a (Newton)
    uint64_t x = a;
    for (int k = 0; k < 6; ++k) x *= 2 - a * x;
    return x;
}
constexpr uint64_t kP32_1Inv = inv_odd64(P32_1);
static_assert(kP32_1Inv * P32_1 == 1, "P32_1 inverse");
__device__ __forceinline__ uint64_t scramble1(uint64_t a, uint64_t s) {
    a ^= a >> 47;
    a ^= s;
    return a * P32_1;
}

template <bool ALIGNED>
__device__ __forceinline__ void ld16(const uint8_t *q, uint64_t &a, uint64_t &b) {
    if (ALIGNED) {
        const v2u64 x = *(const __attribute__((address_space(1))) v2u64 *)q;
        a = x.x;
        b = x.y;
    } else {
        a = rd64(q);
        b = rd64(q + 8);
    }
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

// The scramble chain of the split long path over nb blocks' accumulator sums S[8 blk + c], starting
// from accumulator value acc_in (lane l: accumulator c = l & 7, replicated over the lane's 8 groups);
// returns the accumulator after the last block's scramble.  Lane l loads the sum of block g + (l >> 3)
// for its accumulator (one coalesced 512-byte load per 8 blocks, sixteen loads in flight); the
// per-block values reach the lanes of their accumulator by shuffles that do not depend on the
// accumulators.  One scramble chain per lane per block.
__device__ __forceinline__ uint64_t scramble_chain(const uint64_t *S, uint64_t nb, uint64_t acc_in, uint64_t stv, int lane) {
    const int c8 = lane & 7, s8 = lane >> 3;
    const uint64_t accv = acc_in;
    constexpr int G = 8, DS = 16;
    // loads are unconditional (addresses clamped to the last block) so that the wait before a
    // group's shuffles counts only that group's load: DS groups stay in flight
    auto ldg = [&](uint64_t g) -> uint64_t {
        uint64_t blk = g * G + (uint64_t)s8;
        blk = blk < nb ? blk : nb - 1;
        return *(const __attribute__((address_space(1))) uint64_t *)(S + blk * 8 + c8);
    };
    // the chain carries u = acc + v (the next block's sum already added): per block
    //   a = u ^ (u >> 47) ^ key;  u' = a * P32_1 + v_next
    // = one v_xor3 after the shift, then v_mad_u64_u32 (low half, v_next as the addend) beside
    // v_mul_lo_u32 (high half), then one add
    const uint32_t kl = (uint32_t)stv, kh = (uint32_t)(stv >> 32);
    auto step = [&](uint32_t &ul, uint32_t &uh, uint64_t vnext) {
        const uint32_t al = ul ^ (uh >> 15) ^ kl, ah = uh ^ kh;
        uint32_t c = ah * (uint32_t)P32_1;
        asm("" : "+v"(c));  // keep the high product off the low mad's chain
        const uint64_t m = (uint64_t)al * (uint32_t)P32_1 + vnext;
        ul = (uint32_t)m;
        uh = (uint32_t)(m >> 32) + c;
    };
    // start from the state whose step yields accv + v0: a = accv * P^-1, u0 = xorshift^-1(a ^ key)
    // (x ^ (x >> 47) is its own inverse on 64 bits), so every block is the same step
    const uint64_t b0 = (accv * kP32_1Inv) ^ stv, u0 = b0 ^ (b0 >> 47);
    uint32_t ul = (uint32_t)u0, uh = (uint32_t)(u0 >> 32);
    uint64_t ya[G], yb[G];
    auto perm = [&](uint64_t xv, uint64_t (&v)[G]) {
#pragma unroll
        for (int j = 0; j < G; ++j) v[j] = shfl64(xv, 8 * j + c8);
    };
    uint64_t x[DS];
#pragma unroll
    for (int d = 0; d < DS; ++d) x[d] = ldg(d);
    const uint64_t ng = (nb + G - 1) / G, nround = (nb / G) / DS;
    uint64_t g = 0;
    perm(x[0], ya);
    for (uint64_t r = 0; r < nround; ++r, g += DS) {
#pragma unroll
        for (int d = 0; d < DS; ++d) {
            uint64_t (&cur)[G] = (d & 1) ? yb : ya;
            uint64_t (&nxt)[G] = (d & 1) ? ya : yb;
            perm(x[(d + 1) % DS], nxt);  // group g + d + 1 (x[0] already holds g + DS)
            x[d] = ldg(g + DS + d);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < G; ++j) step(ul, uh, cur[j]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // at most DS groups remain (the last may be partial); their sums are in the ring, and the
    // first of them already in ya (DS is even)
#pragma unroll
    for (int d = 0; d < DS; ++d) {
        if (g + d < ng) {
            uint64_t (&cur)[G] = (d & 1) ? yb : ya;
            uint64_t (&nxt)[G] = (d & 1) ? ya : yb;
            if (d + 1 < DS && g + d + 1 < ng) perm(x[d + 1], nxt);
            const uint64_t cnt = nb - (g + d) * G < (uint64_t)G ? nb - (g + d) * G : (uint64_t)G;
#pragma unroll
            for (int j = 0; j < G; ++j)
                if ((uint64_t)j < cnt) step(ul, uh, cur[j]);
        }
    }
    step(ul, uh, 0);  // the last block's scramble
    return ((uint64_t)uh << 32) | ul;
}

// SPLIT: the full blocks' class sums were written by xxh3_blocksum_kernel (64 B per block at
// p.d_sums + 8 (i nb + blk)); this wave only scrambles (scramble_chain: one accumulator per lane,
// against two in the 4-class layout of the one-pass path, halves the serial instruction stream of a
// block).
template <int BITS, bool ALIGNED, bool SPLIT = false>
__device__ void xxh3_long_wave(const XxhParams &p, uint64_t i, const uint8_t *ptr, uint64_t n, uint64_t seed, int lane) {
    const int s = lane >> 2, wp = lane & 3;
    const uint64_t ks0 = sec64(8 * s + 16 * wp, seed), ks1 = sec64(8 * s + 16 * wp + 8, seed);
    const uint64_t st0 = sec64(128 + 16 * wp, seed), st1 = sec64(136 + 16 * wp, seed);
    const uint64_t init[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
    uint64_t acc0 = init[2 * wp], acc1 = init[2 * wp + 1];
    const uint64_t nb = (n - 1) / 1024;
    const uint8_t *q = ptr + 16 * lane;
    uint64_t accv = 0;  // SPLIT: accumulator l & 7
    if (SPLIT) {
        accv = scramble_chain(p.d_sums + i * nb * 8, nb, init[lane & 7], sec64(128 + 8 * (lane & 7), seed), lane);
    } else {
        // D blocks per round: their lane contributions and class sums are independent of the
        // accumulators, so all D reductions issue together and only the scrambles stay serial
        constexpr int D = 8;  // blocks in flight
        uint64_t w0[D], w1[D];
    #pragma unroll
        for (int d = 0; d < D; ++d)
            if ((uint64_t)d < nb) ld16<ALIGNED>(q + 1024 * d, w0[d], w1[d]);
        uint64_t blk = 0;
        for (; blk + D <= nb; blk += D) {
            uint64_t c0[D], c1[D];
    #pragma unroll
            for (int d = 0; d < D; ++d) {
                c0[d] = mul32x32(w0[d] ^ ks0) + w1[d];
                c1[d] = mul32x32(w1[d] ^ ks1) + w0[d];
                if (blk + D + d < nb) ld16<ALIGNED>(q + 1024 * (blk + D + d), w0[d], w1[d]);
            }
    #pragma unroll
            for (int d = 0; d < D; ++d) {
                c0[d] = class_sum(c0[d]);
                c1[d] = class_sum(c1[d]);
            }
    #pragma unroll
            for (int d = 0; d < D; ++d) {
                acc0 = scramble1(acc0 + c0[d], st0);
                acc1 = scramble1(acc1 + c1[d], st1);
            }
        }
    #pragma unroll
        for (int d = 0; d < D; ++d) {
            if (blk + d < nb) {
                const uint64_t c0 = mul32x32(w0[d] ^ ks0) + w1[d], c1 = mul32x32(w1[d] ^ ks1) + w0[d];
                acc0 = scramble1(acc0 + class_sum(c0), st0);
                acc1 = scramble1(acc1 + class_sum(c1), st1);
            }
        }
    }
    // the partial last block (no scramble) and the last stripe, read at n - 64 (lanes 0..3)
    const uint64_t ns = ((n - 1) - 1024 * nb) / 64;
    uint64_t c0 = 0, c1 = 0;
    if ((uint64_t)s < ns) {
        uint64_t a, b;
        ld16<ALIGNED>(q + 1024 * nb, a, b);
        c0 = mul32x32(a ^ ks0) + b;
        c1 = mul32x32(b ^ ks1) + a;
    }
    if (s == 0) {
        uint64_t a, b;
        ld16<false>(ptr + n - 64 + 16 * wp, a, b);
        c0 += mul32x32(a ^ sec64(121 + 16 * wp, seed)) + b;
        c1 += mul32x32(b ^ sec64(129 + 16 * wp, seed)) + a;
    }
    acc0 += class_sum(c0);
    acc1 += class_sum(c1);
    // lanes 0..3 hold accumulators {0,1}, {2,3}, {4,5}, {6,7} (the partial block's and last stripe's
    // contributions, plus, in the one-pass layout, the full blocks'); SPLIT: lanes 0..7 hold the
    // scrambled accumulators 0..7 of the full blocks
    auto rl64 = [](uint64_t v, int l) -> uint64_t {
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    };
    uint64_t acc[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        acc[2 * k] = rl64(acc0, k);
        acc[2 * k + 1] = rl64(acc1, k);
        if (SPLIT) {
            acc[2 * k] += rl64(accv, 2 * k) - init[2 * k];  // acc0 / acc1 started from init, accv too
            acc[2 * k + 1] += rl64(accv, 2 * k + 1) - init[2 * k + 1];
        }
    }
    if (lane != 0) return;
    auto mergeacc = [&](int off, uint64_t start) {
        uint64_t r = start;
#pragma unroll
        for (int k = 0; k < 4; ++k) r += fold64(acc[2 * k] ^ sec64(off + 16 * k, seed), acc[2 * k + 1] ^ sec64(off + 16 * k + 8, seed));
        return avalanche3(r);
    };
    if (BITS == 64) {
        p.d_out[i] = mergeacc(11, n * P64_1);
    } else {
        p.d_out[2 * i] = mergeacc(117, ~(n * P64_2));  // canonical order: high half first
        p.d_out[2 * i + 1] = mergeacc(11, n * P64_1);
    }
}

// Phase 1 of the split long path (strided batches of long buffers): wave w sums the lane
// contributions of kSumBlocks consecutive full blocks of one buffer (the accumulate step is a pure
// addition within a block) and writes each block's eight accumulator sums (64 B) for the scramble
// pass; all CUs stream the payload instead of one wave per buffer.
constexpr uint64_t kSumBlocks = 64;
template <bool ALIGNED>
__global__ __launch_bounds__(256) void xxh3_blocksum_kernel(const XxhParams p) {
    const uint64_t nb = (p.len - 1) / 1024;
    const uint64_t wpb = (nb + kSumBlocks - 1) / kSumBlocks;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= p.nbuf * wpb) return;
    const uint64_t i = w / wpb, b0 = (w - i * wpb) * kSumBlocks;
    const uint64_t b1 = b0 + kSumBlocks < nb ? b0 + kSumBlocks : nb;
    const int lane = threadIdx.x & 63, s = lane >> 2, wp = lane & 3;
    const uint64_t seed = p.d_seeds ? p.d_seeds[i] : p.seed_all;
    const uint64_t ks0 = sec64(8 * s + 16 * wp, seed), ks1 = sec64(8 * s + 16 * wp + 8, seed);
    const uint8_t *q = (const uint8_t *)(p.base + i * p.stride) + 16 * lane;
    uint64_t *S = p.d_sums + i * nb * 8 + 2 * wp;
    constexpr int D = 8;
    for (uint64_t blk = b0; blk < b1; blk += D) {
        uint64_t c0[D], c1[D];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            uint64_t a = 0, b = 0;
            if (blk + d < b1) ld16<ALIGNED>(q + 1024 * (blk + d), a, b);
            c0[d] = mul32x32(a ^ ks0) + b;
            c1[d] = mul32x32(b ^ ks1) + a;
        }
#pragma unroll
        for (int d = 0; d < D; ++d) {
            c0[d] = class_sum(c0[d]);
            c1[d] = class_sum(c1[d]);
        }
        if (s == 0) {
#pragma unroll
            for (int d = 0; d < D; ++d)
                if (blk + d < b1) {
                    v2u64 v;
                    v.x = c0[d];
                    v.y = c1[d];
                    *(__attribute__((address_space(1))) v2u64 *)(S + (blk + d) * 8) = v;
                }
        }
    }
}

template <int BITS>
__global__ __launch_bounds__(256) void xxh3_wave_kernel(const XxhParams p) {
    const uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= p.nbuf) return;
    const uint8_t *ptr = (const uint8_t *)(p.d_ptrs ? p.d_ptrs[i] : p.base + i * p.stride);
    const uint64_t n = p.d_ptrs ? p.d_lens[i] : p.len;
    const uint64_t seed = p.d_seeds ? p.d_seeds[i] : p.seed_all;
    if (n <= 240) {  // short inputs: the scalar published code paths, one lane
        if (lane == 0) {
            if (BITS == 64) {
                p.d_out[i] = xxh3_64(ptr, n, seed);
            } else {
                const U128 h = xxh3_128(ptr, n, seed);
                p.d_out[2 * i] = h.hi;
                p.d_out[2 * i + 1] = h.lo;
            }
        }
        return;
    }
    if (p.d_sums)  // phase 2 of the split long path (strided batches only)
        xxh3_long_wave<BITS, false, true>(p, i, ptr, n, seed, lane);
    else if (((uintptr_t)ptr & 15) == 0)
        xxh3_long_wave<BITS, true>(p, i, ptr, n, seed, lane);
    else
        xxh3_long_wave<BITS, false>(p, i, ptr, n, seed, lane);
}

// Streaming XXH3 (aws_xxhash_update on device memory, abi_single.cpp): the stream's accumulators
// acc_io[8] (device memory) absorb nb whole blocks whose sums xxh3_blocksum_kernel wrote to S; one
// wave, every block scrambled.
__global__ __launch_bounds__(64) void xxh3_stream_scramble_kernel(const uint64_t *S, uint64_t nb, uint64_t seed, uint64_t *acc_io) {
    const int lane = threadIdx.x;
    const int c8 = lane & 7;
    const uint64_t accv = scramble_chain(S, nb, acc_io[c8], sec64(128 + 8 * c8, seed), lane);
    if (lane < 8) acc_io[lane] = accv;
}

}  // namespace

// Streaming XXH3: nblocks whole 1 KiB blocks at d_ptr into the accumulators at d_acc (device, 8 x u64):
// the block sums over all CUs (d_sums: nblocks x 64 B), then the scramble chain in one wave.
extern "C" int amdcrc_launch_xxh3_stream(const void *d_ptr, uint64_t nblocks, uint64_t seed, uint64_t *d_sums, uint64_t *d_acc,
                                         void *stream) {
    if (nblocks == 0) return 0;
    XxhParams p{};
    p.base = (uint64_t)(uintptr_t)d_ptr;
    p.stride = 0;
    p.len = nblocks * 1024 + 1;  // (len - 1) / 1024 == nblocks whole blocks
    p.nbuf = 1;
    p.seed_all = seed;
    p.d_sums = d_sums;
    int e = amdcrc_launch_xxh3_blocksum(&p, stream, nullptr);
    if (e) return e;
    hipLaunchKernelGGL(xxh3_stream_scramble_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const uint64_t *)d_sums, nblocks,
                       seed, d_acc);
    return (int)hipGetLastError();
}

// Phase 1 of the split path: one wave per kSumBlocks blocks of every buffer (p->d_sums set, p->len > 240)
extern "C" int amdcrc_launch_xxh3_blocksum(const XxhParams *p, void *stream, void *start_event) {
    const uint64_t nb = (p->len - 1) / 1024;
    const uint64_t waves = p->nbuf * ((nb + kSumBlocks - 1) / kSumBlocks);
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const bool aligned = ((p->base | p->stride) & 15) == 0;
    if (aligned)
        hipExtLaunchKernelGGL(xxh3_blocksum_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, (hipEvent_t)start_event, nullptr, 0, *p);
    else
        hipExtLaunchKernelGGL(xxh3_blocksum_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, (hipEvent_t)start_event, nullptr, 0, *p);
    return (int)hipGetLastError();
}

// One wavefront per buffer (4 per 256-thread block): long buffers use all 64 lanes, short ones lane 0.
extern "C" int amdcrc_launch_xxh3(int bits, const XxhParams *p, void *stream, void *const *ev) {
    const int threads = 256;
    const uint64_t blocks = (p->nbuf + 3) / 4;
    if (blocks == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const bool timed = ev && (ev[0] || ev[1]);
    if (bits == 64) {
        if (timed)
            hipExtLaunchKernelGGL(xxh3_wave_kernel<64>, dim3((unsigned)blocks), dim3(threads), 0, s, (hipEvent_t)ev[0], (hipEvent_t)ev[1], 0, *p);
        else
            hipLaunchKernelGGL(xxh3_wave_kernel<64>, dim3((unsigned)blocks), dim3(threads), 0, s, *p);
    } else {
        if (timed)
            hipExtLaunchKernelGGL(xxh3_wave_kernel<128>, dim3((unsigned)blocks), dim3(threads), 0, s, (hipEvent_t)ev[0], (hipEvent_t)ev[1], 0, *p);
        else
            hipLaunchKernelGGL(xxh3_wave_kernel<128>, dim3((unsigned)blocks), dim3(threads), 0, s, *p);
    }
    return (int)hipGetLastError();
}
