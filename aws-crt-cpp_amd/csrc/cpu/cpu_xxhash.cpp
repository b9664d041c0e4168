// Host xxHash64 / XXH3-64 / XXH3-128, one-shot and streaming (published xxHash 0.8 algorithms;
// reference entry points source/checksum/XXHash.cpp:15-71, known answers tests/XXHashTest.cpp).
//
// XXH64 is four serial multiply chains per stream, so one host core (~5-10 GB/s) beats the GPU's
// per-buffer rate by an order of magnitude: few-buffer XXH64 and every streaming update stay here.
// XXH3's stripe accumulation vectorises (AVX-512: one stripe per instruction group; AVX2: two
// halves); its scramble runs once per 1 KiB block.
//
// Streaming states hold O(1) memory (cpu_checksums.h): XXH64 keeps its four lanes and a 32-byte
// tail; XXH3 keeps its eight accumulators, up to 256 unconsumed bytes (all of the input while the
// total is <= 240, where the one-shot short paths apply) and the 64 bytes consumed last, which the
// final overlapping stripe may need.  A stripe is consumed only once at least one more byte is known
// to follow it, exactly as the one-shot loop's (len - 1) bounds.
#include <immintrin.h>
#include <string.h>

#include <algorithm>

#include "cpu_checksums.h"

namespace amdcrc {
namespace cpu {

namespace {

constexpr uint64_t P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full, P3 = 0x165667B19E3779F9ull,
                   P4 = 0x85EBCA77C2B2AE63ull, P5 = 0x27D4EB2F165667C5ull;
constexpr uint64_t Q1 = 0x9E3779B1u, Q2 = 0x85EBCA77u, Q3 = 0xC2B2AE3Du;  // 32-bit primes
constexpr uint64_t MX1 = 0x165667919E3779F9ull, MX2 = 0x9FB21C651E98DF25ull;

alignas(64) const uint8_t kSecret[192] = {
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

inline uint64_t r64(const uint8_t *p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}
inline uint32_t r32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
inline void w64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }
inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

// ---------------------------------------------------------------- XXH64
inline uint64_t round64(uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; }
inline uint64_t merge64(uint64_t h, uint64_t v) { return (h ^ round64(0, v)) * P1 + P4; }

uint64_t xxh64_finish(uint64_t h, const uint8_t *p, size_t n) {
    for (; n >= 8; n -= 8, p += 8) h = rotl(h ^ round64(0, r64(p)), 27) * P1 + P4;
    if (n >= 4) {
        h = rotl(h ^ (uint64_t)r32(p) * P1, 23) * P2 + P3;
        p += 4, n -= 4;
    }
    for (; n; --n, ++p) h = rotl(h ^ *p * P5, 11) * P1;
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    return h ^ (h >> 32);
}

inline uint64_t xxh64_converge(const uint64_t v[4]) {
    uint64_t h = rotl(v[0], 1) + rotl(v[1], 7) + rotl(v[2], 12) + rotl(v[3], 18);
    for (int i = 0; i < 4; ++i) h = merge64(h, v[i]);
    return h;
}

// ---------------------------------------------------------------- XXH3 building blocks
struct U128 {
    uint64_t lo, hi;
};
inline U128 mul128(uint64_t a, uint64_t b) {
    const unsigned __int128 m = (unsigned __int128)a * b;
    return {(uint64_t)m, (uint64_t)(m >> 64)};
}
inline uint64_t fold64(uint64_t a, uint64_t b) {
    const U128 m = mul128(a, b);
    return m.lo ^ m.hi;
}
inline uint64_t avalanche3(uint64_t h) {
    h ^= h >> 37;
    h *= MX1;
    return h ^ (h >> 32);
}
inline uint64_t avalanche64(uint64_t h) {
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    return h ^ (h >> 32);
}
inline uint64_t rrmxmx(uint64_t h, uint64_t len) {
    h ^= rotl(h, 49) ^ rotl(h, 24);
    h *= MX2;
    h ^= (h >> 35) + len;
    h *= MX2;
    return h ^ (h >> 28);
}
inline uint64_t mix16(const uint8_t *in, const uint8_t *sec, uint64_t seed) {
    return fold64(r64(in) ^ (r64(sec) + seed), r64(in + 8) ^ (r64(sec + 8) - seed));
}
inline void mix32(U128 &acc, const uint8_t *a, const uint8_t *b, const uint8_t *sec, uint64_t seed) {
    acc.lo += mix16(a, sec, seed);
    acc.lo ^= r64(b) + r64(b + 8);
    acc.hi += mix16(b, sec + 16, seed);
    acc.hi ^= r64(a) + r64(a + 8);
}

// short inputs (<= 240 bytes) use kSecret and the seed directly
uint64_t x3_64_short(const uint8_t *p, size_t n, uint64_t seed) {
    const uint8_t *s = kSecret;
    if (n <= 16) {
        if (n > 8) {
            const uint64_t lo = r64(p) ^ ((r64(s + 24) ^ r64(s + 32)) + seed);
            const uint64_t hi = r64(p + n - 8) ^ ((r64(s + 40) ^ r64(s + 48)) - seed);
            return avalanche3(n + __builtin_bswap64(lo) + hi + fold64(lo, hi));
        }
        if (n >= 4) {
            const uint64_t sd = seed ^ ((uint64_t)__builtin_bswap32((uint32_t)seed) << 32);
            const uint64_t in64 = r32(p + n - 4) + ((uint64_t)r32(p) << 32);
            return rrmxmx(in64 ^ ((r64(s + 8) ^ r64(s + 16)) - sd), n);
        }
        if (n) {
            const uint32_t c = ((uint32_t)p[0] << 16) | ((uint32_t)p[n >> 1] << 24) | p[n - 1] | ((uint32_t)n << 8);
            return avalanche64((uint64_t)c ^ ((uint64_t)(r32(s) ^ r32(s + 4)) + seed));
        }
        return avalanche64(seed ^ (r64(s + 56) ^ r64(s + 64)));
    }
    uint64_t acc = n * P1;
    if (n <= 128) {
        if (n > 32) {
            if (n > 64) {
                if (n > 96) acc += mix16(p + 48, s + 96, seed) + mix16(p + n - 64, s + 112, seed);
                acc += mix16(p + 32, s + 64, seed) + mix16(p + n - 48, s + 80, seed);
            }
            acc += mix16(p + 16, s + 32, seed) + mix16(p + n - 32, s + 48, seed);
        }
        acc += mix16(p, s, seed) + mix16(p + n - 16, s + 16, seed);
        return avalanche3(acc);
    }
    for (int i = 0; i < 8; ++i) acc += mix16(p + 16 * i, s + 16 * i, seed);
    acc = avalanche3(acc);
    for (int i = 8; i < (int)(n / 16); ++i) acc += mix16(p + 16 * i, s + 16 * (i - 8) + 3, seed);
    acc += mix16(p + n - 16, s + 119, seed);
    return avalanche3(acc);
}

U128 x3_128_short(const uint8_t *p, size_t n, uint64_t seed) {
    const uint8_t *s = kSecret;
    if (n <= 16) {
        if (n > 8) {
            const uint64_t bfl = (r64(s + 32) ^ r64(s + 40)) - seed, bfh = (r64(s + 48) ^ r64(s + 56)) + seed;
            uint64_t ilo = r64(p), ihi = r64(p + n - 8);
            U128 m = mul128(ilo ^ ihi ^ bfl, P1);
            m.lo += (uint64_t)(n - 1) << 54;
            ihi ^= bfh;
            m.hi += ihi + (uint64_t)(uint32_t)ihi * (Q2 - 1);
            m.lo ^= __builtin_bswap64(m.hi);
            U128 h = mul128(m.lo, P2);
            h.hi += m.hi * P2;
            return {avalanche3(h.lo), avalanche3(h.hi)};
        }
        if (n >= 4) {
            const uint64_t sd = seed ^ ((uint64_t)__builtin_bswap32((uint32_t)seed) << 32);
            const uint64_t in64 = r32(p) + ((uint64_t)r32(p + n - 4) << 32);
            U128 m = mul128(in64 ^ ((r64(s + 16) ^ r64(s + 24)) + sd), P1 + (n << 2));
            m.hi += m.lo << 1;
            m.lo ^= m.hi >> 3;
            m.lo ^= m.lo >> 35;
            m.lo *= MX2;
            m.lo ^= m.lo >> 28;
            return {m.lo, avalanche3(m.hi)};
        }
        if (n) {
            const uint32_t cl = ((uint32_t)p[0] << 16) | ((uint32_t)p[n >> 1] << 24) | p[n - 1] | ((uint32_t)n << 8);
            const uint32_t sw = __builtin_bswap32(cl), ch = (sw << 13) | (sw >> 19);
            return {avalanche64((uint64_t)cl ^ ((uint64_t)(r32(s) ^ r32(s + 4)) + seed)),
                    avalanche64((uint64_t)ch ^ ((uint64_t)(r32(s + 8) ^ r32(s + 12)) - seed))};
        }
        return {avalanche64(seed ^ (r64(s + 64) ^ r64(s + 72))), avalanche64(seed ^ (r64(s + 80) ^ r64(s + 88)))};
    }
    U128 acc{n * P1, 0};
    if (n <= 128) {
        if (n > 32) {
            if (n > 64) {
                if (n > 96) mix32(acc, p + 48, p + n - 64, s + 96, seed);
                mix32(acc, p + 32, p + n - 48, s + 64, seed);
            }
            mix32(acc, p + 16, p + n - 32, s + 32, seed);
        }
        mix32(acc, p, p + n - 16, s, seed);
    } else {
        for (int i = 0; i < 4; ++i) mix32(acc, p + 32 * i, p + 32 * i + 16, s + 32 * i, seed);
        acc.lo = avalanche3(acc.lo);
        acc.hi = avalanche3(acc.hi);
        for (int i = 4; i < (int)(n / 32); ++i) mix32(acc, p + 32 * i, p + 32 * i + 16, s + 3 + 32 * (i - 4), seed);
        mix32(acc, p + n - 16, p + n - 32, s + 103, 0ull - seed);
    }
    const uint64_t hl = acc.lo + acc.hi;
    const uint64_t hh = acc.lo * P1 + acc.hi * P4 + (n - seed) * P2;
    return {avalanche3(hl), 0ull - avalanche3(hh)};
}

// ---- long-input stripe machinery: `count` consecutive stripes, stripe i keyed at sec + 8 (s0 + i)
typedef void (*StripesFn)(uint64_t *acc, const uint8_t *in, const uint8_t *sec, size_t count);
typedef void (*ScrambleFn)(uint64_t *acc, const uint8_t *key);

void stripes_scalar(uint64_t *acc, const uint8_t *in, const uint8_t *sec, size_t count) {
    for (size_t s = 0; s < count; ++s, in += 64, sec += 8)
        for (int i = 0; i < 8; ++i) {
            const uint64_t v = r64(in + 8 * i), k = v ^ r64(sec + 8 * i);
            acc[i ^ 1] += v;
            acc[i] += (k & 0xFFFFFFFFull) * (k >> 32);
        }
}
void scramble_scalar(uint64_t *acc, const uint8_t *key) {
    for (int i = 0; i < 8; ++i) acc[i] = (acc[i] ^ (acc[i] >> 47) ^ r64(key + 8 * i)) * Q1;
}

__attribute__((target("avx2"))) void stripes_avx2(uint64_t *acc, const uint8_t *in, const uint8_t *sec, size_t count) {
    __m256i a0 = _mm256_loadu_si256((const __m256i *)acc), a1 = _mm256_loadu_si256((const __m256i *)(acc + 4));
    for (size_t s = 0; s < count; ++s, in += 64, sec += 8) {
        const __m256i d0 = _mm256_loadu_si256((const __m256i *)in), d1 = _mm256_loadu_si256((const __m256i *)(in + 32));
        const __m256i k0 = _mm256_xor_si256(d0, _mm256_loadu_si256((const __m256i *)sec));
        const __m256i k1 = _mm256_xor_si256(d1, _mm256_loadu_si256((const __m256i *)(sec + 32)));
        // (k lo32) * (k hi32) per 64-bit word; acc[i ^ 1] += data: swap the words of each 128-bit half
        const __m256i m0 = _mm256_mul_epu32(k0, _mm256_srli_epi64(k0, 32)), m1 = _mm256_mul_epu32(k1, _mm256_srli_epi64(k1, 32));
        a0 = _mm256_add_epi64(a0, _mm256_add_epi64(m0, _mm256_shuffle_epi32(d0, _MM_SHUFFLE(1, 0, 3, 2))));
        a1 = _mm256_add_epi64(a1, _mm256_add_epi64(m1, _mm256_shuffle_epi32(d1, _MM_SHUFFLE(1, 0, 3, 2))));
    }
    _mm256_storeu_si256((__m256i *)acc, a0);
    _mm256_storeu_si256((__m256i *)(acc + 4), a1);
}
__attribute__((target("avx2"))) void scramble_avx2(uint64_t *acc, const uint8_t *key) {
    const __m256i q = _mm256_set1_epi64x((long long)Q1);
    for (int h = 0; h < 2; ++h) {
        __m256i a = _mm256_loadu_si256((const __m256i *)(acc + 4 * h));
        a = _mm256_xor_si256(_mm256_xor_si256(a, _mm256_srli_epi64(a, 47)), _mm256_loadu_si256((const __m256i *)(key + 32 * h)));
        // a * Q1 mod 2^64 with a 32-bit Q1: lo(a) * Q1 + (hi(a) * Q1) << 32
        const __m256i lo = _mm256_mul_epu32(a, q), hi = _mm256_mul_epu32(_mm256_srli_epi64(a, 32), q);
        _mm256_storeu_si256((__m256i *)(acc + 4 * h), _mm256_add_epi64(lo, _mm256_slli_epi64(hi, 32)));
    }
}

__attribute__((target("avx512f,avx512bw"))) void stripes_avx512(uint64_t *acc, const uint8_t *in, const uint8_t *sec, size_t count) {
    __m512i a = _mm512_loadu_si512(acc);
    for (size_t s = 0; s < count; ++s, in += 64, sec += 8) {
        const __m512i d = _mm512_loadu_si512(in);
        const __m512i k = _mm512_xor_si512(d, _mm512_loadu_si512(sec));
        const __m512i m = _mm512_mul_epu32(k, _mm512_srli_epi64(k, 32));
        a = _mm512_add_epi64(a, _mm512_add_epi64(m, _mm512_shuffle_epi32(d, (_MM_PERM_ENUM)_MM_SHUFFLE(1, 0, 3, 2))));
    }
    _mm512_storeu_si512(acc, a);
}
__attribute__((target("avx512f,avx512bw"))) void scramble_avx512(uint64_t *acc, const uint8_t *key) {
    const __m512i q = _mm512_set1_epi64((long long)Q1);
    __m512i a = _mm512_loadu_si512(acc);
    a = _mm512_ternarylogic_epi64(a, _mm512_srli_epi64(a, 47), _mm512_loadu_si512(key), 0x96);
    const __m512i lo = _mm512_mul_epu32(a, q), hi = _mm512_mul_epu32(_mm512_srli_epi64(a, 32), q);
    _mm512_storeu_si512(acc, _mm512_add_epi64(lo, _mm512_slli_epi64(hi, 32)));
}

struct X3Impl {
    StripesFn stripes;
    ScrambleFn scramble;
};
const X3Impl &x3impl() {
    static const X3Impl impl = [] {
        const Features &f = features();
        if (f.avx512) return X3Impl{stripes_avx512, scramble_avx512};
        if (f.avx2) return X3Impl{stripes_avx2, scramble_avx2};
        return X3Impl{stripes_scalar, scramble_scalar};
    }();
    return impl;
}

inline void acc_init(uint64_t *acc) {
    acc[0] = Q3, acc[1] = P1, acc[2] = P2, acc[3] = P3, acc[4] = P4, acc[5] = Q2, acc[6] = P5, acc[7] = Q1;
}

void derive_secret(uint8_t *out, uint64_t seed) {
    for (int i = 0; i < 12; ++i) {
        w64(out + 16 * i, r64(kSecret + 16 * i) + seed);
        w64(out + 16 * i + 8, r64(kSecret + 16 * i + 8) - seed);
    }
}

// consume `k` stripes at `in` into (acc, stripes-in-block), scrambling after every 16th
void consume(uint64_t *acc, uint32_t &stripes, const uint8_t *in, size_t k, const uint8_t *sec) {
    const X3Impl &x = x3impl();
    while (k) {
        const size_t take = k < 16 - (size_t)stripes ? k : 16 - (size_t)stripes;
        x.stripes(acc, in, sec + 8 * stripes, take);
        in += 64 * take, k -= take, stripes += (uint32_t)take;
        if (stripes == 16) {
            x.scramble(acc, sec + 128);
            stripes = 0;
        }
    }
}

uint64_t merge_acc(const uint64_t *acc, const uint8_t *sec, uint64_t start) {
    uint64_t r = start;
    for (int i = 0; i < 4; ++i) r += fold64(acc[2 * i] ^ r64(sec + 16 * i), acc[2 * i + 1] ^ r64(sec + 16 * i + 8));
    return avalanche3(r);
}

// long inputs (> 240 bytes): accumulators after every stripe, including the final overlapping one
void long_acc(uint64_t *acc, const uint8_t *p, size_t n, const uint8_t *sec) {
    acc_init(acc);
    uint32_t stripes = 0;
    consume(acc, stripes, p, (n - 1) / 64, sec);
    x3impl().stripes(acc, p + n - 64, sec + 121, 1);
}

const uint8_t *long_secret(uint64_t seed, uint8_t *buf) {
    if (!seed) return kSecret;
    derive_secret(buf, seed);
    return buf;
}

}  // namespace

// ---------------------------------------------------------------- public
uint64_t xxh64(const uint8_t *p, size_t n, uint64_t seed) {
    uint64_t h;
    const uint8_t *q = p;
    size_t m = n;
    if (n >= 32) {
        uint64_t v[4] = {seed + P1 + P2, seed + P2, seed, seed - P1};
        for (; m >= 32; m -= 32, q += 32)
            for (int i = 0; i < 4; ++i) v[i] = round64(v[i], r64(q + 8 * i));
        h = xxh64_converge(v);
    } else {
        h = seed + P5;
    }
    return xxh64_finish(h + n, q, m);
}

void xxh64_reset(Xxh64State *s, uint64_t seed) {
    memset(s, 0, sizeof(*s));
    s->seed = seed;
    s->v[0] = seed + P1 + P2, s->v[1] = seed + P2, s->v[2] = seed, s->v[3] = seed - P1;
}

void xxh64_update(Xxh64State *s, const uint8_t *p, size_t n) {
    s->total += n;
    if (s->memn + n < 32) {
        memcpy(s->mem + s->memn, p, n);
        s->memn += (uint32_t)n;
        return;
    }
    if (s->memn) {
        const size_t fill = 32 - s->memn;
        memcpy(s->mem + s->memn, p, fill);
        for (int i = 0; i < 4; ++i) s->v[i] = round64(s->v[i], r64(s->mem + 8 * i));
        p += fill, n -= fill;
        s->memn = 0;
    }
    for (; n >= 32; n -= 32, p += 32)
        for (int i = 0; i < 4; ++i) s->v[i] = round64(s->v[i], r64(p + 8 * i));
    memcpy(s->mem, p, n);
    s->memn = (uint32_t)n;
}

uint64_t xxh64_digest(const Xxh64State *s) {
    const uint64_t h = s->total >= 32 ? xxh64_converge(s->v) : s->seed + P5;
    return xxh64_finish(h + s->total, s->mem, s->memn);
}

uint64_t xxh3_64(const uint8_t *p, size_t n, uint64_t seed) {
    if (n <= 240) return x3_64_short(p, n, seed);
    alignas(64) uint8_t buf[192];
    const uint8_t *sec = long_secret(seed, buf);
    alignas(64) uint64_t acc[8];
    long_acc(acc, p, n, sec);
    return merge_acc(acc, sec + 11, n * P1);
}

void xxh3_128(const uint8_t *p, size_t n, uint64_t seed, uint64_t out[2]) {
    if (n <= 240) {
        const U128 h = x3_128_short(p, n, seed);
        out[0] = h.hi, out[1] = h.lo;
        return;
    }
    alignas(64) uint8_t buf[192];
    const uint8_t *sec = long_secret(seed, buf);
    alignas(64) uint64_t acc[8];
    long_acc(acc, p, n, sec);
    out[1] = merge_acc(acc, sec + 11, n * P1);
    out[0] = merge_acc(acc, sec + 192 - 64 - 11, ~(n * P2));
}

void xxh3_reset(Xxh3State *s, uint64_t seed) {
    memset(s, 0, sizeof(*s));
    s->seed = seed;
    acc_init(s->acc);
    if (seed)
        derive_secret(s->secret, seed);
    else
        memcpy(s->secret, kSecret, 192);
}

void xxh3_update(Xxh3State *s, const uint8_t *p, size_t n) {
    s->total += n;
    if (s->bufn + n <= sizeof(s->buf)) {
        memcpy(s->buf + s->bufn, p, n);
        s->bufn += (uint32_t)n;
        return;
    }
    if (s->bufn) {  // top the buffer up and consume all of it: more input follows
        const size_t fill = sizeof(s->buf) - s->bufn;
        memcpy(s->buf + s->bufn, p, fill);
        p += fill, n -= fill;
        consume(s->acc, s->stripes, s->buf, sizeof(s->buf) / 64, s->secret);
        memcpy(s->last, s->buf + sizeof(s->buf) - 64, 64);
        s->bufn = 0;
    }
    if (n > sizeof(s->buf)) {  // bulk from the caller's memory, leaving 1..64 bytes
        const size_t k = (n - 1) / 64;
        consume(s->acc, s->stripes, p, k, s->secret);
        memcpy(s->last, p + 64 * k - 64, 64);
        p += 64 * k, n -= 64 * k;
    }
    memcpy(s->buf, p, n);
    s->bufn = (uint32_t)n;
}

void xxh3_consume(Xxh3State *s, const uint8_t *p, size_t k) {
    if (!k) return;
    consume(s->acc, s->stripes, p, k, s->secret);
    memcpy(s->last, p + 64 * k - 64, 64);
}

// xxh3_update's steps with the bulk of whole blocks handed to src.blocks (the device)
bool xxh3_update_source(Xxh3State *st, uint64_t n, const Xxh3Source &src) {
    Xxh3State s = *st;
    alignas(64) uint8_t tmp[64 * 15];
    if (s.bufn + n <= sizeof(s.buf)) {
        if (n && !src.read(src.ctx, s.buf + s.bufn, 0, (size_t)n)) return false;
        s.bufn += (uint32_t)n;
        s.total += n;
        *st = s;
        return true;
    }
    uint64_t off = 0;
    if (s.bufn) {  // top the buffer up and consume all of it: more input follows
        const size_t fill = sizeof(s.buf) - s.bufn;
        if (!src.read(src.ctx, s.buf + s.bufn, 0, fill)) return false;
        off = fill;
        consume(s.acc, s.stripes, s.buf, sizeof(s.buf) / 64, s.secret);
        memcpy(s.last, s.buf + sizeof(s.buf) - 64, 64);
        s.bufn = 0;
    }
    if (n - off > sizeof(s.buf)) {  // bulk, leaving 1..64 bytes
        uint64_t k = (n - off - 1) / 64;
        const uint64_t h = std::min<uint64_t>((16 - s.stripes) % 16, k);  // stripes up to a block boundary
        if (h) {
            if (!src.read(src.ctx, tmp, off, (size_t)(64 * h))) return false;
            xxh3_consume(&s, tmp, (size_t)h);
            off += 64 * h, k -= h;
        }
        const uint64_t nbl = k / 16;  // whole blocks (s.stripes is 0 whenever nbl > 0)
        if (nbl) {
            if (!src.blocks(src.ctx, &s, off, nbl)) return false;
            s.stripes = 0;
            off += 1024 * nbl, k -= 16 * nbl;
            if (!src.read(src.ctx, s.last, off - 64, 64)) return false;
        }
        if (k) {
            if (!src.read(src.ctx, tmp, off, (size_t)(64 * k))) return false;
            xxh3_consume(&s, tmp, (size_t)k);
            off += 64 * k;
        }
    }
    if (!src.read(src.ctx, s.buf, off, (size_t)(n - off))) return false;
    s.bufn = (uint32_t)(n - off);
    s.total += n;
    *st = s;
    return true;
}

namespace {
// accumulators of a long stream at digest time (the state itself is left untouched)
void digest_acc(const Xxh3State *s, uint64_t *acc) {
    memcpy(acc, s->acc, 64);
    uint32_t stripes = s->stripes;
    const size_t k = (s->bufn - 1) / 64;
    consume(acc, stripes, s->buf, k, s->secret);
    alignas(64) uint8_t lastw[64];
    const uint8_t *ls;
    if (s->bufn >= 64) {
        ls = s->buf + s->bufn - 64;
    } else {
        memcpy(lastw, s->last + s->bufn, 64 - s->bufn);
        memcpy(lastw + 64 - s->bufn, s->buf, s->bufn);
        ls = lastw;
    }
    x3impl().stripes(acc, ls, s->secret + 121, 1);
}
}  // namespace

uint64_t xxh3_64_digest(const Xxh3State *s) {
    if (s->total <= 240) return x3_64_short(s->buf, (size_t)s->total, s->seed);
    alignas(64) uint64_t acc[8];
    digest_acc(s, acc);
    return merge_acc(acc, s->secret + 11, s->total * P1);
}

void xxh3_128_digest(const Xxh3State *s, uint64_t out[2]) {
    if (s->total <= 240) {
        const U128 h = x3_128_short(s->buf, (size_t)s->total, s->seed);
        out[0] = h.hi, out[1] = h.lo;
        return;
    }
    alignas(64) uint64_t acc[8];
    digest_acc(s, acc);
    out[1] = merge_acc(acc, s->secret + 11, s->total * P1);
    out[0] = merge_acc(acc, s->secret + 192 - 64 - 11, ~(s->total * P2));
}

}  // namespace cpu
}  // namespace amdcrc
