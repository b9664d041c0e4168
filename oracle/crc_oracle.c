/*
 * oracle/crc_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the checksum arithmetic that aws-crt-cpp's Aws::Crt::Checksum API
 * forwards to (the un-vendored aws-checksums C library).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this file's shared object; the product path
 * (aws-crt-cpp_amd/) never links or calls it.
 *
 * Reference call sites this restates (aws-checksums source itself is absent):
 *   ComputeCRC32      -> aws_checksums_crc32_ex        source/checksum/CRC.cpp:15-18
 *   ComputeCRC32C     -> aws_checksums_crc32c_ex       source/checksum/CRC.cpp:20-23
 *   ComputeCRC64NVME  -> aws_checksums_crc64nvme_ex    source/checksum/CRC.cpp:25-28
 *   CombineCRC32/32C/64NVME -> aws_checksums_*_combine source/checksum/CRC.cpp:30-43
 *   ComputeXXHash64   -> aws_xxhash64_compute          source/checksum/XXHash.cpp:15-18
 * Semantics: include/aws/crt/checksum/CRC.h:15-51 (reflected CRCs, ~0 init/xorout,
 * previousCRC = finalised CRC of the prefix; CRC64NVME poly comment CRC.h:33-35).
 *
 * Parity pins: tests/CRCTest.cpp:16,29,42 (32 zero bytes), tests/XXHashTest.cpp:13-28
 * ("Hello world"), standard check values of "123456789", zlib 1.2.11 crc32/crc32_combine,
 * the SSE4.2 crc32 instruction (Castagnoli by ISA definition) and python xxhash 3.8.1.
 *
 * Three tiers per CRC:
 *   *_bitwise : one bit per step, the definition (slow; pins the others)
 *   *_sw      : slice-by-8 tables (aws-checksums' portable SW path technique)
 *   *_hw      : PCLMULQDQ 4x128-bit folding (CRC32, CRC32C, CRC64NVME) and SSE4.2 crc32q
 *               3-way interleave (CRC32C) -- the technique class aws-checksums dispatches to on
 *               x86; used as the timed CPU baseline (kind "port").
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <pthread.h>

#if defined(__x86_64__)
#include <immintrin.h>
#include <cpuid.h>
#define ORACLE_X86 1
#endif

#define POLY32 0xEDB88320u             /* reflected 0x04C11DB7 (gzip/Ethernet)      */
#define POLY32C 0x82F63B78u            /* reflected 0x1EDC6F41 (Castagnoli)         */
#define POLY64NVME 0x9A6C9329AC4BC9B5ull /* reflected 0xAD93D23594C93659 (CRC.h:33-35) */

/* ------------------------------------------------------------------ bitwise definition */

static uint64_t crc_bitwise(const uint8_t *p, size_t n, uint64_t prev, uint64_t poly, int width) {
    uint64_t mask = width == 64 ? ~0ull : ((1ull << width) - 1);
    uint64_t r = (~prev) & mask;
    for (size_t i = 0; i < n; ++i) {
        r ^= p[i];
        for (int b = 0; b < 8; ++b)
            r = (r & 1) ? (r >> 1) ^ poly : (r >> 1);
    }
    return (~r) & mask;
}

uint32_t oracle_crc32_bitwise(const uint8_t *p, size_t n, uint32_t prev) {
    return (uint32_t)crc_bitwise(p, n, prev, POLY32, 32);
}
uint32_t oracle_crc32c_bitwise(const uint8_t *p, size_t n, uint32_t prev) {
    return (uint32_t)crc_bitwise(p, n, prev, POLY32C, 32);
}
uint64_t oracle_crc64nvme_bitwise(const uint8_t *p, size_t n, uint64_t prev) {
    return crc_bitwise(p, n, prev, POLY64NVME, 64);
}

/* ------------------------------------------------------------------ GF(2) shift algebra */
/* Reflected representation: bit (W-1-i) holds the coefficient of x^i.  mulmod follows the
 * zlib multmodp formulation; combine(c1,c2,len2) = c1 * x^(8*len2) mod P  ^  c2
 * (the convention behind aws_checksums_*_combine, CRC.cpp:30-43). */

static uint64_t gf2_mulmod(uint64_t a, uint64_t b, uint64_t poly, int width) {
    uint64_t m = 1ull << (width - 1), p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0)
                break;
        }
        m >>= 1;
        if (!m)
            break;
        b = (b & 1) ? (b >> 1) ^ poly : (b >> 1);
    }
    return p;
}

/* x^(8*nbytes) mod P, by repeated squaring of x^(2^k). */
static uint64_t gf2_xpow8n(uint64_t nbytes, uint64_t poly, int width) {
    uint64_t one = 1ull << (width - 1);
    uint64_t result = one;
    uint64_t sq = one >> 8; /* x^8: in reflected form, one shifted right by 8 (no reduction for W>=16) */
    while (nbytes) {
        if (nbytes & 1)
            result = gf2_mulmod(result, sq, poly, width);
        sq = gf2_mulmod(sq, sq, poly, width);
        nbytes >>= 1;
    }
    return result;
}

uint32_t oracle_crc32_combine(uint32_t c1, uint32_t c2, uint64_t len2) {
    return (uint32_t)(gf2_mulmod(c1, gf2_xpow8n(len2, POLY32, 32), POLY32, 32) ^ c2);
}
uint32_t oracle_crc32c_combine(uint32_t c1, uint32_t c2, uint64_t len2) {
    return (uint32_t)(gf2_mulmod(c1, gf2_xpow8n(len2, POLY32C, 32), POLY32C, 32) ^ c2);
}
uint64_t oracle_crc64nvme_combine(uint64_t c1, uint64_t c2, uint64_t len2) {
    return gf2_mulmod(c1, gf2_xpow8n(len2, POLY64NVME, 64), POLY64NVME, 64) ^ c2;
}
uint64_t oracle_xpow8n(uint64_t nbytes, int alg) {
    switch (alg) {
        case 0: return gf2_xpow8n(nbytes, POLY32, 32);
        case 1: return gf2_xpow8n(nbytes, POLY32C, 32);
        default: return gf2_xpow8n(nbytes, POLY64NVME, 64);
    }
}
uint64_t oracle_mulmod(uint64_t a, uint64_t b, int alg) {
    switch (alg) {
        case 0: return gf2_mulmod(a, b, POLY32, 32);
        case 1: return gf2_mulmod(a, b, POLY32C, 32);
        default: return gf2_mulmod(a, b, POLY64NVME, 64);
    }
}

/* ------------------------------------------------------------------ slice-by-8 tables */

static uint32_t T32[8][256], T32C[8][256];
static uint64_t T64[8][256];
static pthread_once_t tables_once = PTHREAD_ONCE_INIT;

static void build_tables(void) {
    for (int b = 0; b < 256; ++b) {
        uint32_t c = (uint32_t)b, cc = (uint32_t)b;
        uint64_t c64 = (uint64_t)b;
        for (int k = 0; k < 8; ++k) {
            c = (c & 1) ? (c >> 1) ^ POLY32 : (c >> 1);
            cc = (cc & 1) ? (cc >> 1) ^ POLY32C : (cc >> 1);
            c64 = (c64 & 1) ? (c64 >> 1) ^ POLY64NVME : (c64 >> 1);
        }
        T32[0][b] = c;
        T32C[0][b] = cc;
        T64[0][b] = c64;
    }
    for (int k = 1; k < 8; ++k)
        for (int b = 0; b < 256; ++b) {
            T32[k][b] = (T32[k - 1][b] >> 8) ^ T32[0][T32[k - 1][b] & 0xff];
            T32C[k][b] = (T32C[k - 1][b] >> 8) ^ T32C[0][T32C[k - 1][b] & 0xff];
            T64[k][b] = (T64[k - 1][b] >> 8) ^ T64[0][T64[k - 1][b] & 0xff];
        }
}

static inline uint64_t load_le64(const uint8_t *p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}

static uint32_t crc32_sb8_raw(uint32_t r, const uint8_t *p, size_t n, uint32_t (*T)[256]) {
    while (n && ((uintptr_t)p & 7)) {
        r = (r >> 8) ^ T[0][(r ^ *p++) & 0xff];
        --n;
    }
    while (n >= 8) {
        uint64_t w = load_le64(p) ^ r;
        r = T[7][w & 0xff] ^ T[6][(w >> 8) & 0xff] ^ T[5][(w >> 16) & 0xff] ^ T[4][(w >> 24) & 0xff] ^
            T[3][(w >> 32) & 0xff] ^ T[2][(w >> 40) & 0xff] ^ T[1][(w >> 48) & 0xff] ^ T[0][w >> 56];
        p += 8;
        n -= 8;
    }
    while (n--)
        r = (r >> 8) ^ T[0][(r ^ *p++) & 0xff];
    return r;
}

static uint64_t crc64_sb8_raw(uint64_t r, const uint8_t *p, size_t n) {
    while (n && ((uintptr_t)p & 7)) {
        r = (r >> 8) ^ T64[0][(r ^ *p++) & 0xff];
        --n;
    }
    while (n >= 8) {
        uint64_t w = load_le64(p) ^ r;
        r = T64[7][w & 0xff] ^ T64[6][(w >> 8) & 0xff] ^ T64[5][(w >> 16) & 0xff] ^ T64[4][(w >> 24) & 0xff] ^
            T64[3][(w >> 32) & 0xff] ^ T64[2][(w >> 40) & 0xff] ^ T64[1][(w >> 48) & 0xff] ^ T64[0][w >> 56];
        p += 8;
        n -= 8;
    }
    while (n--)
        r = (r >> 8) ^ T64[0][(r ^ *p++) & 0xff];
    return r;
}

uint32_t oracle_crc32_sw(const uint8_t *p, size_t n, uint32_t prev) {
    pthread_once(&tables_once, build_tables);
    return ~crc32_sb8_raw(~prev, p, n, T32);
}
uint32_t oracle_crc32c_sw(const uint8_t *p, size_t n, uint32_t prev) {
    pthread_once(&tables_once, build_tables);
    return ~crc32_sb8_raw(~prev, p, n, T32C);
}
uint64_t oracle_crc64nvme_sw(const uint8_t *p, size_t n, uint64_t prev) {
    pthread_once(&tables_once, build_tables);
    return ~crc64_sb8_raw(~prev, p, n);
}

/* ------------------------------------------------------------------ x86 accelerated tier */
#if ORACLE_X86

static int cpu_has(int leaf, int sub, int reg, int bit) {
    unsigned a, b, c, d;
    if (!__get_cpuid_count(leaf, sub, &a, &b, &c, &d))
        return 0;
    unsigned r = reg == 0 ? a : reg == 1 ? b : reg == 2 ? c : d;
    return (r >> bit) & 1;
}

int oracle_hw_available(void) {
    /* SSE4.2 = CPUID.1:ECX[20], PCLMULQDQ = CPUID.1:ECX[1] */
    return cpu_has(1, 0, 2, 20) && cpu_has(1, 0, 2, 1);
}

/* Folding constants: with reflected 64-bit operands, clmul(a, refl(x^(T-1) mod P)) places
 * a*x^T in the 128-bit reflected convention (bit k <-> degree 127-k).  For W=32 the 32-bit
 * reflected residue sits in the upper half of the 64-bit operand. */
typedef struct {
    uint64_t k_fold512_hi, k_fold512_lo; /* x^(512+64-1), x^(512-1)  */
    uint64_t k_fold128_hi, k_fold128_lo; /* x^(128+64-1), x^(128-1)  */
    int width;
    uint64_t poly;
} fold_consts;

static uint64_t xpow_bits(uint64_t nbits, uint64_t poly, int width) {
    /* x^nbits mod P, reflected */
    uint64_t one = 1ull << (width - 1), result = one, sq = one >> 1; /* x^1 */
    while (nbits) {
        if (nbits & 1)
            result = gf2_mulmod(result, sq, poly, width);
        sq = gf2_mulmod(sq, sq, poly, width);
        nbits >>= 1;
    }
    return result;
}

static uint64_t as_refl64(uint64_t r, int width) { return width == 64 ? r : (r << 32); }

static void make_fold_consts(fold_consts *fc, uint64_t poly, int width) {
    fc->width = width;
    fc->poly = poly;
    fc->k_fold512_hi = as_refl64(xpow_bits(512 + 64 - 1, poly, width), width);
    fc->k_fold512_lo = as_refl64(xpow_bits(512 - 1, poly, width), width);
    fc->k_fold128_hi = as_refl64(xpow_bits(128 + 64 - 1, poly, width), width);
    fc->k_fold128_lo = as_refl64(xpow_bits(128 - 1, poly, width), width);
}

static fold_consts FC32, FC32C, FC64;
static pthread_once_t fold_once = PTHREAD_ONCE_INIT;
static void build_fold(void) {
    make_fold_consts(&FC32, POLY32, 32);
    make_fold_consts(&FC32C, POLY32C, 32);
    make_fold_consts(&FC64, POLY64NVME, 64);
}

__attribute__((target("pclmul,sse4.1"))) static inline __m128i fold128(__m128i a, __m128i k /* lo=hi-const, hi=lo-const */) {
    /* a.lo64 holds degrees 127..64 (A_hi), a.hi64 holds 63..0 (A_lo) */
    __m128i t_hi = _mm_clmulepi64_si128(a, k, 0x00); /* A_hi * x^(F+64) */
    __m128i t_lo = _mm_clmulepi64_si128(a, k, 0x11); /* A_lo * x^F      */
    return _mm_xor_si128(t_hi, t_lo);
}

/* Raw (no init/xorout) CRC state r over data, PCLMUL folding for the bulk, slice-by-8 for
 * the tail.  Requires n >= 64. */
__attribute__((target("pclmul,sse4.1"))) static uint64_t fold_crc_raw(uint64_t r, const uint8_t *p, size_t n,
                                                                        const fold_consts *fc) {
    const int w = fc->width;
    __m128i k512 = _mm_set_epi64x((long long)fc->k_fold512_lo, (long long)fc->k_fold512_hi);
    __m128i k128 = _mm_set_epi64x((long long)fc->k_fold128_lo, (long long)fc->k_fold128_hi);
    __m128i x0 = _mm_loadu_si128((const __m128i *)(p + 0));
    __m128i x1 = _mm_loadu_si128((const __m128i *)(p + 16));
    __m128i x2 = _mm_loadu_si128((const __m128i *)(p + 32));
    __m128i x3 = _mm_loadu_si128((const __m128i *)(p + 48));
    /* inject the running state into the first W/8 bytes (state r then data == 0 then data^r) */
    x0 = _mm_xor_si128(x0, w == 64 ? _mm_set_epi64x(0, (long long)r) : _mm_cvtsi32_si128((int)(uint32_t)r));
    p += 64;
    n -= 64;
    while (n >= 64) {
        x0 = _mm_xor_si128(fold128(x0, k512), _mm_loadu_si128((const __m128i *)(p + 0)));
        x1 = _mm_xor_si128(fold128(x1, k512), _mm_loadu_si128((const __m128i *)(p + 16)));
        x2 = _mm_xor_si128(fold128(x2, k512), _mm_loadu_si128((const __m128i *)(p + 32)));
        x3 = _mm_xor_si128(fold128(x3, k512), _mm_loadu_si128((const __m128i *)(p + 48)));
        p += 64;
        n -= 64;
    }
    x1 = _mm_xor_si128(fold128(x0, k128), x1);
    x2 = _mm_xor_si128(fold128(x1, k128), x2);
    x3 = _mm_xor_si128(fold128(x2, k128), x3);
    while (n >= 16) {
        x3 = _mm_xor_si128(fold128(x3, k128), _mm_loadu_si128((const __m128i *)p));
        p += 16;
        n -= 16;
    }
    /* x3 (16 bytes, congruent to the consumed prefix) -> CRC register via the byte tables */
    uint8_t blk[16];
    _mm_storeu_si128((__m128i *)blk, x3);
    uint64_t s;
    if (w == 64) {
        s = crc64_sb8_raw(0, blk, 16);
        s = crc64_sb8_raw(s, p, n);
    } else {
        uint32_t (*T)[256] = fc->poly == POLY32 ? T32 : T32C;
        s = crc32_sb8_raw(0, blk, 16, T);
        s = crc32_sb8_raw((uint32_t)s, p, n, T);
    }
    return s;
}

uint32_t oracle_crc32_hw(const uint8_t *p, size_t n, uint32_t prev) {
    pthread_once(&tables_once, build_tables);
    pthread_once(&fold_once, build_fold);
    if (n < 64 || !oracle_hw_available())
        return ~crc32_sb8_raw(~prev, p, n, T32);
    return ~(uint32_t)fold_crc_raw((uint32_t)~prev, p, n, &FC32);
}

uint64_t oracle_crc64nvme_hw(const uint8_t *p, size_t n, uint64_t prev) {
    pthread_once(&tables_once, build_tables);
    pthread_once(&fold_once, build_fold);
    if (n < 64 || !oracle_hw_available())
        return ~crc64_sb8_raw(~prev, p, n);
    return ~fold_crc_raw(~prev, p, n, &FC64);
}

uint32_t oracle_crc32c_fold(const uint8_t *p, size_t n, uint32_t prev) {
    pthread_once(&tables_once, build_tables);
    pthread_once(&fold_once, build_fold);
    if (n < 64 || !oracle_hw_available())
        return ~crc32_sb8_raw(~prev, p, n, T32C);
    return ~(uint32_t)fold_crc_raw((uint32_t)~prev, p, n, &FC32C);
}

/* SSE4.2 crc32q, three independent streams over equal blocks, merged with x^(8*blk) shifts
 * (Intel's "3-way interleave"; the shift multiply uses PCLMUL + table reduction). */
__attribute__((target("sse4.2"))) static uint32_t crc32c_hw1(uint32_t r, const uint8_t *p, size_t n) {
    while (n && ((uintptr_t)p & 7)) {
        r = _mm_crc32_u8(r, *p++);
        --n;
    }
    uint64_t r64 = r;
    while (n >= 8) {
        r64 = _mm_crc32_u64(r64, load_le64(p));
        p += 8;
        n -= 8;
    }
    r = (uint32_t)r64;
    while (n--)
        r = _mm_crc32_u8(r, *p++);
    return r;
}

__attribute__((target("sse4.2,pclmul"))) static uint32_t shift_crc32c(uint32_t r, uint64_t k /* refl64(x^(8*blk-33)) */) {
    /* r * x^(8*blk) mod P: clmul to a 64-bit product, then reduce it with crc32q of zero */
    __m128i prod = _mm_clmulepi64_si128(_mm_cvtsi32_si128((int)r), _mm_cvtsi64_si128((long long)k), 0x00);
    return (uint32_t)_mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(prod));
}

__attribute__((target("sse4.2,pclmul"))) uint32_t oracle_crc32c_hw(const uint8_t *p, size_t n, uint32_t prev) {
    pthread_once(&tables_once, build_tables);
    if (!oracle_hw_available())
        return ~crc32_sb8_raw(~prev, p, n, T32C);
    uint32_t r = ~prev;
    const size_t BLK = 8192; /* bytes per stream per round */
    static uint64_t kshift = 0;
    if (!kshift) {
        /* want r*x^(8*BLK).  crc32q(0, v) = v(x)*x^32 (64-bit LE word, degree 63..0 reflected)
         * mod P, and clmul of two reflected 32-bit values yields a 63-bit product positioned so
         * that multiplying by refl(x^(8*BLK - 33)) ends up as r*x^(8*BLK). */
        uint64_t c = xpow_bits(8 * BLK - 33, POLY32C, 32); /* reflected 32-bit */
        kshift = c;                                      /* low 32 bits of the 64-bit operand */
    }
    while (n >= 3 * BLK) {
        uint64_t a = r, b = 0, c = 0;
        const uint8_t *pa = p, *pb = p + BLK, *pc = p + 2 * BLK;
        for (size_t i = 0; i < BLK; i += 8) {
            a = _mm_crc32_u64(a, load_le64(pa + i));
            b = _mm_crc32_u64(b, load_le64(pb + i));
            c = _mm_crc32_u64(c, load_le64(pc + i));
        }
        r = shift_crc32c(shift_crc32c((uint32_t)a, kshift) ^ (uint32_t)b, kshift) ^ (uint32_t)c;
        p += 3 * BLK;
        n -= 3 * BLK;
    }
    return ~crc32c_hw1(r, p, n);
}

#else
int oracle_hw_available(void) { return 0; }
uint32_t oracle_crc32_hw(const uint8_t *p, size_t n, uint32_t prev) { return oracle_crc32_sw(p, n, prev); }
uint32_t oracle_crc32c_hw(const uint8_t *p, size_t n, uint32_t prev) { return oracle_crc32c_sw(p, n, prev); }
uint32_t oracle_crc32c_fold(const uint8_t *p, size_t n, uint32_t prev) { return oracle_crc32c_sw(p, n, prev); }
uint64_t oracle_crc64nvme_hw(const uint8_t *p, size_t n, uint64_t prev) { return oracle_crc64nvme_sw(p, n, prev); }
#endif

/* ------------------------------------------------------------------ xxHash64 */
/* XXH64 as published by xxHash (Yann Collet), restated; aws-checksums wraps it
 * (aws_xxhash64_compute, XXHash.cpp:17).  Digest is written big-endian by the API. */
static const uint64_t XP1 = 0x9E3779B185EBCA87ull, XP2 = 0xC2B2AE3D27D4EB4Full, XP3 = 0x165667B19E3779F9ull,
                      XP4 = 0x85EBCA77C2B2AE63ull, XP5 = 0x27D4EB2F165667C5ull;
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t xround(uint64_t acc, uint64_t in) {
    acc += in * XP2;
    acc = rotl64(acc, 31);
    return acc * XP1;
}
static inline uint64_t xmerge(uint64_t acc, uint64_t v) {
    acc ^= xround(0, v);
    return acc * XP1 + XP4;
}

uint64_t oracle_xxh64(const uint8_t *p, size_t n, uint64_t seed) {
    const uint8_t *end = p + n;
    uint64_t h;
    if (n >= 32) {
        uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
        do {
            v1 = xround(v1, load_le64(p));
            v2 = xround(v2, load_le64(p + 8));
            v3 = xround(v3, load_le64(p + 16));
            v4 = xround(v4, load_le64(p + 24));
            p += 32;
        } while (p + 32 <= end);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xmerge(h, v1);
        h = xmerge(h, v2);
        h = xmerge(h, v3);
        h = xmerge(h, v4);
    } else {
        h = seed + XP5;
    }
    h += (uint64_t)n;
    while (p + 8 <= end) {
        h ^= xround(0, load_le64(p));
        h = rotl64(h, 27) * XP1 + XP4;
        p += 8;
    }
    if (p + 4 <= end) {
        uint32_t v;
        memcpy(&v, p, 4);
        h ^= (uint64_t)v * XP1;
        h = rotl64(h, 23) * XP2 + XP3;
        p += 4;
    }
    while (p < end) {
        h ^= (*p++) * XP5;
        h = rotl64(h, 11) * XP1;
    }
    h ^= h >> 33;
    h *= XP2;
    h ^= h >> 29;
    h *= XP3;
    h ^= h >> 32;
    return h;
}

/* ------------------------------------------------------------------ batched (threaded) baseline */

typedef struct {
    int alg; /* 0 crc32, 1 crc32c, 2 crc64nvme, 3 xxh64 */
    const uint8_t *const *ptrs;
    const size_t *lens;
    uint64_t *out;
    size_t n, tid, nthreads;
} batch_job;

static void *batch_worker(void *arg) {
    batch_job *j = (batch_job *)arg;
    for (size_t i = j->tid; i < j->n; i += j->nthreads) {
        const uint8_t *p = j->ptrs[i];
        size_t len = j->lens[i];
        switch (j->alg) {
            case 0: j->out[i] = oracle_crc32_hw(p, len, 0); break;
            case 1: j->out[i] = oracle_crc32c_hw(p, len, 0); break;
            case 2: j->out[i] = oracle_crc64nvme_hw(p, len, 0); break;
            default: j->out[i] = oracle_xxh64(p, len, 0); break;
        }
    }
    return NULL;
}

/* Round-robin buffers over nthreads std-style threads (protocol item 2). */
int oracle_batch(int alg, const uint8_t *const *ptrs, const size_t *lens, uint64_t *out, size_t n, int nthreads) {
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    pthread_t th[256];
    batch_job jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (batch_job){alg, ptrs, lens, out, n, (size_t)t, (size_t)nthreads};
        if (t > 0 && pthread_create(&th[t], NULL, batch_worker, &jobs[t]) != 0)
            return -1;
    }
    batch_worker(&jobs[0]);
    for (int t = 1; t < nthreads; ++t)
        pthread_join(th[t], NULL);
    return 0;
}

/* ------------------------------------------------------------------ XXH3 (64 / 128) */
/* Restatement of the published XXH3 algorithm (xxHash 0.8, Yann Collet) behind
 * aws_xxhash3_64_compute / aws_xxhash3_128_compute (XXHash.cpp:22,27).  Pinned by
 * tests/XXHashTest.cpp:44 and :73-74 and by python xxhash 3.8.1 over every length class. */
static const uint8_t XXH3_SECRET[192] = {
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
static const uint64_t XQ32_1 = 0x9E3779B1u, XQ32_2 = 0x85EBCA77u, XQ32_3 = 0xC2B2AE3Du;
static const uint64_t XMX1 = 0x165667919E3779F9ull, XMX2 = 0x9FB21C651E98DF25ull;

static inline uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }
static inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
static inline uint64_t mul128_fold64(uint64_t a, uint64_t b) {
    __uint128_t p = (__uint128_t)a * b;
    return (uint64_t)p ^ (uint64_t)(p >> 64);
}
static inline uint64_t x3_avalanche(uint64_t h) { h ^= h >> 37; h *= XMX1; return h ^ (h >> 32); }
static inline uint64_t x64_avalanche(uint64_t h) {
    h ^= h >> 33; h *= XP2; h ^= h >> 29; h *= XP3; return h ^ (h >> 32);
}
static inline uint64_t rrmxmx(uint64_t h, uint64_t len) {
    h ^= rotl64(h, 49) ^ rotl64(h, 24);
    h *= XMX2;
    h ^= (h >> 35) + len;
    h *= XMX2;
    return h ^ (h >> 28);
}
static inline uint64_t mix16(const uint8_t *in, const uint8_t *sec, uint64_t seed) {
    return mul128_fold64(load_le64(in) ^ (load_le64(sec) + seed), load_le64(in + 8) ^ (load_le64(sec + 8) - seed));
}

static void x3_accumulate_512(uint64_t *acc, const uint8_t *in, const uint8_t *sec) {
    for (int i = 0; i < 8; ++i) {
        uint64_t v = load_le64(in + 8 * i), k = v ^ load_le64(sec + 8 * i);
        acc[i ^ 1] += v;
        acc[i] += (k & 0xFFFFFFFFull) * (k >> 32);
    }
}
static void x3_scramble(uint64_t *acc, const uint8_t *sec) {
    for (int i = 0; i < 8; ++i) {
        uint64_t a = acc[i];
        a ^= a >> 47;
        a ^= load_le64(sec + 8 * i);
        acc[i] = a * XQ32_1;
    }
}
static void x3_long_loop(uint64_t *acc, const uint8_t *in, size_t len, const uint8_t *sec) {
    const size_t stripes_per_block = (192 - 64) / 8, block = 64 * stripes_per_block;
    const size_t nb = (len - 1) / block;
    for (size_t n = 0; n < nb; ++n) {
        for (size_t s = 0; s < stripes_per_block; ++s) x3_accumulate_512(acc, in + n * block + 64 * s, sec + 8 * s);
        x3_scramble(acc, sec + 192 - 64);
    }
    const size_t ns = ((len - 1) - block * nb) / 64;
    for (size_t s = 0; s < ns; ++s) x3_accumulate_512(acc, in + nb * block + 64 * s, sec + 8 * s);
    x3_accumulate_512(acc, in + len - 64, sec + 192 - 64 - 7);
}
static uint64_t x3_merge(const uint64_t *acc, const uint8_t *sec, uint64_t start) {
    uint64_t r = start;
    for (int i = 0; i < 4; ++i)
        r += mul128_fold64(acc[2 * i] ^ load_le64(sec + 16 * i), acc[2 * i + 1] ^ load_le64(sec + 16 * i + 8));
    return x3_avalanche(r);
}
static void x3_custom_secret(uint8_t *out, uint64_t seed) {
    for (int i = 0; i < 12; ++i) {
        uint64_t lo = load_le64(XXH3_SECRET + 16 * i) + seed, hi = load_le64(XXH3_SECRET + 16 * i + 8) - seed;
        memcpy(out + 16 * i, &lo, 8);
        memcpy(out + 16 * i + 8, &hi, 8);
    }
}
static void x3_long_acc(uint64_t *acc, const uint8_t *p, size_t n, uint64_t seed, uint8_t *secbuf, const uint8_t **sec) {
    const uint64_t init[8] = {XQ32_3, XP1, XP2, XP3, XP4, XQ32_2, XP5, XQ32_1};
    memcpy(acc, init, sizeof(init));
    *sec = XXH3_SECRET;
    if (seed) {
        x3_custom_secret(secbuf, seed);
        *sec = secbuf;
    }
    x3_long_loop(acc, p, n, *sec);
}

uint64_t oracle_xxh3_64(const uint8_t *p, size_t n, uint64_t seed) {
    const uint8_t *s = XXH3_SECRET;
    if (n <= 16) {
        if (n > 8) {
            uint64_t bf1 = (load_le64(s + 24) ^ load_le64(s + 32)) + seed;
            uint64_t bf2 = (load_le64(s + 40) ^ load_le64(s + 48)) - seed;
            uint64_t lo = load_le64(p) ^ bf1, hi = load_le64(p + n - 8) ^ bf2;
            return x3_avalanche(n + bswap64(lo) + hi + mul128_fold64(lo, hi));
        }
        if (n >= 4) {
            uint64_t sd = seed ^ ((uint64_t)bswap32((uint32_t)seed) << 32);
            uint64_t in64 = ld32(p + n - 4) + ((uint64_t)ld32(p) << 32);
            uint64_t bf = (load_le64(s + 8) ^ load_le64(s + 16)) - sd;
            return rrmxmx(in64 ^ bf, n);
        }
        if (n > 0) {
            uint32_t c = ((uint32_t)p[0] << 16) | ((uint32_t)p[n >> 1] << 24) | p[n - 1] | ((uint32_t)n << 8);
            uint64_t bf = (uint64_t)(ld32(s) ^ ld32(s + 4)) + seed;
            return x64_avalanche((uint64_t)c ^ bf);
        }
        return x64_avalanche(seed ^ (load_le64(s + 56) ^ load_le64(s + 64)));
    }
    if (n <= 128) {
        uint64_t acc = n * XP1;
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
        return x3_avalanche(acc);
    }
    if (n <= 240) {
        uint64_t acc = n * XP1;
        const int rounds = (int)(n / 16);
        for (int i = 0; i < 8; ++i) acc += mix16(p + 16 * i, s + 16 * i, seed);
        acc = x3_avalanche(acc);
        for (int i = 8; i < rounds; ++i) acc += mix16(p + 16 * i, s + 16 * (i - 8) + 3, seed);
        acc += mix16(p + n - 16, s + 136 - 17, seed);
        return x3_avalanche(acc);
    }
    uint64_t acc[8];
    uint8_t secbuf[192];
    const uint8_t *sec;
    x3_long_acc(acc, p, n, seed, secbuf, &sec);
    return x3_merge(acc, sec + 11, n * XP1);
}

static void mix32(uint64_t *lo, uint64_t *hi, const uint8_t *a, const uint8_t *b, const uint8_t *sec, uint64_t seed) {
    *lo += mix16(a, sec, seed);
    *lo ^= load_le64(b) + load_le64(b + 8);
    *hi += mix16(b, sec + 16, seed);
    *hi ^= load_le64(a) + load_le64(a + 8);
}

/* out[0] = high 64 bits, out[1] = low 64 bits */
void oracle_xxh3_128(const uint8_t *p, size_t n, uint64_t seed, uint64_t *out) {
    const uint8_t *s = XXH3_SECRET;
    uint64_t lo, hi;
    if (n <= 16) {
        if (n > 8) {
            uint64_t bfl = (load_le64(s + 32) ^ load_le64(s + 40)) - seed;
            uint64_t bfh = (load_le64(s + 48) ^ load_le64(s + 56)) + seed;
            uint64_t ilo = load_le64(p), ihi = load_le64(p + n - 8);
            __uint128_t m = (__uint128_t)(ilo ^ ihi ^ bfl) * XP1;
            uint64_t mlo = (uint64_t)m, mhi = (uint64_t)(m >> 64);
            mlo += (uint64_t)(n - 1) << 54;
            ihi ^= bfh;
            mhi += ihi + (uint64_t)(uint32_t)ihi * (XQ32_2 - 1);
            mlo ^= bswap64(mhi);
            __uint128_t h = (__uint128_t)mlo * XP2;
            lo = (uint64_t)h;
            hi = (uint64_t)(h >> 64) + mhi * XP2;
            out[0] = x3_avalanche(hi);
            out[1] = x3_avalanche(lo);
            return;
        }
        if (n >= 4) {
            uint64_t sd = seed ^ ((uint64_t)bswap32((uint32_t)seed) << 32);
            uint64_t in64 = ld32(p) + ((uint64_t)ld32(p + n - 4) << 32);
            uint64_t bf = (load_le64(s + 16) ^ load_le64(s + 24)) + sd;
            __uint128_t m = (__uint128_t)(in64 ^ bf) * (XP1 + ((uint64_t)n << 2));
            uint64_t mlo = (uint64_t)m, mhi = (uint64_t)(m >> 64);
            mhi += mlo << 1;
            mlo ^= mhi >> 3;
            mlo ^= mlo >> 35;
            mlo *= XMX2;
            mlo ^= mlo >> 28;
            out[0] = x3_avalanche(mhi);
            out[1] = mlo;
            return;
        }
        if (n > 0) {
            uint32_t cl = ((uint32_t)p[0] << 16) | ((uint32_t)p[n >> 1] << 24) | p[n - 1] | ((uint32_t)n << 8);
            uint32_t sw = bswap32(cl);
            uint32_t ch = (sw << 13) | (sw >> 19);
            uint64_t bfl = (uint64_t)(ld32(s) ^ ld32(s + 4)) + seed;
            uint64_t bfh = (uint64_t)(ld32(s + 8) ^ ld32(s + 12)) - seed;
            out[0] = x64_avalanche((uint64_t)ch ^ bfh);
            out[1] = x64_avalanche((uint64_t)cl ^ bfl);
            return;
        }
        out[1] = x64_avalanche(seed ^ (load_le64(s + 64) ^ load_le64(s + 72)));
        out[0] = x64_avalanche(seed ^ (load_le64(s + 80) ^ load_le64(s + 88)));
        return;
    }
    if (n <= 128) {
        lo = n * XP1;
        hi = 0;
        if (n > 32) {
            if (n > 64) {
                if (n > 96) mix32(&lo, &hi, p + 48, p + n - 64, s + 96, seed);
                mix32(&lo, &hi, p + 32, p + n - 48, s + 64, seed);
            }
            mix32(&lo, &hi, p + 16, p + n - 32, s + 32, seed);
        }
        mix32(&lo, &hi, p, p + n - 16, s, seed);
    } else if (n <= 240) {
        const int rounds = (int)(n / 32);
        lo = n * XP1;
        hi = 0;
        for (int i = 0; i < 4; ++i) mix32(&lo, &hi, p + 32 * i, p + 32 * i + 16, s + 32 * i, seed);
        lo = x3_avalanche(lo);
        hi = x3_avalanche(hi);
        for (int i = 4; i < rounds; ++i) mix32(&lo, &hi, p + 32 * i, p + 32 * i + 16, s + 3 + 32 * (i - 4), seed);
        mix32(&lo, &hi, p + n - 16, p + n - 32, s + 136 - 17 - 16, 0ull - seed);
    } else {
        uint64_t acc[8];
        uint8_t secbuf[192];
        const uint8_t *sec;
        x3_long_acc(acc, p, n, seed, secbuf, &sec);
        out[1] = x3_merge(acc, sec + 11, n * XP1);
        out[0] = x3_merge(acc, sec + 192 - 64 - 11, ~(n * XP2));
        return;
    }
    uint64_t rl = lo + hi;
    uint64_t rh = lo * XP1 + hi * XP4 + (n - seed) * XP2;
    out[1] = x3_avalanche(rl);
    out[0] = 0ull - x3_avalanche(rh);
}
