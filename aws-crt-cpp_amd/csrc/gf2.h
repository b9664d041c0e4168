// GF(2) polynomial arithmetic for reflected CRCs, shared by host (constant tables) and device.
//
// Representation: a W-bit register where bit (W-1-i) holds the coefficient of x^i (the
// "reflected" convention of CRC-32 / CRC-32C / CRC-64/NVME, include/aws/crt/checksum/CRC.h:15-35).
// Multiplying by x is a right shift with conditional XOR of the reflected polynomial.
//
// The identities the engine relies on (all linear over GF(2)):
//   state after bytes m from state v        = v * x^(8|m|)  ^  R(m)          (R = raw CRC, state 0)
//   CRC(A||B) = Combine(CRC(A), CRC(B), |B|) = CRC(A) * x^(8|B|) ^ CRC(B)    (CRC.cpp:30-43 semantics)
//   leading zero bytes do not change R(m)                                   (front padding is free)
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GF2_HD __host__ __device__ constexpr inline
#else
#define GF2_HD constexpr inline
#endif

namespace amdcrc {

enum Alg : int { ALG_CRC32 = 0, ALG_CRC32C = 1, ALG_CRC64NVME = 2 };

constexpr uint32_t kPoly32 = 0xEDB88320u;              // reflected 0x04C11DB7
constexpr uint32_t kPoly32C = 0x82F63B78u;             // reflected 0x1EDC6F41
constexpr uint64_t kPoly64Nvme = 0x9A6C9329AC4BC9B5ull; // reflected 0xAD93D23594C93659

GF2_HD uint64_t alg_poly(int alg) { return alg == ALG_CRC32 ? kPoly32 : alg == ALG_CRC32C ? kPoly32C : kPoly64Nvme; }
GF2_HD int alg_width(int alg) { return alg == ALG_CRC64NVME ? 64 : 32; }
GF2_HD uint64_t alg_mask(int alg) { return alg == ALG_CRC64NVME ? ~0ull : 0xFFFFFFFFull; }

// v * x mod P
GF2_HD uint64_t gf2_mulx(uint64_t v, uint64_t poly) { return (v >> 1) ^ ((v & 1) ? poly : 0); }

// a * b mod P (zlib multmodp formulation, generalised to width W)
GF2_HD uint64_t gf2_mulmod(uint64_t a, uint64_t b, uint64_t poly, int width) {
    uint64_t m = 1ull << (width - 1), p = 0;
    while (m) {
        if (a & m) p ^= b;
        m >>= 1;
        b = gf2_mulx(b, poly);
    }
    return p;
}

// x^(8*nbytes) mod P by square-and-multiply
GF2_HD uint64_t gf2_xpow8n(uint64_t nbytes, uint64_t poly, int width) {
    uint64_t result = 1ull << (width - 1);  // x^0
    uint64_t sq = result >> 8;              // x^8
    while (nbytes) {
        if (nbytes & 1) result = gf2_mulmod(result, sq, poly, width);
        sq = gf2_mulmod(sq, sq, poly, width);
        nbytes >>= 1;
    }
    return result;
}

// slice table entry T_k[e]: byte e followed by k zero bytes, i.e. e * x^(8(k+1)) in register form
GF2_HD uint64_t gf2_table_entry(uint32_t e, int k, uint64_t poly) {
    uint64_t c = e;
    for (int i = 0; i < 8 * (k + 1); ++i) c = gf2_mulx(c, poly);
    return c;
}

}  // namespace amdcrc
