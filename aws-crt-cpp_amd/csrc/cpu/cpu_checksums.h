// Host (x86-64) checksum path of the engine: the part of aws-checksums' job that stays on the CPU.
//
// The reference computes every checksum on the calling thread with a CPU implementation chosen
// by hardware capability at aws_checksums_library_init (include/aws/crt/checksum/CRC.h:17-19,
// source/Api.cpp:53).  This engine keeps the same contract: small host buffers, few-buffer xxHash
// and every call on a machine without a usable gfx950 device run here; device-resident data and
// large batches go to the GPU (engine.cpp dispatch).  Product code: nothing here comes from or
// links oracle/ (the test-only restatement).
//
// Tiers, picked once from CPUID:
//   CRC32 / CRC32C / CRC64NVME   AVX-512 VPCLMULQDQ folding (4 x 512-bit accumulators, 256 B per
//                                iteration) > PCLMULQDQ folding (4 x 128-bit) > slice-by-8 tables;
//                                CRC32C short inputs use the SSE4.2 crc32 instruction.
//   XXH64                        scalar (four serial chains: nothing to vectorise)
//   XXH3-64 / XXH3-128           AVX-512 > AVX2 > scalar stripe accumulation
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <functional>

namespace amdcrc {
namespace cpu {

struct Features {
    bool sse42, pclmul, avx2, avx512, vpclmul;
};
const Features &features();

enum Tier { TIER_TABLE = 0, TIER_PCLMUL = 1, TIER_VPCLMUL = 2 };
// Highest CRC tier this host supports (the one the API uses), and a way to force a lower one
// (tests and the CPU baseline compare tiers; the arithmetic is identical).
Tier best_tier();

// CRC_ex semantics (CRC.h:20-36): previous = finalised CRC of the preceding bytes.
uint32_t crc32(const uint8_t *p, size_t n, uint32_t previous);
uint32_t crc32c(const uint8_t *p, size_t n, uint32_t previous);
uint64_t crc64nvme(const uint8_t *p, size_t n, uint64_t previous);
// alg 0/1/2 as engine.h; tier <= best_tier()
uint64_t crc_tier(int alg, const uint8_t *p, size_t n, uint64_t previous, Tier tier);

// xxHash (published algorithms; XXHash.h:21-37)
uint64_t xxh64(const uint8_t *p, size_t n, uint64_t seed);
uint64_t xxh3_64(const uint8_t *p, size_t n, uint64_t seed);
void xxh3_128(const uint8_t *p, size_t n, uint64_t seed, uint64_t out_hi_lo[2]);

// Streaming states: O(1) memory whatever the stream length (XXHash.h:40-91).
struct Xxh64State {
    uint64_t v[4];
    uint64_t seed, total;
    uint8_t mem[32];
    uint32_t memn;
};
void xxh64_reset(Xxh64State *s, uint64_t seed);
void xxh64_update(Xxh64State *s, const uint8_t *p, size_t n);
uint64_t xxh64_digest(const Xxh64State *s);

struct Xxh3State {
    uint64_t acc[8];
    uint64_t seed, total;
    uint8_t secret[192];  // kSecret, or the seed-derived secret
    uint8_t buf[256];     // unconsumed input (all of it while total <= 240)
    uint8_t last[64];     // the 64 bytes consumed just before buf (for the final overlapping stripe)
    uint32_t bufn, stripes;  // bytes in buf; stripes consumed in the current 1 KiB block
};
void xxh3_reset(Xxh3State *s, uint64_t seed);
void xxh3_update(Xxh3State *s, const uint8_t *p, size_t n);
// k stripes at the state's stripe position (scrambling at block ends); `last` becomes p's final stripe
void xxh3_consume(Xxh3State *s, const uint8_t *p, size_t k);
// xxh3_update over input the host cannot address directly (device memory): `read` copies bytes
// [off, off + len) of the input into host memory; `blocks` absorbs `nblocks` whole 1 KiB blocks at
// offset off into s->acc (called with s->stripes == 0, which it leaves 0).  Every byte outside
// those blocks (the buffer top-up, stripes up to a block boundary, the last partial block and the
// 1..64 buffered bytes) goes through `read` and the host path, so the result is xxh3_update's
// exactly.  The state is updated only if every callback succeeds.
struct Xxh3Source {
    void *ctx;
    bool (*read)(void *ctx, uint8_t *dst, uint64_t off, size_t len);
    bool (*blocks)(void *ctx, Xxh3State *s, uint64_t off, uint64_t nblocks);
};
bool xxh3_update_source(Xxh3State *s, uint64_t n, const Xxh3Source &src);
uint64_t xxh3_64_digest(const Xxh3State *s);
void xxh3_128_digest(const Xxh3State *s, uint64_t out_hi_lo[2]);

// Batch of host buffers over `threads` std::threads (buffers round-robin), results as uint64_t per
// buffer (XXH3-128: two words, high then low).  alg as aws_crt_amd_algorithm.  seeds may be null.
void batch(int alg, const uint8_t *const *ptrs, const size_t *lens, const uint64_t *seeds, uint64_t *out, size_t count,
           int threads);

// fn(0) .. fn(n - 1) on the host batch's persistent worker threads (fn(0) on the calling thread), or
// on threads of their own when the pool is busy.  node >= 0 (from home_node): every index on pool
// workers placed on that NUMA node's CPUs, the calling thread only waiting.
void parallel(size_t n, const std::function<void(size_t)> &fn, int node = -1);

// The NUMA node holding >= 3/4 of a job's bytes (64 pages sampled, move_pages), when the process's
// CPU mask spans more than one node, that node has `threads` CPUs of it and the job is >= 16 MiB;
// else -1.  AWS_CRT_AMD_NUMA=0: always -1; =force: one node counts too (tests).
int home_node(const uint8_t *const *ptrs, const size_t *lens, size_t count, size_t threads);

// The process's CPU share: the CPUs it may run on (its allowed-CPU list, /proc/self/status, else the
// affinity mask), capped by OMP_NUM_THREADS; computed once.  The host path's thread counts and
// home_node's placement use this one figure.
size_t share();

}  // namespace cpu
}  // namespace amdcrc
