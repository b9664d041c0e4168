// aws-checksums single-buffer C ABI (include/aws/checksums/crc.h, xxhash.h) with the engine's
// CPU / GPU dispatch -- the layer the reference's wrappers call (source/checksum/CRC.cpp:17-42,
// source/checksum/XXHash.cpp:17-65) and aws-c-s3 / aws-c-event-stream would call directly.
//
// The reference contract (include/aws/crt/checksum/CRC.h:17-19): "selects a suitable
// implementation based on hardware capabilities", value-only, noexcept -- so every call must
// return the right value.  Dispatch (include/aws_crt_amd/checksums_batch.h):
//   * device-resident input           -> the gfx950 kernels (engine.cpp)
//   * host input                      -> the host path (csrc/cpu/), unless the dispatch mode is
//                                        AWS_CRT_AMD_DISPATCH_GPU (then staged through the GPU)
//   * no usable device, or any HIP error on the GPU path -> the host path (counted in
//     aws_crt_amd_fallback_count); device memory is then read back in bounded pieces.
// The mode only selects where the arithmetic runs; every path computes the same function.
#include <aws/checksums/crc.h>
#include <aws/checksums/xxhash.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>

#include "abi_guard.h"
#include "cpu/cpu_checksums.h"
#include "gf2.h"

#define AWS_CRT_AMD_BUILD 1
#include <aws_crt_amd/checksums_batch.h>

using namespace amdcrc;

// engine.cpp (GPU side)
extern "C" int amdcrc_gpu_usable(void);
extern "C" int amdcrc_is_device_ptr(const void *p);
extern "C" int amdcrc_gpu_single(int alg, const void *input, size_t len, uint64_t seed, uint64_t *out);
extern "C" int amdcrc_copy_to_host(void *dst, const void *src, size_t n);
extern "C" int amdcrc_gpu_xxh3_blocks(const void *d_ptr, uint64_t nblocks, uint64_t seed, uint64_t acc[8]);

using amdcrc::guarded;

namespace {

void no_sink(const char *) noexcept {}

std::atomic<int> g_mode{-1};
std::atomic<unsigned long long> g_fallbacks{0};

int mode() {
    int m = g_mode.load(std::memory_order_relaxed);
    if (m >= 0) return m;
    m = AWS_CRT_AMD_DISPATCH_AUTO;
    if (const char *e = std::getenv("AWS_CRT_AMD_DISPATCH")) {
        if (!std::strcmp(e, "cpu")) m = AWS_CRT_AMD_DISPATCH_CPU;
        if (!std::strcmp(e, "gpu")) m = AWS_CRT_AMD_DISPATCH_GPU;
    }
    int expect = -1;
    g_mode.compare_exchange_strong(expect, m);
    return g_mode.load();
}

uint64_t cpu_one(int alg, const uint8_t *p, size_t n, uint64_t seed, uint64_t *hi_lo) {
    switch (alg) {
        case AWS_CRT_AMD_CRC32: return cpu::crc32(p, n, (uint32_t)seed);
        case AWS_CRT_AMD_CRC32C: return cpu::crc32c(p, n, (uint32_t)seed);
        case AWS_CRT_AMD_CRC64NVME: return cpu::crc64nvme(p, n, seed);
        case AWS_CRT_AMD_XXH64: return cpu::xxh64(p, n, seed);
        case AWS_CRT_AMD_XXH3_64: return cpu::xxh3_64(p, n, seed);
        default: cpu::xxh3_128(p, n, seed, hi_lo); return hi_lo[0];
    }
}

// Device memory on the host path (GPU failed): read back through a bounded bounce buffer.  CRCs
// chain through their running value; xxHash through the streaming states.
bool cpu_from_device(int alg, const void *src, size_t n, uint64_t seed, uint64_t *out) {
    constexpr size_t kChunk = 4u << 20;
    uint8_t *bounce = (uint8_t *)std::malloc(n < kChunk ? (n ? n : 1) : kChunk);
    if (!bounce) return false;
    cpu::Xxh64State x64;
    cpu::Xxh3State *x3 = nullptr;
    if (alg == AWS_CRT_AMD_XXH64) cpu::xxh64_reset(&x64, seed);
    if (alg >= AWS_CRT_AMD_XXH3_64) {
        x3 = (cpu::Xxh3State *)std::malloc(sizeof(cpu::Xxh3State));
        if (!x3) {
            std::free(bounce);
            return false;
        }
        cpu::xxh3_reset(x3, seed);
    }
    uint64_t crc = seed;
    bool ok = true;
    for (size_t off = 0; off < n && ok; off += kChunk) {
        const size_t m = n - off < kChunk ? n - off : kChunk;
        if (amdcrc_copy_to_host(bounce, (const uint8_t *)src + off, m) != 0) {
            ok = false;
            break;
        }
        if (alg <= AWS_CRT_AMD_CRC64NVME)
            crc = cpu::crc_tier(alg, bounce, m, crc, cpu::best_tier());
        else if (alg == AWS_CRT_AMD_XXH64)
            cpu::xxh64_update(&x64, bounce, m);
        else
            cpu::xxh3_update(x3, bounce, m);
    }
    if (ok) {
        if (alg <= AWS_CRT_AMD_CRC64NVME) out[0] = crc;
        else if (alg == AWS_CRT_AMD_XXH64) out[0] = cpu::xxh64_digest(&x64);
        else if (alg == AWS_CRT_AMD_XXH3_64) out[0] = cpu::xxh3_64_digest(x3);
        else cpu::xxh3_128_digest(x3, out);
    }
    std::free(x3);
    std::free(bounce);
    return ok;
}

// One buffer, any memory.  out[0] (out[1]: XXH3-128 low half).  Never fails for host memory.
bool checksum_one(int alg, const void *input, size_t len, uint64_t seed, uint64_t *out) {
    out[0] = out[1] = 0;
    const bool on_device = len && input && amdcrc_is_device_ptr(input);
    if (on_device || mode() == AWS_CRT_AMD_DISPATCH_GPU) {
        if (amdcrc_gpu_usable() && amdcrc_gpu_single(alg, input, len, seed, out) == 0) return true;
        g_fallbacks.fetch_add(1, std::memory_order_relaxed);
        if (on_device) {
            if (cpu_from_device(alg, input, len, seed, out)) return true;
            std::fprintf(stderr, "aws-crt-cpp_amd: device buffer %p (%zu bytes) is unreadable: %s\n", input, len,
                         aws_crt_amd_last_error());
            return false;
        }
    }
    uint64_t hl[2] = {0, 0};
    out[0] = cpu_one(alg, (const uint8_t *)input, len, seed, hl);
    if (alg == AWS_CRT_AMD_XXH3_128) out[1] = hl[1];
    return true;
}

uint64_t crc_value(int alg, const uint8_t *input, size_t len, uint64_t previous) {
    if (!len) return previous;
    uint64_t r[2];
    if (checksum_one(alg, input, len, previous, r)) return r[0];
    // Device memory that neither the GPU nor a read-back can reach.  CRC.h:20-36 is value-only, so
    // the failure goes to the thread's aws error (Aws::Crt::LastError(), ref source/Api.cpp:469-472):
    // a caller that resets the error before the call and checks it after can tell this value apart
    // from a real CRC.  The value returned is the seed, unchanged.
    aws_raise_error(AWS_ERROR_UNSUPPORTED_OPERATION);
    return previous;
}

// ---- xxhash ABI
enum Kind { K_XXH64 = 0, K_XXH3_64 = 1, K_XXH3_128 = 2 };
int kind_alg(Kind k) { return k == K_XXH64 ? AWS_CRT_AMD_XXH64 : k == K_XXH3_64 ? AWS_CRT_AMD_XXH3_64 : AWS_CRT_AMD_XXH3_128; }

int write_digest(Kind k, const uint64_t *v, aws_byte_buf *out) {
    const size_t need = k == K_XXH3_128 ? 16 : 8;
    if (!out || out->capacity - out->len < need) return aws_raise_error(AWS_ERROR_SHORT_BUFFER);
    aws_byte_buf_write_be64(out, v[0]);  // XXH3-128: high 64 bits first (canonical form)
    if (k == K_XXH3_128) aws_byte_buf_write_be64(out, v[1]);
    return AWS_OP_SUCCESS;
}

int compute(Kind k, uint64_t seed, const uint8_t *p, size_t n, aws_byte_buf *out) {
    const size_t need = k == K_XXH3_128 ? 16 : 8;
    if (!out || out->capacity - out->len < need) return aws_raise_error(AWS_ERROR_SHORT_BUFFER);
    uint64_t v[2];
    if (!checksum_one(kind_alg(k), p, n, seed, v)) return aws_raise_error(AWS_ERROR_UNSUPPORTED_OPERATION);
    return write_digest(k, v, out);
}

}  // namespace

// Streaming object: the host states of cpu_checksums.h (O(1) memory).  Device-resident chunks of an
// XXH3 stream of at least kDeviceStreamBytes are absorbed on the GPU: XXH3's accumulate step is a
// pure sum within each 1 KiB block, so the chunk's whole blocks are summed by all CUs and one wave
// runs the scramble chain from the stream's accumulators (xxh3_kernels.hip), while the few hundred
// bytes around them go through the host state (cpu::xxh3_update_source).  XXH64 is one serial
// chain per stream (four lanes, each round depending on the last), so its device chunks are read
// back through a bounded bounce buffer and hashed on the host.
constexpr size_t kDeviceStreamBytes = 1u << 20;

namespace {
struct DeviceChunk {
    const uint8_t *d;
};
bool chunk_read(void *ctx, uint8_t *dst, uint64_t off, size_t len) {
    return !len || amdcrc_copy_to_host(dst, ((DeviceChunk *)ctx)->d + off, len) == 0;
}
bool chunk_blocks(void *ctx, cpu::Xxh3State *s, uint64_t off, uint64_t nblocks) {
    const uint8_t *d = ((DeviceChunk *)ctx)->d + off;
    if (amdcrc_gpu_usable() && amdcrc_gpu_xxh3_blocks(d, nblocks, s->seed, s->acc) == 0) return true;
    // the GPU path failed: the same blocks on the host path, read back in bounded pieces
    g_fallbacks.fetch_add(1, std::memory_order_relaxed);
    constexpr uint64_t kPiece = 1024;  // blocks (1 MiB)
    uint8_t *bounce = (uint8_t *)std::malloc(kPiece * 1024);
    if (!bounce) return false;
    bool ok = true;
    for (uint64_t b = 0; b < nblocks && ok; b += kPiece) {
        const uint64_t m = nblocks - b < kPiece ? nblocks - b : kPiece;
        ok = amdcrc_copy_to_host(bounce, d + 1024 * b, (size_t)(1024 * m)) == 0;
        if (ok) cpu::xxh3_consume(s, bounce, (size_t)(16 * m));
    }
    std::free(bounce);
    return ok;
}
}  // namespace

struct aws_xxhash {
    aws_allocator *allocator;
    Kind kind;
    bool finalized;
    union {
        cpu::Xxh64State x64;
        cpu::Xxh3State x3;
    };
};

extern "C" {

AWS_CRT_AMD_API int aws_crt_amd_set_dispatch(int m) {
    if (m < AWS_CRT_AMD_DISPATCH_AUTO || m > AWS_CRT_AMD_DISPATCH_GPU) return AWS_CRT_AMD_ERR_INVALID_ARG;
    g_mode.store(m);
    return 0;
}
AWS_CRT_AMD_API int aws_crt_amd_get_dispatch(void) { return mode(); }
AWS_CRT_AMD_API unsigned long long aws_crt_amd_fallback_count(void) { return g_fallbacks.load(); }
// internal (ingest.cpp): a host job whose devices failed was served by the host path
void amdcrc_note_fallback(void) { g_fallbacks.fetch_add(1, std::memory_order_relaxed); }

AWS_CRT_AMD_API int aws_crt_amd_cpu_batch(int alg, const void *const *h_ptrs, const size_t *lens, size_t count,
                                          const uint64_t *seeds, uint64_t *out, int threads) {
    return guarded(no_sink, [&]() -> int {
        if (alg < 0 || alg > 5) return AWS_CRT_AMD_ERR_INVALID_ARG;
        if (count && (!h_ptrs || !lens || !out)) return AWS_CRT_AMD_ERR_INVALID_ARG;
        cpu::batch(alg, (const uint8_t *const *)h_ptrs, lens, seeds, out, count, threads);
        return 0;
    });
}

AWS_CRT_AMD_API const char *aws_crt_amd_cpu_tier(void) {
    switch (cpu::best_tier()) {
        case cpu::TIER_VPCLMUL: return "avx512-vpclmulqdq";
        case cpu::TIER_PCLMUL: return "pclmulqdq";
        default: return "slice-by-8";
    }
}

#if AWS_CRT_AMD_DIAG
// Diagnostic library only: one CRC on a given host tier (0 tables, 1 PCLMULQDQ, 2 AVX-512
// VPCLMULQDQ; clamped to what the host supports), so every tier is checked on any host.
AWS_CRT_AMD_API uint64_t aws_crt_amd_debug_cpu_crc(int alg, int tier, const uint8_t *p, size_t n, uint64_t previous) {
    return cpu::crc_tier(alg, p, n, previous, (cpu::Tier)tier);
}
#endif

// ---- aws-checksums CRC ABI (include/aws/checksums/crc.h)
AWS_CRT_AMD_API void aws_checksums_library_init(struct aws_allocator *) {
    (void)cpu::best_tier();  // CPU capability dispatch, as at source/Api.cpp:53
}
AWS_CRT_AMD_API void aws_checksums_library_clean_up(void) {}

AWS_CRT_AMD_API uint32_t aws_checksums_crc32_ex(const uint8_t *input, size_t length, uint32_t previous) {
    return (uint32_t)crc_value(AWS_CRT_AMD_CRC32, input, length, previous);
}
AWS_CRT_AMD_API uint32_t aws_checksums_crc32c_ex(const uint8_t *input, size_t length, uint32_t previous) {
    return (uint32_t)crc_value(AWS_CRT_AMD_CRC32C, input, length, previous);
}
AWS_CRT_AMD_API uint64_t aws_checksums_crc64nvme_ex(const uint8_t *input, size_t length, uint64_t previous) {
    return crc_value(AWS_CRT_AMD_CRC64NVME, input, length, previous);
}
AWS_CRT_AMD_API uint32_t aws_checksums_crc32(const uint8_t *input, int length, uint32_t previous) {
    return aws_checksums_crc32_ex(input, length < 0 ? 0 : (size_t)length, previous);
}
AWS_CRT_AMD_API uint32_t aws_checksums_crc32c(const uint8_t *input, int length, uint32_t previous) {
    return aws_checksums_crc32c_ex(input, length < 0 ? 0 : (size_t)length, previous);
}
AWS_CRT_AMD_API uint64_t aws_checksums_crc64nvme(const uint8_t *input, int length, uint64_t previous) {
    return aws_checksums_crc64nvme_ex(input, length < 0 ? 0 : (size_t)length, previous);
}

// Combine is O(log len2) GF(2) algebra on two 4/8-byte values (CRC.cpp:30-43); batched device form:
// aws_crt_amd_crc_combine_batch.
AWS_CRT_AMD_API uint32_t aws_checksums_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
    return (uint32_t)(gf2_mulmod(crc1, gf2_xpow8n(len2, kPoly32, 32), kPoly32, 32) ^ crc2);
}
AWS_CRT_AMD_API uint32_t aws_checksums_crc32c_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
    return (uint32_t)(gf2_mulmod(crc1, gf2_xpow8n(len2, kPoly32C, 32), kPoly32C, 32) ^ crc2);
}
AWS_CRT_AMD_API uint64_t aws_checksums_crc64nvme_combine(uint64_t crc1, uint64_t crc2, uint64_t len2) {
    return gf2_mulmod(crc1, gf2_xpow8n(len2, kPoly64Nvme, 64), kPoly64Nvme, 64) ^ crc2;
}

// ---- aws-checksums xxhash ABI (include/aws/checksums/xxhash.h)
AWS_XXHASH_API int aws_xxhash64_compute(uint64_t seed, aws_byte_cursor data, aws_byte_buf *out) {
    return compute(K_XXH64, seed, data.ptr, data.len, out);
}
AWS_XXHASH_API int aws_xxhash3_64_compute(uint64_t seed, aws_byte_cursor data, aws_byte_buf *out) {
    return compute(K_XXH3_64, seed, data.ptr, data.len, out);
}
AWS_XXHASH_API int aws_xxhash3_128_compute(uint64_t seed, aws_byte_cursor data, aws_byte_buf *out) {
    return compute(K_XXH3_128, seed, data.ptr, data.len, out);
}

static aws_xxhash *make(aws_allocator *a, Kind k, uint64_t seed) {
    if (!a) a = aws_default_allocator();
    void *mem = aws_mem_acquire(a, sizeof(aws_xxhash));
    if (!mem) {
        aws_raise_error(AWS_ERROR_OOM);
        return nullptr;
    }
    aws_xxhash *h = static_cast<aws_xxhash *>(mem);
    std::memset(h, 0, sizeof(*h));
    h->allocator = a;
    h->kind = k;
    if (k == K_XXH64)
        cpu::xxh64_reset(&h->x64, seed);
    else
        cpu::xxh3_reset(&h->x3, seed);
    return h;
}

AWS_XXHASH_API aws_xxhash *aws_xxhash64_new(aws_allocator *a, uint64_t seed) { return make(a, K_XXH64, seed); }
AWS_XXHASH_API aws_xxhash *aws_xxhash3_64_new(aws_allocator *a, uint64_t seed) { return make(a, K_XXH3_64, seed); }
AWS_XXHASH_API aws_xxhash *aws_xxhash3_128_new(aws_allocator *a, uint64_t seed) { return make(a, K_XXH3_128, seed); }

AWS_XXHASH_API int aws_xxhash_update(aws_xxhash *h, aws_byte_cursor data) {
    if (!h || h->finalized) return aws_raise_error(AWS_ERROR_INVALID_STATE);
    if (!data.len) return AWS_OP_SUCCESS;
    if (!data.ptr) return aws_raise_error(AWS_ERROR_INVALID_ARGUMENT);
    auto feed = [h](const uint8_t *p, size_t n) {
        if (h->kind == K_XXH64)
            cpu::xxh64_update(&h->x64, p, n);
        else
            cpu::xxh3_update(&h->x3, p, n);
    };
    if (!amdcrc_is_device_ptr(data.ptr)) {
        feed(data.ptr, data.len);
        return AWS_OP_SUCCESS;
    }
    if (h->kind != K_XXH64 && data.len >= kDeviceStreamBytes) {
        DeviceChunk ctx{data.ptr};
        const cpu::Xxh3Source src{&ctx, chunk_read, chunk_blocks};
        return cpu::xxh3_update_source(&h->x3, data.len, src) ? AWS_OP_SUCCESS : aws_raise_error(AWS_ERROR_UNSUPPORTED_OPERATION);
    }
    constexpr size_t kChunk = 1u << 20;
    uint8_t *bounce = (uint8_t *)std::malloc(data.len < kChunk ? data.len : kChunk);
    if (!bounce) return aws_raise_error(AWS_ERROR_OOM);
    int rc = AWS_OP_SUCCESS;
    for (size_t off = 0; off < data.len; off += kChunk) {
        const size_t m = data.len - off < kChunk ? data.len - off : kChunk;
        if (amdcrc_copy_to_host(bounce, data.ptr + off, m) != 0) {
            rc = aws_raise_error(AWS_ERROR_UNSUPPORTED_OPERATION);
            break;
        }
        feed(bounce, m);
    }
    std::free(bounce);
    return rc;
}

AWS_XXHASH_API int aws_xxhash_finalize(aws_xxhash *h, aws_byte_buf *out) {
    if (!h || h->finalized) return aws_raise_error(AWS_ERROR_INVALID_STATE);
    uint64_t v[2] = {0, 0};
    if (h->kind == K_XXH64)
        v[0] = cpu::xxh64_digest(&h->x64);
    else if (h->kind == K_XXH3_64)
        v[0] = cpu::xxh3_64_digest(&h->x3);
    else
        cpu::xxh3_128_digest(&h->x3, v);
    const int rc = write_digest(h->kind, v, out);
    if (rc == AWS_OP_SUCCESS) h->finalized = true;
    return rc;
}

AWS_XXHASH_API void aws_xxhash_destroy(aws_xxhash *h) {
    if (!h) return;
    aws_mem_release(h->allocator, h);
}

}  // extern "C"
