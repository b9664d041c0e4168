// aws-checksums xxhash C ABI (include/aws/checksums/xxhash.h) over the MI355X engine.
// Reference call sites: source/checksum/XXHash.cpp:17-65.
//
// One-shot digests run on the GPU (engine.cpp single path).  The streaming object keeps the bytes
// it is given and hashes them on the GPU at finalize: XXH64/XXH3 state updates are a serial chain
// per stream, so a device round trip per Update() would buy nothing.
#include <aws/checksums/xxhash.h>

#include <cstring>
#include <new>
#include <vector>

extern "C" int aws_crt_amd_xxh64_single(const void *input, size_t len, uint64_t seed, uint64_t *out);
extern "C" int aws_crt_amd_xxh3_single(int bits, const void *input, size_t len, uint64_t seed, uint64_t *out_hi_lo);

namespace {

enum Kind { K_XXH64 = 0, K_XXH3_64 = 1, K_XXH3_128 = 2 };

int write_digest(Kind k, const uint64_t *v, aws_byte_buf *out) {
    const size_t need = k == K_XXH3_128 ? 16 : 8;
    if (!out || out->capacity - out->len < need) return aws_raise_error(AWS_ERROR_SHORT_BUFFER);
    if (k == K_XXH3_128) {
        aws_byte_buf_write_be64(out, v[0]);  // high 64 bits first (canonical XXH128 form)
        aws_byte_buf_write_be64(out, v[1]);
    } else {
        aws_byte_buf_write_be64(out, v[0]);
    }
    return AWS_OP_SUCCESS;
}

int compute(Kind k, uint64_t seed, const uint8_t *p, size_t n, aws_byte_buf *out) {
    const size_t need = k == K_XXH3_128 ? 16 : 8;
    if (!out || out->capacity - out->len < need) return aws_raise_error(AWS_ERROR_SHORT_BUFFER);
    uint64_t v[2] = {0, 0};
    int rc = k == K_XXH64 ? aws_crt_amd_xxh64_single(p, n, seed, v)
                          : aws_crt_amd_xxh3_single(k == K_XXH3_64 ? 64 : 128, p, n, seed, v);
    if (rc != 0) return aws_raise_error(AWS_ERROR_UNSUPPORTED_OPERATION);
    return write_digest(k, v, out);
}

}  // namespace

struct aws_xxhash {
    aws_allocator *allocator;
    Kind kind;
    uint64_t seed;
    bool finalized;
    std::vector<uint8_t> data;
};

extern "C" {

int aws_xxhash64_compute(uint64_t seed, aws_byte_cursor data, aws_byte_buf *out) {
    return compute(K_XXH64, seed, data.ptr, data.len, out);
}
int aws_xxhash3_64_compute(uint64_t seed, aws_byte_cursor data, aws_byte_buf *out) {
    return compute(K_XXH3_64, seed, data.ptr, data.len, out);
}
int aws_xxhash3_128_compute(uint64_t seed, aws_byte_cursor data, aws_byte_buf *out) {
    return compute(K_XXH3_128, seed, data.ptr, data.len, out);
}

static aws_xxhash *make(aws_allocator *a, Kind k, uint64_t seed) {
    void *mem = aws_mem_acquire(a, sizeof(aws_xxhash));
    if (!mem) return nullptr;
    return new (mem) aws_xxhash{a, k, seed, false, {}};
}

aws_xxhash *aws_xxhash64_new(aws_allocator *a, uint64_t seed) { return make(a, K_XXH64, seed); }
aws_xxhash *aws_xxhash3_64_new(aws_allocator *a, uint64_t seed) { return make(a, K_XXH3_64, seed); }
aws_xxhash *aws_xxhash3_128_new(aws_allocator *a, uint64_t seed) { return make(a, K_XXH3_128, seed); }

int aws_xxhash_update(aws_xxhash *h, aws_byte_cursor data) {
    if (!h || h->finalized) return aws_raise_error(AWS_ERROR_INVALID_STATE);
    if (data.len) h->data.insert(h->data.end(), data.ptr, data.ptr + data.len);
    return AWS_OP_SUCCESS;
}

int aws_xxhash_finalize(aws_xxhash *h, aws_byte_buf *out) {
    if (!h || h->finalized) return aws_raise_error(AWS_ERROR_INVALID_STATE);
    int rc = compute(h->kind, h->seed, h->data.data(), h->data.size(), out);
    if (rc == AWS_OP_SUCCESS) {
        h->finalized = true;
        std::vector<uint8_t>().swap(h->data);
    }
    return rc;
}

void aws_xxhash_destroy(aws_xxhash *h) {
    if (!h) return;
    aws_allocator *a = h->allocator;
    h->~aws_xxhash();
    aws_mem_release(a, h);
}

}  // extern "C"
