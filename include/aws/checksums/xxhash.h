#pragma once
/*
 * aws-checksums xxhash C ABI, re-implemented on MI355X (gfx950).  Declarations inferred from the
 * reference's call sites (aws-checksums is un-vendored):
 *   aws_xxhash64_compute    <- source/checksum/XXHash.cpp:17    (ComputeXXHash64)
 *   aws_xxhash3_64_compute  <- source/checksum/XXHash.cpp:22    (ComputeXXHash3_64)
 *   aws_xxhash3_128_compute <- source/checksum/XXHash.cpp:27    (ComputeXXHash3_128)
 *   aws_xxhash64_new / aws_xxhash3_64_new / aws_xxhash3_128_new <- XXHash.cpp:40,45,50
 *   aws_xxhash_update       <- XXHash.cpp:55
 *   aws_xxhash_finalize     <- XXHash.cpp:65
 *   aws_xxhash_destroy      <- XXHash.cpp:30 (ScopedResource deleter)
 * Digests are appended to `out` in canonical (big-endian) byte order (XXHashTest.cpp:15).
 * Return AWS_OP_SUCCESS / AWS_OP_ERR with aws_last_error() set (AWS_ERROR_SHORT_BUFFER when `out`
 * lacks room).
 */
#include <aws/common/common.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(AWS_CRT_AMD_BUILD)
#    define AWS_XXHASH_API __attribute__((visibility("default")))
#else
#    define AWS_XXHASH_API
#endif

struct aws_xxhash;

AWS_XXHASH_API int aws_xxhash64_compute(uint64_t seed, struct aws_byte_cursor data, struct aws_byte_buf *out);
AWS_XXHASH_API int aws_xxhash3_64_compute(uint64_t seed, struct aws_byte_cursor data, struct aws_byte_buf *out);
AWS_XXHASH_API int aws_xxhash3_128_compute(uint64_t seed, struct aws_byte_cursor data, struct aws_byte_buf *out);

AWS_XXHASH_API struct aws_xxhash *aws_xxhash64_new(struct aws_allocator *allocator, uint64_t seed);
AWS_XXHASH_API struct aws_xxhash *aws_xxhash3_64_new(struct aws_allocator *allocator, uint64_t seed);
AWS_XXHASH_API struct aws_xxhash *aws_xxhash3_128_new(struct aws_allocator *allocator, uint64_t seed);
AWS_XXHASH_API int aws_xxhash_update(struct aws_xxhash *hash, struct aws_byte_cursor data);
AWS_XXHASH_API int aws_xxhash_finalize(struct aws_xxhash *hash, struct aws_byte_buf *out);
AWS_XXHASH_API void aws_xxhash_destroy(struct aws_xxhash *hash);

#ifdef __cplusplus
}
#endif
