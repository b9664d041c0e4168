#pragma once
/*
 * aws-checksums CRC C ABI, re-implemented on MI355X (gfx950).
 *
 * Names and signatures are the ones the reference binds (aws-checksums itself is an un-vendored
 * submodule, .gitmodules:25-27, so the declarations are inferred from the call sites):
 *   aws_checksums_crc32_ex        <- source/checksum/CRC.cpp:17   (ComputeCRC32)
 *   aws_checksums_crc32c_ex       <- source/checksum/CRC.cpp:22   (ComputeCRC32C)
 *   aws_checksums_crc64nvme_ex    <- source/checksum/CRC.cpp:27   (ComputeCRC64NVME)
 *   aws_checksums_crc32_combine   <- source/checksum/CRC.cpp:32   (CombineCRC32)
 *   aws_checksums_crc32c_combine  <- source/checksum/CRC.cpp:37   (CombineCRC32C)
 *   aws_checksums_crc64nvme_combine <- source/checksum/CRC.cpp:42 (CombineCRC64NVME)
 *   aws_checksums_library_init / _clean_up <- source/Api.cpp:53 / :84
 *
 * `input` may be host memory or a device address.  Device-resident input is scanned in place by the
 * gfx950 kernels; host input runs on the host path chosen from CPUID (AVX-512 VPCLMULQDQ /
 * PCLMULQDQ folding, SSE4.2 crc32, tables), as aws-checksums does (CRC.h:17-19), unless
 * aws_crt_amd_set_dispatch(AWS_CRT_AMD_DISPATCH_GPU) routes it through the GPU.  The *_ex functions
 * have no error channel (CRC.h:20-51 are noexcept, value-only): any GPU failure, or no device at
 * all, falls back to the host path; they never abort.
 */
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct aws_allocator;

#if defined(AWS_CRT_AMD_BUILD)
#    define AWS_CHECKSUMS_API __attribute__((visibility("default")))
#else
#    define AWS_CHECKSUMS_API
#endif

AWS_CHECKSUMS_API void aws_checksums_library_init(struct aws_allocator *allocator);
AWS_CHECKSUMS_API void aws_checksums_library_clean_up(void);

AWS_CHECKSUMS_API uint32_t aws_checksums_crc32_ex(const uint8_t *input, size_t length, uint32_t previous_crc32);
AWS_CHECKSUMS_API uint32_t aws_checksums_crc32c_ex(const uint8_t *input, size_t length, uint32_t previous_crc32c);
AWS_CHECKSUMS_API uint64_t aws_checksums_crc64nvme_ex(const uint8_t *input, size_t length, uint64_t previous_crc64);

/* int-length legacy forms (aws-checksums keeps them next to the _ex forms) */
AWS_CHECKSUMS_API uint32_t aws_checksums_crc32(const uint8_t *input, int length, uint32_t previous_crc32);
AWS_CHECKSUMS_API uint32_t aws_checksums_crc32c(const uint8_t *input, int length, uint32_t previous_crc32c);
AWS_CHECKSUMS_API uint64_t aws_checksums_crc64nvme(const uint8_t *input, int length, uint64_t previous_crc64);

AWS_CHECKSUMS_API uint32_t aws_checksums_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);
AWS_CHECKSUMS_API uint32_t aws_checksums_crc32c_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);
AWS_CHECKSUMS_API uint64_t aws_checksums_crc64nvme_combine(uint64_t crc1, uint64_t crc2, uint64_t len2);

#ifdef __cplusplus
}
#endif
