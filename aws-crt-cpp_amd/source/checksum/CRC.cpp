/*
 * Aws::Crt::Checksum CRC API (reference source/checksum/CRC.cpp:13-45) over the MI355X engine.
 * Each call forwards to the aws-checksums-named C ABI (include/aws/checksums/crc.h): device inputs
 * are scanned in place by the gfx950 kernels; host inputs run on the engine's host path in the
 * default (AUTO) dispatch, and are staged through pinned memory to the GPU only when the GPU
 * dispatch is forced (AWS_CRT_AMD_DISPATCH=gpu).
 */
#include <aws/checksums/crc.h>
#include <aws/crt/checksum/CRC.h>

namespace Aws
{
namespace Crt
{
namespace Checksum
{
    uint32_t ComputeCRC32(ByteCursor input, uint32_t previousCRC32) noexcept
    {
        return aws_checksums_crc32_ex(input.ptr, input.len, previousCRC32);
    }

    uint32_t ComputeCRC32C(ByteCursor input, uint32_t previousCRC32C) noexcept
    {
        return aws_checksums_crc32c_ex(input.ptr, input.len, previousCRC32C);
    }

    uint64_t ComputeCRC64NVME(ByteCursor input, uint64_t previousCRC64NVME) noexcept
    {
        return aws_checksums_crc64nvme_ex(input.ptr, input.len, previousCRC64NVME);
    }

    uint32_t CombineCRC32(uint32_t crc1, uint32_t crc2, uint64_t len2) noexcept
    {
        return aws_checksums_crc32_combine(crc1, crc2, len2);
    }

    uint32_t CombineCRC32C(uint32_t crc1, uint32_t crc2, uint64_t len2) noexcept
    {
        return aws_checksums_crc32c_combine(crc1, crc2, len2);
    }

    uint64_t CombineCRC64NVME(uint64_t crc1, uint64_t crc2, uint64_t len2) noexcept
    {
        return aws_checksums_crc64nvme_combine(crc1, crc2, len2);
    }
} // namespace Checksum
} // namespace Crt
} // namespace Aws
