#pragma once
/*
 * Aws::Crt::Checksum CRC entry points -- same declarations as the reference
 * include/aws/crt/checksum/CRC.h:20-51, computed on MI355X by aws-crt-cpp_amd.
 *
 *   CRC32      Ethernet/gzip, reflected 0x04C11DB7
 *   CRC32C     Castagnoli/iSCSI, reflected 0x1EDC6F41
 *   CRC64NVME  reflected form of 0xAD93D23594C93659 (a.k.a. CRC64-Rocksoft)
 * All three invert the register on entry and exit.  previous* is the finalised CRC of the bytes
 * that precede `input` (0 to start).  Combine*(crc1, crc2, len2) is the CRC of A||B given
 * crc1 = CRC(A), crc2 = CRC(B) and len2 = |B|.
 */
#include <aws/crt/Exports.h>
#include <aws/crt/Types.h>

namespace Aws
{
namespace Crt
{
namespace Checksum
{
    uint32_t AWS_CRT_CPP_API ComputeCRC32(ByteCursor input, uint32_t previousCRC32 = 0) noexcept;
    uint32_t AWS_CRT_CPP_API ComputeCRC32C(ByteCursor input, uint32_t previousCRC32C = 0) noexcept;
    uint64_t AWS_CRT_CPP_API ComputeCRC64NVME(ByteCursor input, uint64_t previousCRC64NVME = 0) noexcept;

    uint32_t AWS_CRT_CPP_API CombineCRC32(uint32_t crc1, uint32_t crc2, uint64_t len2) noexcept;
    uint32_t AWS_CRT_CPP_API CombineCRC32C(uint32_t crc1, uint32_t crc2, uint64_t len2) noexcept;
    uint64_t AWS_CRT_CPP_API CombineCRC64NVME(uint64_t crc1, uint64_t crc2, uint64_t len2) noexcept;
} // namespace Checksum
} // namespace Crt
} // namespace Aws
