#pragma once
/*
 * Aws::Crt::Checksum xxHash entry points -- same declarations as the reference
 * include/aws/crt/checksum/XXHash.h:16-91.  One-shot functions append the canonical (big-endian)
 * digest to `output` and return false with Aws::Crt::LastError() set on failure.  XXHash is the
 * move-only streaming form: Update() any number of times, then Digest() once.
 */
#include <aws/crt/Exports.h>
#include <aws/crt/Types.h>

struct aws_xxhash;

namespace Aws
{
namespace Crt
{
namespace Checksum
{
    bool AWS_CRT_CPP_API ComputeXXHash64(const ByteCursor &input, ByteBuf &output, uint64_t seed = 0) noexcept;
    bool AWS_CRT_CPP_API ComputeXXHash3_64(const ByteCursor &input, ByteBuf &output, uint64_t seed = 0) noexcept;
    bool AWS_CRT_CPP_API ComputeXXHash3_128(const ByteCursor &input, ByteBuf &output, uint64_t seed = 0) noexcept;

    class AWS_CRT_CPP_API XXHash final
    {
      public:
        XXHash(const XXHash &) = delete;
        XXHash &operator=(const XXHash &) = delete;
        XXHash(XXHash &&toMove) noexcept = default;
        XXHash &operator=(XXHash &&toMove) noexcept = default;

        /* aws error of the last failed operation on this object */
        inline int LastError() const noexcept { return m_lastError; }

        static XXHash CreateXXHash64(uint64_t seed = 0, Allocator *allocator = ApiAllocator()) noexcept;
        static XXHash CreateXXHash3_64(uint64_t seed = 0, Allocator *allocator = ApiAllocator()) noexcept;
        static XXHash CreateXXHash3_128(uint64_t seed = 0, Allocator *allocator = ApiAllocator()) noexcept;

        bool Update(const ByteCursor &toHash) noexcept;
        bool Digest(ByteBuf &output) noexcept;

      private:
        explicit XXHash(aws_xxhash *hash) noexcept;
        XXHash() = delete;

        ScopedResource<struct aws_xxhash> m_hash;
        int m_lastError;
    };
} // namespace Checksum
} // namespace Crt
} // namespace Aws
