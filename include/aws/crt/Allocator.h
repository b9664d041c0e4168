#pragma once
/* Allocator subset of the reference's include/aws/crt/Allocator.h:14-44. */
#include <aws/common/common.h>
#include <aws/crt/Exports.h>

namespace Aws
{
namespace Crt
{
    using Allocator = aws_allocator;

    /* Allocator used by objects created without an explicit one (set by ApiHandle). */
    AWS_CRT_CPP_API Allocator *ApiAllocator() noexcept;
    AWS_CRT_CPP_API Allocator *DefaultAllocatorImplementation() noexcept;
    AWS_CRT_CPP_API Allocator *DefaultAllocator() noexcept;
    extern AWS_CRT_CPP_API Allocator *g_allocator;
} // namespace Crt
} // namespace Aws
