#pragma once
/*
 * ApiHandle / error subset of the reference's include/aws/crt/Api.h (:47-259).  For the checksum
 * path the handle sets the default allocator and brings the MI355X engine up
 * (aws_checksums_library_init, reference source/Api.cpp:53) and down (:84).
 */
#include <aws/crt/Allocator.h>
#include <aws/crt/Exports.h>
#include <aws/crt/Types.h>

namespace Aws
{
namespace Crt
{
    class AWS_CRT_CPP_API ApiHandle
    {
      public:
        ApiHandle(Allocator *allocator) noexcept;
        ApiHandle() noexcept;
        ~ApiHandle();
        ApiHandle(const ApiHandle &) = delete;
        ApiHandle(ApiHandle &&) = delete;
        ApiHandle &operator=(const ApiHandle &) = delete;
        ApiHandle &operator=(ApiHandle &&) = delete;
    };

    AWS_CRT_CPP_API const char *ErrorDebugString(int error) noexcept;
    AWS_CRT_CPP_API const char *ErrorName(int error) noexcept;
    /* last aws error raised on this thread (0 if none), reference Api.h:251 */
    AWS_CRT_CPP_API int LastError() noexcept;
    AWS_CRT_CPP_API int LastErrorOrUnknown() noexcept;
} // namespace Crt
} // namespace Aws
