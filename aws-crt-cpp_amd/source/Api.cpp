/*
 * ApiHandle, allocator and error subset (reference source/Api.cpp:43-94, :459-480;
 * source/Allocator.cpp:13-28; source/Types.cpp:13-76) for the checksum path.
 */
#include <aws/checksums/crc.h>
#include <aws/crt/Api.h>

namespace Aws
{
namespace Crt
{
    Allocator *g_allocator = nullptr;

    Allocator *DefaultAllocatorImplementation() noexcept { return aws_default_allocator(); }
    Allocator *DefaultAllocator() noexcept { return DefaultAllocatorImplementation(); }
    Allocator *ApiAllocator() noexcept { return g_allocator ? g_allocator : DefaultAllocatorImplementation(); }

    ApiHandle::ApiHandle(Allocator *allocator) noexcept
    {
        g_allocator = allocator;
        aws_checksums_library_init(allocator);
    }

    ApiHandle::ApiHandle() noexcept : ApiHandle(DefaultAllocator()) {}

    ApiHandle::~ApiHandle()
    {
        g_allocator = nullptr;
        aws_checksums_library_clean_up();
    }

    const char *ErrorDebugString(int error) noexcept { return aws_error_debug_str(error); }
    const char *ErrorName(int error) noexcept { return aws_error_name(error); }
    int LastError() noexcept { return aws_last_error(); }
    int LastErrorOrUnknown() noexcept
    {
        int e = aws_last_error();
        return e == AWS_ERROR_SUCCESS ? AWS_ERROR_UNKNOWN : e;
    }

    ByteCursor ByteCursorFromCString(const char *str) noexcept { return aws_byte_cursor_from_c_str(str); }
    ByteCursor ByteCursorFromArray(const uint8_t *array, size_t len) noexcept
    {
        return aws_byte_cursor_from_array(array, len);
    }
    ByteCursor ByteCursorFromByteBuf(const ByteBuf &buf) noexcept { return aws_byte_cursor_from_buf(&buf); }
    ByteBuf ByteBufFromArray(const uint8_t *array, size_t capacity) noexcept
    {
        return aws_byte_buf_from_array(array, capacity);
    }
    ByteBuf ByteBufInit(Allocator *alloc, size_t len)
    {
        ByteBuf b;
        aws_byte_buf_init(&b, alloc, len);
        return b;
    }
    void ByteBufDelete(ByteBuf &buf) { aws_byte_buf_clean_up(&buf); }
} // namespace Crt
} // namespace Aws
