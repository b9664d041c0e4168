#pragma once
/*
 * Trimmed Types.h: only what the checksum path needs from the reference's
 * include/aws/crt/Types.h -- the ByteBuf / ByteCursor aliases (:30-31) and ScopedResource (:168).
 * The reference version also pulls in aws/io/socket.h and aws/mqtt/mqtt.h (:11-12), which are out
 * of scope here.
 */
#include <aws/common/common.h>
#include <aws/crt/Allocator.h>
#include <aws/crt/Exports.h>

#include <functional>
#include <memory>

namespace Aws::Crt
{
    using ByteBuf = aws_byte_buf;
    using ByteCursor = aws_byte_cursor;

    template <typename T> using ScopedResource = std::unique_ptr<T, std::function<void(T *)>>;

    AWS_CRT_CPP_API ByteCursor ByteCursorFromCString(const char *str) noexcept;
    AWS_CRT_CPP_API ByteCursor ByteCursorFromArray(const uint8_t *array, size_t len) noexcept;
    AWS_CRT_CPP_API ByteCursor ByteCursorFromByteBuf(const ByteBuf &) noexcept;
    AWS_CRT_CPP_API ByteBuf ByteBufFromArray(const uint8_t *array, size_t capacity) noexcept;
    AWS_CRT_CPP_API ByteBuf ByteBufInit(Allocator *alloc, size_t len);
    AWS_CRT_CPP_API void ByteBufDelete(ByteBuf &);
} // namespace Aws::Crt
