#pragma once
/*
 * Trimmed Types.h: only what the checksum path needs from the reference's
 * include/aws/crt/Types.h -- the ByteBuf / ByteCursor aliases (:30-31), ScopedResource (:168) and the
 * Base64 helpers that carry checksums on the S3 wire (:70-75).
 * The reference version also pulls in aws/io/socket.h and aws/mqtt/mqtt.h (:11-12), which are out
 * of scope here.  String / Vector are bound to StlAllocator exactly as
 * in the reference (:45-53), so their types and mangled names match a real aws-crt-cpp build.
 * C++11, like the reference (CMakeLists.txt:34-36).
 */
#include <aws/common/common.h>
#include <aws/crt/Allocator.h>
#include <aws/crt/Exports.h>
#include <aws/crt/StlAllocator.h>

#include <functional>
#include <memory>
#include <string>
#include <vector>

namespace Aws
{
namespace Crt
{
    using ByteBuf = aws_byte_buf;
    using ByteCursor = aws_byte_cursor;

    using String = std::basic_string<char, std::char_traits<char>, StlAllocator<char>>;
    template <typename T> using Vector = std::vector<T, StlAllocator<T>>;

    template <typename T> using ScopedResource = std::unique_ptr<T, std::function<void(T *)>>;

    AWS_CRT_CPP_API ByteCursor ByteCursorFromCString(const char *str) noexcept;
    AWS_CRT_CPP_API ByteCursor ByteCursorFromArray(const uint8_t *array, size_t len) noexcept;
    AWS_CRT_CPP_API ByteCursor ByteCursorFromByteBuf(const ByteBuf &) noexcept;
    AWS_CRT_CPP_API ByteBuf ByteBufFromArray(const uint8_t *array, size_t capacity) noexcept;
    AWS_CRT_CPP_API ByteBuf ByteBufInit(Allocator *alloc, size_t len);
    AWS_CRT_CPP_API void ByteBufDelete(ByteBuf &);
    AWS_CRT_CPP_API ByteCursor ByteCursorFromString(const String &str) noexcept;

    // RFC 4648 base64 with padding.  Decode returns an empty vector on malformed input (length not a
    // multiple of 4, a character outside the alphabet, or misplaced padding), as the reference does.
    AWS_CRT_CPP_API Vector<uint8_t> Base64Decode(const String &decode) noexcept;
    AWS_CRT_CPP_API Vector<uint8_t> Base64Decode(ByteCursor decode) noexcept;
    AWS_CRT_CPP_API size_t Base64DecodedLength(ByteCursor decode) noexcept;
    AWS_CRT_CPP_API String Base64Encode(const Vector<uint8_t> &encode) noexcept;
    AWS_CRT_CPP_API String Base64Encode(ByteCursor encode) noexcept;
    AWS_CRT_CPP_API size_t Base64EncodedLength(ByteCursor encode) noexcept;
} // namespace Crt
} // namespace Aws
