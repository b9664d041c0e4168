/*
 * Base64 helpers of the reference's Types.h:70-75 (Types.cpp:78-145 there delegates to
 * aws-c-common's aws_base64_*).  Host code: a checksum's wire form is 4 or 8 bytes, not payload.
 *   encoded length = 4 * ceil(n / 3), no terminator;
 *   decoded length = 3 * (len / 4) minus the '=' padding, 0 when len is not a multiple of 4.
 */
#include <aws/crt/Types.h>

namespace Aws
{
namespace Crt
{
    namespace
    {
        constexpr char kAlphabet[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

        int sextet(uint8_t c)
        {
            if (c >= 'A' && c <= 'Z')
                return c - 'A';
            if (c >= 'a' && c <= 'z')
                return c - 'a' + 26;
            if (c >= '0' && c <= '9')
                return c - '0' + 52;
            if (c == '+')
                return 62;
            if (c == '/')
                return 63;
            return -1;
        }

        // decoded size, or -1 when the input cannot be base64
        long decoded_size(ByteCursor in)
        {
            if (in.len % 4 != 0)
                return -1;
            if (in.len == 0)
                return 0;
            size_t pad = 0;
            if (in.ptr[in.len - 1] == '=')
                pad = in.ptr[in.len - 2] == '=' ? 2 : 1;
            return (long)(in.len / 4 * 3 - pad);
        }
    } // namespace

    ByteCursor ByteCursorFromString(const String &str) noexcept
    {
        return aws_byte_cursor_from_array((const void *)str.data(), str.size());
    }

    size_t Base64EncodedLength(ByteCursor encode) noexcept { return (encode.len + 2) / 3 * 4; }

    size_t Base64DecodedLength(ByteCursor decode) noexcept
    {
        const long n = decoded_size(decode);
        return n < 0 ? 0 : (size_t)n;
    }

    String Base64Encode(ByteCursor encode) noexcept
    {
        String out;
        out.reserve(Base64EncodedLength(encode));
        size_t i = 0;
        for (; i + 3 <= encode.len; i += 3)
        {
            const uint32_t v = (uint32_t)encode.ptr[i] << 16 | (uint32_t)encode.ptr[i + 1] << 8 | encode.ptr[i + 2];
            out.push_back(kAlphabet[v >> 18]);
            out.push_back(kAlphabet[(v >> 12) & 63]);
            out.push_back(kAlphabet[(v >> 6) & 63]);
            out.push_back(kAlphabet[v & 63]);
        }
        const size_t rest = encode.len - i;
        if (rest)
        {
            const uint32_t v = (uint32_t)encode.ptr[i] << 16 | (rest == 2 ? (uint32_t)encode.ptr[i + 1] << 8 : 0u);
            out.push_back(kAlphabet[v >> 18]);
            out.push_back(kAlphabet[(v >> 12) & 63]);
            out.push_back(rest == 2 ? kAlphabet[(v >> 6) & 63] : '=');
            out.push_back('=');
        }
        return out;
    }

    String Base64Encode(const Vector<uint8_t> &encode) noexcept
    {
        return Base64Encode(aws_byte_cursor_from_array(encode.data(), encode.size()));
    }

    Vector<uint8_t> Base64Decode(ByteCursor decode) noexcept
    {
        const long n = decoded_size(decode);
        if (n <= 0)
            return {};
        Vector<uint8_t> out;
        out.reserve((size_t)n);
        for (size_t i = 0; i < decode.len; i += 4)
        {
            const bool last = i + 4 == decode.len;
            int s[4];
            for (int k = 0; k < 4; ++k)
            {
                const uint8_t c = decode.ptr[i + k];
                // '=' is only valid as the last one or two characters of the final quantum
                s[k] = (c == '=' && last && k >= 2 && (k == 3 || decode.ptr[i + 3] == '=')) ? 0 : sextet(c);
                if (s[k] < 0)
                    return {};
            }
            const uint32_t v = (uint32_t)s[0] << 18 | (uint32_t)s[1] << 12 | (uint32_t)s[2] << 6 | (uint32_t)s[3];
            out.push_back((uint8_t)(v >> 16));
            if (out.size() < (size_t)n)
                out.push_back((uint8_t)(v >> 8));
            if (out.size() < (size_t)n)
                out.push_back((uint8_t)v);
        }
        return out;
    }

    Vector<uint8_t> Base64Decode(const String &decode) noexcept { return Base64Decode(ByteCursorFromString(decode)); }
} // namespace Crt
} // namespace Aws
