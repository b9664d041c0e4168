/*
 * The few aws-c-common functions the checksum path uses (byte cursor / buffer, default allocator,
 * thread-local last error).  aws-c-common is un-vendored in the reference (.gitmodules:1-4); a
 * full CRT build links the real library instead of this file.
 */
#include <aws/common/common.h>

#include <cstdlib>
#include <cstring>

namespace
{
    void *s_acquire(aws_allocator *, size_t size) { return std::malloc(size); }
    void s_release(aws_allocator *, void *ptr) { std::free(ptr); }
    void *s_realloc(aws_allocator *, void *old, size_t, size_t newsize) { return std::realloc(old, newsize); }
    void *s_calloc(aws_allocator *, size_t num, size_t size) { return std::calloc(num, size); }
    aws_allocator s_default = {s_acquire, s_release, s_realloc, s_calloc, nullptr};
    thread_local int s_last_error = 0;
} // namespace

extern "C"
{
    aws_allocator *aws_default_allocator(void) { return &s_default; }

    void *aws_mem_acquire(aws_allocator *a, size_t size)
    {
        void *p = (a ? a : &s_default)->mem_acquire(a, size);
        if (!p) aws_raise_error(AWS_ERROR_OOM);
        return p;
    }
    void *aws_mem_calloc(aws_allocator *a, size_t num, size_t size)
    {
        a = a ? a : &s_default;
        void *p = a->mem_calloc ? a->mem_calloc(a, num, size) : nullptr;
        if (!p && !a->mem_calloc)
        {
            p = a->mem_acquire(a, num * size);
            if (p) std::memset(p, 0, num * size);
        }
        if (!p) aws_raise_error(AWS_ERROR_OOM);
        return p;
    }
    void aws_mem_release(aws_allocator *a, void *ptr)
    {
        if (ptr) (a ? a : &s_default)->mem_release(a, ptr);
    }

    int aws_last_error(void) { return s_last_error; }
    int aws_raise_error(int err)
    {
        s_last_error = err;
        return AWS_OP_ERR;
    }
    void aws_reset_error(void) { s_last_error = 0; }
    const char *aws_error_name(int err)
    {
        switch (err)
        {
            case AWS_ERROR_SUCCESS: return "AWS_ERROR_SUCCESS";
            case AWS_ERROR_OOM: return "AWS_ERROR_OOM";
            case AWS_ERROR_SHORT_BUFFER: return "AWS_ERROR_SHORT_BUFFER";
            case AWS_ERROR_INVALID_ARGUMENT: return "AWS_ERROR_INVALID_ARGUMENT";
            case AWS_ERROR_UNSUPPORTED_OPERATION: return "AWS_ERROR_UNSUPPORTED_OPERATION";
            case AWS_ERROR_INVALID_STATE: return "AWS_ERROR_INVALID_STATE";
            default: return "AWS_ERROR_UNKNOWN";
        }
    }
    const char *aws_error_debug_str(int err) { return aws_error_name(err); }

    aws_byte_cursor aws_byte_cursor_from_array(const void *bytes, size_t len)
    {
        aws_byte_cursor c;
        c.len = len;
        c.ptr = (uint8_t *)bytes;
        return c;
    }
    aws_byte_cursor aws_byte_cursor_from_c_str(const char *s)
    {
        return aws_byte_cursor_from_array(s, s ? std::strlen(s) : 0);
    }
    aws_byte_cursor aws_byte_cursor_from_buf(const aws_byte_buf *b) { return aws_byte_cursor_from_array(b->buffer, b->len); }

    int aws_byte_buf_init(aws_byte_buf *buf, aws_allocator *a, size_t capacity)
    {
        buf->buffer = capacity ? (uint8_t *)aws_mem_acquire(a, capacity) : nullptr;
        if (capacity && !buf->buffer) return AWS_OP_ERR;
        buf->len = 0;
        buf->capacity = capacity;
        buf->allocator = a;
        return AWS_OP_SUCCESS;
    }
    void aws_byte_buf_clean_up(aws_byte_buf *buf)
    {
        if (buf->allocator && buf->buffer) aws_mem_release(buf->allocator, buf->buffer);
        buf->buffer = nullptr;
        buf->len = buf->capacity = 0;
        buf->allocator = nullptr;
    }
    void aws_byte_buf_reset(aws_byte_buf *buf, bool zero)
    {
        if (zero && buf->buffer) std::memset(buf->buffer, 0, buf->capacity);
        buf->len = 0;
    }
    aws_byte_buf aws_byte_buf_from_array(const void *bytes, size_t len)
    {
        aws_byte_buf b;
        b.len = len;
        b.buffer = (uint8_t *)bytes;
        b.capacity = len;
        b.allocator = nullptr;
        return b;
    }
    aws_byte_buf aws_byte_buf_from_empty_array(const void *bytes, size_t capacity)
    {
        aws_byte_buf b = aws_byte_buf_from_array(bytes, capacity);
        b.len = 0;
        return b;
    }
    bool aws_byte_buf_write(aws_byte_buf *buf, const uint8_t *src, size_t len)
    {
        if (buf->capacity - buf->len < len) return false;
        if (len) std::memcpy(buf->buffer + buf->len, src, len);
        buf->len += len;
        return true;
    }
    bool aws_byte_buf_write_be64(aws_byte_buf *buf, uint64_t x)
    {
        uint8_t be[8];
        for (int i = 0; i < 8; ++i) be[i] = (uint8_t)(x >> (56 - 8 * i));
        return aws_byte_buf_write(buf, be, 8);
    }
} // extern "C"
