#pragma once
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <aws/common/allocator.h>

#ifdef __cplusplus
extern "C" {
#endif

/* field order of aws-c-common's structs (evidenced by ByteCursor{0, nullptr}, source/s3/S3.cpp:820) */
struct aws_byte_cursor {
    size_t len;
    uint8_t *ptr;
};

struct aws_byte_buf {
    size_t len;
    uint8_t *buffer;
    size_t capacity;
    struct aws_allocator *allocator;
};

AWS_COMMON_SHIM_API struct aws_byte_cursor aws_byte_cursor_from_array(const void *bytes, size_t len);
AWS_COMMON_SHIM_API struct aws_byte_cursor aws_byte_cursor_from_c_str(const char *c_str);
AWS_COMMON_SHIM_API struct aws_byte_cursor aws_byte_cursor_from_buf(const struct aws_byte_buf *buf);

AWS_COMMON_SHIM_API int aws_byte_buf_init(struct aws_byte_buf *buf, struct aws_allocator *allocator, size_t capacity);
AWS_COMMON_SHIM_API void aws_byte_buf_clean_up(struct aws_byte_buf *buf);
AWS_COMMON_SHIM_API void aws_byte_buf_reset(struct aws_byte_buf *buf, bool zero_contents);
AWS_COMMON_SHIM_API struct aws_byte_buf aws_byte_buf_from_array(const void *bytes, size_t len);
AWS_COMMON_SHIM_API struct aws_byte_buf aws_byte_buf_from_empty_array(const void *bytes, size_t capacity);
AWS_COMMON_SHIM_API bool aws_byte_buf_write_be64(struct aws_byte_buf *buf, uint64_t x);
AWS_COMMON_SHIM_API bool aws_byte_buf_write(struct aws_byte_buf *buf, const uint8_t *src, size_t len);

#ifdef __cplusplus
}
#endif
