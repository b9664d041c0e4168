#pragma once
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(AWS_CRT_AMD_BUILD)
#    define AWS_COMMON_SHIM_API __attribute__((visibility("default")))
#else
#    define AWS_COMMON_SHIM_API
#endif

/* field layout of aws-c-common's struct aws_allocator */
struct aws_allocator {
    void *(*mem_acquire)(struct aws_allocator *allocator, size_t size);
    void (*mem_release)(struct aws_allocator *allocator, void *ptr);
    void *(*mem_realloc)(struct aws_allocator *allocator, void *oldptr, size_t oldsize, size_t newsize);
    void *(*mem_calloc)(struct aws_allocator *allocator, size_t num, size_t size);
    void *impl;
};

AWS_COMMON_SHIM_API struct aws_allocator *aws_default_allocator(void);
AWS_COMMON_SHIM_API void *aws_mem_acquire(struct aws_allocator *allocator, size_t size);
AWS_COMMON_SHIM_API void *aws_mem_calloc(struct aws_allocator *allocator, size_t num, size_t size);
AWS_COMMON_SHIM_API void aws_mem_release(struct aws_allocator *allocator, void *ptr);

#ifdef __cplusplus
}
#endif
