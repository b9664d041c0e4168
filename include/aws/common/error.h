#pragma once
#include <aws/common/allocator.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AWS_OP_SUCCESS (0)
#define AWS_OP_ERR (-1)

/* error codes (values of aws-c-common's enum aws_common_error) */
enum {
    AWS_ERROR_SUCCESS = 0,
    AWS_ERROR_OOM = 1,
    AWS_ERROR_NO_SPACE = 2,
    AWS_ERROR_UNKNOWN = 3,
    AWS_ERROR_SHORT_BUFFER = 4,
    AWS_ERROR_INVALID_ARGUMENT = 34,
    AWS_ERROR_UNSUPPORTED_OPERATION = 39,
    AWS_ERROR_INVALID_STATE = 44,
};

AWS_COMMON_SHIM_API int aws_last_error(void);
AWS_COMMON_SHIM_API int aws_raise_error(int err);
AWS_COMMON_SHIM_API void aws_reset_error(void);
AWS_COMMON_SHIM_API const char *aws_error_name(int err);
AWS_COMMON_SHIM_API const char *aws_error_debug_str(int err);

#ifdef __cplusplus
}
#endif
