#pragma once
/*
 * Symbol visibility for the Aws::Crt drop-in (behaviour of the reference's
 * include/aws/crt/Exports.h:18-38 on ELF: default visibility only when building the shared
 * library with import/export enabled).
 */
#if defined(AWS_CRT_CPP_USE_IMPORT_EXPORT) && defined(AWS_CRT_CPP_EXPORTS)
#    define AWS_CRT_CPP_API __attribute__((visibility("default")))
#else
#    define AWS_CRT_CPP_API
#endif
