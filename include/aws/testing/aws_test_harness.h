#pragma once
/*
 * Minimal stand-in for aws-c-common's aws/testing/aws_test_harness.h, enough for the checksum
 * tests (reference tests/CRCTest.cpp:7, tests/XXHashTest.cpp:7) to compile unmodified against the
 * MI355X drop-in.  Test functions have the aws-c-common signature
 *   int fn(struct aws_allocator *allocator, void *ctx)
 * and are registered by AWS_TEST_CASE(name, fn); tests/cpp/test_main.cpp runs them by name.
 */
#include <aws/common/common.h>

#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#define AWS_OP_SKIP (-2)

namespace aws_test_harness
{
    using test_fn = int (*)(struct aws_allocator *, void *);
    struct entry
    {
        const char *name;
        test_fn fn;
    };
    inline std::vector<entry> &registry()
    {
        static std::vector<entry> r;
        return r;
    }
    struct registrar
    {
        registrar(const char *name, test_fn fn) { registry().push_back({name, fn}); }
    };
} // namespace aws_test_harness

#define AWS_TEST_CASE(name, fn) static aws_test_harness::registrar s_aws_test_reg_##name(#name, fn);

#define AWS_HARNESS_FAIL(...)                                                                                          \
    do                                                                                                                 \
    {                                                                                                                  \
        std::fprintf(stderr, "***FAILURE*** %s:%d: ", __FILE__, __LINE__);                                             \
        std::fprintf(stderr, __VA_ARGS__);                                                                             \
        std::fprintf(stderr, "\n");                                                                                    \
        return AWS_OP_ERR;                                                                                             \
    } while (0)

#define ASSERT_TRUE(cond, ...)                                                                                         \
    do                                                                                                                 \
    {                                                                                                                  \
        if (!(cond))                                                                                                   \
            AWS_HARNESS_FAIL("expected true: %s", #cond);                                                              \
    } while (0)

#define ASSERT_FALSE(cond, ...) ASSERT_TRUE(!(cond))

#define ASSERT_UINT_EQUALS(expected, got, ...)                                                                         \
    do                                                                                                                 \
    {                                                                                                                  \
        const uint64_t e_ = (uint64_t)(expected);                                                                      \
        const uint64_t g_ = (uint64_t)(got);                                                                           \
        if (e_ != g_)                                                                                                  \
            AWS_HARNESS_FAIL("expected 0x%" PRIx64 " got 0x%" PRIx64 " (%s)", e_, g_, #got);                          \
    } while (0)

#define ASSERT_INT_EQUALS(expected, got, ...)                                                                          \
    do                                                                                                                 \
    {                                                                                                                  \
        const long long e_ = (long long)(expected);                                                                    \
        const long long g_ = (long long)(got);                                                                         \
        if (e_ != g_)                                                                                                  \
            AWS_HARNESS_FAIL("expected %lld got %lld (%s)", e_, g_, #got);                                             \
    } while (0)

#define ASSERT_SUCCESS(expr, ...) ASSERT_INT_EQUALS(AWS_OP_SUCCESS, (expr))

#define ASSERT_BIN_ARRAYS_EQUALS(expected, expected_len, got, got_len, ...)                                            \
    do                                                                                                                 \
    {                                                                                                                  \
        const size_t el_ = (size_t)(expected_len);                                                                     \
        const size_t gl_ = (size_t)(got_len);                                                                          \
        if (el_ != gl_)                                                                                                \
            AWS_HARNESS_FAIL("length mismatch: expected %zu got %zu", el_, gl_);                                       \
        if (el_ && std::memcmp((const void *)(expected), (const void *)(got), el_) != 0)                               \
            AWS_HARNESS_FAIL("byte arrays differ (%s vs %s)", #expected, #got);                                        \
    } while (0)
