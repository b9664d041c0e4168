// Test driver for AWS_TEST_CASE-registered tests (the role aws-c-common's generated
// aws-crt-cpp-tests driver plays in the reference, tests/CMakeLists.txt:9,373).
//   ./checksum_tests            run every registered test
//   ./checksum_tests NAME ...   run the named tests
#include <aws/common/common.h>
#include <aws/testing/aws_test_harness.h>
#include <aws_crt_amd/checksums_batch.h>

#include <cstdio>
#include <cstring>

int main(int argc, char **argv)
{
    int failed = 0, ran = 0;
    for (const auto &e : aws_test_harness::registry())
    {
        bool want = argc <= 1;
        for (int i = 1; i < argc; ++i)
            want = want || std::strcmp(argv[i], e.name) == 0;
        if (!want)
            continue;
        ++ran;
        int rc = e.fn(aws_default_allocator(), nullptr);
        std::printf("[%s] %s\n", rc == AWS_OP_SUCCESS ? "PASS" : (rc == AWS_OP_SKIP ? "SKIP" : "FAIL"), e.name);
        if (rc != AWS_OP_SUCCESS && rc != AWS_OP_SKIP)
            ++failed;
    }
    std::printf("%d ran, %d failed\n", ran, failed);
    // where the single-buffer ABI ran (tests/test_cpp_dropin.py checks a forced-GPU run fell back 0 times)
    std::printf("dispatch %d, gpu fallbacks %llu\n", aws_crt_amd_get_dispatch(), aws_crt_amd_fallback_count());
    return failed ? 1 : (ran ? 0 : 2);
}
