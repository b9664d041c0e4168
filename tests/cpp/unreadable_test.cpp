// A device buffer that neither the GPU nor a read-back can reach (tests/cpp/unreadable_stubs.cpp).
// The reference's CRC calls are value-only (include/aws/crt/checksum/CRC.h:20-36), so the failure
// must reach the caller through the thread's aws error (Aws::Crt::LastError(), reference
// source/Api.cpp:469-472); xxHash calls return false.  A host buffer afterwards is served.
#include <aws/crt/Api.h>
#include <aws/crt/checksum/CRC.h>
#include <aws/crt/checksum/XXHash.h>
#include <aws/testing/aws_test_harness.h>

using namespace Aws::Crt;

extern "C" const uint8_t g_unreadable[256];

static int s_UnreadableDeviceBufferRaises(struct aws_allocator *allocator, void *)
{
    ApiHandle handle(allocator);
    ByteCursor bad = aws_byte_cursor_from_array(g_unreadable, sizeof(g_unreadable));
    aws_reset_error();
    ASSERT_UINT_EQUALS(0x1234u, Checksum::ComputeCRC32C(bad, 0x1234u));
    ASSERT_INT_EQUALS(AWS_ERROR_UNSUPPORTED_OPERATION, LastError());
    aws_reset_error();
    (void)Checksum::ComputeCRC32(bad);
    ASSERT_INT_EQUALS(AWS_ERROR_UNSUPPORTED_OPERATION, LastError());
    aws_reset_error();
    (void)Checksum::ComputeCRC64NVME(bad);
    ASSERT_INT_EQUALS(AWS_ERROR_UNSUPPORTED_OPERATION, LastError());

    uint8_t out[16];
    ByteBuf buf = aws_byte_buf_from_empty_array(out, sizeof(out));
    aws_reset_error();
    ASSERT_FALSE(Checksum::ComputeXXHash64(bad, buf));
    ASSERT_INT_EQUALS(AWS_ERROR_UNSUPPORTED_OPERATION, LastError());

    // a host buffer is unaffected and raises nothing (reference tests/CRCTest.cpp known answer)
    const uint8_t digits[] = {'1', '2', '3', '4', '5', '6', '7', '8', '9'};
    aws_reset_error();
    ASSERT_UINT_EQUALS(0xE3069283u, Checksum::ComputeCRC32C(aws_byte_cursor_from_array(digits, sizeof(digits))));
    ASSERT_INT_EQUALS(0, LastError());
    return AWS_OP_SUCCESS;
}
AWS_TEST_CASE(UnreadableDeviceBufferRaises, s_UnreadableDeviceBufferRaises)
