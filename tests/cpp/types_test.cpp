// Base64 helpers of the Types surface (reference include/aws/crt/Types.h:70-75), CPU only.
// The first case is the reference's own Base64RoundTrip vector (tests/TypesTest.cpp:17-31); the
// rest are the RFC 4648 section 10 vectors, the S3 wire forms of the CRC check values, and
// malformed inputs (empty result, as aws_base64_decode failing makes the reference return {}).
#include <aws/crt/Types.h>
#include <aws/testing/aws_test_harness.h>

#include <cstring>

using namespace Aws::Crt;

static int s_base64_round_trip(struct aws_allocator *, void *)
{
    const String test_data = "foobar", expected = "Zm9vYmFy";
    const Vector<uint8_t> v(test_data.begin(), test_data.end());
    const String enc = Base64Encode(v);
    ASSERT_BIN_ARRAYS_EQUALS(expected.data(), expected.size(), enc.data(), enc.size());
    ASSERT_UINT_EQUALS(enc.size(), Base64EncodedLength(ByteCursorFromArray(v.data(), v.size())));
    const Vector<uint8_t> dec = Base64Decode(enc);
    ASSERT_BIN_ARRAYS_EQUALS(v.data(), v.size(), dec.data(), dec.size());
    ASSERT_UINT_EQUALS(dec.size(), Base64DecodedLength(ByteCursorFromString(enc)));
    return 0;
}
AWS_TEST_CASE(Base64RoundTrip, s_base64_round_trip)

static int s_base64_rfc4648(struct aws_allocator *, void *)
{
    const char *plain[] = {"", "f", "fo", "foo", "foob", "fooba", "foobar"};
    const char *coded[] = {"", "Zg==", "Zm8=", "Zm9v", "Zm9vYg==", "Zm9vYmE=", "Zm9vYmFy"};
    for (int i = 0; i < 7; ++i)
    {
        const String p = plain[i], c = coded[i];
        const String e = Base64Encode(ByteCursorFromString(p));
        ASSERT_BIN_ARRAYS_EQUALS(c.data(), c.size(), e.data(), e.size());
        const Vector<uint8_t> d = Base64Decode(c);
        ASSERT_BIN_ARRAYS_EQUALS(p.data(), p.size(), d.data(), d.size());
        ASSERT_UINT_EQUALS(p.size(), Base64DecodedLength(ByteCursorFromString(c)));
    }
    return 0;
}
AWS_TEST_CASE(Base64Rfc4648, s_base64_rfc4648)

static int s_base64_checksum_wire_forms(struct aws_allocator *, void *)
{
    // big-endian bytes of the check values ("123456789"): CRC32C 0xE3069283, CRC32 0xCBF43926,
    // CRC64NVME 0xAE8B14860A799888
    const uint8_t c32c[] = {0xE3, 0x06, 0x92, 0x83}, c32[] = {0xCB, 0xF4, 0x39, 0x26};
    const uint8_t c64[] = {0xAE, 0x8B, 0x14, 0x86, 0x0A, 0x79, 0x98, 0x88};
    const String a = Base64Encode(ByteCursorFromArray(c32c, 4)), b = Base64Encode(ByteCursorFromArray(c32, 4));
    const String c = Base64Encode(ByteCursorFromArray(c64, 8));
    ASSERT_TRUE(a == "4waSgw==");
    ASSERT_TRUE(b == "y/Q5Jg==");
    ASSERT_TRUE(c == "rosUhgp5mIg=");
    return 0;
}
AWS_TEST_CASE(Base64ChecksumWireForms, s_base64_checksum_wire_forms)

static int s_base64_malformed(struct aws_allocator *, void *)
{
    const char *bad[] = {"Zm9", "Zm9v!A==", "Z===", "Zg=a", "=Zm9", "Zm=v"};
    for (const char *b : bad)
        ASSERT_UINT_EQUALS(0, Base64Decode(String(b)).size());
    ASSERT_UINT_EQUALS(0, Base64DecodedLength(ByteCursorFromString(String("abc"))));
    return 0;
}
AWS_TEST_CASE(Base64Malformed, s_base64_malformed)
