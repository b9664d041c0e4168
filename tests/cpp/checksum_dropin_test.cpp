// Aws::Crt::Checksum drop-in tests for the MI355X engine, written against the same public API
// and known answers as the reference's tests/CRCTest.cpp and tests/XXHashTest.cpp, plus the
// running-CRC and Combine semantics those tests leave unpinned.
#include <aws/crt/Api.h>
#include <aws/crt/checksum/CRC.h>
#include <aws/crt/checksum/XXHash.h>
#include <aws/testing/aws_test_harness.h>

#include <vector>

using namespace Aws::Crt;

static std::vector<uint8_t> s_bytes(size_t n, uint64_t seed)
{
    std::vector<uint8_t> v(n);
    uint64_t x = seed;
    for (size_t i = 0; i < n; ++i)
    {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        v[i] = (uint8_t)(x >> 56);
    }
    return v;
}

static int s_ZeroBlockKnownAnswers(struct aws_allocator *allocator, void *)
{
    ApiHandle handle(allocator);
    uint8_t zeros[32] = {0};
    ByteCursor cur = aws_byte_cursor_from_array(zeros, sizeof(zeros));
    // known answers of reference tests/CRCTest.cpp:16, :29, :42
    ASSERT_UINT_EQUALS(0x190A55AD, Checksum::ComputeCRC32(cur));
    ASSERT_UINT_EQUALS(0x8A9136AA, Checksum::ComputeCRC32C(cur));
    ASSERT_UINT_EQUALS(0xCF3473434D4ECF3Bull, Checksum::ComputeCRC64NVME(cur));
    return AWS_OP_SUCCESS;
}
AWS_TEST_CASE(DropInZeroBlockKnownAnswers, s_ZeroBlockKnownAnswers)

static int s_CheckStrings(struct aws_allocator *allocator, void *)
{
    ApiHandle handle(allocator);
    ByteCursor cur = aws_byte_cursor_from_c_str("123456789");
    ASSERT_UINT_EQUALS(0xCBF43926, Checksum::ComputeCRC32(cur));
    ASSERT_UINT_EQUALS(0xE3069283, Checksum::ComputeCRC32C(cur));
    ASSERT_UINT_EQUALS(0xAE8B14860A799888ull, Checksum::ComputeCRC64NVME(cur));
    return AWS_OP_SUCCESS;
}
AWS_TEST_CASE(DropInCheckStrings, s_CheckStrings)

static int s_RunningAndCombine(struct aws_allocator *allocator, void *)
{
    ApiHandle handle(allocator);
    std::vector<uint8_t> data = s_bytes(300000, 42);
    for (size_t split : {size_t(0), size_t(1), size_t(15), size_t(4096), size_t(123457), data.size()})
    {
        ByteCursor all = aws_byte_cursor_from_array(data.data(), data.size());
        ByteCursor a = aws_byte_cursor_from_array(data.data(), split);
        ByteCursor b = aws_byte_cursor_from_array(data.data() + split, data.size() - split);

        uint32_t c32 = Checksum::ComputeCRC32(all), c32c = Checksum::ComputeCRC32C(all);
        uint64_t c64 = Checksum::ComputeCRC64NVME(all);
        ASSERT_UINT_EQUALS(c32, Checksum::ComputeCRC32(b, Checksum::ComputeCRC32(a)));
        ASSERT_UINT_EQUALS(c32c, Checksum::ComputeCRC32C(b, Checksum::ComputeCRC32C(a)));
        ASSERT_UINT_EQUALS(c64, Checksum::ComputeCRC64NVME(b, Checksum::ComputeCRC64NVME(a)));
        ASSERT_UINT_EQUALS(
            c32, Checksum::CombineCRC32(Checksum::ComputeCRC32(a), Checksum::ComputeCRC32(b), b.len));
        ASSERT_UINT_EQUALS(
            c32c, Checksum::CombineCRC32C(Checksum::ComputeCRC32C(a), Checksum::ComputeCRC32C(b), b.len));
        ASSERT_UINT_EQUALS(
            c64,
            Checksum::CombineCRC64NVME(Checksum::ComputeCRC64NVME(a), Checksum::ComputeCRC64NVME(b), b.len));
    }
    return AWS_OP_SUCCESS;
}
AWS_TEST_CASE(DropInRunningAndCombine, s_RunningAndCombine)

static int s_XXHash64(struct aws_allocator *allocator, void *)
{
    ApiHandle handle(allocator);
    ByteCursor cur = aws_byte_cursor_from_c_str("Hello world");
    const uint8_t want[] = {0xc5, 0x00, 0xb0, 0xc9, 0x12, 0xb3, 0x76, 0xd8};  // XXHashTest.cpp:15
    ByteBuf out;
    aws_byte_buf_init(&out, allocator, 8);
    ASSERT_TRUE(Checksum::ComputeXXHash64(cur, out));
    ASSERT_BIN_ARRAYS_EQUALS(want, sizeof(want), out.buffer, out.len);
    aws_byte_buf_reset(&out, false);
    auto h = Checksum::XXHash::CreateXXHash64(0, allocator);
    ASSERT_TRUE(h.Update(aws_byte_cursor_from_c_str("Hello ")));
    ASSERT_TRUE(h.Update(aws_byte_cursor_from_c_str("world")));
    ASSERT_TRUE(h.Digest(out));
    ASSERT_BIN_ARRAYS_EQUALS(want, sizeof(want), out.buffer, out.len);
    // a full buffer is refused with AWS_ERROR_SHORT_BUFFER
    ASSERT_FALSE(Checksum::ComputeXXHash64(cur, out));
    ASSERT_INT_EQUALS(AWS_ERROR_SHORT_BUFFER, LastError());
    aws_byte_buf_clean_up(&out);
    return AWS_OP_SUCCESS;
}
AWS_TEST_CASE(DropInXXHash64, s_XXHash64)

static int s_XXHash3(struct aws_allocator *allocator, void *)
{
    ApiHandle handle(allocator);
    ByteCursor cur = aws_byte_cursor_from_c_str("Hello world");
    const uint8_t want64[] = {0xb6, 0xac, 0xb9, 0xd8, 0x4a, 0x38, 0xff, 0x74};  // XXHashTest.cpp:44
    const uint8_t want128[] = {0x73, 0x51, 0xf8, 0x98, 0x12, 0xf9, 0x73, 0x82,
                               0xb9, 0x1d, 0x05, 0xb3, 0x1e, 0x04, 0xdd, 0x7f};  // XXHashTest.cpp:73-74
    ByteBuf out;
    aws_byte_buf_init(&out, allocator, 16);
    ASSERT_TRUE(Checksum::ComputeXXHash3_64(cur, out));
    ASSERT_BIN_ARRAYS_EQUALS(want64, sizeof(want64), out.buffer, out.len);
    aws_byte_buf_reset(&out, false);
    ASSERT_TRUE(Checksum::ComputeXXHash3_128(cur, out));
    ASSERT_BIN_ARRAYS_EQUALS(want128, sizeof(want128), out.buffer, out.len);
    aws_byte_buf_reset(&out, false);
    auto h = Checksum::XXHash::CreateXXHash3_128(0, allocator);
    ASSERT_TRUE(h.Update(cur));
    ASSERT_TRUE(h.Digest(out));
    ASSERT_BIN_ARRAYS_EQUALS(want128, sizeof(want128), out.buffer, out.len);
    ASSERT_FALSE(h.Digest(out));  // unusable after Digest (XXHash.h:40-42)
    aws_byte_buf_clean_up(&out);
    return AWS_OP_SUCCESS;
}
AWS_TEST_CASE(DropInXXHash3, s_XXHash3)
