// Streaming XXH3 over "device" chunks (tests/cpp/devstream_stubs.cpp): every split of a 4 MiB input
// into host-sized and >= 1 MiB device chunks, starting the device chunks at every buffer fill and
// stripe position class, must digest to the one-shot value of the same bytes (reference
// include/aws/crt/checksum/XXHash.h:40-91: Update any number of times, then Digest).
#include <aws/crt/Api.h>
#include <aws/crt/checksum/XXHash.h>
#include <aws/testing/aws_test_harness.h>
#include <aws_crt_amd/checksums_batch.h>

#include <vector>

using namespace Aws::Crt;

extern "C" uint8_t g_fake_dev[];
extern "C" int g_fail_blocks;
extern "C" unsigned long long g_blocks_calls, g_blocks_absorbed;

static const size_t kN = 4u << 20;

static void s_fill()
{
    uint64_t x = 0x1234567887654321ull;
    for (size_t i = 0; i < kN + 4096; ++i)
    {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        g_fake_dev[i] = (uint8_t)(x >> 56);
    }
}

// digest of g_fake_dev[0, n) streamed in `sizes` chunks (the last chunk takes the rest)
static bool s_stream(bool x128, uint64_t seed, size_t n, const std::vector<size_t> &sizes, ByteBuf &out)
{
    Checksum::XXHash h = x128 ? Checksum::XXHash::CreateXXHash3_128(seed) : Checksum::XXHash::CreateXXHash3_64(seed);
    size_t off = 0;
    for (size_t s : sizes)
    {
        if (off + s > n)
            s = n - off;
        if (!h.Update(aws_byte_cursor_from_array(g_fake_dev + off, s)))
            return false;
        off += s;
    }
    if (off < n && !h.Update(aws_byte_cursor_from_array(g_fake_dev + off, n - off)))
        return false;
    return h.Digest(out);
}

static int s_check_all(bool fail_blocks)
{
    s_fill();
    g_fail_blocks = fail_blocks ? 1 : 0;
    std::vector<uint8_t> host(g_fake_dev, g_fake_dev + kN);
    const size_t M = 1u << 20;
    // prefixes put the first device chunk at every length class and buffer / stripe position
    const size_t prefixes[] = {0, 1, 16, 100, 128, 240, 241, 255, 256, 257, 300, 511, 1000, 1023, 1024, 1025, 1087, 1088,
                               4095, 4096, 9000, 15 * 64 + 1};
    for (int x128 = 0; x128 < 2; ++x128)
    {
        for (uint64_t seed : {0ull, 0x9E3779B97F4A7C15ull})
        {
            for (size_t n : {kN, kN - 1, 2 * M + 777, M + 64 * 16 + 5})
            {
                uint8_t want_b[16], got_b[16];
                ByteBuf want = aws_byte_buf_from_empty_array(want_b, 16);
                ByteCursor hc = aws_byte_cursor_from_array(host.data(), n);
                ASSERT_TRUE(x128 ? Checksum::ComputeXXHash3_128(hc, want, seed) : Checksum::ComputeXXHash3_64(hc, want, seed));
                for (size_t pre : prefixes)
                {
                    std::vector<std::vector<size_t>> splits = {
                        {pre},                               // prefix (host-sized), then the rest on the device path
                        {pre, M + 13},                       // two device chunks
                        {pre, M, 64, M + 1000},              // device, small, device
                        {pre, 3, M - 1, 17, M + 64 * 7 + 1}, // device chunks at shifted stripe positions
                    };
                    for (const auto &sp : splits)
                    {
                        ByteBuf got = aws_byte_buf_from_empty_array(got_b, 16);
                        ASSERT_TRUE(s_stream(x128 != 0, seed, n, sp, got));
                        ASSERT_UINT_EQUALS(want.len, got.len);
                        ASSERT_BIN_ARRAYS_EQUALS(want_b, want.len, got_b, got.len);
                    }
                }
            }
        }
    }
    g_fail_blocks = 0;
    return AWS_OP_SUCCESS;
}

static int s_DeviceStreamXxh3Splits(struct aws_allocator *allocator, void *)
{
    ApiHandle handle(allocator);
    const unsigned long long before = aws_crt_amd_fallback_count();
    ASSERT_SUCCESS(s_check_all(false));
    ASSERT_TRUE(g_blocks_calls > 0 && g_blocks_absorbed > 0);  // the block path was taken
    ASSERT_TRUE(aws_crt_amd_fallback_count() == before);
    return AWS_OP_SUCCESS;
}
AWS_TEST_CASE(DeviceStreamXxh3Splits, s_DeviceStreamXxh3Splits)

static int s_DeviceStreamXxh3Fallback(struct aws_allocator *allocator, void *)
{
    ApiHandle handle(allocator);
    const unsigned long long before = aws_crt_amd_fallback_count();
    ASSERT_SUCCESS(s_check_all(true));
    ASSERT_TRUE(aws_crt_amd_fallback_count() > before);  // every device chunk fell back, counted
    return AWS_OP_SUCCESS;
}
AWS_TEST_CASE(DeviceStreamXxh3Fallback, s_DeviceStreamXxh3Fallback)
