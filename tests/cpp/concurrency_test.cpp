// Concurrent callers of the value-only API (SURVEY.md 8(b) "Threading": reentrant, callable from
// any thread, e.g. aws-c-s3 event-loop threads).  Eight threads race on first use (the host path's
// one-time CPU dispatch and table setup) and then checksum their own buffers and run their own
// streaming XXHash objects; every result must equal the single-threaded one.  Run under TSan
// (tests/test_host_sanitizers.py) and in the normal driver.
#include <aws/crt/Api.h>
#include <aws/crt/checksum/CRC.h>
#include <aws/crt/checksum/XXHash.h>
#include <aws/testing/aws_test_harness.h>

#include <atomic>
#include <thread>
#include <vector>

using namespace Aws::Crt;

namespace
{
    struct Result
    {
        uint32_t c32, c32c;
        uint64_t c64, x64;
        uint8_t x3[16];
    };

    std::vector<uint8_t> s_make(size_t n, uint64_t seed)
    {
        std::vector<uint8_t> v(n);
        uint64_t x = seed | 1;
        for (size_t i = 0; i < n; ++i)
        {
            x ^= x << 13;
            x ^= x >> 7;
            x ^= x << 17;
            v[i] = (uint8_t)x;
        }
        return v;
    }

    Result s_compute(const std::vector<uint8_t> &v)
    {
        Result r;
        ByteCursor cur = aws_byte_cursor_from_array(v.data(), v.size());
        r.c32 = Checksum::ComputeCRC32(cur);
        r.c32c = Checksum::ComputeCRC32C(cur, 0x1234u);
        r.c64 = Checksum::ComputeCRC64NVME(cur);
        Checksum::XXHash h = Checksum::XXHash::CreateXXHash64(7);
        for (size_t off = 0; off < v.size(); off += 1000)
        {
            ByteCursor part = aws_byte_cursor_from_array(v.data() + off, v.size() - off < 1000 ? v.size() - off : 1000);
            h.Update(part);
        }
        uint8_t d[8];
        ByteBuf out = aws_byte_buf_from_array(d, sizeof(d));
        out.len = 0;
        h.Digest(out);
        r.x64 = 0;
        for (int i = 0; i < 8; ++i)
            r.x64 = (r.x64 << 8) | d[i];
        ByteBuf o3 = aws_byte_buf_from_array(r.x3, sizeof(r.x3));
        o3.len = 0;
        Checksum::ComputeXXHash3_128(cur, o3, 99);
        return r;
    }
} // namespace

static int s_ConcurrentCallers(struct aws_allocator *allocator, void *)
{
    ApiHandle handle(allocator);
    const int kThreads = 8, kBufs = 6;
    std::vector<std::vector<uint8_t>> bufs;
    for (int i = 0; i < kBufs; ++i)
        bufs.push_back(s_make(37 + (size_t)i * 40009, 0xABCDu + (uint64_t)i));
    std::vector<Result> seq(kBufs), par((size_t)kThreads * kBufs);
    std::atomic<int> go(0);
    std::vector<std::thread> pool;
    for (int t = 0; t < kThreads; ++t)
        pool.emplace_back([&, t] {
            while (!go.load())
            {
            }
            for (int k = 0; k < kBufs; ++k)
                par[(size_t)t * kBufs + (size_t)((k + t) % kBufs)] = s_compute(bufs[(size_t)((k + t) % kBufs)]);
        });
    go.store(1);
    for (auto &th : pool)
        th.join();
    for (int k = 0; k < kBufs; ++k)
        seq[(size_t)k] = s_compute(bufs[(size_t)k]);
    for (int t = 0; t < kThreads; ++t)
        for (int k = 0; k < kBufs; ++k)
        {
            const Result &a = seq[(size_t)k], &b = par[(size_t)t * kBufs + (size_t)k];
            ASSERT_UINT_EQUALS(a.c32, b.c32);
            ASSERT_UINT_EQUALS(a.c32c, b.c32c);
            ASSERT_UINT_EQUALS(a.c64, b.c64);
            ASSERT_UINT_EQUALS(a.x64, b.x64);
            ASSERT_BIN_ARRAYS_EQUALS(a.x3, 16, b.x3, 16);
        }
    return AWS_OP_SUCCESS;
}
AWS_TEST_CASE(ConcurrentCallers, s_ConcurrentCallers)
