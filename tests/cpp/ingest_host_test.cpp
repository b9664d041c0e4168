// Host-ingest jobs on the host path (ndevices < 0) under ThreadSanitizer (tests/test_host_sanitizers.py):
// several threads submit and wait jobs at once -- uncut jobs whose results go straight to the caller's
// array, jobs with buffers cut into pieces joined with Combine, seeds on all -- so finished jobs and
// their vectors are reused across threads and the coordinators run on the shared runner threads.
// Every result must equal the single-buffer host path's.
#include <aws/checksums/crc.h>
#include <aws_crt_amd/checksums_batch.h>
#include <aws/testing/aws_test_harness.h>

#include <atomic>
#include <thread>
#include <vector>

namespace
{
    std::vector<uint8_t> s_bytes(size_t n, uint64_t seed)
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

    // one job of `nbuf` buffers cut from `data` (lengths from `len_of`); true when every value matches
    bool s_job(int alg, const std::vector<uint8_t> &data, size_t nbuf, size_t (*len_of)(size_t), uint64_t salt)
    {
        std::vector<const void *> ptrs;
        std::vector<size_t> lens;
        std::vector<uint64_t> seeds64;
        std::vector<uint32_t> seeds32;
        size_t off = 0;
        for (size_t i = 0; i < nbuf; ++i)
        {
            const size_t n = len_of(i + salt) % (data.size() - off + 1);
            ptrs.push_back(data.data() + off);
            lens.push_back(n);
            seeds64.push_back(i * 0x9E3779B97F4A7C15ull + salt);
            seeds32.push_back((uint32_t)(i * 2654435761u + salt));
            off += n / 2;  // buffers overlap: any bytes will do
        }
        const bool w64 = alg == AWS_CRT_AMD_CRC64NVME;
        std::vector<uint64_t> out(nbuf, 0);
        struct aws_crt_amd_ingest_options opt = {-1, 4, nullptr};
        struct aws_crt_amd_job *job = nullptr;
        if (aws_crt_amd_host_submit_ex(alg, ptrs.data(), lens.data(), nbuf, w64 ? (const void *)seeds64.data() : seeds32.data(),
                                       out.data(), &opt, &job) != 0)
            return false;
        if (aws_crt_amd_job_wait(job) != 0)
            return false;
        for (size_t i = 0; i < nbuf; ++i)
        {
            const uint8_t *p = (const uint8_t *)ptrs[i];
            uint64_t want;
            if (alg == AWS_CRT_AMD_CRC32)
                want = aws_checksums_crc32_ex(p, lens[i], seeds32[i]);
            else if (alg == AWS_CRT_AMD_CRC32C)
                want = aws_checksums_crc32c_ex(p, lens[i], seeds32[i]);
            else
                want = aws_checksums_crc64nvme_ex(p, lens[i], seeds64[i]);
            const uint64_t got = w64 ? out[i] : ((const uint32_t *)out.data())[i];
            if (got != want)
                return false;
        }
        return true;
    }

    size_t s_short(size_t i) { return 1 + (i * 7919) % 70000; }          // uncut: every buffer within a piece
    size_t s_long(size_t i) { return (9u << 20) + (i * 104729) % (3u << 20); }  // cut into 8 MiB pieces
}

static int s_test_concurrent_host_jobs(struct aws_allocator *allocator, void *ctx)
{
    (void)allocator;
    (void)ctx;
    const std::vector<uint8_t> data = s_bytes(40u << 20, 0xC0FFEE);
    std::atomic<int> bad{0};
    std::vector<std::thread> ts;
    for (int t = 0; t < 6; ++t)
        ts.emplace_back(
            [&, t]
            {
                const int alg = t % 3 == 0 ? AWS_CRT_AMD_CRC32 : t % 3 == 1 ? AWS_CRT_AMD_CRC32C : AWS_CRT_AMD_CRC64NVME;
                for (int r = 0; r < 4; ++r)
                {
                    if (!s_job(alg, data, 300, s_short, (uint64_t)(t * 10 + r)))
                        bad.fetch_add(1);
                    if (!s_job(alg, data, 4, s_long, (uint64_t)(t * 10 + r)))
                        bad.fetch_add(1);
                }
            });
    for (auto &th : ts)
        th.join();
    ASSERT_INT_EQUALS(0, bad.load());
    return AWS_OP_SUCCESS;
}
AWS_TEST_CASE(ConcurrentHostJobs, s_test_concurrent_host_jobs)
