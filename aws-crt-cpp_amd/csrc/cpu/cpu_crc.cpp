// Host CRC32 / CRC32C / CRC64NVME (see cpu_checksums.h for where this sits in the engine).
//
// Folding (PCLMULQDQ / VPCLMULQDQ), the technique aws-checksums dispatches to on x86-64
// ("Where time goes today"), derived here for any reflected CRC of width 32 or 64:
//
//   A 16-byte block loaded little-endian into a 128-bit X holds the message polynomial relative to
//   the block's end with bit p <-> x^(127-p).  Its low qword H and high qword L are 64-bit reflected
//   values (bit b <-> x^(63-b)) with X = H x^64 + L.  Moving X forward by D bytes,
//       X x^(8D) = H x^(64+8D) + L x^(8D)   (mod P),
//   is two carry-less products.  clmul of two 64-bit reflected values yields bit k <-> x^(126-k), one
//   short of the 128-bit convention, so the constants carry one power of x less:
//       K_D = { x^(64+8D-1) mod P , x^(8D-1) mod P }  (64-bit reflected; W=32 values shifted up 32).
//   Products stay below degree 128, so the folded X is congruent (mod P) to everything it absorbed.
//   The register is XORed into the first W bits of the first block (a reflected CRC's register lines
//   up with the next bytes), and at the end the register equals the CRC register of X's 16 bytes
//   taken from state 0 -- a table (or crc32 instruction) pass over 16 bytes.
//
// Accumulators: AVX-512 four zmm (256 B per iteration, D = 256), reduced with D = 192/128/64 and the
// four 128-bit lanes with D = 48/32/16; SSE four xmm (64 B per iteration).  Tails and short inputs:
// slice-by-8 tables, or the SSE4.2 crc32 instruction for CRC32C.
#include <immintrin.h>
#include <cpuid.h>
#include <pthread.h>
#include <sched.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <fstream>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../gf2.h"
#include "cpu_checksums.h"

namespace amdcrc {
namespace cpu {

namespace {

uint64_t xgetbv0() {
    uint32_t lo, hi;
    __asm__ volatile("xgetbv" : "=a"(lo), "=d"(hi) : "c"(0));
    return ((uint64_t)hi << 32) | lo;
}

Features detect() {
    Features f{};
    unsigned a = 0, b = 0, c = 0, d = 0;
    if (!__get_cpuid(1, &a, &b, &c, &d)) return f;
    f.sse42 = (c & bit_SSE4_2) != 0;
    f.pclmul = (c & bit_PCLMUL) != 0 && f.sse42;
    const bool osxsave = (c & bit_OSXSAVE) != 0;
    const uint64_t xcr0 = osxsave ? xgetbv0() : 0;
    const bool ymm_os = (xcr0 & 0x6) == 0x6, zmm_os = (xcr0 & 0xE6) == 0xE6;
    if (__get_cpuid_count(7, 0, &a, &b, &c, &d)) {
        f.avx2 = ymm_os && (b & bit_AVX2) != 0;
        f.avx512 = zmm_os && (b & bit_AVX512F) != 0 && (b & bit_AVX512BW) != 0 && (b & bit_AVX512VL) != 0;
        f.vpclmul = f.avx512 && f.pclmul && (c & bit_VPCLMULQDQ) != 0;
    }
    return f;
}

// x^n mod P for any bit exponent n, W-bit reflected register form
uint64_t xpow_bits(uint64_t n, uint64_t poly, int w) {
    uint64_t result = 1ull << (w - 1), base = result >> 1;  // x^0, x^1
    while (n) {
        if (n & 1) result = gf2_mulmod(result, base, poly, w);
        base = gf2_mulmod(base, base, poly, w);
        n >>= 1;
    }
    return result;
}

struct PolyTables {
    int alg, w;
    uint64_t poly;
    uint64_t t[8][256];  // t[k][e] = e * x^(8(k+1)): byte e followed by k zero bytes
    // fold constants {high-qword multiplier, low-qword multiplier} for D bytes
    alignas(16) uint64_t k16[2], k32[2], k48[2], k64[2], k128[2], k192[2], k256[2];

    explicit PolyTables(int a) : alg(a), w(alg_width(a)), poly(alg_poly(a)) {
        for (int e = 0; e < 256; ++e) {
            uint64_t c = (uint64_t)e;
            for (int k = 0; k < 8; ++k) {
                for (int i = 0; i < 8; ++i) c = gf2_mulx(c, poly);
                t[k][e] = c;
            }
        }
        set(k16, 16), set(k32, 32), set(k48, 48), set(k64, 64), set(k128, 128), set(k192, 192), set(k256, 256);
    }
    void set(uint64_t *k, uint64_t d) {
        const int sh = 64 - w;
        k[0] = xpow_bits(64 + 8 * d - 1, poly, w) << sh;
        k[1] = xpow_bits(8 * d - 1, poly, w) << sh;
    }
};

const PolyTables &tables(int alg) {
    static const PolyTables t32(ALG_CRC32), t32c(ALG_CRC32C), t64(ALG_CRC64NVME);
    return alg == ALG_CRC32 ? t32 : alg == ALG_CRC32C ? t32c : t64;
}

inline uint64_t rd64(const uint8_t *p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}

// register r advanced over n bytes with the slice-by-8 tables
uint64_t tab_update(const PolyTables &T, uint64_t r, const uint8_t *p, size_t n) {
    for (; n >= 8; n -= 8, p += 8) {
        const uint64_t x = rd64(p) ^ r;
        r = T.t[7][x & 0xff] ^ T.t[6][(x >> 8) & 0xff] ^ T.t[5][(x >> 16) & 0xff] ^ T.t[4][(x >> 24) & 0xff] ^
            T.t[3][(x >> 32) & 0xff] ^ T.t[2][(x >> 40) & 0xff] ^ T.t[1][(x >> 48) & 0xff] ^ T.t[0][x >> 56];
    }
    for (; n; --n, ++p) r = (r >> 8) ^ T.t[0][(r ^ *p) & 0xff];
    return r;
}

// CRC32C register over n bytes with the SSE4.2 crc32 instruction
__attribute__((target("sse4.2"))) uint64_t crc32c_hw(uint64_t r, const uint8_t *p, size_t n) {
    uint64_t c = (uint32_t)r;
    for (; n >= 8; n -= 8, p += 8) c = _mm_crc32_u64(c, rd64(p));
    uint32_t c32 = (uint32_t)c;
    for (; n; --n, ++p) c32 = _mm_crc32_u8(c32, *p);
    return c32;
}

// register of X's 16 bytes from state 0
uint64_t finish16(const PolyTables &T, const uint8_t *x16) {
    if (T.alg == ALG_CRC32C && features().sse42) return crc32c_hw(0, x16, 16);
    return tab_update(T, 0, x16, 16);
}

__attribute__((target("sse4.2,pclmul"))) inline __m128i fold128(__m128i x, __m128i k) {
    return _mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11));
}

// register after the first (n & ~15) bytes; n >= 32
__attribute__((target("sse4.2,pclmul"))) uint64_t fold_sse(const PolyTables &T, uint64_t r, const uint8_t *p, size_t n) {
    const __m128i rv = _mm_set_epi64x(0, (long long)r);
    const __m128i K16 = _mm_load_si128((const __m128i *)T.k16);
    __m128i x;
    if (n >= 128) {
        const __m128i K64 = _mm_load_si128((const __m128i *)T.k64);
        __m128i a0 = _mm_xor_si128(_mm_loadu_si128((const __m128i *)p), rv);
        __m128i a1 = _mm_loadu_si128((const __m128i *)(p + 16));
        __m128i a2 = _mm_loadu_si128((const __m128i *)(p + 32));
        __m128i a3 = _mm_loadu_si128((const __m128i *)(p + 48));
        p += 64, n -= 64;
        for (; n >= 64; n -= 64, p += 64) {
            a0 = _mm_xor_si128(fold128(a0, K64), _mm_loadu_si128((const __m128i *)p));
            a1 = _mm_xor_si128(fold128(a1, K64), _mm_loadu_si128((const __m128i *)(p + 16)));
            a2 = _mm_xor_si128(fold128(a2, K64), _mm_loadu_si128((const __m128i *)(p + 32)));
            a3 = _mm_xor_si128(fold128(a3, K64), _mm_loadu_si128((const __m128i *)(p + 48)));
        }
        x = _mm_xor_si128(_mm_xor_si128(fold128(a0, _mm_load_si128((const __m128i *)T.k48)),
                                        fold128(a1, _mm_load_si128((const __m128i *)T.k32))),
                          _mm_xor_si128(fold128(a2, K16), a3));
    } else {
        x = _mm_xor_si128(_mm_loadu_si128((const __m128i *)p), rv);
        p += 16, n -= 16;
    }
    for (; n >= 16; n -= 16, p += 16) x = _mm_xor_si128(fold128(x, K16), _mm_loadu_si128((const __m128i *)p));
    alignas(16) uint8_t b[16];
    _mm_store_si128((__m128i *)b, x);
    return finish16(T, b);
}

#define CPU_AVX512_TARGET "avx512f,avx512bw,avx512vl,vpclmulqdq,pclmul,sse4.2"

__attribute__((target(CPU_AVX512_TARGET))) inline __m512i fold512(__m512i x, __m512i k) {
    return _mm512_xor_si512(_mm512_clmulepi64_epi128(x, k, 0x00), _mm512_clmulepi64_epi128(x, k, 0x11));
}
__attribute__((target(CPU_AVX512_TARGET))) inline __m512i bcast(const uint64_t *k) {
    return _mm512_broadcast_i32x4(_mm_load_si128((const __m128i *)k));
}
// a ^ fold(x, k): one ternary-logic XOR of the two products and a
__attribute__((target(CPU_AVX512_TARGET))) inline __m512i fold512_x(__m512i x, __m512i k, __m512i a) {
    return _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x, k, 0x00), _mm512_clmulepi64_epi128(x, k, 0x11), a, 0x96);
}

// register after the first (n & ~15) bytes; n >= 256
__attribute__((target(CPU_AVX512_TARGET))) uint64_t fold_avx512(const PolyTables &T, uint64_t r, const uint8_t *p, size_t n) {
    const __m512i K256 = bcast(T.k256), K64 = bcast(T.k64);
    __m512i z0 = _mm512_xor_si512(_mm512_loadu_si512(p), _mm512_set_epi64(0, 0, 0, 0, 0, 0, 0, (long long)r));
    __m512i z1 = _mm512_loadu_si512(p + 64), z2 = _mm512_loadu_si512(p + 128), z3 = _mm512_loadu_si512(p + 192);
    p += 256, n -= 256;
    for (; n >= 256; n -= 256, p += 256) {
        z0 = fold512_x(z0, K256, _mm512_loadu_si512(p));
        z1 = fold512_x(z1, K256, _mm512_loadu_si512(p + 64));
        z2 = fold512_x(z2, K256, _mm512_loadu_si512(p + 128));
        z3 = fold512_x(z3, K256, _mm512_loadu_si512(p + 192));
    }
    __m512i z = _mm512_ternarylogic_epi64(fold512(z0, bcast(T.k192)), fold512(z1, bcast(T.k128)), fold512_x(z2, K64, z3), 0x96);
    for (; n >= 64; n -= 64, p += 64) z = fold512_x(z, K64, _mm512_loadu_si512(p));
    // lanes l0 (oldest) .. l3: l0 x^(8*48) + l1 x^(8*32) + l2 x^(8*16) + l3
    const __m128i l0 = _mm512_extracti32x4_epi32(z, 0), l1 = _mm512_extracti32x4_epi32(z, 1);
    const __m128i l2 = _mm512_extracti32x4_epi32(z, 2), l3 = _mm512_extracti32x4_epi32(z, 3);
    const __m128i K16 = _mm_load_si128((const __m128i *)T.k16);
    __m128i x = _mm_xor_si128(_mm_xor_si128(fold128(l0, _mm_load_si128((const __m128i *)T.k48)),
                                            fold128(l1, _mm_load_si128((const __m128i *)T.k32))),
                              _mm_xor_si128(fold128(l2, K16), l3));
    for (; n >= 16; n -= 16, p += 16) x = _mm_xor_si128(fold128(x, K16), _mm_loadu_si128((const __m128i *)p));
    alignas(16) uint8_t b[16];
    _mm_store_si128((__m128i *)b, x);
    return finish16(T, b);
}

uint64_t update(int alg, uint64_t r, const uint8_t *p, size_t n, Tier tier) {
    const PolyTables &T = tables(alg);
    if (tier == TIER_VPCLMUL && n >= 256) {
        const size_t m = n & ~(size_t)15;
        r = fold_avx512(T, r, p, m);
        p += m, n -= m;
    } else if (tier >= TIER_PCLMUL && n >= (alg == ALG_CRC32C ? 256 : 32)) {
        const size_t m = n & ~(size_t)15;
        r = fold_sse(T, r, p, m);
        p += m, n -= m;
    }
    if (!n) return r;
    if (alg == ALG_CRC32C && tier != TIER_TABLE && features().sse42) return crc32c_hw(r, p, n);
    return tab_update(T, r, p, n);
}

}  // namespace

const Features &features() {
    static const Features f = detect();
    return f;
}

Tier best_tier() {
    static const Tier t = [] {
        const Features &f = features();
        return f.vpclmul ? TIER_VPCLMUL : f.pclmul ? TIER_PCLMUL : TIER_TABLE;
    }();
    return t;
}

uint64_t crc_tier(int alg, const uint8_t *p, size_t n, uint64_t previous, Tier tier) {
    if (tier > best_tier()) tier = best_tier();
    const uint64_t mask = alg_mask(alg);
    if (!n) return previous & mask;
    return ~update(alg, ~previous & mask, p, n, tier) & mask;
}

uint32_t crc32(const uint8_t *p, size_t n, uint32_t previous) { return (uint32_t)crc_tier(ALG_CRC32, p, n, previous, best_tier()); }
uint32_t crc32c(const uint8_t *p, size_t n, uint32_t previous) {
    return (uint32_t)crc_tier(ALG_CRC32C, p, n, previous, best_tier());
}
uint64_t crc64nvme(const uint8_t *p, size_t n, uint64_t previous) {
    return crc_tier(ALG_CRC64NVME, p, n, previous, best_tier());
}

namespace {

// NUMA placement of the host path.  A checksum pass reads every byte once, so it runs at the
// bandwidth its threads see to the buffer's memory: on the pool's two-socket hosts (16-CPU share,
// affinity over both sockets) threads left to float read a one-node buffer at 104-153 GiB/s, and at
// 324-399 GiB/s when they all run on the buffer's node (profiles/r04/numa).  The node CPU sets are
// the process's affinity mask at first use split by /sys/devices/system/node/node*/cpulist;
// AWS_CRT_AMD_NUMA=0 turns placement off, =force places jobs on a one-node host too (tests).
struct Numa {
    std::vector<cpu_set_t> node_cpus;  // allowed CPUs per node (may be empty)
    bool on = false;
};

bool parse_cpulist(const std::string &s, cpu_set_t *set) {
    size_t i = 0;
    while (i < s.size()) {
        char *end = nullptr;
        const long a = std::strtol(s.c_str() + i, &end, 10);
        if (end == s.c_str() + i) return false;
        i = (size_t)(end - s.c_str());
        long b = a;
        if (i < s.size() && s[i] == '-') {
            b = std::strtol(s.c_str() + i + 1, &end, 10);
            i = (size_t)(end - s.c_str());
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET((int)c, set);
        while (i < s.size() && (s[i] == ',' || s[i] == '\n' || s[i] == ' ')) ++i;
    }
    return true;
}

// The CPUs the process may run on: the allowed-CPU list of /proc/self/status (the process's mask,
// whichever thread asks; sched_getaffinity(0) would return the calling thread's own, possibly pinned,
// mask), else that of the calling thread.
bool process_cpus(cpu_set_t *set) {
    CPU_ZERO(set);
    std::ifstream f("/proc/self/status");
    std::string line;
    while (std::getline(f, line))
        if (line.compare(0, 19, "Cpus_allowed_list:\t") == 0 && parse_cpulist(line.substr(19), set) && CPU_COUNT(set) > 0)
            return true;
    CPU_ZERO(set);
    return sched_getaffinity(0, sizeof(cpu_set_t), set) == 0;
}

const cpu_set_t &allowed_cpus() {
    static const cpu_set_t s = [] {
        cpu_set_t c;
        if (!process_cpus(&c)) CPU_ZERO(&c);
        return c;
    }();
    return s;
}

const Numa &numa() {
    static const Numa n = [] {
        Numa m;
        const char *env = std::getenv("AWS_CRT_AMD_NUMA");
        const cpu_set_t &all = allowed_cpus();
        if ((env && env[0] == '0') || CPU_COUNT(&all) == 0) return m;
        int populated = 0;
        for (int node = 0; node < 64; ++node) {
            std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
            if (!f) break;
            std::string line;
            std::getline(f, line);
            cpu_set_t set;
            CPU_ZERO(&set);
            if (!parse_cpulist(line, &set)) break;
            CPU_AND(&set, &set, &all);
            populated += CPU_COUNT(&set) > 0;
            m.node_cpus.push_back(set);
        }
        m.on = populated >= (env && strcmp(env, "force") == 0 ? 1 : 2);
        return m;
    }();
    return n;
}

// Persistent workers for batch(): spawning a std::thread costs tens of microseconds, as much as
// checksumming a few hundred KiB, so the threads stay parked between calls.  One batch at a time
// uses the pool; a call that finds it busy runs on threads of its own.  A batch placed on a NUMA
// node runs every index on workers moved onto that node's CPUs (the caller only waits: its own
// thread's mask is not ours to change); a worker moves back when a batch has no node.
class Pool {
  public:
    bool try_run(size_t n, const std::function<void(size_t)> &fn, int node) {
        std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
        if (!busy.owns_lock()) return false;
        const size_t shift = node >= 0 ? 1 : 0;  // worker idx runs fn(idx - shift)
        size_t nw;
        {
            std::lock_guard<std::mutex> g(mu_);
            try {
                while (workers_.size() + 1 - shift < n) workers_.emplace_back([this, i = workers_.size() + 1] { loop(i); });
            } catch (...) {
                // fewer workers than asked for: the indices without one run on this thread below
            }
            nw = workers_.size();
            fn_ = &fn;
            n_ = n;
            shift_ = shift;
            node_ = node;
            pending_ = std::min(nw, n + shift - 1);
            ++gen_;
        }
        cv_.notify_all();
        if (!shift) fn(0);
        for (size_t i = nw + 1 - shift; i < n; ++i) fn(i);
        std::unique_lock<std::mutex> g(mu_);
        done_.wait(g, [this] { return pending_ == 0; });
        fn_ = nullptr;
        return true;
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : workers_) t.join();
    }

  private:
    void loop(size_t idx) {
        uint64_t seen = 0;
        int placed = -1;  // the node this thread's mask is on (-1: its mask at creation)
        cpu_set_t own;    // what the worker returns to after a placed batch
        const bool have_own = pthread_getaffinity_np(pthread_self(), sizeof(cpu_set_t), &own) == 0;
        for (;;) {
            const std::function<void(size_t)> *fn;
            size_t shift;
            int node;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                if (idx >= n_ + shift_) continue;  // not part of this batch
                fn = fn_;
                shift = shift_;
                node = node_;
            }
            if (node != placed && (node >= 0 || have_own)) {
                const Numa &m = numa();
                pthread_setaffinity_np(pthread_self(), sizeof(cpu_set_t), node >= 0 ? &m.node_cpus[(size_t)node] : &own);
                placed = node;
            }
            (*fn)(idx - shift);
            std::lock_guard<std::mutex> g(mu_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> workers_;
    const std::function<void(size_t)> *fn_ = nullptr;
    size_t n_ = 0, pending_ = 0, shift_ = 0;
    int node_ = -1;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

Pool &pool() {
    static Pool p;
    return p;
}

}  // namespace

int home_node(const uint8_t *const *ptrs, const size_t *lens, size_t count, size_t threads) {
    constexpr size_t kMinBytes = (size_t)16 << 20;  // below this a job is too short to gain
    constexpr size_t kSamples = 64;
    const Numa &m = numa();
    if (!m.on || threads < 2) return -1;
    size_t total = 0;
    for (size_t i = 0; i < count; ++i) total += lens[i];
    if (total < kMinBytes) return -1;
    // one page at each of kSamples evenly spaced byte offsets of the job
    const uintptr_t page = (uintptr_t)sysconf(_SC_PAGESIZE);
    void *pages[kSamples];
    int status[kSamples];
    size_t k = 0, i = 0, before = 0;
    for (size_t s = 0; s < kSamples; ++s) {
        const size_t off = (2 * s + 1) * (total / (2 * kSamples));
        while (i < count && before + lens[i] <= off) before += lens[i++];
        if (i == count) break;
        pages[k++] = (void *)(((uintptr_t)ptrs[i] + (off - before)) & ~(page - 1));
    }
    if (!k || syscall(SYS_move_pages, 0, (unsigned long)k, pages, nullptr, status, 0) != 0) return -1;
    size_t votes[64] = {0}, valid = 0;
    for (size_t s = 0; s < k; ++s)
        if (status[s] >= 0 && status[s] < 64) ++votes[status[s]], ++valid;
    const size_t best = (size_t)(std::max_element(votes, votes + 64) - votes);
    // one node holding >= 3/4 of the sampled pages, with a CPU of the process's mask per thread
    if (valid * 2 < k || votes[best] * 4 < valid * 3 || best >= m.node_cpus.size()) return -1;
    if ((size_t)CPU_COUNT(&m.node_cpus[best]) < threads) return -1;
    return (int)best;
}

size_t share() {
    static const size_t s = [] {
        size_t t = (size_t)CPU_COUNT(&allowed_cpus());
        if (t == 0) t = std::max(1u, std::thread::hardware_concurrency());
        if (const char *e = std::getenv("OMP_NUM_THREADS")) {
            const long v = std::strtol(e, nullptr, 10);
            if (v > 0) t = std::min<size_t>(t, (size_t)v);
        }
        return std::max<size_t>(1, t);
    }();
    return s;
}

void parallel(size_t n, const std::function<void(size_t)> &fn, int node) {
    if (n == 0) return;
    if (n == 1 || pool().try_run(n, fn, node)) {
        if (n == 1) fn(0);
        return;
    }
    std::vector<std::thread> ts;
    size_t spawned = 1;
    try {
        for (; spawned < n; ++spawned) ts.emplace_back(fn, spawned);
    } catch (...) {
    }
    fn(0);
    for (auto &t : ts) t.join();
    for (size_t i = spawned; i < n; ++i) fn(i);  // threads that could not be started
}

// Host batch (aws_crt_amd_cpu_batch).  Work items are claimed dynamically by `threads` threads.  A
// CRC buffer longer than the piece size is cut into pieces, each checksummed from seed 0 (the first
// from the caller's seed) and folded in order with Combine (CRC.h:41-51) -- so a batch of fewer
// buffers than threads, such as 8 x 64 MiB, still keeps every thread busy.  A hash is one serial
// chain per buffer: one item per buffer.
void batch(int alg, const uint8_t *const *ptrs, const size_t *lens, const uint64_t *seeds, uint64_t *out, size_t count,
           int threads) {
    auto one = [&](size_t i) {
        const uint64_t s = seeds ? seeds[i] : 0;
        switch (alg) {
            case 0: out[i] = crc32(ptrs[i], lens[i], (uint32_t)s); break;
            case 1: out[i] = crc32c(ptrs[i], lens[i], (uint32_t)s); break;
            case 2: out[i] = crc64nvme(ptrs[i], lens[i], s); break;
            case 3: out[i] = xxh64(ptrs[i], lens[i], s); break;
            case 4: out[i] = xxh3_64(ptrs[i], lens[i], s); break;
            default: xxh3_128(ptrs[i], lens[i], s, out + 2 * i); break;
        }
    };
    const size_t nt = threads <= 1 ? 1 : (size_t)threads;
    if (nt == 1 || count == 0) {
        for (size_t i = 0; i < count; ++i) one(i);
        return;
    }
    // items: (buffer, piece) with pieces only for CRCs
    size_t total = 0;
    for (size_t i = 0; i < count; ++i) total += lens[i];
    const bool crc = alg <= 2;
    const size_t piece = crc ? std::max<size_t>((size_t)1 << 20, (total / (4 * nt) + 4095) & ~(size_t)4095) : ~(size_t)0;
    std::vector<size_t> first(count + 1, 0);  // first item of buffer i
    for (size_t i = 0; i < count; ++i) first[i + 1] = first[i] + (lens[i] > piece ? (lens[i] + piece - 1) / piece : 1);
    const size_t nitems = first[count];
    if (nitems == count && count == 1) {
        one(0);
        return;
    }
    std::vector<uint64_t> pv(crc ? nitems : 0);
    // items are claimed in runs (one shared counter touched by every thread of a two-socket host
    // costs more than checksumming a short buffer): about 16 claims per thread, at least one item
    const size_t run = std::max<size_t>(1, nitems / (16 * nt));
    std::atomic<size_t> next{0};
    auto work = [&](size_t) {
        for (;;) {
            const size_t it0 = next.fetch_add(run, std::memory_order_relaxed);
            if (it0 >= nitems) return;
            const size_t it1 = std::min(nitems, it0 + run);
            size_t i = (size_t)(std::upper_bound(first.begin(), first.end(), it0) - first.begin()) - 1;
            for (size_t it = it0; it < it1; ++it) {
                while (first[i + 1] <= it) ++i;
                if (!crc || first[i + 1] - first[i] == 1) {
                    one(i);
                    if (crc) pv[it] = out[i];
                    continue;
                }
                const size_t k = it - first[i], off = k * piece, n = std::min(piece, lens[i] - off);
                const uint64_t s = k == 0 && seeds ? seeds[i] : 0;
                pv[it] = alg == 0   ? crc32(ptrs[i] + off, n, (uint32_t)s)
                         : alg == 1 ? crc32c(ptrs[i] + off, n, (uint32_t)s)
                                    : crc64nvme(ptrs[i] + off, n, s);
            }
        }
    };
    const size_t nrun = std::min(nt, nitems);
    if (!pool().try_run(nrun, work, home_node(ptrs, lens, count, nrun))) {
        std::vector<std::thread> ts;
        for (size_t t = 1; t < nrun; ++t) ts.emplace_back(work, t);
        work(0);
        for (auto &th : ts) th.join();
    }
    if (!crc) return;
    // fold the pieces of every split buffer: crc = Combine(crc, piece, |piece|)
    const uint64_t poly = alg_poly(alg);
    const int w = alg_width(alg);
    for (size_t i = 0; i < count; ++i) {
        const size_t np = first[i + 1] - first[i];
        if (np == 1) continue;
        uint64_t acc = pv[first[i]];
        for (size_t k = 1; k < np; ++k) {
            const size_t n = std::min(piece, lens[i] - k * piece);
            acc = gf2_mulmod(acc, gf2_xpow8n(n, poly, w), poly, w) ^ pv[first[i] + k];
        }
        out[i] = acc;
    }
}

}  // namespace cpu
}  // namespace amdcrc
