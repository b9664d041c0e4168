// Host ingest and in-process multi-device fan-out (include/aws_crt_amd/checksums_batch.h).
//
// the CRT's part buffers (S3BufferTicket, include/aws/crt/s3/S3BufferTicket.h:20-30;
// async S3MetaRequest::Write, source/s3/S3.cpp:1133-1149) start in host memory.  A host job shards
// the caller's buffers round-robin over the visible GPUs (north_star: one HIP stream per GPU, no
// collective) and, per device, runs a three-slot pipeline on two streams:
//
//     copy stream     H2D slot k+1   (DMA straight from registered / pinned memory; pageable bytes are
//                                     first copied into the slot's pinned mirror by the worker thread)
//     compute stream  scan slot k    (one ragged list launch over the pieces packed into the slot)
//                     D2H piece results
//
// Buffers longer than a piece are cut into pieces; every piece is scanned from seed 0 (the caller's
// seed for a buffer's first piece) and the pieces of a buffer are folded on the host with Combine
// (CRC.h:41-51), O(log n) scalar algebra per piece.  xxHash cannot be split that way and is a serial
// chain per buffer, so a job's xxHash buffers run on the engine's host path.
//
// Hybrid jobs (round 4, the default): the data starts in host memory, where the host path checksums
// it at 20-45 GiB/s per core while one device lane is bound by PCIe (~50 GiB/s).  So the CPU share's
// threads and the device lanes both take pieces from one cursor over the job (work stealing by
// claims of contiguous pieces): a device claims a slot's part of its share of what is left (its PCIe
// rate against the host threads'), a host thread a run of about 1 MiB.  Offloading is then never slower
// than the host path alone, and the devices add their PCIe rate on top.
//
// Device-resident lists spanning several devices (aws_crt_amd_checksum_list_devices) are grouped by
// the device that owns each buffer; one host thread per device stages and launches that device's
// list and copies its results back, and the results are scattered in caller order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "abi_guard.h"
#include "cpu/cpu_checksums.h"
#include "gf2.h"
#include "runner.h"

#define AWS_CRT_AMD_BUILD 1
#include <aws_crt_amd/checksums_batch.h>

using namespace amdcrc;

extern "C" int amdcrc_gpu_usable(void);      // engine.cpp
extern "C" void amdcrc_note_fallback(void);  // abi_single.cpp: aws_crt_amd_fallback_count

namespace {

thread_local std::string t_err;
void job_err_sink(const char *m) noexcept {
    try {
        t_err = m;
    } catch (...) {
    }
}

constexpr size_t kSlotBytes = 32u << 20;  // device slot / pinned mirror per pipeline stage
constexpr int kSlots = 3;
constexpr size_t kMaxPiecesPerSlot = 8192;

inline bool is_crc(int alg) { return alg <= AWS_CRT_AMD_CRC64NVME; }
inline int out_words(int alg) { return alg == AWS_CRT_AMD_XXH3_128 ? 2 : 1; }

bool host_pinned(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;  // hipHostMalloc'd or hipHostRegister'ed
}

struct Piece {
    size_t buf;          // caller's buffer index
    size_t off, len;     // bytes [off, off + len) of that buffer
    uint64_t seed;       // the caller's seed for the first piece, 0 otherwise
};

// One device's pipeline state
struct Lane {
    int dev = -1;
    hipStream_t copy = nullptr, comp = nullptr;
    void *dslot[kSlots] = {};
    void *hmirror[kSlots] = {};
    void *dres[kSlots] = {}, *dseed[kSlots] = {};
    void *hres[kSlots] = {}, *hseed[kSlots] = {};
    hipEvent_t copied[kSlots] = {}, done[kSlots] = {};
    bool used[kSlots] = {};
};

struct JobImpl {
    int alg = 0;
    const void *const *ptrs = nullptr;
    const size_t *lens = nullptr;
    size_t count = 0;
    const void *h_seeds = nullptr;  // the caller's seeds (u32 or u64 per buffer) or null
    bool seed64 = false;
    uint64_t seed_of(size_t i) const {
        return !h_seeds ? 0 : seed64 ? ((const uint64_t *)h_seeds)[i] : ((const uint32_t *)h_seeds)[i];
    }
    void *h_out = nullptr;
    // Pieces: with no buffer cut (every buffer within a piece) piece q is buffer q and its value goes
    // straight to h_out (`direct`: no piece records, no join pass -- a C4-shard job of 131,072 parts
    // spent ~20 % of its time building and folding them); otherwise the records below.
    bool direct = false;
    size_t npieces = 0;
    std::vector<Piece> pieces;
    std::vector<uint64_t> piece_val;    // per piece (CRC jobs, not direct)
    std::vector<uint64_t> piece_start;  // byte offset of each piece in the job (npieces + 1)
    Piece piece(size_t q) const { return direct ? Piece{q, 0, lens[q], seed_of(q)} : pieces[q]; }
    void put(size_t q, uint64_t v) {
        if (!direct)
            piece_val[q] = v;
        else if (alg == AWS_CRT_AMD_CRC64NVME)
            ((uint64_t *)h_out)[q] = v;
        else
            ((uint32_t *)h_out)[q] = (uint32_t)v;
    }
    std::atomic<size_t> cursor{0};      // the next unclaimed piece
    int ndev = 0;                       // device lanes of the job
    size_t hthreads = 0;                // host threads taking pieces beside them
    int numa_node = -1;                 // the NUMA node the host threads run on (-1: not placed)
    std::atomic<uint64_t> dev_bytes{0};
    // AWS_CRT_AMD_INGEST_TRACE=1: one stderr line per job (claims and when each side ran out of work)
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    std::atomic<uint64_t> lane_claims{0}, lane_end_ns{0}, host_end_ns{0}, host_claims{0};
    std::atomic<uint64_t> lane_wait_ns{0}, lane_issue_ns{0}, lane_first_ns{0}, lane_stage_ns{0};
    std::atomic<uint64_t> lane_mirror_bytes{0}, lane_pin_checks{0}, lane_pin_ns{0};
    uint64_t since_ns() const {
        return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    }
    static void atomic_max(std::atomic<uint64_t> &a, uint64_t v) {
        uint64_t c = a.load(std::memory_order_relaxed);
        while (c < v && !a.compare_exchange_weak(c, v, std::memory_order_relaxed)) {
        }
    }
    uint64_t *dev_bytes_out = nullptr;  // options: bytes the devices scanned, set by job_wait
    std::vector<std::thread> workers;
    // the host coordinator posted to the runner: done when it has returned
    std::mutex host_mu;
    std::condition_variable host_cv;
    bool host_running = false;
    void host_wait() {
        std::unique_lock<std::mutex> g(host_mu);
        host_cv.wait(g, [this] { return !host_running; });
    }
    std::atomic<int> rc{0};
    std::string err;
    std::mutex err_mu;
    // back to a fresh job, keeping the vectors' storage (a C2 job's 20,480 pieces are ~1 MiB of
    // vectors: fresh pages on every job cost ~0.3 ms of faults)
    void reset() {
        alg = 0, ptrs = nullptr, lens = nullptr, count = 0, h_out = nullptr;
        h_seeds = nullptr, seed64 = false, direct = false, npieces = 0;
        pieces.clear(), piece_val.clear(), piece_start.clear();
        cursor.store(0), ndev = 0, hthreads = 0, numa_node = -1, dev_bytes.store(0), dev_bytes_out = nullptr;
        workers.clear(), rc.store(0), err.clear(), host_running = false;
        t0 = std::chrono::steady_clock::now();
        lane_claims.store(0), lane_end_ns.store(0), host_end_ns.store(0), host_claims.store(0);
        lane_wait_ns.store(0), lane_issue_ns.store(0), lane_first_ns.store(0), lane_stage_ns.store(0);
        lane_mirror_bytes.store(0), lane_pin_checks.store(0), lane_pin_ns.store(0);
    }
    void set_error(int code, const char *m) noexcept {
        std::lock_guard<std::mutex> g(err_mu);
        if (rc.load() == 0) {
            rc.store(code);
            try {
                err = m;
            } catch (...) {
            }
        }
    }
    void set_error(int code, const std::string &m) noexcept { set_error(code, m.c_str()); }
    // start a worker; on failure join the ones already started (the job must not be freed under them)
    template <class... A>
    void spawn(A &&...a) {
        try {
            workers.emplace_back(std::forward<A>(a)...);
        } catch (...) {
            for (auto &t : workers) t.join();
            workers.clear();
            throw;
        }
    }
};

#define LANE_TRY(expr)                                                                                     \
    do {                                                                                                   \
        hipError_t e_ = (expr);                                                                            \
        if (e_ != hipSuccess) {                                                                            \
            job->set_error(AWS_CRT_AMD_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_));           \
            return;                                                                                        \
        }                                                                                                  \
    } while (0)

// Lanes are cached per device and reused by later jobs: pinning 96 MiB of mirrors and allocating the
// device slots costs tens of milliseconds, as much as moving a few GiB over PCIe.
std::mutex g_lane_mu;
std::vector<std::vector<Lane *>> g_free_lanes;

void lane_free(Lane &L);

Lane *lane_take(int dev) {
    std::lock_guard<std::mutex> g(g_lane_mu);
    if ((int)g_free_lanes.size() <= dev) g_free_lanes.resize((size_t)dev + 1);
    auto &v = g_free_lanes[(size_t)dev];
    if (v.empty()) return new Lane;
    Lane *l = v.back();
    v.pop_back();
    return l;
}
void lane_give(Lane *l, bool healthy) {
    if (!healthy) {
        lane_free(*l);
        delete l;
        return;
    }
    std::lock_guard<std::mutex> g(g_lane_mu);
    g_free_lanes[(size_t)l->dev].push_back(l);
}

void lane_free(Lane &L) {
    // nothing may still be queued on the lane's streams when its buffers go (an early error return)
    if (L.copy) (void)hipStreamSynchronize(L.copy);
    if (L.comp) (void)hipStreamSynchronize(L.comp);
    for (int k = 0; k < kSlots; ++k) {
        if (L.dslot[k]) (void)hipFree(L.dslot[k]);
        if (L.dres[k]) (void)hipFree(L.dres[k]);
        if (L.dseed[k]) (void)hipFree(L.dseed[k]);
        if (L.hmirror[k]) (void)hipHostFree(L.hmirror[k]);
        if (L.hres[k]) (void)hipHostFree(L.hres[k]);
        if (L.hseed[k]) (void)hipHostFree(L.hseed[k]);
        if (L.copied[k]) (void)hipEventDestroy(L.copied[k]);
        if (L.done[k]) (void)hipEventDestroy(L.done[k]);
    }
    if (L.copy) (void)hipStreamDestroy(L.copy);
    if (L.comp) (void)hipStreamDestroy(L.comp);
}

Runner &runner() {
    static Runner r;
    return r;
}

constexpr size_t kHybridPiece = 8u << 20;  // piece size of hybrid jobs (host threads claim whole pieces)
constexpr uint64_t kMinDevClaim = 1u << 20;
constexpr uint64_t kHostClaim = 1u << 20;
constexpr uint64_t kHostClaimMax = 64u << 20;
constexpr size_t kAutoLanesMaxShare = 12;  // auto jobs use device lanes below this many host threads

// Claim the next run of pieces [*a, *b): at least one, at most max_pieces, at most `budget` bytes
// past the first.  false when the job has no unclaimed piece left.
bool claim(JobImpl *job, uint64_t budget, size_t max_pieces, size_t *a, size_t *b) {
    const size_t n = job->npieces;
    size_t cur = job->cursor.load(std::memory_order_relaxed);
    for (;;) {
        if (cur >= n) return false;
        const uint64_t lim = job->piece_start[cur] + std::max<uint64_t>(budget, 1);
        size_t e = (size_t)(std::upper_bound(job->piece_start.begin() + (long)cur + 1, job->piece_start.end(), lim) -
                            job->piece_start.begin()) - 1;
        e = std::min(std::max(e, cur + 1), max_pieces >= n - cur ? n : cur + max_pieces);
        if (job->cursor.compare_exchange_weak(cur, e, std::memory_order_relaxed)) {
            *a = cur;
            *b = e;
            return true;
        }
    }
}

// A device lane's claim: its share of the unclaimed bytes, at one lane's PCIe rate (~50 GiB/s)
// against a host thread's CRC rate over DRAM-resident parts (~17 GiB/s on the pool's EPYC boxes):
// 3 : 1 per lane and thread, spread over the lane's kSlots claims in flight (round 4: one claim of
// the whole share per slot gave the lane 21 % of a C2 job and left the host threads waiting for it,
// profiles/r04/e).  Devices alone: a whole slot.
uint64_t dev_budget(const JobImpl *job) {
    if (!job->hthreads) return kSlotBytes;
    const size_t c = std::min(job->cursor.load(std::memory_order_relaxed), job->npieces);
    const uint64_t rem = job->piece_start.back() - job->piece_start[c];
    const uint64_t share = rem * 3 / ((3 * (uint64_t)job->ndev + (uint64_t)job->hthreads) * kSlots);
    return std::min<uint64_t>(kSlotBytes, std::max(kMinDevClaim, share));
}

// Worker for one device: claimed runs of pieces through the 3-slot ring
void device_worker_body(JobImpl *job, int dev);
void device_worker(JobImpl *job, int dev) noexcept {
    try {
        device_worker_body(job, dev);
    } catch (const std::bad_alloc &) {
        job->set_error(AWS_CRT_AMD_ERR_OOM, "out of host memory");
    } catch (...) {
        job->set_error(AWS_CRT_AMD_ERR_HIP, "internal error in a device worker");
    }
}
void device_worker_body(JobImpl *job, int dev) {
    Lane *lp = lane_take(dev);
    Lane &L = *lp;
    struct Guard {
        Lane *l;
        JobImpl *job;
        ~Guard() { lane_give(l, job->rc.load() == 0); }
    } guard{lp, job};
    LANE_TRY(hipSetDevice(dev));
    const size_t osz = job->alg == AWS_CRT_AMD_CRC64NVME ? 8 : 4;
    if (L.dev < 0) {  // a new lane (the pinned mirrors are allocated on first pageable use)
        L.dev = dev;
        LANE_TRY(hipStreamCreateWithFlags(&L.copy, hipStreamNonBlocking));
        LANE_TRY(hipStreamCreateWithFlags(&L.comp, hipStreamNonBlocking));
        for (int k = 0; k < kSlots; ++k) {
            LANE_TRY(hipMalloc(&L.dslot[k], kSlotBytes));
            LANE_TRY(hipMalloc(&L.dres[k], kMaxPiecesPerSlot * 8));
            LANE_TRY(hipMalloc(&L.dseed[k], kMaxPiecesPerSlot * 8));
            LANE_TRY(hipHostMalloc(&L.hres[k], kMaxPiecesPerSlot * 8, hipHostMallocDefault));
            LANE_TRY(hipHostMalloc(&L.hseed[k], kMaxPiecesPerSlot * 8, hipHostMallocDefault));
            LANE_TRY(hipEventCreateWithFlags(&L.copied[k], hipEventDisableTiming));
            // the lane thread waits on done[k] (harvest): blocking, so it sleeps instead of spinning on
            // a CPU of the share the host threads run on
            LANE_TRY(hipEventCreateWithFlags(&L.done[k], hipEventDisableTiming | hipEventBlockingSync));
        }
    }
    std::vector<const void *> dptrs;
    std::vector<size_t> dlens;
    std::vector<size_t> slot_pieces[kSlots];
    // copy a slot's results back into the job once its scan has completed
    auto harvest = [&](int k) {
        if (!L.used[k]) return true;
        const uint64_t w0 = job->since_ns();
        if (hipEventSynchronize(L.done[k]) != hipSuccess) return false;
        job->lane_wait_ns.fetch_add(job->since_ns() - w0, std::memory_order_relaxed);
        const std::vector<size_t> &ps = slot_pieces[k];
        for (size_t j = 0; j < ps.size(); ++j)
            job->put(ps[j], osz == 8 ? ((const uint64_t *)L.hres[k])[j] : ((const uint32_t *)L.hres[k])[j]);
        L.used[k] = false;
        return true;
    };
    int k = 0;
    while (job->rc.load() == 0) {
        if (!harvest(k)) {
            job->set_error(AWS_CRT_AMD_ERR_HIP, "slot results");
            return;
        }
        // claim a run of pieces for slot k: contiguous in the slot, in order (pieces are at most a slot)
        size_t a, b;
        if (!claim(job, dev_budget(job), kMaxPiecesPerSlot, &a, &b)) break;
        const uint64_t i0 = job->since_ns();
        if (job->lane_claims.fetch_add(1, std::memory_order_relaxed) == 0) job->lane_first_ns.store(i0);
        std::vector<size_t> &ps = slot_pieces[k];
        ps.clear();
        for (size_t q = a; q < b; ++q) ps.push_back(q);
        job->dev_bytes.fetch_add(job->piece_start[b] - job->piece_start[a], std::memory_order_relaxed);
        // H2D: runs of host-contiguous pinned pieces go straight from the caller's memory; the rest
        // through the pinned mirror (memcpy by this thread, then one DMA per run)
        size_t off = 0;
        dptrs.clear();
        dlens.clear();
        uint8_t *slot = (uint8_t *)L.dslot[k], *mir = (uint8_t *)L.hmirror[k];
        size_t run_dev = 0, run_len = 0;
        const uint8_t *run_src = nullptr;
        auto flush = [&]() -> bool {
            if (run_len && hipMemcpyAsync(slot + run_dev, run_src, run_len, hipMemcpyHostToDevice, L.copy) != hipSuccess) return false;
            run_len = 0;
            return true;
        };
        // pinned or not is asked once per run of host-contiguous pieces (it only decides between a
        // direct DMA and the mirror: hipMemcpyAsync is correct from pageable memory too)
        bool cur_pinned = false;
        const uint8_t *src_end = nullptr;
        for (size_t j = 0; j < ps.size(); ++j) {
            const Piece pc = job->piece(ps[j]);
            const uint8_t *src = (const uint8_t *)job->ptrs[pc.buf] + pc.off;
            if (src != src_end) {
                const uint64_t c0 = job->since_ns();
                cur_pinned = pc.len && host_pinned(src);
                job->lane_pin_checks.fetch_add(1, std::memory_order_relaxed);
                job->lane_pin_ns.fetch_add(job->since_ns() - c0, std::memory_order_relaxed);
            }
            src_end = src + pc.len;
            const uint8_t *from = src;
            if (pc.len && !cur_pinned) {
                if (!mir) {
                    LANE_TRY(hipHostMalloc(&L.hmirror[k], kSlotBytes, hipHostMallocDefault));
                    mir = (uint8_t *)L.hmirror[k];
                }
                std::memcpy(mir + off, src, pc.len);
                job->lane_mirror_bytes.fetch_add(pc.len, std::memory_order_relaxed);
                from = mir + off;
            }
            if (run_len && run_src + run_len == from && run_dev + run_len == off) {
                run_len += pc.len;
            } else {
                if (!flush()) {
                    job->set_error(AWS_CRT_AMD_ERR_HIP, "host-to-device copy");
                    return;
                }
                run_src = from, run_dev = off, run_len = pc.len;
            }
            dptrs.push_back(slot + off);
            dlens.push_back(pc.len);
            if (osz == 8)
                ((uint64_t *)L.hseed[k])[j] = pc.seed;
            else
                ((uint32_t *)L.hseed[k])[j] = (uint32_t)pc.seed;
            off += pc.len;
        }
        if (!flush()) {
            job->set_error(AWS_CRT_AMD_ERR_HIP, "host-to-device copy");
            return;
        }
        job->lane_stage_ns.fetch_add(job->since_ns() - i0, std::memory_order_relaxed);
        LANE_TRY(hipMemcpyAsync(L.dseed[k], L.hseed[k], ps.size() * osz, hipMemcpyHostToDevice, L.copy));
        LANE_TRY(hipEventRecord(L.copied[k], L.copy));
        LANE_TRY(hipStreamWaitEvent(L.comp, L.copied[k], 0));
        // pieces of one length (part buffers of one size) lie back to back in the slot: a strided
        // batch, with no per-buffer descriptors to build and stage
        bool uniform = dlens[0] % 16 == 0 || ps.size() == 1;
        for (size_t j = 1; uniform && j < dlens.size(); ++j) uniform = dlens[j] == dlens[0];
        const int rc = uniform ? aws_crt_amd_checksum_strided(job->alg, dptrs[0], dlens[0], dlens[0], ps.size(), L.dseed[k], L.dres[k], L.comp)
                               : aws_crt_amd_checksum_list(job->alg, dptrs.data(), dlens.data(), ps.size(), L.dseed[k], L.dres[k], L.comp);
        if (rc) {
            job->set_error(rc, aws_crt_amd_last_error());
            return;
        }
        LANE_TRY(hipMemcpyAsync(L.hres[k], L.dres[k], ps.size() * osz, hipMemcpyDeviceToHost, L.comp));
        LANE_TRY(hipEventRecord(L.done[k], L.comp));
        // the slot's copy stream must not overwrite it before the scan has read it: the next use of
        // slot k waits on done[k] in harvest(); the copy stream also waits for it explicitly
        L.used[k] = true;
        job->lane_issue_ns.fetch_add(job->since_ns() - i0, std::memory_order_relaxed);
        k = (k + 1) % kSlots;
        LANE_TRY(hipStreamWaitEvent(L.copy, L.done[k], 0));  // slot k (next) free on the device side
    }
    for (int j = 0; j < kSlots; ++j)
        if (!harvest(j)) job->set_error(AWS_CRT_AMD_ERR_HIP, "slot results");
    JobImpl::atomic_max(job->lane_end_ns, job->since_ns());
}

// A hybrid CRC job's host thread: claimed runs of pieces on the host path, into piece_val like a lane
void crc_host_worker(JobImpl *job) noexcept {
    size_t a, b;
    while (job->rc.load() == 0) {
        const size_t c = std::min(job->cursor.load(std::memory_order_relaxed), job->npieces);
        const uint64_t rem = job->piece_start.back() - job->piece_start[c];
        // guided: a quarter of an even share of what is left, at least kHostClaim or an eighth of an
        // even share of the job (one shared cursor claimed in 1 MiB runs cost a C2 job ~4,000
        // contended claims; a 1 MiB floor left a 1 MiB job to one thread)
        const uint64_t workers = job->hthreads + (size_t)job->ndev;
        const uint64_t floor = std::min<uint64_t>(kHostClaim, std::max<uint64_t>(job->piece_start.back() / (8 * workers), 1));
        const uint64_t budget = std::min<uint64_t>(kHostClaimMax, std::max<uint64_t>(rem / (4 * workers), floor));
        if (!claim(job, budget, SIZE_MAX, &a, &b)) break;
        job->host_claims.fetch_add(1, std::memory_order_relaxed);
        for (size_t q = a; q < b; ++q) {
            const Piece pc = job->piece(q);
            const uint8_t *p = (const uint8_t *)job->ptrs[pc.buf] + pc.off;
            switch (job->alg) {
                case AWS_CRT_AMD_CRC32: job->put(q, cpu::crc32(p, pc.len, (uint32_t)pc.seed)); break;
                case AWS_CRT_AMD_CRC32C: job->put(q, cpu::crc32c(p, pc.len, (uint32_t)pc.seed)); break;
                default: job->put(q, cpu::crc64nvme(p, pc.len, pc.seed)); break;
            }
        }
    }
    JobImpl::atomic_max(job->host_end_ns, job->since_ns());
}

// A job's buffers on the host path (xxHash, or no device): buffers round-robin over `threads`
void host_worker(JobImpl *job, size_t t, size_t threads) {
    for (size_t i = t; i < job->count; i += threads) {
        uint64_t r[2] = {0, 0};
        const uint8_t *p = (const uint8_t *)job->ptrs[i];
        const size_t n = job->lens[i];
        const uint64_t sd = job->seed_of(i);
        switch (job->alg) {
            case AWS_CRT_AMD_CRC32: ((uint32_t *)job->h_out)[i] = cpu::crc32(p, n, (uint32_t)sd); continue;
            case AWS_CRT_AMD_CRC32C: ((uint32_t *)job->h_out)[i] = cpu::crc32c(p, n, (uint32_t)sd); continue;
            case AWS_CRT_AMD_CRC64NVME: ((uint64_t *)job->h_out)[i] = cpu::crc64nvme(p, n, sd); continue;
            case AWS_CRT_AMD_XXH64: r[0] = cpu::xxh64(p, n, sd); break;
            case AWS_CRT_AMD_XXH3_64: r[0] = cpu::xxh3_64(p, n, sd); break;
            default: cpu::xxh3_128(p, n, sd, r); break;
        }
        uint64_t *o = (uint64_t *)job->h_out;
        if (job->alg == AWS_CRT_AMD_XXH3_128)
            o[2 * i] = r[0], o[2 * i + 1] = r[1];
        else
            o[i] = r[0];
    }
}

// Worker streams of the fan-out calls (aws_crt_amd_checksum_list_devices / _checksum_devices),
// cached per device like the ingest lanes: the engine keys its per-stream staging, workspaces and
// sums by stream handle, so a stream created and destroyed per call would leave those behind on every
// call.  A pooled stream carries the call's device result / seed buffer, grown geometrically.
struct FanStream {
    int dev = -1;
    hipStream_t st = nullptr;
    void *buf = nullptr;
    size_t bytes = 0;
};
std::mutex g_fan_mu;
std::vector<std::vector<FanStream *>> g_fan_free;

// the calling thread's current device must be `dev`
FanStream *fan_take(int dev) {
    {
        std::lock_guard<std::mutex> g(g_fan_mu);
        if ((int)g_fan_free.size() <= dev) g_fan_free.resize((size_t)dev + 1);
        auto &v = g_fan_free[(size_t)dev];
        if (!v.empty()) {
            FanStream *f = v.back();
            v.pop_back();
            return f;
        }
    }
    std::unique_ptr<FanStream> f(new FanStream);
    f->dev = dev;
    if (hipStreamCreateWithFlags(&f->st, hipStreamNonBlocking) != hipSuccess) return nullptr;
    return f.release();
}
void fan_give(FanStream *f) {
    if (!f) return;
    std::lock_guard<std::mutex> g(g_fan_mu);
    g_fan_free[(size_t)f->dev].push_back(f);
}
bool fan_reserve(FanStream *f, size_t bytes) {
    if (f->bytes >= bytes) return true;
    if (f->buf) {
        if (hipStreamSynchronize(f->st) != hipSuccess) return false;  // nothing queued may still use it
        (void)hipFree(f->buf);
        f->buf = nullptr;
        f->bytes = 0;
    }
    const size_t cap = std::max<size_t>(bytes, 2 * f->bytes);
    if (hipMalloc(&f->buf, cap) != hipSuccess) return false;
    f->bytes = cap;
    return true;
}

// host-path threads for a job that runs on the CPU: the process's CPU share (cpu::share: its allowed
// CPUs capped by OMP_NUM_THREADS, the figure home_node places by), at most one per buffer
size_t host_threads(size_t count) { return std::max<size_t>(1, std::min(cpu::share(), std::max<size_t>(count, 1))); }

int visible_devices() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

}  // namespace

struct aws_crt_amd_job {
    JobImpl impl;
};

namespace {
// finished jobs kept for reuse (their vectors' storage), at most 4, none over 1 Mi pieces; freed at exit
struct JobCache {
    std::mutex mu;
    std::vector<aws_crt_amd_job *> v;
    ~JobCache() {
        for (aws_crt_amd_job *j : v) delete j;
    }
};
JobCache &job_cache() {
    static JobCache c;
    return c;
}
aws_crt_amd_job *job_take() {
    {
        JobCache &c = job_cache();
        std::lock_guard<std::mutex> g(c.mu);
        if (!c.v.empty()) {
            aws_crt_amd_job *j = c.v.back();
            c.v.pop_back();
            return j;
        }
    }
    return new (std::nothrow) aws_crt_amd_job;
}
void job_give(aws_crt_amd_job *j) noexcept {
    if (!j) return;
    if (j->impl.pieces.capacity() <= ((size_t)1 << 20)) {
        try {
            j->impl.reset();
            JobCache &c = job_cache();
            std::lock_guard<std::mutex> g(c.mu);
            if (c.v.size() < 4) {
                c.v.push_back(j);
                return;
            }
        } catch (...) {
        }
    }
    delete j;
}
}  // namespace

extern "C" {

AWS_CRT_AMD_API int aws_crt_amd_register_host(void *p, size_t n) {
    if (!p || !n) return AWS_CRT_AMD_ERR_INVALID_ARG;
    if (visible_devices() <= 0) return AWS_CRT_AMD_ERR_NO_DEVICE;
    // portable: the registration is visible to every device's DMA engines
    return hipHostRegister(p, n, hipHostRegisterPortable) == hipSuccess ? 0 : AWS_CRT_AMD_ERR_HIP;
}

AWS_CRT_AMD_API int aws_crt_amd_unregister_host(void *p) {
    if (!p) return AWS_CRT_AMD_ERR_INVALID_ARG;
    return hipHostUnregister(p) == hipSuccess ? 0 : AWS_CRT_AMD_ERR_HIP;
}

AWS_CRT_AMD_API int aws_crt_amd_host_submit_ex(int alg, const void *const *h_ptrs, const size_t *lens, size_t count,
                                               const void *h_seeds, void *h_out, const struct aws_crt_amd_ingest_options *opt,
                                               struct aws_crt_amd_job **job_out) {
    return guarded(job_err_sink, [&]() -> int {
        if (!job_out) return AWS_CRT_AMD_ERR_INVALID_ARG;
        *job_out = nullptr;
        if (alg < 0 || alg > 5) return AWS_CRT_AMD_ERR_INVALID_ARG;
        if (count && (!h_ptrs || !lens || !h_out)) return AWS_CRT_AMD_ERR_INVALID_ARG;
        for (size_t i = 0; i < count; ++i)
            if (lens[i] && !h_ptrs[i]) return AWS_CRT_AMD_ERR_INVALID_ARG;
        const int ndevices = opt ? opt->ndevices : 0;
        const int want_host = opt ? opt->host_threads : -1;
        std::unique_ptr<aws_crt_amd_job, void (*)(aws_crt_amd_job *)> job(job_take(), job_give);
        if (!job) return AWS_CRT_AMD_ERR_OOM;
        JobImpl &J = job->impl;
        J.alg = alg;
        J.ptrs = h_ptrs;
        J.lens = lens;
        J.count = count;
        J.h_out = h_out;
        J.dev_bytes_out = opt ? opt->device_bytes : nullptr;
        if (J.dev_bytes_out) *J.dev_bytes_out = 0;
        const bool seed64 = alg != AWS_CRT_AMD_CRC32 && alg != AWS_CRT_AMD_CRC32C;
        J.h_seeds = h_seeds;
        J.seed64 = seed64;
        const int vis = ndevices < 0 ? 0 : visible_devices();
        int G = ndevices < 0 ? 0 : ndevices == 0 ? vis : std::min(ndevices, vis);  // < 0: the host path only
        if (is_crc(alg) && G > 0 && !amdcrc_gpu_usable()) {
            amdcrc_note_fallback();  // a visible device the engine cannot use (not gfx950, HIP error)
            G = 0;
        }
        if (!is_crc(alg)) {
            // xxHash: the host path on the process's CPU share, a thread per buffer at a time
            const size_t threads = host_threads(count);
            for (size_t t = 0; t < threads; ++t) J.spawn(host_worker, &J, t, threads);
            *job_out = job.release();
            return 0;
        }
        // host threads beside the lanes: the CPU share less one thread per lane (auto), or as asked;
        // with no usable device the CPU share alone takes every piece
        if (G < 0) G = 0;
        uint64_t total = 0;
        for (size_t i = 0; i < count; ++i) total += lens[i];
        const size_t share = host_threads(SIZE_MAX);
        // Auto (ndevices 0, host_threads -1): device lanes only for a CPU-poor share.  A lane moves
        // ~50 GiB/s over PCIe, about what 2.5 host threads fold (~20 GiB/s each, AVX-512 VPCLMULQDQ),
        // and takes a thread plus headroom for the HIP runtime beside it; on the pool's 16-CPU share
        // the hybrid job measured 107-306 GiB/s against 284-348 host-only (profiles/r04/m-o), so the
        // default there is the host path.  Lanes stay on when asked for explicitly.
        if (ndevices == 0 && want_host < 0 && share >= kAutoLanesMaxShare) G = 0;
        // (auto: one CPU of the share per lane for its thread and three for the HIP runtime's own
        // threads while lanes run -- a share run full by host threads stalled the lane's staging of a
        // 32 MiB claim for ~1 ms: C2 parts from pinned memory at 116 GiB/s with 14 host threads, 191
        // with 12, profiles/r04/l)
        const size_t reserve = G ? 4 * (size_t)G : 0;
        size_t H = want_host < 0 || G == 0 ? (share > reserve ? share - reserve : 1) : (size_t)want_host;
        if (G == 0) H = std::max<size_t>(H, 1);
        const size_t piece = H ? kHybridPiece : kSlotBytes;
        // pieces, buffer by buffer, in job order (none recorded when no buffer is cut)
        size_t maxlen = 0;
        for (size_t i = 0; i < count; ++i) maxlen = std::max(maxlen, lens[i]);
        J.direct = maxlen <= piece;
        if (J.direct) {
            J.npieces = count;
            J.piece_start.resize(count + 1);
            J.piece_start[0] = 0;
            for (size_t i = 0; i < count; ++i) J.piece_start[i + 1] = J.piece_start[i] + lens[i];
        } else {
            J.pieces.reserve(count + (size_t)(total / piece));
            for (size_t i = 0; i < count; ++i) {
                size_t off = 0;
                do {
                    const size_t n = std::min(piece, lens[i] - off);
                    J.pieces.push_back({i, off, n, off == 0 ? J.seed_of(i) : 0});
                    off += n;
                } while (off < lens[i]);
            }
            J.npieces = J.pieces.size();
            J.piece_start.resize(J.npieces + 1, 0);
            for (size_t q = 0; q < J.npieces; ++q) J.piece_start[q + 1] = J.piece_start[q] + J.pieces[q].len;
            J.piece_val.assign(J.npieces, 0);
        }
        H = std::min(H, J.npieces);
        if (G) G = (int)std::min<size_t>((size_t)G, std::max<size_t>(1, (size_t)(total / kMinDevClaim)));  // tiny jobs: fewer lanes
        // a hybrid job smaller than one slot finishes on the host threads before a lane's first copy
        // and launch would (tens of microseconds): no lane
        if (H > 0 && total < kSlotBytes) G = 0;
        J.ndev = G;
        J.hthreads = H;
        for (int g = 0; g < G; ++g) J.spawn(device_worker, &J, g);
        // the host threads: the host path's persistent pool (a std::thread per job thread cost its
        // creation on every job), driven by one coordinator thread the job joins
        if (H) {
            // the host threads on the NUMA node holding the job's bytes (cpu::home_node)
            J.numa_node = cpu::home_node((const uint8_t *const *)h_ptrs, lens, count, H);
            J.host_running = true;
            JobImpl *jp = &J;
            try {
                runner().post([jp, H] {
                    cpu::parallel(H, [jp](size_t) { crc_host_worker(jp); }, jp->numa_node);
                    std::lock_guard<std::mutex> g(jp->host_mu);
                    jp->host_running = false;
                    jp->host_cv.notify_all();
                });
            } catch (...) {
                // no runner thread: the job must not be released under the lanes already started
                J.host_running = false;
                J.set_error(AWS_CRT_AMD_ERR_OOM, "no host thread for the job");
                for (auto &t : J.workers) t.join();
                J.workers.clear();
                throw;
            }
        }
        *job_out = job.release();
        return 0;
    });
}

AWS_CRT_AMD_API int aws_crt_amd_host_submit(int alg, const void *const *h_ptrs, const size_t *lens, size_t count,
                                            const void *h_seeds, void *h_out, int ndevices, struct aws_crt_amd_job **job_out) {
    const struct aws_crt_amd_ingest_options opt = {ndevices, -1, nullptr};
    return aws_crt_amd_host_submit_ex(alg, h_ptrs, lens, count, h_seeds, h_out, &opt, job_out);
}

AWS_CRT_AMD_API int aws_crt_amd_job_wait(struct aws_crt_amd_job *job) {
    return guarded(job_err_sink, [&]() -> int {
        if (!job) return AWS_CRT_AMD_ERR_INVALID_ARG;
        JobImpl &J = job->impl;
        for (auto &t : J.workers) t.join();
        J.workers.clear();
        J.host_wait();
        int rc = J.rc.load();
        if ((rc == AWS_CRT_AMD_ERR_HIP || rc == AWS_CRT_AMD_ERR_NO_DEVICE) && is_crc(J.alg)) {
            // a device worker failed: the whole job on the host path instead, as the single-buffer ABI
            // does (counted in aws_crt_amd_fallback_count); the value is the same function
            const size_t threads = host_threads(J.count);
            for (size_t t = 0; t < threads; ++t) J.spawn(host_worker, &J, t, threads);
            for (auto &t : J.workers) t.join();
            amdcrc_note_fallback();
            rc = 0;
        } else if (rc == 0 && is_crc(J.alg) && J.dev_bytes_out) {
            *J.dev_bytes_out = J.dev_bytes.load();
        }
        if (rc == 0 && is_crc(J.alg) && !J.direct && !J.pieces.empty() && J.workers.empty()) {
            // fold each buffer's pieces: crc = Combine(crc, piece, |piece|)
            const uint64_t poly = alg_poly(J.alg);
            const int w = alg_width(J.alg);
            size_t p = 0;
            for (size_t i = 0; i < J.count; ++i) {
                uint64_t acc = J.piece_val[p++];
                while (p < J.pieces.size() && J.pieces[p].buf == i) {
                    acc = gf2_mulmod(acc, gf2_xpow8n(J.pieces[p].len, poly, w), poly, w) ^ J.piece_val[p];
                    ++p;
                }
                if (w == 64)
                    ((uint64_t *)J.h_out)[i] = acc;
                else
                    ((uint32_t *)J.h_out)[i] = (uint32_t)acc;
            }
        }
        const char *trace = std::getenv("AWS_CRT_AMD_INGEST_TRACE");
        if (trace && *trace && *trace != '0')
            std::fprintf(stderr,
                         "{\"ingest_trace\": 1, \"pieces\": %zu, \"host_threads\": %zu, \"lanes\": %d, \"device_bytes\": %llu, "
                         "\"lane_claims\": %llu, \"host_claims\": %llu, \"host_end_ms\": %.3f, \"lane_end_ms\": %.3f, \"wait_ms\": %.3f, "
                         "\"lane_first_ms\": %.3f, \"lane_issue_ms\": %.3f, \"lane_stage_ms\": %.3f, \"lane_wait_ms\": %.3f, "
                         "\"lane_mirror_bytes\": %llu, \"lane_pin_checks\": %llu, \"lane_pin_ms\": %.3f, \"numa_node\": %d}\n",
                         J.npieces, J.hthreads, J.ndev, (unsigned long long)J.dev_bytes.load(),
                         (unsigned long long)J.lane_claims.load(), (unsigned long long)J.host_claims.load(), J.host_end_ns.load() * 1e-6,
                         J.lane_end_ns.load() * 1e-6, J.since_ns() * 1e-6, J.lane_first_ns.load() * 1e-6,
                         J.lane_issue_ns.load() * 1e-6, J.lane_stage_ns.load() * 1e-6, J.lane_wait_ns.load() * 1e-6,
                         (unsigned long long)J.lane_mirror_bytes.load(), (unsigned long long)J.lane_pin_checks.load(),
                         J.lane_pin_ns.load() * 1e-6, J.numa_node);
        if (rc) t_err = J.err;
        job_give(job);
        return rc;
    });
}

AWS_CRT_AMD_API const char *aws_crt_amd_job_last_error(void) { return t_err.c_str(); }

// Device-resident buffers on any of the visible devices: grouped by owning device, one host thread
// per device stages and launches that device's list on its own stream and copies the results back;
// results are scattered in caller order into h_out.  Synchronous.
AWS_CRT_AMD_API int aws_crt_amd_checksum_list_devices(int alg, const void *const *d_ptrs, const size_t *lens, size_t count,
                                                      const void *h_seeds, void *h_out) {
    return guarded(job_err_sink, [&]() -> int {
        if (alg < 0 || alg > 5) return AWS_CRT_AMD_ERR_INVALID_ARG;
        if (!count) return 0;
        if (!d_ptrs || !lens || !h_out) return AWS_CRT_AMD_ERR_INVALID_ARG;
        const int vis = visible_devices();
        if (vis <= 0) return AWS_CRT_AMD_ERR_NO_DEVICE;
        std::vector<std::vector<size_t>> by_dev((size_t)vis);
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) return AWS_CRT_AMD_ERR_HIP;
        for (size_t i = 0; i < count; ++i) {
            int dev = cur;  // zero-length entries may carry any pointer
            if (lens[i]) {
                hipPointerAttribute_t a;
                if (!d_ptrs[i] || hipPointerGetAttributes(&a, d_ptrs[i]) != hipSuccess || a.type != hipMemoryTypeDevice) {
                    (void)hipGetLastError();
                    t_err = "aws_crt_amd_checksum_list_devices: buffer " + std::to_string(i) + " is not device memory";
                    return AWS_CRT_AMD_ERR_INVALID_ARG;
                }
                dev = a.device;
            }
            by_dev[(size_t)dev].push_back(i);
        }
        const int per = out_words(alg);
        const size_t osz = alg == AWS_CRT_AMD_CRC32 || alg == AWS_CRT_AMD_CRC32C ? 4 : 8 * (size_t)per;
        const size_t ssz = alg == AWS_CRT_AMD_CRC32 || alg == AWS_CRT_AMD_CRC32C ? 4 : 8;
        std::atomic<int> rc{0};
        std::vector<std::thread> pool;
        for (int g = 0; g < vis; ++g) {
            if (by_dev[(size_t)g].empty()) continue;
            auto body = [&, g] {
                const std::vector<size_t> &ix = by_dev[(size_t)g];
                const size_t n = ix.size();
                std::vector<const void *> ptrs(n);
                std::vector<size_t> ls(n);
                std::vector<uint8_t> seeds(n * ssz), res(n * osz);
                for (size_t j = 0; j < n; ++j) {
                    ptrs[j] = d_ptrs[ix[j]];
                    ls[j] = lens[ix[j]];
                    if (h_seeds) std::memcpy(seeds.data() + j * ssz, (const uint8_t *)h_seeds + ix[j] * ssz, ssz);
                }
                FanStream *fs = hipSetDevice(g) == hipSuccess ? fan_take(g) : nullptr;
                int e = fs && fan_reserve(fs, n * (osz + ssz)) ? 0 : AWS_CRT_AMD_ERR_HIP;
                hipStream_t st = fs ? fs->st : nullptr;
                void *dbuf = e ? nullptr : fs->buf;
                void *dseed = dbuf ? (uint8_t *)dbuf + n * osz : nullptr;
                if (!e && h_seeds && hipMemcpyAsync(dseed, seeds.data(), n * ssz, hipMemcpyHostToDevice, st) != hipSuccess)
                    e = AWS_CRT_AMD_ERR_HIP;
                if (!e) e = aws_crt_amd_checksum_list(alg, ptrs.data(), ls.data(), n, h_seeds ? dseed : nullptr, dbuf, st);
                if (!e && (hipMemcpyAsync(res.data(), dbuf, n * osz, hipMemcpyDeviceToHost, st) != hipSuccess ||
                           hipStreamSynchronize(st) != hipSuccess))
                    e = AWS_CRT_AMD_ERR_HIP;
                if (!e)
                    for (size_t j = 0; j < n; ++j) std::memcpy((uint8_t *)h_out + ix[j] * osz, res.data() + j * osz, osz);
                if (st && e) (void)hipStreamSynchronize(st);  // nothing of this call stays queued
                fan_give(fs);
                if (e) {
                    int z = 0;
                    rc.compare_exchange_strong(z, e);
                }
            };
            auto worker = [&rc, body] {
                try {
                    body();
                } catch (...) {  // host allocation inside the worker
                    int z = 0;
                    rc.compare_exchange_strong(z, (int)AWS_CRT_AMD_ERR_OOM);
                }
            };
            try {
                pool.emplace_back(worker);
            } catch (...) {
                for (auto &t : pool) t.join();
                throw;
            }
        }
        for (auto &t : pool) t.join();
        (void)hipSetDevice(cur);
        return rc.load();
    });
}

// Per-device uniform batches, all devices at once: each entry is launched on its device (one stream
// per device: the entry's, or one the call creates), then every device is awaited.  Synchronous.
AWS_CRT_AMD_API int aws_crt_amd_checksum_devices(int alg, const struct aws_crt_amd_device_batch *b, size_t n) {
    return guarded(job_err_sink, [&]() -> int {
        if (alg < 0 || alg > 5 || (n && !b)) return AWS_CRT_AMD_ERR_INVALID_ARG;
        const int vis = visible_devices();
        if (n && vis <= 0) return AWS_CRT_AMD_ERR_NO_DEVICE;
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) return AWS_CRT_AMD_ERR_HIP;
        std::vector<FanStream *> own(n, nullptr);
        int rc = 0;
        for (size_t i = 0; i < n && !rc; ++i) {
            if (b[i].device < 0 || b[i].device >= vis) {
                rc = AWS_CRT_AMD_ERR_INVALID_ARG;
                break;
            }
            if (hipSetDevice(b[i].device) != hipSuccess) {
                rc = AWS_CRT_AMD_ERR_HIP;
                break;
            }
            hipStream_t st = (hipStream_t)b[i].hip_stream;
            if (!st) {
                if (!(own[i] = fan_take(b[i].device))) {
                    rc = AWS_CRT_AMD_ERR_HIP;
                    break;
                }
                st = own[i]->st;
            }
            rc = aws_crt_amd_checksum_strided(alg, b[i].d_base, b[i].stride, b[i].len, b[i].count, b[i].d_seeds, b[i].d_out, st);
        }
        for (size_t i = 0; i < n; ++i) {  // await every device (also after a failure: nothing stays queued)
            if (hipSetDevice(b[i].device) != hipSuccess) continue;
            hipStream_t st = own[i] ? own[i]->st : (hipStream_t)b[i].hip_stream;
            if (hipStreamSynchronize(st) != hipSuccess && !rc) rc = AWS_CRT_AMD_ERR_HIP;
            fan_give(own[i]);
        }
        (void)hipSetDevice(cur);
        return rc;
    });
}

}  // extern "C"
