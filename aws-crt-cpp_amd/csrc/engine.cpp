// Host side of the MI355X checksum engine: device bring-up, constant tables, workspaces, batch
// planning and the batched C ABI (include/aws_crt_amd/checksums_batch.h).
//
// The reference's equivalent is one synchronous CPU call per buffer
// (source/checksum/CRC.cpp:15-43 -> aws-checksums).  Here the checksums of device-resident batches
// are computed by the gfx950 kernels in crc_kernels.hip / xxh3_kernels.hip; this file plans work and
// moves descriptors.  The single-buffer aws-checksums ABI and its CPU / GPU dispatch live in
// abi_single.cpp; the host path in csrc/cpu/.
//
// No library call synchronises the whole device.  Growing a cached table or workspace never frees
// memory that queued kernels may still read: the old allocation is retired (kept until process
// exit; growth is geometric, so retired memory is bounded by the live size).
#include "variant_guard.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "abi_guard.h"
#include "cpu/cpu_checksums.h"
#include "engine.h"
#include "gf2.h"
#include "ptr_class.h"
#include "runner.h"
#include "stream_states.h"

#define AWS_CRT_AMD_BUILD 1
#include <aws_crt_amd/checksums_batch.h>

using namespace amdcrc;

namespace {

thread_local std::string g_last_error;
// measurement hook (aws_crt_amd_debug_time_next_launch): events stamped by the next scan dispatch
thread_local void *g_time_events[2] = {nullptr, nullptr};

// Prepared launches (aws_crt_amd_plan_*): while a plan is being built, the strided scan planner
// records each launch it would make instead of making it.  A launch that needs the per-stream
// cross-tile workspace records its size; the workspace is looked up on the stream at launch time.
struct PlannedLaunch {
    int alg = 0;
    int kind = 0;  // 0: amdcrc_launch_scan(ScanParams), 1: amdcrc_launch_lanes(LaneParams)
    amdcrc::ScanParams p{};
    amdcrc::LaneParams lp{};
    uint64_t blocks = 0;
    bool ws = false;  // patch d_acc / d_cnt (/ acc1, cnt1, claim) from the stream's workspace
    uint64_t ws_nbuf = 0, ws_tiles = 0;
};
thread_local std::vector<PlannedLaunch> *t_plan = nullptr;

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}
void err_sink(const char *m) noexcept {
    try {
        g_last_error = m;
    } catch (...) {
    }
}

#define HIP_TRY(expr)                                                                                      \
    do {                                                                                                   \
        hipError_t e_ = (expr);                                                                            \
        if (e_ != hipSuccess) return fail(AWS_CRT_AMD_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

// Per-stream cross-tile workspace.  Kernels on one stream are serialised, and each launch leaves
// the words it touched at zero, so a workspace is reusable by the next launch on its stream.  A
// launch captured into a HIP graph keeps its capture stream's workspace: replay such a graph on the
// capture stream, or while no eager launch of the capture stream runs.
struct Workspace {
    unsigned long long *acc = nullptr;   // per buffer
    unsigned int *cnt = nullptr;         // per buffer
    unsigned long long *acc1 = nullptr;  // per tile (32-tile group slots of the braided scans)
    unsigned int *cnt1 = nullptr;        // per tile (W=64 group arrival counts)
    unsigned int *claim = nullptr;       // workgroup tile pools: 2 words per shard
    size_t cap = 0, cap_tiles = 0;
};

// Per-stream descriptor staging: three (pinned host, device) slots used round-robin, each with the
// event of its last upload, so a call waits only for the upload of the call three before it.
constexpr int kStageSlots = 3;
struct Stage {
    DevBuf dev[kStageSlots], host[kStageSlots];
    hipEvent_t done[kStageSlots] = {nullptr, nullptr, nullptr};
    int next = 0, cur = 0;
};

// Everything the engine keeps per caller stream (stream_states.h): scratch that launches on one stream
// share in stream order, and the fence recorded after the last launch that read it.
struct StreamState {
    Workspace ws;
    Stage st;
    DevBuf xsums;   // split XXH3 long path: per-block accumulator sums
    DevBuf mp_out;  // multipart part results
    // held by a multipart call on the stream from its list launch until its results are on the host:
    // two calls on one stream would otherwise queue launch A, launch B, then A's copy of B's results
    std::mutex mp_mu;
    hipEvent_t fence = nullptr;  // recorded after the last launch that read this state
    bool fenced = false;
    bool pinned = false;         // read by a launch captured into a graph: never handed to another stream
    uint64_t tick = 0;
};
struct StatePolicy {
    static bool idle(StreamState &s) {
        if (s.pinned) return false;
        if (!s.mp_mu.try_lock()) return false;
        s.mp_mu.unlock();
        if (!s.fenced) return true;
        const hipError_t e = hipEventQuery(s.fence);
        if (e == hipSuccess) {
            s.fenced = false;
            return true;
        }
        (void)hipGetLastError();
        return false;
    }
};
constexpr size_t kMaxStreamStates = 64;

struct Device {
    int id = -1;
    int cus = 0;
    uint64_t max_pitch = 0;  // hipDeviceProp_t::memPitch: the largest pitch a 2D copy accepts
    std::mutex mu;
    std::map<int, DevBuf> braid;                       // alg -> W=32 braided-scan constants
    std::map<int, DevBuf> braid64;                     // alg -> W=64 braided-scan constants
    std::map<std::pair<int, uint64_t>, DevBuf> pcols;  // (alg, tile) -> tmax x W x u64
    std::map<std::pair<int, uint64_t>, uint64_t> pcols_tmax;
    std::map<std::pair<int, uint64_t>, DevBuf> xcd;    // (alg, waves per XCD) -> crc64_xcd_kernel constants
    std::vector<DevBuf> retired;                       // outgrown buffers queued kernels may still read
    StreamStates<hipStream_t, StreamState, StatePolicy> states{kMaxStreamStates};  // under mu
    // single path (GPU-dispatched host buffers, device buffers through the aws-checksums ABI)
    hipStream_t own_stream = nullptr;
    void *pin[2] = {nullptr, nullptr};
    void *dbuf[2] = {nullptr, nullptr};
    hipEvent_t pin_free[2] = {nullptr, nullptr};
    size_t stage_bytes = 0;
    DevBuf hash_stage;        // whole-buffer device copy for GPU-dispatched host xxHash
    DevBuf xstream_sums;      // streaming XXH3 on device chunks: block sums of one pass
    DevBuf ceil_sink;         // read-ceiling diagnostics: one word per wave
    DevBuf es_imgs;           // eventstream_flat_kernel's nibble images (get_es_images)
    void *d_small = nullptr;  // results / seeds for the single path
    void *h_res = nullptr;    // pinned, coherent host slot the single path's last launch stores into
    std::mutex single_mu;
};

std::mutex g_mu;
std::map<int, std::unique_ptr<Device>> g_devices;

int device_count_noinit() {
    static const int n = [] {
        int c = 0;
        if (hipGetDeviceCount(&c) != hipSuccess) {
            (void)hipGetLastError();
            return 0;
        }
        return c;
    }();
    return n;
}

int get_device(Device **out) {
    if (device_count_noinit() <= 0) return fail(AWS_CRT_AMD_ERR_NO_DEVICE, "no HIP device visible");
    int id = 0;
    HIP_TRY(hipGetDevice(&id));
    std::lock_guard<std::mutex> g(g_mu);
    auto &slot = g_devices[id];
    if (!slot) {
        hipDeviceProp_t prop;
        HIP_TRY(hipGetDeviceProperties(&prop, id));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return fail(AWS_CRT_AMD_ERR_NO_DEVICE, std::string("device is ") + prop.gcnArchName + ", engine is built for gfx950");
        auto d = std::make_unique<Device>();
        d->id = id;
        d->cus = prop.multiProcessorCount;
        d->max_pitch = prop.memPitch ? (uint64_t)prop.memPitch : (1ull << 31) - 1;
        slot = std::move(d);
    }
    *out = slot.get();
    return 0;
}

inline int width_of(int alg) { return alg == ALG_CRC64NVME ? 64 : 32; }

// hipStreamIsCapturing: paths that allocate or synchronise refuse captured streams (the caller
// warms the engine up on the stream before capturing)
bool capturing(hipStream_t s) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return st != hipStreamCaptureStatusNone;
}

// The per-stream state the launch about to be made reads (set by get_workspace / stage_begin / the
// XXH3 sums, under the device mutex); fence_after records the state's fence behind that launch.
thread_local StreamState *t_used = nullptr;

void fence_after(hipStream_t s) {
    StreamState *u = t_used;
    t_used = nullptr;
    if (!u) return;
    if (capturing(s)) {
        u->pinned = true;  // a graph may replay it at any time
        return;
    }
    if ((!u->fence && hipEventCreateWithFlags(&u->fence, hipEventDisableTiming) != hipSuccess) ||
        hipEventRecord(u->fence, s) != hipSuccess) {
        (void)hipGetLastError();
        u->pinned = true;  // unknown completion: never handed over
        return;
    }
    u->fenced = true;
}

int upload_new(DevBuf &b, const void *host, size_t bytes) {
    HIP_TRY(hipMalloc(&b.p, bytes));
    b.bytes = bytes;
    HIP_TRY(hipMemcpy(b.p, host, bytes, hipMemcpyHostToDevice));
    return 0;
}

// x^-1 * t : inverse of gf2_mulx (the reflected polynomial's top bit is the x^0 coefficient, 1)
inline uint32_t inv_mulx32(uint32_t t, uint32_t poly) { return (t & 0x80000000u) ? (((t ^ poly) << 1) | 1u) : (t << 1); }
inline uint64_t inv_mulx64(uint64_t t, uint64_t poly) { return (t >> 63) ? (((t ^ poly) << 1) | 1u) : (t << 1); }

// Nibble image of a GF(2) matrix given by its W columns (col(j) is the product of operand bit W-1-j):
// entry 16 i + v is the product of nibble i's value v, i.e. of bits W-1-4i .. W-4-4i (the kernels'
// mul_nib: one scalar load per nibble, all issued together)
template <class T, int W, class Col>
void nib_image(T *out, Col col) {
    for (int i = 0; i < W / 4; ++i)
        for (int v = 0; v < 16; ++v) {
            T e = 0;
            for (int k = 0; k < 4; ++k)
                if ((v >> (3 - k)) & 1) e ^= (T)col(4 * i + k);
            out[16 * i + v] = e;
        }
}

// W=32 braided-scan constants (layout: engine.h kBraidConstWords): the K image of x^(-32 l) (32 matrix
// columns per lane), T' (the row step's slice-by-4 tables) and T0 (byte table)
int get_braid_consts(Device *d, int alg, const uint64_t **out) {
    auto it = d->braid.find(alg);
    if (it == d->braid.end()) {
        const uint32_t poly = (uint32_t)alg_poly(alg);
        std::vector<uint32_t> c(kBraidConstWords, 0);
        uint32_t kl = 0x80000000u;  // x^0, then x^(-32 l)
        for (int l = 0; l < 64; ++l) {
            uint32_t col = kl;
            for (int j = 0; j < 32; ++j) {
                c[((j >> 2) * 64 + l) * 4 + (j & 3)] = col;
                col = (uint32_t)gf2_mulx(col, poly);
            }
            for (int i = 0; i < 32; ++i) kl = inv_mulx32(kl, poly);
        }
        const uint64_t skip = gf2_xpow8n(kBraidRow - 4, poly, 32);
        for (int i = 0; i < 1024; ++i)
            c[2048 + i] = (uint32_t)gf2_mulmod(gf2_table_entry(i & 255, i >> 8, poly), skip, poly, 32);
        for (int e = 0; e < 256; ++e) c[3072 + e] = (uint32_t)gf2_table_entry(e, 0, poly);
        // the streaming scan's lanes own 8-byte words (K_l = x^(-64 l)) or 16-byte words (x^(-128 l))
        for (const int wbits : {64, 128}) {
            const int base = wbits == 64 ? kBraidK64Word : kBraidK128Word;
            kl = 0x80000000u;
            for (int l = 0; l < 64; ++l) {
                uint32_t col = kl;
                for (int j = 0; j < 32; ++j) {
                    c[base + ((j >> 2) * 64 + l) * 4 + (j & 3)] = col;
                    col = (uint32_t)gf2_mulx(col, poly);
                }
                for (int i = 0; i < wbits; ++i) kl = inv_mulx32(kl, poly);
            }
        }
        // X^(-j) columns (X = x^(8*512), the 8-byte-word row step), u64 each: column i = X^(-j) * x^i
        uint32_t xj = 0x80000000u;  // x^0
        for (int j = 0; j < 8; ++j) {
            uint32_t col = xj;
            for (int i = 0; i < 32; ++i) {
                c[kBraidXinvWord + 2 * (32 * j + i)] = col;
                col = (uint32_t)gf2_mulx(col, poly);
            }
            for (int i = 0; i < 8 * 512; ++i) xj = inv_mulx32(xj, poly);
        }
        // columns of x^(8*4096*2^i), i < 32 (the list streaming scan's part shifts)
        uint64_t sq = gf2_xpow8n(4096, poly, 32);
        for (int i = 0; i < 32; ++i) {
            uint32_t col = (uint32_t)sq;
            for (int j = 0; j < 32; ++j) {
                c[kBraidGshiftWord + 2 * (32 * i + j)] = col;
                col = (uint32_t)gf2_mulx(col, poly);
            }
            sq = gf2_mulmod(sq, sq, poly, 32);
        }
        // columns of x^(8*4096*m), m < kBraidGmCount
        const uint64_t g1 = gf2_xpow8n(4096, poly, 32);
        uint64_t gm = 0x80000000u;  // x^0
        for (int m = 0; m < kBraidGmCount; ++m) {
            uint32_t col = (uint32_t)gm;
            for (int j = 0; j < 32; ++j) {
                c[kBraidGmWord + 2 * (32 * m + j)] = col;
                col = (uint32_t)gf2_mulx(col, poly);
            }
            gm = gf2_mulmod(gm, g1, poly, 32);
        }
        // the three sets again as nibble images (one-round-trip products, round 5)
        for (int j = 0; j < 8; ++j)
            nib_image<uint32_t, 32>(&c[kBraidNibXinvWord + 128 * j], [&](int k) { return c[kBraidXinvWord + 2 * (32 * j + k)]; });
        for (int i = 0; i < 32; ++i)
            nib_image<uint32_t, 32>(&c[kBraidNibGshiftWord + 128 * i], [&](int k) { return c[kBraidGshiftWord + 2 * (32 * i + k)]; });
        for (int m = 0; m < kBraidGmCount; ++m)
            nib_image<uint32_t, 32>(&c[kBraidNibGmWord + 128 * m], [&](int k) { return c[kBraidGmWord + 2 * (32 * m + k)]; });
        // x^(-8 t), t < 8: the list scans' masked edges (crc_kernels.hip lbuf_at)
        uint32_t xn = 0x80000000u;  // x^0, then x^(-8 t)
        for (int t = 0; t < 8; ++t) {
            const uint32_t base = xn;
            nib_image<uint32_t, 32>(&c[kBraidNibXneg8Word + 128 * t], [&](int k) {
                uint32_t col = base;
                for (int i = 0; i < k; ++i) col = (uint32_t)gf2_mulx(col, poly);
                return col;
            });
            for (int i = 0; i < 8; ++i) xn = inv_mulx32(xn, poly);
        }
        DevBuf b;
        int rc = upload_new(b, c.data(), c.size() * 4);
        if (rc) return rc;
        it = d->braid.emplace(alg, b).first;
    }
    *out = (const uint64_t *)it->second.p;
    return 0;
}

// eventstream_flat_kernel's products (engine.h kEsImages): nibble images of x^(64 v 16^d) -- the word
// distances between a message's end word and its previous record or a chunk end, one image per hex
// digit -- and of x^(-8 t), t = 1..7 (the end word's overshoot past the span end).  CRC32 only.
int get_es_images(Device *d, const uint32_t **out) {
    if (!d->es_imgs.p) {
        const uint32_t poly = (uint32_t)alg_poly(ALG_CRC32);
        std::vector<uint32_t> c(128 * kEsImages, 0);
        auto image = [&](int slot, uint32_t k) {
            nib_image<uint32_t, 32>(&c[128 * slot], [&](int j) {
                uint32_t col = k;
                for (int i = 0; i < j; ++i) col = (uint32_t)gf2_mulx(col, poly);
                return col;
            });
        };
        for (int dg = 0; dg < 4; ++dg)
            for (uint32_t v = 1; v < 16; ++v) image(15 * dg + (int)v - 1, (uint32_t)gf2_xpow8n(8ull * v << (4 * dg), poly, 32));
        uint32_t xn = 0x80000000u;  // x^0, then x^(-8 t)
        for (int t = 1; t < 8; ++t) {
            for (int i = 0; i < 8; ++i) xn = inv_mulx32(xn, poly);
            image(60 + t - 1, xn);
        }
        int rc = upload_new(d->es_imgs, c.data(), c.size() * 4);
        if (rc) return rc;
    }
    *out = (const uint32_t *)d->es_imgs.p;
    return 0;
}

// W=64 braided-scan constants: K_l = x^(-64 l), l < 64, then zeros to 16 KiB (a wave without
// payload primes its ring from this block: two groups of its words stay inside)
int get_braid64_consts(Device *d, int alg, const uint64_t **out) {
    auto it = d->braid64.find(alg);
    if (it == d->braid64.end()) {
        const uint64_t poly = alg_poly(alg);
        std::vector<uint64_t> c(2048, 0);
        uint64_t kl = 1ull << 63;  // x^0
        for (int l = 0; l < 64; ++l) {
            c[l] = kl;
            for (int i = 0; i < 64; ++i) kl = inv_mulx64(kl, poly);
        }
        DevBuf b;
        int rc = upload_new(b, c.data(), c.size() * 8);
        if (rc) return rc;
        it = d->braid64.emplace(alg, b).first;
    }
    *out = (const uint64_t *)it->second.p;
    return 0;
}

// crc64_xcd_kernel constants for nwx waves per XCD (u64): [0, 256) the nibble tables of the chunk
// jump J = x^(8 * chunk * (nwx - 1)), entry 16 n + v = (v << 4n) * J; then 40 x 64 columns of
// x^(8 * chunk * 2^i) * x^j; then [level < 4][v < 256] x 64 columns of x^(8 * chunk * v * 256^level) * x^j
// (a part's shift to its buffer end: a byte of the distance per product); then the list scan's X^(-j)
// columns, x^(8*4096*2^i) columns and x^(8*4096*m) columns (m < kBraidGmCount); then the nibble
// images of the last three sets (engine.h kXcdNib*)
int get_xcd_consts(Device *d, int alg, uint64_t nwx, const uint64_t **out) {
    const auto key = std::make_pair(alg, nwx);
    auto it = d->xcd.find(key);
    if (it == d->xcd.end()) {
        const uint64_t poly = alg_poly(alg);
        std::vector<uint64_t> c(kXcdConstU64, 0);
        const uint64_t J = gf2_xpow8n((uint64_t)kXcdChunkBytes * (nwx - 1), poly, 64);
        for (int n = 0; n < 16; ++n)
            for (uint64_t v = 0; v < 16; ++v) c[16 * n + v] = gf2_mulmod(v << (4 * n), J, poly, 64);
        uint64_t sq = gf2_xpow8n(kXcdChunkBytes, poly, 64);
        for (int i = 0; i < 40; ++i) {
            uint64_t col = sq;
            for (int j = 0; j < 64; ++j) {
                c[256 + 64 * i + j] = col;
                col = gf2_mulx(col, poly);
            }
            sq = gf2_mulmod(sq, sq, poly, 64);
        }
        uint64_t base = gf2_xpow8n(kXcdChunkBytes, poly, 64);  // x^(8 * chunk * 256^level)
        for (int L = 0; L < 4; ++L) {
            uint64_t pv = 1ull << 63;  // x^0, then base^v
            for (int v = 0; v < 256; ++v) {
                uint64_t col = pv;
                for (int j = 0; j < 64; ++j) {
                    c[256 + 40 * 64 + (256 * L + v) * 64 + j] = col;
                    col = gf2_mulx(col, poly);
                }
                pv = gf2_mulmod(pv, base, poly, 64);
            }
            base = pv;  // base^256
        }
        // X^(-jr) columns, X = x^(8*512), jr < 32: the head state's entry behind a front pad
        uint64_t xj = 1ull << 63;  // x^0
        for (int jr = 0; jr < 32; ++jr) {
            uint64_t col = xj;
            for (int j = 0; j < 64; ++j) {
                c[256 + 40 * 64 + 4 * 256 * 64 + 64 * jr + j] = col;
                col = gf2_mulx(col, poly);
            }
            for (int i = 0; i < 8 * 512; ++i) xj = inv_mulx64(xj, poly);
        }
        // columns of x^(8*4096*2^i), i < 40: crc64_list_stream_kernel's part shifts (4 KiB groups)
        uint64_t gq = gf2_xpow8n(4096, poly, 64);
        for (int i = 0; i < 40; ++i) {
            uint64_t col = gq;
            for (int j = 0; j < 64; ++j) {
                c[256 + 40 * 64 + 4 * 256 * 64 + 32 * 64 + 64 * i + j] = col;
                col = gf2_mulx(col, poly);
            }
            gq = gf2_mulmod(gq, gq, poly, 64);
        }
        // columns of x^(8*4096*m), m < kBraidGmCount: the same shifts in one product (round 4)
        const uint64_t g1 = gf2_xpow8n(4096, poly, 64);
        uint64_t gm = 1ull << 63;  // x^0
        for (int m = 0; m < kBraidGmCount; ++m) {
            uint64_t col = gm;
            for (int j = 0; j < 64; ++j) {
                c[256 + 40 * 64 + 4 * 256 * 64 + 32 * 64 + 40 * 64 + 64 * m + j] = col;
                col = gf2_mulx(col, poly);
            }
            gm = gf2_mulmod(gm, g1, poly, 64);
        }
        // nibble images (256 u64 per matrix) of X^(-jr), x^(8*4096*2^i) and x^(8*4096*m): the list
        // scan's mul_nib64 (two scalar round trips instead of eight, round 5)
        constexpr uint64_t kXinv = 256 + 40 * 64 + 4 * 256 * 64, kGsh = kXinv + 32 * 64, kGm = kGsh + 40 * 64;
        static_assert(kGm + kBraidGmCount * 64 == kXcdNibXinvU64, "xcd constant layout");
        for (uint64_t m = 0; m < 32; ++m)
            nib_image<uint64_t, 64>(&c[kXcdNibXinvU64 + 256 * m], [&](int k) { return c[kXinv + 64 * m + k]; });
        for (uint64_t m = 0; m < 40; ++m)
            nib_image<uint64_t, 64>(&c[kXcdNibGshiftU64 + 256 * m], [&](int k) { return c[kGsh + 64 * m + k]; });
        for (uint64_t m = 0; m < (uint64_t)kBraidGmCount; ++m)
            nib_image<uint64_t, 64>(&c[kXcdNibGmU64 + 256 * m], [&](int k) { return c[kGm + 64 * m + k]; });
        uint64_t xn = 1ull << 63;  // x^0, then x^(-8 t), t < 8: the list scan's masked edges
        for (int t = 0; t < 8; ++t) {
            const uint64_t base = xn;
            nib_image<uint64_t, 64>(&c[kXcdNibXneg8U64 + 256 * t], [&](int k) {
                uint64_t col = base;
                for (int i = 0; i < k; ++i) col = gf2_mulx(col, poly);
                return col;
            });
            for (int i = 0; i < 8; ++i) xn = inv_mulx64(xn, poly);
        }
        DevBuf b;
        int rc = upload_new(b, c.data(), c.size() * 8);
        if (rc) return rc;
        it = d->xcd.emplace(key, b).first;
    }
    *out = (const uint64_t *)it->second.p;
    return 0;
}

// column j of P_k = x^(8*tile*k) * x^j, k < tmax : moves tile k's partial to its buffer end
int get_pcols(Device *d, int alg, uint64_t tile, uint64_t tmax, hipStream_t s, const uint64_t **out) {
    auto key = std::make_pair(alg, tile);
    auto it = d->pcols_tmax.find(key);
    if (it == d->pcols_tmax.end() || it->second < tmax) {
        if (capturing(s)) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "engine tables must be warmed up before stream capture");
        uint64_t want = std::max<uint64_t>(tmax, 64);
        if (it != d->pcols_tmax.end()) want = std::max(want, it->second * 2);
        const uint64_t poly = alg_poly(alg);
        const int w = width_of(alg);
        std::vector<uint64_t> cols(want * w);
        const uint64_t step = gf2_xpow8n(tile, poly, w);
        uint64_t pk = 1ull << (w - 1);  // x^0
        for (uint64_t k = 0; k < want; ++k) {
            uint64_t c = pk;
            for (int j = 0; j < w; ++j) {
                cols[k * w + j] = c;
                c = gf2_mulx(c, poly);
            }
            pk = gf2_mulmod(pk, step, poly, w);
        }
        DevBuf nb;
        int rc = upload_new(nb, cols.data(), cols.size() * 8);
        if (rc) return rc;
        DevBuf &b = d->pcols[key];
        if (b.p) d->retired.push_back(b);  // queued kernels on other streams may still read it
        b = nb;
        d->pcols_tmax[key] = want;
    }
    *out = (const uint64_t *)d->pcols[key].p;
    return 0;
}

// zero-initialised device words, ordered before the stream's next kernel
template <class T>
int alloc_zero(T **p, size_t n, hipStream_t s) {
    HIP_TRY(hipMalloc((void **)p, n * sizeof(T)));
    HIP_TRY(hipMemsetAsync(*p, 0, n * sizeof(T), s));
    return 0;
}

int get_workspace(Device *d, hipStream_t s, size_t nbuf, size_t ntiles, Workspace **out) {
    StreamState *ss = d->states.get(s);
    t_used = ss;
    Workspace &w = ss->ws;
    const bool grow = w.cap_tiles < ntiles || !w.claim || w.cap < nbuf;
    if (grow && capturing(s)) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "engine workspace must be warmed up before stream capture");
    int rc;
    if (w.cap_tiles < ntiles) {
        const size_t cap = std::max<size_t>(ntiles, w.cap_tiles * 2);
        if (w.acc1) d->retired.push_back({w.acc1, 0}), d->retired.push_back({w.cnt1, 0});
        if ((rc = alloc_zero(&w.acc1, cap, s)) || (rc = alloc_zero(&w.cnt1, cap, s))) return rc;
        w.cap_tiles = cap;
    }
    if (!w.claim && (rc = alloc_zero(&w.claim, 2 * 1024, s))) return rc;  // >= 2 x (max workgroups / kShardBlocks)
    if (w.cap < nbuf) {
        const size_t cap = std::max<size_t>(nbuf, w.cap * 2);
        if (w.acc) d->retired.push_back({w.acc, 0}), d->retired.push_back({w.cnt, 0});
        if ((rc = alloc_zero(&w.acc, cap, s)) || (rc = alloc_zero(&w.cnt, cap, s))) return rc;
        w.cap = cap;
    }
    *out = &w;
    return 0;
}

// main region of a buffer (see engine.h): 16-aligned [H, E)
inline uint64_t main_len(uint64_t ptr, uint64_t n) {
    const uint64_t H = (ptr + 15) & ~15ull, E = (ptr + n) & ~15ull;
    return E > H ? E - H : 0;
}
// the list streaming scans' main regions: a buffer of >= 16 bytes as the 8-byte words [ptr & ~7, end & ~7)
// (crc_kernels.hip lbuf_at: the bytes in front of ptr are masked in the registers)
inline uint64_t main_len_list(uint64_t ptr, uint64_t n) {
    return n >= 16 ? ((ptr + n) & ~7ull) - (ptr & ~7ull) : 0;
}

// Bytes per lane per tile.  A tile is 64*seg bytes; pick the largest seg (fewest partials to
// combine) that still gives every wavefront slot on the chip a tile and does not exceed the
// typical buffer.  per_slot: tiles wanted per wave slot (2 when a workgroup pool balances the
// waves); waves_per_cu: the launch's wave slots per CU.
uint32_t choose_seg(const Device *d, uint64_t total_main, uint64_t typical_main, uint64_t per_slot = 1,
                    uint64_t waves_per_cu = kWavesPerBlock) {
    const uint64_t slots = (uint64_t)d->cus * waves_per_cu * per_slot;
    uint64_t seg = 4096;
    while (seg > kGroupBytes && (total_main / (seg * kWave) < slots || seg * kWave > std::max<uint64_t>(typical_main, 1)))
        seg >>= 1;
    return (uint32_t)std::max<uint64_t>(seg, kGroupBytes);
}

inline bool is_hash(int alg) { return alg >= AWS_CRT_AMD_XXH64; }

// Launch geometry of the scan kernels.  The W=32 scans run 512-thread workgroups (8 waves, 77-80 KiB
// LDS), two of which fit a CU.  A small batch (under 256 MiB of main bytes) launches one per CU: a
// single launch then takes 6 % longer (19.0 vs 17.9 us for 1024 x 64 KiB), but launches queued on
// other streams find a free workgroup slot on every CU, so one launch's prologue and drain overlap
// another's streaming (4950 vs 4290 GiB/s with 3 streams).  Large batches are long
// enough to amortise their own ramp and use both slots.  The W=64 streaming scan runs 512-thread
// workgroups two per CU (66 KiB of LDS); the W=64 braided scan one 1024-thread workgroup per CU.
#ifndef AMDCRC_SMALL_BATCH  // compile-time only (geometry experiments build a variant)
#define AMDCRC_SMALL_BATCH (256ull << 20)
#endif
constexpr uint64_t kSmallBatchBytes = AMDCRC_SMALL_BATCH;
// W=32 streaming scans of at least kSmallBatchBytes on 16-byte words (crc_kernels.hip Braid32W16,
// AMDCRC_STREAM_W16 in engine.h): measured 1-5 % slower than the 8-byte-word kernel, so off
constexpr bool kStreamW16 = AMDCRC_STREAM_W16 != 0;
// Strided CRC64NVME batches of many short buffers (main regions of whole 1 KiB groups, at most
// kRows16MaxBytes, at least a set of four buffers per wave slot) take crc64_rows16_kernel
#ifndef AMDCRC_ROWS16  // compile-time only (A/B builds)
#define AMDCRC_ROWS16 1
#endif
constexpr bool kRows16 = AMDCRC_ROWS16 != 0;
// Strided CRC64NVME batches whose main regions are whole chunks, at least kXcdMinChunks of them, take
// crc64_xcd_kernel (XCD-window chunk order)
#ifndef AMDCRC_XCD  // compile-time only (A/B builds)
#define AMDCRC_XCD 1
#endif
constexpr bool kXcd = AMDCRC_XCD != 0;
#ifndef AMDCRC_XCD_MIN_CHUNKS  // compile-time only (A/B builds)
#define AMDCRC_XCD_MIN_CHUNKS 256
#endif
constexpr uint64_t kXcdMinChunks = AMDCRC_XCD_MIN_CHUNKS;
// W=32 streaming scans in XCD-window tile order (16 KiB tiles)
#ifndef AMDCRC_STREAM_XCD  // compile-time only (A/B builds)
#define AMDCRC_STREAM_XCD 0
#endif
constexpr bool kStreamXcd = AMDCRC_STREAM_XCD != 0;
#ifndef AMDCRC_STREAM_XCD_TILE  // tile bytes of the XCD-window order (A/B builds)
#define AMDCRC_STREAM_XCD_TILE 16384
#endif
constexpr uint64_t kXoTile = AMDCRC_STREAM_XCD_TILE;
#ifndef AMDCRC_STREAM_XCD_MIN  // smallest launch (main bytes) taking the XCD-window order
#define AMDCRC_STREAM_XCD_MIN 0
#endif
constexpr uint64_t kXoMinBytes = AMDCRC_STREAM_XCD_MIN;
constexpr uint64_t kRows16MinBuffers = 4 * 4096;
constexpr uint64_t kRows16MaxBytes = 256u << 10;
// Ragged lists whose buffers are all at most this long take the lane-per-buffer scan
#ifndef AMDCRC_LANE_LIST_MAX  // compile-time only (launch-shape sweeps build a variant; no run-time switch)
#define AMDCRC_LANE_LIST_MAX 4096
#endif
constexpr uint64_t kLaneMaxBytes = AMDCRC_LANE_LIST_MAX;
// Strided CRC64NVME launches of short buffers take the lane-per-buffer scan once they hold enough
// buffers for a wave per SIMD.  1 GiB steps, lanes vs the streaming scan with the byte-Horner tile
// finish (profiles/r02/lane64_r2/): 3749 vs 1262 GiB/s at 2 KiB, 3754 vs 2933 at 4 KiB, 3738 vs 4259
// at 8 KiB (the C4 shard), so buffers up to 4 KiB.  (Round-2 before the finish rewrite, lanes won at
// 8 KiB too: 3668 vs 2693, profiles/r02/lane64/.)  The W=32 scans stay braided (4 KiB CRC32C: 5561
// braided vs 4029 lanes).
#ifndef AMDCRC_LANE64_MAX  // compile-time only (launch-shape sweeps build a variant; no run-time switch)
#define AMDCRC_LANE64_MAX 4096
#endif
constexpr uint64_t kLaneStrided64Max = AMDCRC_LANE64_MAX;
constexpr uint64_t kLaneStrided64MinBuffers = 65536;
// Strided XXH3 batches whose buffers hold at least this many full 1 KiB blocks take the split path
constexpr uint64_t kXxh3SplitBlocks = 4096;
// Ragged CRC32 / CRC32C lists: crc32_list_stream_kernel (0 keeps crc32_braid_kernel<POLY, true>), on
// two 512-thread workgroups per CU once a list holds kListTwoPerCuBytes of main bytes
#ifndef AMDCRC_LIST_STREAM  // compile-time only (A/B builds)
#define AMDCRC_LIST_STREAM 1
#endif
#ifndef AMDCRC_LIST_TWO_PER_CU
#define AMDCRC_LIST_TWO_PER_CU (64ull << 20)
#endif
constexpr bool kListStream = AMDCRC_LIST_STREAM != 0;
// Ragged CRC64NVME lists on crc64_list_stream_kernel (0 keeps crc64_braid_kernel<POLY, true>)
#ifndef AMDCRC_LIST_STREAM64  // compile-time only (A/B builds)
#define AMDCRC_LIST_STREAM64 1
#endif
constexpr bool kListStream64 = AMDCRC_LIST_STREAM64 != 0;
constexpr uint64_t kListTwoPerCuBytes = AMDCRC_LIST_TWO_PER_CU;
// workgroups of a list launch: 8 waves each, at most one wave per 8 groups (4 KiB each)
uint64_t list_stream_blocks(const Device *d, uint64_t ngroups, uint64_t total_main) {
    const uint64_t per_cu = total_main >= kListTwoPerCuBytes ? 2 : 1;
    return std::max<uint64_t>(1, std::min<uint64_t>((ngroups + 63) / 64, (uint64_t)d->cus * per_cu));
}

struct ScanGeometry {
    uint64_t blocks, waves_per_block;
};
ScanGeometry scan_geometry(const Device *d, int alg, uint64_t ntiles, uint64_t total_main, bool w64_half_blocks = false,
                           bool w16 = false) {
    if (w16) {  // crc32_stream_kernel<POLY, 16>: one 1024-thread workgroup per CU
        const uint64_t blocks = std::min<uint64_t>((ntiles + 15) / 16, (uint64_t)d->cus);
        return {blocks, 16};
    }
    const uint64_t wpb = width_of(alg) == 32 ? 8 : w64_half_blocks ? (uint64_t)kW64StreamBlock / kWave : (uint64_t)kWavesPerBlock;
    const uint64_t per_cu = w64_half_blocks ? 1024 / kW64StreamBlock : width_of(alg) == 32 && total_main >= kSmallBatchBytes ? 2 : 1;
    const uint64_t cap = (uint64_t)d->cus * per_cu;
    const uint64_t blocks = std::min<uint64_t>((ntiles + wpb - 1) / wpb, cap);
    return {blocks, wpb};
}

int launch_hash(int alg, XxhParams &xp, hipStream_t s) {
    int e = alg == AWS_CRT_AMD_XXH64 ? amdcrc_launch_xxh64(&xp, s, g_time_events)
                                     : amdcrc_launch_xxh3(alg == AWS_CRT_AMD_XXH3_64 ? 64 : 128, &xp, s, g_time_events);
    g_time_events[0] = g_time_events[1] = nullptr;
    return e ? fail(AWS_CRT_AMD_ERR_HIP, std::string("hash kernel launch: ") + hipGetErrorString((hipError_t)e)) : 0;
}

// log2(v) + 1 when v is a power of two, else 0 (ScanParams::shifts1)
uint8_t pow2_shift1(uint64_t v) { return v && (v & (v - 1)) == 0 ? (uint8_t)(__builtin_ctzll(v) + 1) : (uint8_t)0; }

// crc32_stream_kernel needs no per-stream workspace when every buffer lies wholly inside one workgroup's
// tiles and that workgroup combines it in LDS (crc_kernels.hip LocalBufs: T <= 32, at most kLocalSlots
// whole buffers per workgroup): the C2 shapes, one batch or twenty.  The launch then takes no stream
// state, so it records no fence event behind itself (round 5: one runtime call less per launch, the
// cost that bounds one-batch-per-launch submission).
// wpb: waves per workgroup of the instantiation (8: 512-thread kBraidBlock; 16: the 1024-thread
// kW16Block of the 16-byte-word variant, p.stream == 2).
bool stream_local_only(const ScanParams &p, uint64_t blocks, uint64_t wpb) {
    const uint64_t T = p.tiles_per_buf, nw = blocks * wpb;
    if (T < 2 || T > 32 || p.nstatic || p.xcd_order || p.list_mode) return false;
    auto split_at = [&](uint64_t w) { return w * p.split_q + std::min<uint64_t>(w, p.split_r); };
    for (uint64_t b = 0; b < blocks; ++b) {
        const uint64_t t0 = split_at(wpb * b), t1 = split_at(std::min(wpb * b + wpb, nw));
        if (t0 % T || t1 % T || (t1 - t0) / T > kStreamLocalSlots) return false;
    }
    return true;
}

int launch_scan(Device *d, int alg, ScanParams &p, uint64_t nbuf, uint64_t tmax, uint64_t total_main, hipStream_t s) {
    const uint64_t tile = (uint64_t)p.seg * kWave;
    int rc = width_of(alg) == 32 ? get_braid_consts(d, alg, &p.d_kvals) : get_braid64_consts(d, alg, &p.d_kvals);
    if (rc) return rc;
    p.d_pcols = nullptr;
    p.pcols_tmax = 0;
    p.d_acc = nullptr;
    p.d_cnt = nullptr;
    p.d_acc1 = nullptr;
    p.d_cnt1 = nullptr;
    p.d_claim = nullptr;
    const bool w64_half = width_of(alg) == 64 && p.stream;  // crc64_stream4_kernel
    uint64_t blocks = scan_geometry(d, alg, p.ntiles, total_main, w64_half, p.stream == 2).blocks;
    if (p.stream == 3) blocks = std::min<uint64_t>((p.nbuf + 4 * 8 - 1) / (4 * 8), 2 * (uint64_t)d->cus);  // 4 buffers per wave
    if (p.list_mode && p.stream == 4) blocks = list_stream_blocks(d, p.ntiles, total_main);  // the waves list_stream split for
    if (blocks == 0) return 0;
    // crc32_stream_kernel's static split (ScanParams::split_q), now that the grid is known.  Every
    // instantiation takes its waves' tiles from the split (the 16-byte-word variant,
    // p.stream == 2, had none and wrote no result), over its own waves per workgroup.
    const bool stream32 = width_of(alg) == 32 && (p.stream == 1 || p.stream == 2) && !p.list_mode;
    const uint64_t wpb = p.stream == 2 ? 16 : 8;
    if (stream32) {
        const uint64_t nw = blocks * wpb;
        p.split_q = p.ntiles / nw;
        p.split_r = (uint32_t)(p.ntiles % nw);
        p.shifts1 = (p.shifts1 & ~0xFFu) | pow2_shift1(p.tiles_per_buf);
    }
    bool ws = false;
    if (tmax > 1 || p.nstatic) {
        if ((rc = get_pcols(d, alg, tile, tmax, s, &p.d_pcols))) return rc;
        p.pcols_tmax = tmax;
        ws = !(stream32 && stream_local_only(p, blocks, wpb));
        if (ws && !t_plan) {
            Workspace *w;
            if ((rc = get_workspace(d, s, nbuf, p.ntiles, &w))) return rc;
            p.d_acc = w->acc;
            p.d_cnt = w->cnt;
            p.d_acc1 = w->acc1;
            p.d_cnt1 = w->cnt1;
            p.d_claim = w->claim;
        }
    }
    // crc64_list_stream_kernel: the head-entry and part-shift columns
    if (p.list_mode && p.stream == 4 && width_of(alg) == 64 && (rc = get_xcd_consts(d, alg, 512, &p.d_pcols))) return rc;
    if (t_plan) {
        PlannedLaunch pl;
        pl.alg = alg, pl.p = p, pl.blocks = blocks, pl.ws = ws, pl.ws_nbuf = nbuf, pl.ws_tiles = p.ntiles;
        t_plan->push_back(pl);
        return 0;
    }
    int e = amdcrc_launch_scan(alg, &p, (int)blocks, s, g_time_events);
    g_time_events[0] = g_time_events[1] = nullptr;
    if (e) return fail(AWS_CRT_AMD_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString((hipError_t)e));
    fence_after(s);
    return 0;
}

// One uniform batch of a strided launch
struct Batch {
    uint64_t base;
    const void *seeds;
    void *out;
};

int scan_batches(Device *d, int alg, const Batch *bs, size_t nb, size_t stride, size_t len, size_t count, uint64_t seed_all,
                 hipStream_t s);

// ---- XXH64 over few long device buffers: the stream-ordered host route.
// XXH64 is one serial chain per buffer (four lanes whose every round depends on the last): on a
// gfx950 SIMD a round is issue-bound at about 41 cycles (experiments/chainbench.hip: 31.5 for the six chain
// instructions, 9 more for the two DPP moves that bring the next stripe's product in), 1.7 GiB/s
// per buffer, against about 1.3 ns per round on one host core.  A batch of at most kX64HostMaxBuffers
// long buffers therefore goes to the host: slices of every buffer (one hipMemcpy2DAsync per slice) are
// copied D2H on the caller's stream into two pinned halves, alternately, each copy gated by a stream
// wait on a signal-memory counter that the host worker advances once it has hashed the slice two back;
// the worker (a runner thread, not HIP's callback thread: round 5) hashes a slice with one pool thread
// per buffer as soon as its copy lands, and the results go back H2D on the caller's stream behind a
// final wait.  The call keeps the batch ABI's asynchronous, stream-ordered contract.
// AWS_CRT_AMD_XXH64_ROUTE=0 (read per call) keeps every batch on the GPU kernels.
#ifndef AMDCRC_X64_HOST_MAX  // compile-time only (A/B builds: 0 keeps every XXH64 batch on the GPU kernels)
#define AMDCRC_X64_HOST_MAX 16
#endif
constexpr size_t kX64HostMaxBuffers = AMDCRC_X64_HOST_MAX;
constexpr size_t kX64HostMinBytes = 1u << 20;
constexpr size_t kX64Half = 32u << 20;             // one pinned half: a slice of every buffer
constexpr size_t kX64StageExtra = 16 * 64;          // seeds, then results (at most 64 buffers)
static_assert(kX64HostMaxBuffers <= 64, "staging extra");

// Staging of one queued job: two pinned halves (+ seeds / results), and two counters in signal memory
// through which the caller's stream and the job's host worker order each other without host
// callbacks (round 5; VERDICT r04: the slices used to be hashed inside hipLaunchHostFunc callbacks,
// which run on the runtime's one async-handler thread, so concurrent jobs on other streams -- and
// every other callback in the process -- waited behind them):
//   copied  the stream writes base + k + 1 once slice k is in its half (hipStreamWriteValue64)
//   hashed  the worker stores base + k + 1 once it has hashed slice k; the copy of slice k + 2 into
//           the same half and the results' H2D wait for it (hipStreamWaitValue64)
// Everything the worker waits for is queued on the caller's stream AHEAD of the wait that waits for
// the worker, so no wait can stand in front of what it depends on -- also when the runtime maps
// several streams onto one hardware queue (a first version copied on a separate stream, whose
// packets could sit behind the caller's wait in a shared queue: a deadlock).  The counters only grow:
// a stage reused by a later job continues from its sequence number.
struct X64Stage {
    int dev = -1;
    uint8_t *pin = nullptr;  // 2 * kX64Half, then kX64StageExtra
    uint64_t *copied = nullptr, *hashed = nullptr;  // signal memory (hipMallocSignalMemory)
    uint64_t seq = 0;                               // counter value reached by the stage's last job
    hipEvent_t done = nullptr;                      // recorded after the results' H2D
};
std::mutex g_x64_mu;
std::vector<X64Stage *> g_x64_free;

struct X64Job {
    X64Stage *st = nullptr;
    size_t count = 0, nslices = 0, slice = 0, len = 0;
    uint64_t base = 0;  // counter value before the job's first slice
    uint64_t *h_seed = nullptr, *h_res = nullptr;
    uint64_t *out_host = nullptr;  // results wanted in host memory: the worker writes them there itself
    std::atomic<bool> submitted{false};  // the submitting thread has queued everything (done recorded)
    bool seeds = false;
    uint64_t seed_all = 0;
    hipStream_t stream = nullptr;  // the caller's stream: polled for errors while the worker waits on it
    std::vector<cpu::Xxh64State> xs;
};

// Route workers never block process exit: the runner is never destroyed (no join at
// static destruction), an exit handler -- registered after the globals above exist, so it runs before
// their destructors -- tells waiting workers to stop and gives running ones a moment to finish, and a
// worker whose stream failed (or whose GPU stopped) gives up instead of spinning forever.
std::atomic<bool> g_x64_stop{false};
std::atomic<int> g_x64_active{0};
std::atomic<unsigned long long> g_x64_abandoned{0};

void x64_at_exit() {
    g_x64_stop.store(true, std::memory_order_release);
    for (int i = 0; i < 200 && g_x64_active.load(std::memory_order_acquire) > 0; ++i)
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
}

Runner &x64_runner() {
    static Runner *r = [] {
        std::atexit(x64_at_exit);
        return new Runner;
    }();
    return *r;
}

inline uint64_t sig_load(const uint64_t *p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline void sig_store(uint64_t *p, uint64_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }

// The job's host worker (a runner thread, never the runtime's callback thread): slice k once the copy
// stream reports it copied, one host thread per buffer; then the stage goes back once the caller's
// stream has taken the results.
// AWS_CRT_AMD_X64_TRACE=1 prints one line per job: time waiting for copies, time hashing.
// Wait until *ctr >= want.  Gives up (false) when the process is exiting or the job's stream has
// failed (hipStreamQuery reports an error other than "not ready", polled about every 5 ms).
bool x64_wait(const X64Job *j, const uint64_t *ctr, uint64_t want) {
    for (unsigned spin = 0; sig_load(ctr) < want; ++spin) {
        if (g_x64_stop.load(std::memory_order_acquire)) return false;
        if (spin < 64) {
            std::this_thread::yield();
            continue;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
        if ((spin & 255) == 0) {
            const hipError_t q = hipStreamQuery(j->stream);
            if (q != hipSuccess && q != hipErrorNotReady) return false;
        }
    }
    return true;
}

// A job whose copies will never land: release every wait the stream holds on the worker (the
// counters jump past the job), drop the stage (the device may still write into it: never reused)
// and count the job.  The stream's own error reports the failure to the caller.
void x64_abandon(X64Job *j) {
    sig_store(j->st->hashed, j->base + j->nslices);
    g_x64_abandoned.fetch_add(1, std::memory_order_relaxed);
    delete j;
    g_x64_active.fetch_sub(1, std::memory_order_acq_rel);
}

void x64_work(X64Job *j) noexcept {
    X64Stage *st = j->st;
    static const bool trace = [] {
        const char *e = getenv("AWS_CRT_AMD_X64_TRACE");
        return e && e[0] == '1';
    }();
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    double wait_us = 0, hash_us = 0, first_us = 0;
    for (size_t k = 0; k < j->nslices; ++k) {
        const uint64_t want = j->base + k + 1;
        const auto w0 = clk::now();
        if (!x64_wait(j, st->copied, want)) return x64_abandon(j);
        const auto w1 = clk::now();
        if (k == 0) first_us = std::chrono::duration<double, std::micro>(w1 - w0).count();
        else wait_us += std::chrono::duration<double, std::micro>(w1 - w0).count();
        const uint8_t *rows = st->pin + (k & 1) * kX64Half;
        const size_t off = k * j->slice, rb = std::min(j->slice, j->len - off);
        const bool first = k == 0, last = k + 1 == j->nslices;
        cpu::parallel(j->count, [&](size_t i) {
            if (first) cpu::xxh64_reset(&j->xs[i], j->seeds ? j->h_seed[i] : j->seed_all);
            cpu::xxh64_update(&j->xs[i], rows + i * rb, rb);
            if (last) j->h_res[i] = cpu::xxh64_digest(&j->xs[i]);
        });
        if (k + 1 == j->nslices && j->out_host) std::memcpy(j->out_host, j->h_res, 8 * j->count);
        sig_store(st->hashed, want);
        hash_us += std::chrono::duration<double, std::micro>(clk::now() - w1).count();
    }
    if (trace)
        fprintf(stderr, "[x64] buffers %zu slices %zu of %zu B: first copy %.0f us, copy waits %.0f us, hashing %.0f us, total %.0f us, threads %zu\n",
                j->count, j->nslices, j->slice, first_us, wait_us, hash_us,
                std::chrono::duration<double, std::micro>(clk::now() - t0).count(), cpu::share());
    while (!j->submitted.load(std::memory_order_acquire)) {
        if (g_x64_stop.load(std::memory_order_acquire)) return x64_abandon(j);
        std::this_thread::yield();
    }
    // the results' H2D has read h_res (polled: a stream that failed or a process exiting ends the wait)
    for (unsigned spin = 0;; ++spin) {
        const hipError_t q = hipEventQuery(st->done);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady || g_x64_stop.load(std::memory_order_acquire)) return x64_abandon(j);
        std::this_thread::sleep_for(std::chrono::microseconds(spin < 64 ? 5 : 50));
    }
    {
        std::lock_guard<std::mutex> g(g_x64_mu);
        try {
            g_x64_free.push_back(st);
        } catch (...) {
            (void)0;  // the stage is dropped (leaked) rather than freed under the lock
        }
    }
    delete j;
    g_x64_active.fetch_sub(1, std::memory_order_acq_rel);
}

int x64_take_stage(int dev, X64Stage **out) {
    std::lock_guard<std::mutex> g(g_x64_mu);
    for (size_t i = 0; i < g_x64_free.size(); ++i)
        if (g_x64_free[i]->dev == dev) {
            *out = g_x64_free[i];
            g_x64_free.erase(g_x64_free.begin() + (long)i);
            return 0;
        }
    std::unique_ptr<X64Stage> st(new X64Stage);
    st->dev = dev;
    HIP_TRY(hipHostMalloc((void **)&st->pin, 2 * kX64Half + kX64StageExtra, hipHostMallocPortable));
    HIP_TRY(hipExtMallocWithFlags((void **)&st->copied, sizeof(uint64_t), hipMallocSignalMemory));
    HIP_TRY(hipExtMallocWithFlags((void **)&st->hashed, sizeof(uint64_t), hipMallocSignalMemory));
    sig_store(st->copied, 0);
    sig_store(st->hashed, 0);
    HIP_TRY(hipEventCreateWithFlags(&st->done, hipEventDisableTiming));
    *out = st.release();
    return 0;
}

// AWS_CRT_AMD_XXH64_ROUTE=0: every XXH64 batch on the kernels (a caller with no spare host CPUs)
bool x64_route_wanted() {
    const char *e = getenv("AWS_CRT_AMD_XXH64_ROUTE");
    return !(e && e[0] == '0' && e[1] == 0);
}

// the device can order its streams on memory values (hipStreamWaitValue64); otherwise the route is off
bool x64_route_usable(int dev) {
    static std::mutex mu;
    static std::map<int, bool> known;
    std::lock_guard<std::mutex> g(mu);
    auto it = known.find(dev);
    if (it != known.end()) return it->second;
    int v = 0;
    const bool ok = hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue, dev) == hipSuccess && v != 0;
    (void)hipGetLastError();
    known[dev] = ok;
    return ok;
}

bool is_device_ptr(const void *p);

int xxh64_host_route(int dev, uint64_t base, size_t stride, size_t len, size_t count, const void *d_seeds, uint64_t seed_all,
                     void *d_out, hipStream_t s) {
    std::unique_ptr<X64Job> j(new X64Job);
    int rc = x64_take_stage(dev, &j->st);
    if (rc) return rc;
    X64Stage *st = j->st;
    j->count = count;
    j->len = len;
    j->h_seed = (uint64_t *)(st->pin + 2 * kX64Half);
    j->h_res = j->h_seed + 64;
    j->seeds = d_seeds != nullptr;
    j->seed_all = seed_all;
    j->xs.resize(count);
    j->slice = std::min<size_t>(len, (kX64Half / count) & ~(size_t)63);
    j->nslices = (len + j->slice - 1) / j->slice;
    j->base = st->seq;
    const uint64_t end = j->base + j->nslices;
    hipError_t e = hipSuccess;
    if (g_time_events[0]) e = hipEventRecord((hipEvent_t)g_time_events[0], s);
    if (!e && d_seeds) e = hipMemcpyAsync(j->h_seed, d_seeds, 8 * count, hipMemcpyDefault, s);
    for (size_t k = 0; !e && k < j->nslices; ++k) {
        const size_t off = k * j->slice, rb = std::min(j->slice, len - off);
        if (k >= 2) e = hipStreamWaitValue64(s, st->hashed, j->base + k - 1, hipStreamWaitValueGte);  // half free
        if (!e)
            e = hipMemcpy2DAsync(st->pin + (k & 1) * kX64Half, rb, (const void *)(uintptr_t)(base + off), stride, rb, count,
                                 hipMemcpyDeviceToHost, s);
        if (!e) e = hipStreamWriteValue64(s, st->copied, j->base + k + 1, 0);
    }
    if (e) {
        // nothing waits for a worker yet: release every wait already queued (the counters jump past
        // the job), let the stream drain, and keep the stage (its sequence continues after this job's)
        sig_store(st->hashed, end);
        (void)hipStreamSynchronize(s);
        st->seq = end;
        sig_store(st->copied, end);
        {
            std::lock_guard<std::mutex> g(g_x64_mu);
            g_x64_free.push_back(st);
        }
        g_time_events[0] = g_time_events[1] = nullptr;
        return fail(AWS_CRT_AMD_ERR_HIP, std::string("xxh64 host route: ") + hipGetErrorString(e));
    }
    st->seq = end;
    // results for host memory (the single-buffer path's pinned slot) are written by the worker: a
    // host-to-host hipMemcpyAsync may be performed by the runtime on this thread once the stream
    // reaches it, i.e. after the worker, which must therefore already be running
    const bool host_out = !is_device_ptr(d_out);
    j->out_host = host_out ? (uint64_t *)d_out : nullptr;
    uint64_t *const h_res = j->h_res;
    j->stream = s;
    X64Job *jp = j.release();
    bool posted = true;
    g_x64_active.fetch_add(1, std::memory_order_acq_rel);
    try {
        x64_runner().post([jp] { x64_work(jp); });
    } catch (...) {
        posted = false;  // hashed on this thread below (x64_work ends the active count either way)
    }
    e = hipStreamWaitValue64(s, st->hashed, end, hipStreamWaitValueGte);  // every slice hashed
    if (!e && !host_out) e = hipMemcpyAsync(d_out, h_res, 8 * count, hipMemcpyHostToDevice, s);
    if (!e && g_time_events[1]) e = hipEventRecord((hipEvent_t)g_time_events[1], s);
    g_time_events[0] = g_time_events[1] = nullptr;
    if (!e) e = hipEventRecord(st->done, s);
    if (e) (void)hipStreamSynchronize(s);  // whatever was queued has run before the worker lets the stage go
    // from here on the worker owns the job and the stage (it may free them at once)
    jp->submitted.store(true, std::memory_order_release);
    if (!posted) x64_work(jp);  // no thread to be had: hash on this thread
    return e ? fail(AWS_CRT_AMD_ERR_HIP, std::string("xxh64 host route: ") + hipGetErrorString(e)) : 0;
}

int strided_impl(Device *d, int alg, uint64_t base, size_t stride, size_t len, size_t count, const void *d_seeds,
                 uint64_t seed_all, void *d_out, hipStream_t s) {
    if (count == 0) return 0;
    if (!d_out || (len && !base)) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null buffer");
    if (!is_hash(alg)) {
        const Batch b{base, d_seeds, d_out};
        return scan_batches(d, alg, &b, 1, stride, len, count, seed_all, s);
    }
    // the route copies rows with hipMemcpy2DAsync (source pitch = stride): overlapping or repeated
    // buffers (stride < len, e.g. stride 0 = one buffer under several seeds) and pitches past the
    // device's 2D-copy limit stay on the kernels
    if (alg == AWS_CRT_AMD_XXH64 && count <= kX64HostMaxBuffers && len >= kX64HostMinBytes && (count == 1 || stride >= len) &&
        x64_route_usable(d->id) && x64_route_wanted() &&
        (count == 1 || stride <= d->max_pitch) && !capturing(s))
        return xxh64_host_route(d->id, base, count == 1 ? len : stride, len, count, d_seeds, seed_all, d_out, s);
    {
        XxhParams xp{};
        xp.base = base;
        xp.stride = stride;
        xp.len = len;
        xp.nbuf = count;
        xp.d_seeds = (const uint64_t *)d_seeds;
        xp.seed_all = seed_all;
        xp.d_out = (uint64_t *)d_out;
        // XXH3 over long uniform buffers: a block-sum pass over all CUs, then one wave per buffer
        // scrambles the 64-byte sums (xxh3_kernels.hip)
        const uint64_t nb = len > 240 ? (len - 1) / 1024 : 0;
        if (alg != AWS_CRT_AMD_XXH64 && nb >= kXxh3SplitBlocks) {
            // the sums are the stream's state: held from their sizing until the fence behind the
            // scramble pass that reads them
            std::lock_guard<std::mutex> g(d->mu);
            StreamState *ss = d->states.get(s);
            t_used = ss;
            DevBuf &xs = ss->xsums;
            const size_t need = count * nb * 64;
            if (xs.bytes < need) {
                if (capturing(s)) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "engine workspace must be warmed up before stream capture");
                if (xs.p) d->retired.push_back(xs);  // queued launches may still read the old sums
                xs = DevBuf{};
                HIP_TRY(hipMalloc(&xs.p, need));
                xs.bytes = need;
            }
            xp.d_sums = (uint64_t *)xs.p;
            int e = amdcrc_launch_xxh3_blocksum(&xp, s, g_time_events[0]);
            g_time_events[0] = nullptr;
            if (e) {
                t_used = nullptr;
                return fail(AWS_CRT_AMD_ERR_HIP, std::string("xxh3 block-sum launch: ") + hipGetErrorString((hipError_t)e));
            }
            const int rc = launch_hash(alg, xp, s);
            if (rc) t_used = nullptr;
            fence_after(s);
            return rc;
        }
        return launch_hash(alg, xp, s);
    }
}

// CRC scan of nb uniform batches (same stride / len / count; bases of one alignment mod 16) in one
// launch: buffer b of the launch is buffer b % count of batch b / count (ScanParams::bbase etc.)
int scan_batches(Device *d, int alg, const Batch *bs, size_t nb, size_t stride, size_t len, size_t count, uint64_t seed_all,
                 hipStream_t s) {
    if (count > 1 && (stride % 16) != 0)
        return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "strided batch needs stride % 16 == 0 (use the list API)");
    if (nb == 0 || nb > (size_t)kMaxBatches) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "bad batch count");
    std::lock_guard<std::mutex> g(d->mu);
    t_used = nullptr;
    const uint64_t base = bs[0].base;
    const uint64_t ml = main_len(base, len);
    ScanParams p{};
    p.nbatch = (uint32_t)nb;
    p.bcount = count;
    p.shifts1 = (uint32_t)pow2_shift1(count) << 8;
    for (size_t j = 0; j < nb; ++j) {
        p.bbase[j] = bs[j].base;
        p.bout[j] = (uint64_t)(uintptr_t)bs[j].out;
        p.bseed[j] = (uint64_t)(uintptr_t)bs[j].seeds;
    }
    count *= nb;  // buffers of the launch
    if (alg == AWS_CRT_AMD_CRC64NVME && len <= kLaneStrided64Max && count >= kLaneStrided64MinBuffers) {
        // short CRC64NVME buffers: one lane per buffer (crc_lanes_kernel) -- the W=64 braided scan's
        // per-tile lane combine (a 64-step GF(2) multiply per lane) costs more than such a tile's scan
        LaneParams lp{};
        lp.nbuf = count;
        lp.seed_all = seed_all;
        lp.stride = stride;
        lp.len = len;
        lp.bcount = p.bcount;
        for (size_t j = 0; j < nb; ++j) lp.bbase[j] = p.bbase[j], lp.bout[j] = p.bout[j], lp.bseed[j] = p.bseed[j];
        if (t_plan) {
            PlannedLaunch pl;
            pl.alg = alg, pl.kind = 1, pl.lp = lp;
            t_plan->push_back(pl);
            return 0;
        }
        int e = amdcrc_launch_lanes(alg, &lp, s, g_time_events);
        g_time_events[0] = g_time_events[1] = nullptr;
        return e ? fail(AWS_CRT_AMD_ERR_HIP, std::string("lane kernel launch: ") + hipGetErrorString((hipError_t)e)) : 0;
    }
    // Batches whose main regions are whole tiles take the streaming scans (crc32_stream_kernel,
    // crc64_stream4_kernel), tiles sized for one per wave slot of the launch: 1024 x 64 KiB CRC32C
    // measured 5250-5315 GiB/s with one 32 KiB tile per wave against 5000-5030 with two of 16 KiB.
    // W=64 small batches: tiles for 4 waves per CU.  A tile that spans a whole buffer finishes without
    // the cross-tile combine (global atomics with return, pcol loads), which costs a W=64 wave more
    // than the idle slots do once other streams' launches fill them: 1024 x 64 KiB CRC64NVME measured
    // 2774 GiB/s with 16 KiB tiles (4 per buffer), 3930 with 32 KiB, 4010 with 64 KiB.
    p.seg = choose_seg(d, ml * count, ml, 1);
    const bool w32 = width_of(alg) == 32;
    const bool small = ml * count < kSmallBatchBytes;
    const uint64_t wpc = w32 ? 8 * (small ? 1 : 2) : small ? 4 : (uint64_t)kWavesPerBlock;
    const uint32_t seg_stream = choose_seg(d, ml * count, ml, 1, wpc);
    const bool stream = ml > 0 && ml % ((uint64_t)seg_stream * kWave) == 0;
    if (stream) p.seg = seg_stream;
    // W=32 braided scan: every wave scans one static tile, then claims tiles from its workgroup's
    // pool, where the pool does not shrink the tiles (smaller tiles cost a tile finish per 8 KiB and
    // measured slower on 1024 x 64 KiB: 3704 vs 4380 GiB/s; on 16 x 256 MiB and 131072 x 8 KiB the
    // pool gains 3-4 % at equal tiles)
    const bool pool = w32 && ml > 0 && choose_seg(d, ml * count, ml, 2) == p.seg;
    const uint64_t tile = (uint64_t)p.seg * kWave;
    const uint64_t T = ml ? (ml + tile - 1) / tile : 1;
    p.base = base;
    p.stride = stride;
    p.len = len;
    p.tiles_per_buf = T;
    p.nbuf = count;
    p.ntiles = T * count;
    p.seed_all = seed_all;
    p.stream = stream && ml % tile == 0 ? 1u : 0u;
    // many short CRC64NVME buffers whose main regions are whole 1 KiB groups: 16 lanes per buffer
    // (crc64_rows16_kernel), one tile finish per four buffers
    if (!w32 && kRows16 && count >= kRows16MinBuffers && ml >= 1024 && ml <= kRows16MaxBytes && ml % 1024 == 0) {
        p.stream = 3;
        p.base = base;
        p.stride = stride;
        p.len = len;
        p.tiles_per_buf = 1;
        p.nbuf = count;
        p.ntiles = count;
        p.seed_all = seed_all;
        return launch_scan(d, alg, p, count, 1, ml * count, s);
    }
    // long CRC64NVME buffers of whole chunks: XCD-window chunk order (crc64_xcd_kernel)
    if (!w32 && kXcd && ml >= kXcdMinChunks * kXcdChunkBytes) {
        const uint64_t blocks = ((uint64_t)d->cus * kXcdBpc) & ~7ull, nwx = blocks * (kXcdBlock / 64) / 8;
        if (blocks >= 8) {
            p.stream = 5;
            p.tiles_per_buf = (ml + kXcdChunkBytes - 1) / kXcdChunkBytes;
            p.xcd_pad = (uint32_t)(p.tiles_per_buf * kXcdChunkBytes - ml);
            p.ntiles = p.tiles_per_buf * count;
            int rc = get_braid64_consts(d, alg, &p.d_kvals);
            if (!rc) rc = get_xcd_consts(d, alg, nwx, &p.d_pcols);
            if (rc) return rc;
            if (t_plan) {
                PlannedLaunch pl;
                pl.alg = alg, pl.p = p, pl.blocks = blocks, pl.ws = true, pl.ws_nbuf = count, pl.ws_tiles = 1;
                t_plan->push_back(pl);
                return 0;
            }
            Workspace *w;
            if ((rc = get_workspace(d, s, count, 1, &w))) return rc;
            p.d_acc = w->acc;
            p.d_cnt = w->cnt;
            int e = amdcrc_launch_scan(alg, &p, (int)blocks, s, g_time_events);
            g_time_events[0] = g_time_events[1] = nullptr;
            if (e) return fail(AWS_CRT_AMD_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString((hipError_t)e));
            fence_after(s);
            return 0;
        }
    }
    // large W=32 launches: 16-byte lane words in one 1024-thread workgroup per CU (the same waves per
    // CU as two 512-thread workgroups; the tiles hold 4 KiB groups either way)
    if (p.stream && w32 && kStreamW16 && !small) p.stream = 2;
    // XCD-window tile order (crc32_stream_kernel, ScanParams::xcd_order): buffers of 1, 2, 4 or 8 tiles
    // of 16 KiB; every XCD eighth a whole number of buffers; each wave's tile count within the LDS slots
    if (kStreamXcd && w32 && !kStreamW16 && ml > 0 && ml % kXoTile == 0 && ml / kXoTile <= 8 &&
        ((ml / kXoTile) & (ml / kXoTile - 1)) == 0 && (kXoMinBytes == 0 || ml * count >= kXoMinBytes)) {
        const uint64_t To = ml / kXoTile, nt = To * count;
        const ScanGeometry geo = scan_geometry(d, alg, nt, ml * count);
        const uint64_t nwx = geo.blocks * geo.waves_per_block / 8;
        const uint64_t rounds = nwx ? (nt / 8 + nwx - 1) / nwx : 0;
        if (geo.blocks % 8 == 0 && geo.waves_per_block == 8 && nt % (8 * To) == 0 && rounds * (8 / To) <= 128) {
            p.seg = (uint32_t)(kXoTile / kWave);
            p.stream = 1;
            p.tiles_per_buf = To;
            p.ntiles = nt;
            p.nstatic = 0;
            p.xcd_order = 1;
            return launch_scan(d, alg, p, count, To, ml * count, s);
        }
    }
    if (pool && !p.stream) {
        // workgroup pools need every wave to own a static tile: ntiles / blocks >= waves per block
        const ScanGeometry geo = scan_geometry(d, alg, p.ntiles, ml * count);
        if (p.ntiles >= 2 * geo.blocks * geo.waves_per_block) p.nstatic = geo.blocks * geo.waves_per_block;
    }
    return launch_scan(d, alg, p, count, T, ml * count, s);
}

// Descriptor staging: returns pinned host memory to fill (slot `cur`); stage_end queues its upload
// on the stream and returns the device copy.  The slot reused is the one three calls old.
int stage_begin(Device *d, hipStream_t s, size_t bytes, void **host) {
    StreamState *ss = d->states.get(s);
    t_used = ss;
    Stage &st = ss->st;
    const int k = st.next;
    st.cur = k;
    st.next = (k + 1) % kStageSlots;
    if (!st.done[k]) {
        HIP_TRY(hipEventCreateWithFlags(&st.done[k], hipEventDisableTiming));
    } else {
        HIP_TRY(hipEventSynchronize(st.done[k]));  // this slot's previous upload has been performed
    }
    if (st.dev[k].bytes < bytes) {
        if (capturing(s)) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "descriptor staging must be warmed up before stream capture");
        if (st.dev[k].p) d->retired.push_back(st.dev[k]);  // the device copy may still be read by queued kernels
        if (st.host[k].p) (void)hipHostFree(st.host[k].p);  // its upload has completed (event above)
        const size_t cap = std::max<size_t>(bytes, st.dev[k].bytes * 2);
        st.dev[k] = DevBuf{};
        st.host[k] = DevBuf{};
        HIP_TRY(hipMalloc(&st.dev[k].p, cap));
        HIP_TRY(hipHostMalloc(&st.host[k].p, cap, hipHostMallocDefault));
        st.dev[k].bytes = st.host[k].bytes = cap;
    }
    *host = st.host[k].p;
    return 0;
}

int stage_end(Device *d, hipStream_t s, size_t bytes, const void **dev) {
    Stage &st = d->states.get(s)->st;
    const int k = st.cur;
    HIP_TRY(hipMemcpyAsync(st.dev[k].p, st.host[k].p, bytes, hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(st.done[k], s));
    *dev = st.dev[k].p;
    return 0;
}

// Ragged CRC32 / CRC32C lists on crc32_list_stream_kernel.  Every buffer's main
// region (the 8-byte words covering it: main_len_list) is front-padded to whole 4 KiB groups; the list is one sequence of groups, split evenly over
// the waves (cut anywhere, also inside a buffer).  Wave w walks buffers [wbuf[w], wbuf[w + 1]) from
// group woff[w] of the first, scans groups [wq[w], wq[w + 1]) of the sequence and folds the buffers
// without a main region whose place in the sequence falls in its range.  Descriptor block:
// ptrs[count] lens[count] wbuf[nw + 1] woff[nw + 1] wq[nw + 1].
int list_stream(Device *d, int alg, const void *const *ptrs, const size_t *lens, size_t count,
                const std::vector<uint64_t> &mains, uint64_t total, const void *d_seeds, void *d_out, hipStream_t s) {
    constexpr uint64_t gb = 4096;  // bytes per wave group
    std::vector<uint64_t> gp(count + 1, 0);
    bool split = false;
    for (size_t i = 0; i < count; ++i) gp[i + 1] = gp[i] + (mains[i] + gb - 1) / gb;
    const uint64_t ng = gp[count];
    const uint64_t blocks = list_stream_blocks(d, ng, total), nw = blocks * 8;
    const size_t words = count * 2 + 4 * (nw + 1);
    uint64_t *h;
    int rc = stage_begin(d, s, words * 8, (void **)&h);
    if (rc) return rc;
    for (size_t i = 0; i < count; ++i) {
        h[i] = (uint64_t)(uintptr_t)ptrs[i];
        h[count + i] = lens[i];
    }
    uint64_t *wbuf = h + 2 * count, *woff = wbuf + nw + 1, *wq = woff + nw + 1;
    // wave w starts at the first buffer that ends past q0 = w * ng / nw, or at a buffer without a main
    // region whose place is q0 (those come first in index order); both cursors only move forward
    size_t b = 0;
    for (uint64_t w = 0; w <= nw; ++w) {
        const uint64_t q0 = w == nw ? ng : w * ng / nw;
        if (w == nw) {
            b = count;
        } else {
            while (b < count && gp[b + 1] <= q0 && !(gp[b + 1] == gp[b] && gp[b] >= q0)) ++b;
        }
        wbuf[w] = b;
        wq[w] = q0;
        woff[w] = b < count && gp[b + 1] > gp[b] ? q0 - gp[b] : 0;
        if (woff[w]) split = true;
    }
    // join descriptors of buffers cut between waves (crc32/64_list_stream_kernel): the parts of such a
    // buffer inside one workgroup (8 waves) meet in an LDS slot -- slot = its first wave in the
    // workgroup, or 8 when it began in an earlier workgroup -- and the last of the `expected` parts
    // to arrive finishes the buffer, or publishes the workgroup's share when the buffer also lies in
    // another workgroup.  Word w: bits 0-15 the descriptor of wave w's first part, 16-31 of its last
    // (bit 15 valid, 0-3 slot, 4-7 expected, 8 global).
    uint64_t *wjoin = wq + nw + 1;
    std::fill(wjoin, wjoin + nw + 1, 0ull);
    if (split) {
        auto wave_of = [&](uint64_t q) {  // the wave whose group range holds group q
            return (uint64_t)(std::upper_bound(wq, wq + nw + 1, q) - wq) - 1;
        };
        for (size_t i = 0; i < count; ++i) {
            if (gp[i + 1] == gp[i]) continue;
            const uint64_t ws = wave_of(gp[i]), we = wave_of(gp[i + 1] - 1);
            if (ws == we) continue;  // whole inside one wave
            for (uint64_t w = ws; w <= we; ++w) {
                if (wq[w + 1] == wq[w]) continue;  // a wave without groups holds no part
                const uint64_t wg0 = w & ~7ull, r0 = std::max(ws, wg0), r1 = std::min(we, wg0 + 7);
                uint64_t parts = 0;
                for (uint64_t v = r0; v <= r1; ++v) parts += wq[v + 1] > wq[v] ? 1 : 0;
                const uint64_t desc = 0x8000u | (ws >= wg0 ? ws - wg0 : 8u) | (parts << 4) |
                                      ((ws < wg0 || we > wg0 + 7) ? 0x100u : 0u);
                if (wq[w] >= gp[i]) wjoin[w] |= desc;              // the buffer is wave w's first part
                if (wq[w + 1] <= gp[i + 1]) wjoin[w] |= desc << 16;  // ... and/or its last part
            }
        }
    }
    const uint64_t *dd;
    if ((rc = stage_end(d, s, words * 8, (const void **)&dd))) return rc;
    ScanParams p{};
    p.seg = kGroupBytes;
    p.list_mode = 1;
    p.stream = 4;
    p.nbatch = 1;
    p.bcount = count;
    p.d_ptrs = dd;
    p.d_lens = dd + count;
    p.d_wave_buf = dd + 2 * count;
    p.d_tile_prefix = dd + 2 * count + nw + 1;
    p.nbuf = count;
    p.ntiles = ng;
    p.d_seeds = d_seeds;
    p.d_out = d_out;
    // a buffer cut between waves combines through the per-buffer accumulator and count (workspace)
    return launch_scan(d, alg, p, count, split ? 2 : 1, total, s);
}

int list_impl(Device *d, int alg, const void *const *ptrs, const size_t *lens, size_t count, const void *d_seeds,
              void *d_out, hipStream_t s) {
    if (count == 0) return 0;
    if (!ptrs || !lens || !d_out) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null argument");
    std::lock_guard<std::mutex> g(d->mu);
    t_used = nullptr;
    // plan: seg from the median main length, tiles per buffer, per-wave starting buffer
    std::vector<uint64_t> mains(count);
    uint64_t total = 0, maxlen = 0;
    for (size_t i = 0; i < count; ++i) {
        if (lens[i] && !ptrs[i]) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null buffer with nonzero length");
        mains[i] = main_len((uint64_t)(uintptr_t)ptrs[i], lens[i]);
        total += mains[i];
        maxlen = std::max<uint64_t>(maxlen, lens[i]);
    }
    const bool xxh = is_hash(alg);
    // lists of short buffers only (event-stream framing): one lane per buffer (crc_lanes_kernel)
    if (!xxh && maxlen <= kLaneMaxBytes) {
        uint64_t *h;
        int rc1 = stage_begin(d, s, count * 16, (void **)&h);
        if (rc1) return rc1;
        for (size_t i = 0; i < count; ++i) {
            h[i] = (uint64_t)(uintptr_t)ptrs[i];
            h[count + i] = lens[i];
        }
        const uint64_t *dl;
        if ((rc1 = stage_end(d, s, count * 16, (const void **)&dl))) return rc1;
        LaneParams lp{};
        lp.d_ptrs = dl, lp.d_lens = dl + count, lp.nbuf = count, lp.d_seeds = d_seeds, lp.d_out = d_out;
        int e = amdcrc_launch_lanes(alg, &lp, s, g_time_events);
        g_time_events[0] = g_time_events[1] = nullptr;
        if (e) return fail(AWS_CRT_AMD_ERR_HIP, std::string("lane kernel launch: ") + hipGetErrorString((hipError_t)e));
        fence_after(s);
        return 0;
    }
    uint32_t seg = kGroupBytes;
    uint64_t tile = 0;
    // CRC64NVME lists whose main regions are all whole 4 KiB groups (no front pads) measured 6 % faster
    // on crc64_braid_kernel<POLY, true>; any padded buffer moves the list to the stream
    bool padded64 = false;
    if (width_of(alg) == 64)
        for (size_t i = 0; i < count && !padded64; ++i) padded64 = mains[i] % (kGroupBytes * kWave) != 0;
    if (kListStream && !xxh && (width_of(alg) == 32 || (kListStream64 && padded64))) {
        uint64_t total8 = 0;
        for (size_t i = 0; i < count; ++i) total8 += (mains[i] = main_len_list((uint64_t)(uintptr_t)ptrs[i], lens[i]));
        return list_stream(d, alg, ptrs, lens, count, mains, total8, d_seeds, d_out, s);
    }
    if (!xxh) {
        std::vector<uint64_t> sorted(mains);
        std::nth_element(sorted.begin(), sorted.begin() + count / 2, sorted.end());
        seg = choose_seg(d, total, sorted[count / 2]);
        tile = (uint64_t)seg * kWave;
    }
    // descriptor block: ptrs[count] lens[count] prefix[count+1] wavebuf[nwaves]
    std::vector<uint64_t> prefix(count + 1, 0);
    uint64_t tmax = 1;
    for (size_t i = 0; i < count; ++i) {
        const uint64_t T = xxh ? 1 : (mains[i] ? (mains[i] + tile - 1) / tile : 1);
        tmax = std::max(tmax, T);
        prefix[i + 1] = prefix[i] + T;
    }
    const uint64_t ntiles = prefix[count];
    const ScanGeometry geo = scan_geometry(d, xxh ? ALG_CRC32 : alg, ntiles, total);
    const uint64_t nw = std::max<uint64_t>(geo.blocks, 1) * geo.waves_per_block;
    // (a workgroup tile pool for lists, as strided batches have, was tried in round 3 and dropped: its
    // claims do not skip tiles without a main region -- empty or sub-16-byte buffers -- which the
    // static walk skips)
    const size_t words = count * 2 + (count + 1) + nw;
    uint64_t *h;
    int rc0 = stage_begin(d, s, words * 8, (void **)&h);
    if (rc0) return rc0;
    for (size_t i = 0; i < count; ++i) {
        h[i] = (uint64_t)(uintptr_t)ptrs[i];
        h[count + i] = lens[i];
    }
    std::memcpy(h + 2 * count, prefix.data(), (count + 1) * 8);
    uint64_t *wb = h + 3 * count + 1;
    for (uint64_t w = 0; w < nw; ++w) {
        const uint64_t t0 = w * ntiles / nw;
        const uint64_t b = (uint64_t)(std::upper_bound(prefix.begin(), prefix.end(), t0) - prefix.begin()) - 1;
        wb[w] = std::min<uint64_t>(b, count - 1);
    }
    const uint64_t *dd;
    if ((rc0 = stage_end(d, s, words * 8, (const void **)&dd))) return rc0;
    if (xxh) {
        XxhParams xp{};
        xp.d_ptrs = dd;
        xp.d_lens = dd + count;
        xp.nbuf = count;
        xp.d_seeds = (const uint64_t *)d_seeds;
        xp.d_out = (uint64_t *)d_out;
        const int rc = launch_hash(alg, xp, s);
        if (!rc) fence_after(s);
        return rc;
    }
    ScanParams p{};
    p.seg = seg;
    p.list_mode = 1;
    p.nbatch = 1;
    p.bcount = count;
    p.d_ptrs = dd;
    p.d_lens = dd + count;
    p.d_tile_prefix = dd + 2 * count;
    p.d_wave_buf = dd + 3 * count + 1;
    p.nbuf = count;
    p.ntiles = ntiles;
    p.d_seeds = d_seeds;
    p.d_out = d_out;
    return launch_scan(d, alg, p, count, tmax, total, s);
}

int ensure_stage(Device *d, size_t bytes) {
    if (!d->own_stream) HIP_TRY(hipStreamCreateWithFlags(&d->own_stream, hipStreamNonBlocking));
    if (!d->d_small) HIP_TRY(hipMalloc(&d->d_small, 64));
    if (!d->h_res) HIP_TRY(hipHostMalloc(&d->h_res, 64, hipHostMallocCoherent));
    if (d->stage_bytes >= bytes) return 0;
    for (int i = 0; i < 2; ++i) {
        if (d->pin[i]) {
            HIP_TRY(hipStreamSynchronize(d->own_stream));  // the engine's own stream only
            (void)hipHostFree(d->pin[i]);
            (void)hipFree(d->dbuf[i]);
        }
        HIP_TRY(hipHostMalloc(&d->pin[i], bytes, hipHostMallocDefault));
        HIP_TRY(hipMalloc(&d->dbuf[i], bytes));
        if (!d->pin_free[i]) HIP_TRY(hipEventCreateWithFlags(&d->pin_free[i], hipEventDisableTiming));
    }
    d->stage_bytes = bytes;
    return 0;
}

// the runtime's view of a pointer (ptr_class.h): 0 unregistered host, 1 runtime-known host, 2 device
int probe_ptr(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged || a.type == hipMemoryTypeUnified) return 2;
    return a.type == hipMemoryTypeUnregistered ? 0 : 1;
}
using Classifier = PtrClass<probe_ptr>;

bool is_device_ptr(const void *p) {
    if (!p || device_count_noinit() <= 0) return false;
    return Classifier::classify(p) == PtrKind::Device;
}

constexpr size_t kStageChunk = 16u << 20;
constexpr size_t kHashStageMax = 64u << 20;  // cached device copy of a GPU-dispatched host hash (kept <= 64 MiB)

// One buffer (host or device memory) on the GPU, synchronous.  Host data streams through two pinned
// slots; chunk i+1 is seeded on the device with chunk i's result, so no host round trip sits
// between chunks (the running-CRC semantics of CRC.h:20).
int single_impl(int alg, const void *input, size_t len, uint64_t seed, uint64_t *result) {
    Device *d;
    int rc = get_device(&d);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(d->single_mu);
    if ((rc = ensure_stage(d, std::min(kStageChunk, std::max<size_t>(len, 4096))))) return rc;
    hipStream_t s = d->own_stream;
    const size_t osz = alg == AWS_CRT_AMD_XXH3_128 ? 16 : (width_of(alg) == 64 || is_hash(alg)) ? 8 : 4;
    char *res = (char *)d->d_small;  // two result slots (ping-pong) + seed slot
    if ((len == 0 || !input) && !is_hash(alg)) {
        *result = seed;  // CRC of nothing is the seed itself
        return 0;
    }
    if (is_hash(alg)) {
        // xxHash is not chunkable by seed: a host buffer is copied whole into device memory.  Up to
        // one staging chunk the copy goes into a cached buffer; a larger one into a buffer of its own
        // that is freed once the call has synchronised, so a large hash never stays pinned in HBM.
        const void *dp = input;
        void *temp = nullptr;
        const bool host_in = len && !is_device_ptr(input);
        // a long XXH64 buffer takes the host route on the device too (strided_impl): one that is
        // already in host memory is hashed where it is, without crossing PCIe twice
        if (host_in && alg == AWS_CRT_AMD_XXH64 && len >= kX64HostMinBytes) {
            result[0] = cpu::xxh64((const uint8_t *)input, len, seed);
            return 0;
        }
        if (host_in) {
            if (len > kHashStageMax) {
                HIP_TRY(hipMalloc(&temp, len));
                dp = temp;
            } else {
                if (d->hash_stage.bytes < len) {
                    // geometric growth up to kHashStageMax: repeated large hashes reuse one buffer
                    const size_t cap = std::min(kHashStageMax, std::max(std::max(len, kStageChunk), d->hash_stage.bytes * 2));
                    if (d->hash_stage.p) (void)hipFree(d->hash_stage.p);  // own stream synchronised after every call
                    d->hash_stage = DevBuf{};
                    HIP_TRY(hipMalloc(&d->hash_stage.p, cap));
                    d->hash_stage.bytes = cap;
                }
                dp = d->hash_stage.p;
            }
            const hipError_t ce = hipMemcpyAsync((void *)dp, input, len, hipMemcpyHostToDevice, s);
            if (ce != hipSuccess) {
                if (temp) (void)hipFree(temp);
                return fail(AWS_CRT_AMD_ERR_HIP, std::string("hash staging copy: ") + hipGetErrorString(ce));
            }
        }
        const uint64_t base = len ? (uint64_t)(uintptr_t)dp : 16;
        rc = strided_impl(d, alg, base, len, len, 1, nullptr, seed, d->h_res, s);
        {
            const hipError_t e = hipStreamSynchronize(s);  // also before a failed launch's staging is freed
            if (!rc && e != hipSuccess) rc = fail(AWS_CRT_AMD_ERR_HIP, hipGetErrorString(e));
        }
        if (temp) (void)hipFree(temp);
        const volatile uint64_t *h = (const volatile uint64_t *)d->h_res;
        result[0] = rc ? 0 : h[0];
        if (osz == 16) result[1] = rc ? 0 : h[1];
        return rc;
    }
    // the last launch stores its result straight into pinned host memory (no device-to-host copy)
    if (is_device_ptr(input)) {
        rc = strided_impl(d, alg, (uint64_t)(uintptr_t)input, len, len, 1, nullptr, seed, d->h_res, s);
        if (rc) return rc;
    } else {
        const char *src = (const char *)input;
        size_t off = 0;
        int i = 0;
        while (off < len) {
            const size_t n = std::min(kStageChunk, len - off);
            const int slot = i & 1;
            HIP_TRY(hipEventSynchronize(d->pin_free[slot]));  // slot's previous H2D copy done
            std::memcpy(d->pin[slot], src + off, n);
            HIP_TRY(hipMemcpyAsync(d->dbuf[slot], d->pin[slot], n, hipMemcpyHostToDevice, s));
            HIP_TRY(hipEventRecord(d->pin_free[slot], s));
            const void *dseed = i == 0 ? nullptr : res + ((i - 1) & 1) * 8;
            const bool last = off + n == len;
            rc = strided_impl(d, alg, (uint64_t)(uintptr_t)d->dbuf[slot], n, n, 1, dseed, seed,
                              last ? d->h_res : (void *)(res + slot * 8), s);
            if (rc) return rc;
            off += n;
            ++i;
        }
    }
    HIP_TRY(hipStreamSynchronize(s));
    const volatile char *h = (const volatile char *)d->h_res;
    *result = osz == 4 ? *(const volatile uint32_t *)h : *(const volatile uint64_t *)h;
    return 0;
}

}  // namespace

// ================================================================== internal (abi_single.cpp)
extern "C" int amdcrc_gpu_usable(void) {
    return guarded(err_sink, [&]() -> int {
        Device *d;
        return get_device(&d) == 0 ? 1 : 0;
    });
}
extern "C" int amdcrc_is_device_ptr(const void *p) { return is_device_ptr(p) ? 1 : 0; }
#if AWS_CRT_AMD_DIAG
// diagnostic library only: runtime pointer probes made by the calling thread (tests: the small-call
// path stays out of the HIP runtime)
extern "C" AWS_CRT_AMD_API unsigned long long aws_crt_amd_debug_pointer_probes(void) { return Classifier::tls().probes; }
#endif
extern "C" int amdcrc_gpu_single(int alg, const void *input, size_t len, uint64_t seed, uint64_t *out) {
    return guarded(err_sink, [&]() -> int {
        return single_impl(alg, input, len, seed, out);
    });
}
extern "C" int amdcrc_copy_to_host(void *dst, const void *src, size_t n) {
    return hipMemcpy(dst, src, n, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
// Streaming XXH3 (abi_single.cpp aws_xxhash_update): nblocks whole 1 KiB blocks of device memory
// absorbed into the stream's eight accumulators acc (in / out), in passes of at most 256 MiB (16 MiB
// of block sums); the accumulators stay on the device between passes.  Synchronous.
extern "C" int amdcrc_gpu_xxh3_blocks(const void *d_ptr, uint64_t nblocks, uint64_t seed, uint64_t acc[8]) {
    return guarded(err_sink, [&]() -> int {
        Device *d;
        int rc = get_device(&d);
        if (rc) return rc;
        if (!is_device_ptr(d_ptr)) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "xxh3 stream: not device memory");
        std::lock_guard<std::mutex> g(d->single_mu);
        if ((rc = ensure_stage(d, 4096))) return rc;
        hipStream_t s = d->own_stream;
        constexpr uint64_t kPassBlocks = 256 * 1024;
        const uint64_t pass = std::min<uint64_t>(nblocks, kPassBlocks);
        if (d->xstream_sums.bytes < pass * 64) {
            if (d->xstream_sums.p) {
                HIP_TRY(hipStreamSynchronize(s));  // the engine's own stream only
                (void)hipFree(d->xstream_sums.p);
            }
            d->xstream_sums = DevBuf{};
            HIP_TRY(hipMalloc(&d->xstream_sums.p, pass * 64));
            d->xstream_sums.bytes = pass * 64;
        }
        uint64_t *d_acc = (uint64_t *)d->d_small;  // 64 B: the single path's slots (under single_mu)
        HIP_TRY(hipMemcpyAsync(d_acc, acc, 64, hipMemcpyHostToDevice, s));
        for (uint64_t b = 0; b < nblocks; b += kPassBlocks) {
            const uint64_t m = std::min(kPassBlocks, nblocks - b);
            const int e = amdcrc_launch_xxh3_stream((const uint8_t *)d_ptr + 1024 * b, m, seed, (uint64_t *)d->xstream_sums.p, d_acc, s);
            if (e) {
                (void)hipStreamSynchronize(s);
                return fail(AWS_CRT_AMD_ERR_HIP, std::string("xxh3 stream launch: ") + hipGetErrorString((hipError_t)e));
            }
        }
        HIP_TRY(hipMemcpyAsync(d->h_res, d_acc, 64, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        std::memcpy(acc, d->h_res, 64);
        return 0;
    });
}

// ================================================================== C ABI
extern "C" {

AWS_CRT_AMD_API int aws_crt_amd_init(void) {
    return guarded(err_sink, [&]() -> int {
        Device *d;
        return get_device(&d);
    });
}

AWS_CRT_AMD_API int aws_crt_amd_device_count(void) { return device_count_noinit(); }

AWS_CRT_AMD_API const char *aws_crt_amd_last_error(void) { return g_last_error.c_str(); }

// Launch profiling (checksums_batch.h): the next launch made by this thread stamps the dispatch's own
// start / end timestamps into these hipEvent_t (hipExtLaunchKernel), the interval a kernel-trace
// profiler reports, without the marker packets of a hipEventRecord pair.
AWS_CRT_AMD_API void aws_crt_amd_profile_next_launch(void *start_event, void *stop_event) {
    g_time_events[0] = start_event;
    g_time_events[1] = stop_event;
}

// Elapsed milliseconds between two events stamped by aws_crt_amd_profile_next_launch (waits for the
// stop event); -1 on failure.
AWS_CRT_AMD_API float aws_crt_amd_profile_elapsed_ms(void *start_event, void *stop_event) {
    float ms = -1.0f;
    if (hipEventSynchronize((hipEvent_t)stop_event) != hipSuccess) return -1.0f;
    if (hipEventElapsedTime(&ms, (hipEvent_t)start_event, (hipEvent_t)stop_event) != hipSuccess) return -1.0f;
    return ms;
}

#if AWS_CRT_AMD_DIAG
// Diagnostic library only: one launch of the streaming-read ceiling kernel (crc_kernels.hip
// read_ceiling_kernel) over [d_base, d_base + bytes), in the W=32 streaming scan's launch shape
// (512-thread workgroups, one per CU below 256 MiB, two above).  Honours
// aws_crt_amd_profile_next_launch.
AWS_CRT_AMD_API int aws_crt_amd_debug_read_ceiling(const void *d_base, size_t bytes, void *hip_stream) {
    return guarded(err_sink, [&]() -> int {
        Device *d;
        int rc = get_device(&d);
        if (rc) return rc;
        const size_t words = (size_t)d->cus * 2 * 8;  // one word per wave (practically never written)
        {
            std::lock_guard<std::mutex> g(d->mu);
            if (!d->ceil_sink.p) {
                HIP_TRY(hipMalloc(&d->ceil_sink.p, words * sizeof(uint32_t)));
                d->ceil_sink.bytes = words * sizeof(uint32_t);
            }
        }
        const int blocks = bytes >= kSmallBatchBytes ? 2 * d->cus : d->cus;
        const int e = amdcrc_launch_read_ceiling(d_base, bytes, (uint32_t *)d->ceil_sink.p, blocks, hip_stream, g_time_events);
        g_time_events[0] = g_time_events[1] = nullptr;
        return e ? fail(AWS_CRT_AMD_ERR_HIP, std::string("read ceiling launch: ") + hipGetErrorString((hipError_t)e)) : 0;
    });
}
#endif

// Per-stream state (stream_states.h): hand a stream's state back (before destroying the stream, or
// when it will not be used with the engine for a while); at most kMaxStreamStates streams per device
// hold state otherwise, the least recently used idle one handing its state to a new stream.
AWS_CRT_AMD_API int aws_crt_amd_stream_release(void *hip_stream) {
    return guarded(err_sink, [&]() -> int {
        std::lock_guard<std::mutex> g(g_mu);
        for (auto &kv : g_devices) {
            Device *d = kv.second.get();
            std::lock_guard<std::mutex> gd(d->mu);
            d->states.release((hipStream_t)hip_stream);
        }
        return 0;
    });
}

AWS_CRT_AMD_API int aws_crt_amd_stream_states(size_t *live, size_t *spare, size_t *created) {
    return guarded(err_sink, [&]() -> int {
        Device *d;
        int rc = get_device(&d);
        if (rc) return rc;
        std::lock_guard<std::mutex> g(d->mu);
        if (live) *live = d->states.live();
        if (spare) *spare = d->states.spares();
        if (created) *created = d->states.created();
        return 0;
    });
}

AWS_CRT_AMD_API int aws_crt_amd_checksum_strided(int alg, const void *d_base, size_t stride, size_t len, size_t count,
                                                 const void *d_seeds, void *d_out, void *hip_stream) {
    return guarded(err_sink, [&]() -> int {
        if (alg < 0 || alg > 5) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "bad algorithm");
        Device *d;
        int rc = get_device(&d);
        if (rc) return rc;
        if (count == 1) stride = len;
        return strided_impl(d, alg, (uint64_t)(uintptr_t)d_base, stride, len, count, d_seeds, 0, d_out, (hipStream_t)hip_stream);
    });
}

AWS_CRT_AMD_API int aws_crt_amd_checksum_batches(int alg, const struct aws_crt_amd_batch *batches, size_t nbatches,
                                                 size_t stride, size_t len, size_t count, void *hip_stream) {
    return guarded(err_sink, [&]() -> int {
        if (alg < 0 || alg > 5) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "bad algorithm");
        if (nbatches && !batches) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null batches");
        Device *d;
        int rc = get_device(&d);
        if (rc) return rc;
        hipStream_t s = (hipStream_t)hip_stream;
        if (count == 1) stride = len;
        for (size_t j = 0; j < nbatches; ++j)
            if (!batches[j].d_out || (len && !batches[j].d_base)) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null buffer");
        if (count == 0 || nbatches == 0) return 0;
        if (is_hash(alg)) {  // the hash kernels run one launch per batch
            for (size_t j = 0; j < nbatches && !rc; ++j)
                rc = strided_impl(d, alg, (uint64_t)(uintptr_t)batches[j].d_base, stride, len, count, batches[j].d_seeds, 0,
                                  batches[j].d_out, s);
            return rc;
        }
        // one launch per run of up to kMaxBatches batches whose bases share their alignment mod 16
        std::vector<Batch> run;
        for (size_t j = 0; j <= nbatches && !rc; ++j) {
            const bool flush = j == nbatches || run.size() == (size_t)kMaxBatches ||
                               (!run.empty() && ((uint64_t)(uintptr_t)batches[j].d_base & 15) != (run[0].base & 15));
            if (flush && !run.empty()) {
                rc = scan_batches(d, alg, run.data(), run.size(), stride, len, count, 0, s);
                run.clear();
            }
            if (j < nbatches) run.push_back({(uint64_t)(uintptr_t)batches[j].d_base, batches[j].d_seeds, batches[j].d_out});
        }
        return rc;
    });
}

// Prepared submissions (checksums_batch.h aws_crt_amd_plan_*): the planning of
// aws_crt_amd_checksum_batches (runs of batches, kernel, tile size, geometry, constants) done once;
// a launch of the plan only looks up the stream's workspace where a kernel needs one and launches.
struct aws_crt_amd_plan {
    Device *dev = nullptr;
    int alg = 0;
    std::vector<PlannedLaunch> launches;
    // hashes: the batch call itself, made at launch (their launches depend on the stream)
    std::vector<aws_crt_amd_batch> batches;
    size_t stride = 0, len = 0, count = 0;
};

AWS_CRT_AMD_API int aws_crt_amd_plan_create(int alg, const struct aws_crt_amd_batch *batches, size_t nbatches, size_t stride,
                                            size_t len, size_t count, aws_crt_amd_plan **out) {
    return guarded(err_sink, [&]() -> int {
        if (!out) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null plan pointer");
        *out = nullptr;
        if (alg < 0 || alg > 5) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "bad algorithm");
        if (nbatches && !batches) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null batches");
        Device *d;
        int rc = get_device(&d);
        if (rc) return rc;
        if (count == 1) stride = len;
        for (size_t j = 0; j < nbatches; ++j)
            if (!batches[j].d_out || (len && !batches[j].d_base)) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null buffer");
        if (count > 1 && (stride % 16) != 0 && !is_hash(alg))
            return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "strided batch needs stride % 16 == 0 (use the list API)");
        std::unique_ptr<aws_crt_amd_plan> pl(new aws_crt_amd_plan);
        pl->dev = d, pl->alg = alg, pl->stride = stride, pl->len = len, pl->count = count;
        if (is_hash(alg) || count == 0) {
            pl->batches.assign(batches, batches + nbatches);
        } else {
            struct Rec {
                explicit Rec(std::vector<PlannedLaunch> *v) { t_plan = v; }
                ~Rec() { t_plan = nullptr; }
            } rec(&pl->launches);
            std::vector<Batch> run;
            for (size_t j = 0; j <= nbatches && !rc; ++j) {
                const bool flush = j == nbatches || run.size() == (size_t)kMaxBatches ||
                                   (!run.empty() && ((uint64_t)(uintptr_t)batches[j].d_base & 15) != (run[0].base & 15));
                if (flush && !run.empty()) {
                    rc = scan_batches(d, alg, run.data(), run.size(), stride, len, count, 0, nullptr);
                    run.clear();
                }
                if (j < nbatches) run.push_back({(uint64_t)(uintptr_t)batches[j].d_base, batches[j].d_seeds, batches[j].d_out});
            }
            if (rc) return rc;
        }
        *out = pl.release();
        return 0;
    });
}

AWS_CRT_AMD_API int aws_crt_amd_plan_launch(aws_crt_amd_plan *pl, void *hip_stream) {
    return guarded(err_sink, [&]() -> int {
        if (!pl) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null plan");
        hipStream_t s = (hipStream_t)hip_stream;
        if (!pl->batches.empty())
            return aws_crt_amd_checksum_batches(pl->alg, pl->batches.data(), pl->batches.size(), pl->stride, pl->len, pl->count,
                                                hip_stream);
        for (const PlannedLaunch &L : pl->launches) {
            int e;
            if (L.kind == 1) {
                e = amdcrc_launch_lanes(L.alg, &L.lp, s, g_time_events);
            } else if (L.ws) {
                ScanParams p = L.p;
                std::lock_guard<std::mutex> g(pl->dev->mu);
                t_used = nullptr;
                Workspace *w;
                const int rc = get_workspace(pl->dev, s, L.ws_nbuf, L.ws_tiles, &w);
                if (rc) {
                    t_used = nullptr;
                    return rc;
                }
                p.d_acc = w->acc, p.d_cnt = w->cnt, p.d_acc1 = w->acc1, p.d_cnt1 = w->cnt1, p.d_claim = w->claim;
                e = amdcrc_launch_scan(L.alg, &p, (int)L.blocks, s, g_time_events);
                if (!e) fence_after(s);
                t_used = nullptr;
            } else {
                e = amdcrc_launch_scan(L.alg, &L.p, (int)L.blocks, s, g_time_events);
            }
            g_time_events[0] = g_time_events[1] = nullptr;
            if (e) return fail(AWS_CRT_AMD_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString((hipError_t)e));
        }
        return 0;
    });
}

AWS_CRT_AMD_API size_t aws_crt_amd_plan_launches(const aws_crt_amd_plan *pl) {
    return pl ? (pl->batches.empty() ? pl->launches.size() : pl->batches.size()) : 0;
}

AWS_CRT_AMD_API void aws_crt_amd_plan_destroy(aws_crt_amd_plan *pl) { delete pl; }

// Submission queue (checksums_batch.h): pushes collect batches of one shape; a full queue
// (max_batches, at most kMaxBatches), an age bound (a flusher thread), a flush or a wait hand them to
// aws_crt_amd_checksum_batches, one launch per run of batches -- and, under the eager policy (the
// default since round 6), so does any push that finds fewer than max_inflight of
// the queue's launches still running.  Round 5's queue launched only at 32 queued batches or at the
// flush: a producer of one batch at a time left the GPU idle through all its pushes (4548-4689 GiB/s,
// below one launch per batch).  Every push gets a ticket; each launch records an event after it on
// the queue's stream, so a ticket's completion (or the error of the launch that dropped it) can be
// asked for and waited on -- and the eager policy asks the newest events whether the stream is busy.
// Eager launches' default minimum batch count.  Measured on the driver's command (20 pushes of one
// C2 batch from Python, then flush; profiles/r06/c/driver1.log): min 1 4955 GiB/s (the first push
// launches a lone one-batch launch at frac ~0.55, 3-4 launches), min 2 5381 (2 launches), min 4 5358,
// two launches in flight 4636, the batched policy 4953, one launch per batch 4834.
constexpr size_t kQueueMinLaunch = 2;
struct aws_crt_amd_queue {
    int alg = 0;
    int device = 0;
    size_t stride = 0, len = 0, count = 0;
    void *stream = nullptr;
    size_t max_batches = kMaxBatches;
    uint64_t max_age_us = 0;
    bool eager = true;        // AWS_CRT_AMD_QUEUE_EAGER
    size_t max_inflight = 1;  // eager: launch on a push while fewer of the queue's launches are running
    size_t min_launch = kQueueMinLaunch;  // eager: ... and at least this many batches are queued
    uint64_t nlaunches = 0;   // launches made (refused ones included)
    std::mutex mu;
    std::condition_variable cv;
    std::vector<aws_crt_amd_batch> pending;
    uint64_t next_ticket = 1;                                  // ticket of the next push
    std::chrono::steady_clock::time_point oldest;              // push time of pending[0]
    struct Launch {
        uint64_t first, end;  // tickets [first, end)
        hipEvent_t ev;        // recorded after the launch (nullptr when it was refused)
        int rc;
    };
    std::deque<Launch> launches;                               // recent launches, oldest first
    std::vector<Launch> failed;                                // pruned refused launches (bounded)
    uint64_t expired_below = 0;                                // tickets below this may have lost their record
    std::vector<hipEvent_t> spare;                             // events of completed, pruned launches
    std::thread flusher;
    bool stop = false;
};

namespace {
constexpr size_t kQueueKeepLaunches = 64;
constexpr size_t kQueueKeepFailures = 1024;

void queue_prune_locked(aws_crt_amd_queue *q) {
    while (q->launches.size() > kQueueKeepLaunches) {
        aws_crt_amd_queue::Launch &L = q->launches.front();
        if (L.rc) {
            // adjacent refused launches with one status share a record; past the bound the oldest
            // record goes and its tickets (and every pruned one below them) report EXPIRED, never 0
            if (!q->failed.empty() && q->failed.back().end == L.first && q->failed.back().rc == L.rc) {
                q->failed.back().end = L.end;
            } else {
                if (q->failed.size() >= kQueueKeepFailures) {
                    q->expired_below = q->failed.front().end;
                    q->failed.erase(q->failed.begin());
                }
                q->failed.push_back(L);
            }
        } else if (hipEventQuery(L.ev) != hipSuccess) {
            (void)hipGetLastError();
            return;  // still running: keep it (and every later one)
        } else {
            q->spare.push_back(L.ev);
        }
        q->launches.pop_front();
    }
}

int queue_flush_locked(aws_crt_amd_queue *q) {
    if (q->pending.empty()) return 0;
    const uint64_t first = q->next_ticket - q->pending.size();
    int rc = aws_crt_amd_checksum_batches(q->alg, q->pending.data(), q->pending.size(), q->stride, q->len, q->count,
                                          q->stream);
    hipEvent_t ev = nullptr;
    if (!rc) {
        if (!q->spare.empty()) {
            ev = q->spare.back();
            q->spare.pop_back();
        } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
            ev = nullptr;
        }
        if (!ev || hipEventRecord(ev, (hipStream_t)q->stream) != hipSuccess) {
            (void)hipGetLastError();
            if (ev) q->spare.push_back(ev);
            ev = nullptr;
            rc = fail(AWS_CRT_AMD_ERR_HIP, "queue: completion event");
        }
    }
    // launched (with its completion event), or refused: its tickets carry the error; not retried
    q->launches.push_back({first, q->next_ticket, ev, rc});
    ++q->nlaunches;
    q->pending.clear();
    queue_prune_locked(q);
    return rc;
}

// The queue's launches still running, newest first, counted up to `limit` (a stream completes its
// launches in order: the first complete one ends the count; refused launches never ran)
size_t queue_inflight_locked(aws_crt_amd_queue *q, size_t limit) {
    size_t n = 0;
    for (auto it = q->launches.rbegin(); it != q->launches.rend() && n < limit; ++it) {
        if (it->rc || !it->ev) continue;
        const hipError_t e = hipEventQuery(it->ev);
        if (e == hipSuccess) break;
        (void)hipGetLastError();
        if (e != hipErrorNotReady) break;  // a failed stream: nothing of it is running any more
        ++n;
    }
    return n;
}

// The age bound: launch what is queued once the oldest push is max_age_us old
void queue_flusher(aws_crt_amd_queue *q) noexcept {
    (void)hipSetDevice(q->device);
    std::unique_lock<std::mutex> g(q->mu);
    while (!q->stop) {
        if (q->pending.empty()) {
            q->cv.wait(g);
            continue;
        }
        const auto due = q->oldest + std::chrono::microseconds(q->max_age_us);
        if (std::chrono::steady_clock::now() >= due) {
            (void)guarded(err_sink, [&]() -> int { return queue_flush_locked(q); });
        } else {
            q->cv.wait_until(g, due);
        }
    }
}

int queue_status_locked(aws_crt_amd_queue *q, uint64_t ticket, hipEvent_t *ev) {
    *ev = nullptr;
    if (ticket == 0 || ticket >= q->next_ticket) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "queue: no such ticket");
    if (ticket >= q->next_ticket - q->pending.size()) return AWS_CRT_AMD_TICKET_QUEUED;
    for (auto it = q->launches.rbegin(); it != q->launches.rend(); ++it) {
        if (ticket < it->first || ticket >= it->end) continue;
        if (it->rc) return it->rc;
        const hipError_t e = hipEventQuery(it->ev);
        if (e == hipSuccess) return 0;
        (void)hipGetLastError();
        *ev = it->ev;
        return e == hipErrorNotReady ? AWS_CRT_AMD_TICKET_LAUNCHED : AWS_CRT_AMD_ERR_HIP;
    }
    for (const auto &L : q->failed)
        if (ticket >= L.first && ticket < L.end) return L.rc;
    if (ticket < q->expired_below) return AWS_CRT_AMD_ERR_TICKET_EXPIRED;  // outcome no longer recorded
    return 0;  // pruned: completed (a launch is pruned only once complete or refused)
}
}  // namespace

AWS_CRT_AMD_API int aws_crt_amd_queue_create_ex(int alg, size_t stride, size_t len, size_t count, void *hip_stream,
                                                const struct aws_crt_amd_queue_options *opt, aws_crt_amd_queue **out) {
    return guarded(err_sink, [&]() -> int {
        if (!out) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null queue pointer");
        *out = nullptr;
        if (alg < 0 || alg > 5) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "bad algorithm");
        if (count > 1 && stride % 16 != 0 && !is_hash(alg))
            return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "strided batch needs stride % 16 == 0 (use the list API)");
        if (opt && opt->max_batches > (size_t)kMaxBatches)
            return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "queue: max_batches above 32");
        if (opt && opt->policy != AWS_CRT_AMD_QUEUE_EAGER && opt->policy != AWS_CRT_AMD_QUEUE_BATCHED)
            return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "queue: unknown policy");
        if (opt && opt->max_inflight > 8) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "queue: max_inflight above 8");
        if (opt && (opt->min_launch > (uint32_t)kMaxBatches || opt->reserved))
            return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "queue: min_launch above 32 or reserved field set");
        std::unique_ptr<aws_crt_amd_queue> q(new aws_crt_amd_queue);
        q->alg = alg, q->stride = stride, q->len = len, q->count = count, q->stream = hip_stream;
        if (opt && opt->max_batches) q->max_batches = opt->max_batches;
        if (opt) q->max_age_us = opt->max_age_us;
        if (opt) q->eager = opt->policy == AWS_CRT_AMD_QUEUE_EAGER;
        if (opt && opt->max_inflight) q->max_inflight = opt->max_inflight;
        if (opt && opt->min_launch) q->min_launch = opt->min_launch;
        if (hipGetDevice(&q->device) != hipSuccess) {
            (void)hipGetLastError();
            q->device = 0;
        }
        q->pending.reserve(kMaxBatches);
        if (q->max_age_us) q->flusher = std::thread(queue_flusher, q.get());
        *out = q.release();
        return 0;
    });
}

AWS_CRT_AMD_API int aws_crt_amd_queue_create(int alg, size_t stride, size_t len, size_t count, void *hip_stream,
                                             aws_crt_amd_queue **out) {
    return aws_crt_amd_queue_create_ex(alg, stride, len, count, hip_stream, nullptr, out);
}

AWS_CRT_AMD_API int aws_crt_amd_queue_push_ex(aws_crt_amd_queue *q, const void *d_base, const void *d_seeds, void *d_out,
                                              uint64_t *ticket) {
    return guarded(err_sink, [&]() -> int {
        if (ticket) *ticket = 0;
        if (!q) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null queue");
        if (!d_out || (q->len && !d_base)) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null buffer");
        std::lock_guard<std::mutex> g(q->mu);
        if (q->pending.empty()) {
            q->oldest = std::chrono::steady_clock::now();
            if (q->max_age_us) q->cv.notify_one();
        }
        q->pending.push_back({d_base, d_seeds, d_out});
        if (ticket) *ticket = q->next_ticket;
        ++q->next_ticket;
        if (q->pending.size() >= q->max_batches) return queue_flush_locked(q);
        // eager: the stream has room (none, or fewer than max_inflight, of the queue's launches running)
        if (q->eager && q->pending.size() >= q->min_launch && queue_inflight_locked(q, q->max_inflight) < q->max_inflight)
            return queue_flush_locked(q);
        return 0;
    });
}

AWS_CRT_AMD_API int aws_crt_amd_queue_push(aws_crt_amd_queue *q, const void *d_base, const void *d_seeds, void *d_out) {
    return aws_crt_amd_queue_push_ex(q, d_base, d_seeds, d_out, nullptr);
}

AWS_CRT_AMD_API int aws_crt_amd_queue_flush(aws_crt_amd_queue *q) {
    return guarded(err_sink, [&]() -> int {
        if (!q) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null queue");
        std::lock_guard<std::mutex> g(q->mu);
        return queue_flush_locked(q);
    });
}

AWS_CRT_AMD_API size_t aws_crt_amd_queue_pending(const aws_crt_amd_queue *q) {
    if (!q) return 0;
    std::lock_guard<std::mutex> g(const_cast<aws_crt_amd_queue *>(q)->mu);
    return q->pending.size();
}

AWS_CRT_AMD_API uint64_t aws_crt_amd_queue_launches(const aws_crt_amd_queue *q) {
    if (!q) return 0;
    std::lock_guard<std::mutex> g(const_cast<aws_crt_amd_queue *>(q)->mu);
    return q->nlaunches;
}

AWS_CRT_AMD_API uint64_t aws_crt_amd_queue_first_pending(const aws_crt_amd_queue *q) {
    if (!q) return 0;
    std::lock_guard<std::mutex> g(const_cast<aws_crt_amd_queue *>(q)->mu);
    return q->next_ticket - q->pending.size();
}

AWS_CRT_AMD_API int aws_crt_amd_queue_status(aws_crt_amd_queue *q, uint64_t ticket) {
    return guarded(err_sink, [&]() -> int {
        if (!q) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null queue");
        std::lock_guard<std::mutex> g(q->mu);
        hipEvent_t ev;
        return queue_status_locked(q, ticket, &ev);
    });
}

AWS_CRT_AMD_API int aws_crt_amd_queue_wait(aws_crt_amd_queue *q, uint64_t ticket) {
    return guarded(err_sink, [&]() -> int {
        if (!q) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null queue");
        hipEvent_t ev;
        {
            std::lock_guard<std::mutex> g(q->mu);
            int st = queue_status_locked(q, ticket, &ev);
            if (st == AWS_CRT_AMD_TICKET_QUEUED) {
                const int rc = queue_flush_locked(q);
                if (rc) return rc;
                st = queue_status_locked(q, ticket, &ev);
            }
            if (st != AWS_CRT_AMD_TICKET_LAUNCHED) return st;
        }
        // the event is never destroyed while the queue lives (pruned events are kept as spares, and a
        // spare is re-recorded only after its launch completed -- waiting on it then returns at once)
        HIP_TRY(hipEventSynchronize(ev));
        std::lock_guard<std::mutex> g(q->mu);
        hipEvent_t ev2;
        const int st = queue_status_locked(q, ticket, &ev2);
        return st == AWS_CRT_AMD_TICKET_LAUNCHED ? 0 : st;
    });
}

AWS_CRT_AMD_API int aws_crt_amd_queue_destroy(aws_crt_amd_queue *q) {
    if (!q) return 0;
    int rc;
    {
        std::lock_guard<std::mutex> g(q->mu);
        q->stop = true;
        q->cv.notify_all();
    }
    if (q->flusher.joinable()) q->flusher.join();
    {
        std::lock_guard<std::mutex> g(q->mu);
        rc = guarded(err_sink, [&]() -> int { return queue_flush_locked(q); });
        // the events may be destroyed while their launches run (HIP releases them after completion)
        for (auto &L : q->launches)
            if (L.ev) (void)hipEventDestroy(L.ev);
        for (hipEvent_t e : q->spare) (void)hipEventDestroy(e);
    }
    delete q;
    return rc;
}

AWS_CRT_AMD_API int aws_crt_amd_checksum_list(int alg, const void *const *d_ptrs, const size_t *lens, size_t count,
                                              const void *d_seeds, void *d_out, void *hip_stream) {
    return guarded(err_sink, [&]() -> int {
        if (alg < 0 || alg > 5) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "bad algorithm");
        Device *d;
        int rc = get_device(&d);
        if (rc) return rc;
        return list_impl(d, alg, d_ptrs, lens, count, d_seeds, d_out, (hipStream_t)hip_stream);
    });
}

AWS_CRT_AMD_API int aws_crt_amd_eventstream_crcs(const void *base, uint64_t limit, const uint64_t *d_offsets, size_t count,
                                                 uint32_t *d_prelude_crc, uint32_t *d_message_crc, uint32_t *d_status,
                                                 void *hip_stream) {
    return guarded(err_sink, [&]() -> int {
        if (count == 0) return 0;
        if (!base || !d_offsets || !d_prelude_crc || !d_message_crc || !d_status)
            return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null argument");
        Device *d;
        int rc = get_device(&d);
        if (rc) return rc;
        const uint32_t *imgs = nullptr;
        {
            std::lock_guard<std::mutex> g(d->mu);
            if (!d->es_imgs.p && capturing((hipStream_t)hip_stream))
                return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "event-stream images must be warmed up before stream capture");
            rc = get_es_images(d, &imgs);
        }
        if (rc) return rc;
        EventStreamParams ep{(const uint8_t *)base, d_offsets, count, limit, d_prelude_crc, d_message_crc, d_status, imgs};
        int e = amdcrc_launch_eventstream(&ep, hip_stream, g_time_events);
        g_time_events[0] = g_time_events[1] = nullptr;
        return e ? fail(AWS_CRT_AMD_ERR_HIP, std::string("event-stream kernel launch: ") + hipGetErrorString((hipError_t)e)) : 0;
    });
}

AWS_CRT_AMD_API int aws_crt_amd_checksum_host(int alg, const void *const *h_ptrs, const size_t *lens, size_t count,
                                              const void *h_seeds, void *h_out) {
    return guarded(err_sink, [&]() -> int {
        if (alg < 0 || alg > 5) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "bad algorithm");
        if (count && (!h_ptrs || !lens || !h_out)) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null argument");
        const bool seed64 = alg != AWS_CRT_AMD_CRC32 && alg != AWS_CRT_AMD_CRC32C;
        const bool gpu = aws_crt_amd_get_dispatch() == AWS_CRT_AMD_DISPATCH_GPU;
        for (size_t i = 0; i < count; ++i) {
            uint64_t seed = 0;
            if (h_seeds) seed = seed64 ? ((const uint64_t *)h_seeds)[i] : ((const uint32_t *)h_seeds)[i];
            uint64_t r[2] = {0, 0};
            if (!gpu || single_impl(alg, h_ptrs[i], lens[i], seed, r) != 0) {
                const uint8_t *p = (const uint8_t *)h_ptrs[i];
                (void)aws_crt_amd_cpu_batch(alg, (const void *const *)&p, &lens[i], 1, &seed, r, 1);
            }
            if (alg == AWS_CRT_AMD_XXH3_128) {
                ((uint64_t *)h_out)[2 * i] = r[0];
                ((uint64_t *)h_out)[2 * i + 1] = r[1];
            } else if (seed64) {
                ((uint64_t *)h_out)[i] = r[0];
            } else {
                ((uint32_t *)h_out)[i] = (uint32_t)r[0];
            }
        }
        return 0;
    });
}

AWS_CRT_AMD_API int aws_crt_amd_crc_combine_batch(int alg, const void *d_crc1, const void *d_crc2, const uint64_t *len2,
                                                  size_t count, void *d_out, void *hip_stream) {
    return guarded(err_sink, [&]() -> int {
        if (alg < 0 || alg > 2) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "combine needs a CRC algorithm");
        if (count == 0) return 0;
        if (!d_crc1 || !d_crc2 || !len2 || !d_out) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "null argument");
        Device *d;
        int rc = get_device(&d);
        if (rc) return rc;
        hipStream_t s = (hipStream_t)hip_stream;
        std::lock_guard<std::mutex> g(d->mu);
        t_used = nullptr;
        // staging: [x^(8*2^i), i < 64][len2[count]]
        uint64_t *h;
        const size_t words = 64 + count;
        if ((rc = stage_begin(d, s, words * 8, (void **)&h))) return rc;
        const uint64_t poly = alg_poly(alg);
        const int w = width_of(alg);
        uint64_t sq = (1ull << (w - 1)) >> 8;
        for (int i = 0; i < 64; ++i) {
            h[i] = sq;
            sq = gf2_mulmod(sq, sq, poly, w);
        }
        std::memcpy(h + 64, len2, count * 8);
        const uint64_t *dd;
        if ((rc = stage_end(d, s, words * 8, (const void **)&dd))) return rc;
        CombineParams cp{d_crc1, d_crc2, dd + 64, count, d_out, dd};
        int e = amdcrc_launch_combine(alg, &cp, s);
        if (e) {
            t_used = nullptr;
            return fail(AWS_CRT_AMD_ERR_HIP, "combine launch failed");
        }
        fence_after(s);
        return 0;
    });
}

// The S3 wire form of a digest: standard base64 with padding (RFC 4648 §4), what the CRT's
// Aws::Crt::Base64Encode (reference include/aws/crt/Types.h:70-75) gives for it.  The engine sits at
// the aws-checksums level and does not call up into the C++ surface.
static std::string wire_base64(const uint8_t *p, size_t n) {
    static const char A[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    std::string out;
    for (size_t i = 0; i < n; i += 3) {
        const uint32_t v = (uint32_t)p[i] << 16 | (i + 1 < n ? (uint32_t)p[i + 1] << 8 : 0) | (i + 2 < n ? p[i + 2] : 0);
        out += A[v >> 18];
        out += A[(v >> 12) & 63];
        out += i + 1 < n ? A[(v >> 6) & 63] : '=';
        out += i + 2 < n ? A[v & 63] : '=';
    }
    return out;
}

// S3 multipart composition (checksums_batch.h): one batched scan over the parts, then the
// Combine fold of the part values (4/8-byte scalars, no payload) into the full-object checksum.
AWS_CRT_AMD_API int aws_crt_amd_multipart_crc(int alg, const void *const *d_parts, const size_t *lens, size_t count,
                                              void *h_part_out, void *h_object_out, char *b64_out, void *hip_stream) {
    return guarded(err_sink, [&]() -> int {
        if (alg < AWS_CRT_AMD_CRC32 || alg > AWS_CRT_AMD_CRC64NVME || !h_object_out || (count && (!d_parts || !lens)))
            return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "multipart: CRC32/CRC32C/CRC64NVME, parts and an object result");
        Device *d;
        int rc = get_device(&d);
        if (rc) return rc;
        const int w = width_of(alg);
        const uint64_t poly = alg_poly(alg);
        std::vector<uint64_t> part(count, 0);
        if (count) {
            const size_t osz = w / 8;
            hipStream_t s = (hipStream_t)hip_stream;
            void *d_out;
            std::unique_lock<std::mutex> call;
            for (;;) {
                StreamState *ss;
                {
                    std::lock_guard<std::mutex> g(d->mu);
                    ss = d->states.get(s);
                }
                // per stream, taken before d->mu (list_impl takes d->mu); a held state is never handed
                // to another stream (StatePolicy::idle), so re-check that it is still this stream's
                call = std::unique_lock<std::mutex>(ss->mp_mu);
                std::lock_guard<std::mutex> g(d->mu);
                if (d->states.get(s) == ss) break;
                call.unlock();
            }
            {
                std::lock_guard<std::mutex> g(d->mu);
                DevBuf &ob = d->states.get(s)->mp_out;
                if (ob.bytes < count * osz) {
                    if (ob.p) d->retired.push_back(ob);
                    ob = DevBuf{};
                    HIP_TRY(hipMalloc(&ob.p, count * osz));
                    ob.bytes = count * osz;
                }
                d_out = ob.p;
            }
            rc = list_impl(d, alg, d_parts, lens, count, nullptr, d_out, s);
            std::vector<uint8_t> h(count * osz);
            if (!rc && hipMemcpyAsync(h.data(), d_out, h.size(), hipMemcpyDeviceToHost, s) == hipSuccess &&
                hipStreamSynchronize(s) == hipSuccess) {
                for (size_t i = 0; i < count; ++i)
                    part[i] = w == 64 ? ((const uint64_t *)h.data())[i] : ((const uint32_t *)h.data())[i];
            } else if (!rc) {
                rc = fail(AWS_CRT_AMD_ERR_HIP, "multipart: result copy failed");
            }
            if (rc) return rc;
        }
        uint64_t obj = 0;  // CRC of zero bytes
        for (size_t i = 0; i < count; ++i)
            obj = gf2_mulmod(obj, gf2_xpow8n(lens[i], poly, w), poly, w) ^ part[i];
        for (size_t i = 0; h_part_out && i < count; ++i) {
            if (w == 64)
                ((uint64_t *)h_part_out)[i] = part[i];
            else
                ((uint32_t *)h_part_out)[i] = (uint32_t)part[i];
        }
        if (w == 64)
            *(uint64_t *)h_object_out = obj;
        else
            *(uint32_t *)h_object_out = (uint32_t)obj;
        if (b64_out) {
            uint8_t be[8];
            for (int i = 0; i < w / 8; ++i) be[i] = (uint8_t)(obj >> (w - 8 * (i + 1)));
            const std::string b64 = wire_base64(be, (size_t)(w / 8));
            std::memcpy(b64_out, b64.c_str(), b64.size() + 1);
        }
        return 0;
    });
}

// S3 multipart checksums for every algorithm S3ChecksumAlgorithm names beside the SHAs
// (include/aws/crt/s3/S3.h:69-81, source/s3/S3.cpp:392-424).  Parts are checksummed on the GPU as
// one ragged list (list_impl); then on the host:
//   FULL_OBJECT (CRC32 / CRC32C / CRC64NVME): the object's checksum by Combine, as
//               aws_crt_amd_multipart_crc;
//   COMPOSITE  (every algorithm): the checksum, with the same algorithm, of the concatenated
//               big-endian part digests (4, 8 or 16 bytes each), wire form base64 + "-" + parts.
// The composite rule is S3's "checksum of checksums"; the reference holds no fixture for it, so its
// parity is unpinned (tests check it against the oracle's own digest of the concatenation).
AWS_CRT_AMD_API int aws_crt_amd_multipart_checksum(int alg, int type, const void *const *d_parts, const size_t *lens,
                                                   size_t count, void *h_part_out, void *h_object_out, char *b64_out,
                                                   void *hip_stream) {
    return guarded(err_sink, [&]() -> int {
        if (alg < 0 || alg > 5 || (type != AWS_CRT_AMD_MULTIPART_FULL_OBJECT && type != AWS_CRT_AMD_MULTIPART_COMPOSITE))
            return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "multipart: bad algorithm or type");
        if (type == AWS_CRT_AMD_MULTIPART_FULL_OBJECT) {
            if (is_hash(alg)) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "multipart: FULL_OBJECT composes CRCs only");
            return aws_crt_amd_multipart_crc(alg, d_parts, lens, count, h_part_out, h_object_out, b64_out, hip_stream);
        }
        if (!h_object_out || (count && (!d_parts || !lens))) return fail(AWS_CRT_AMD_ERR_INVALID_ARG, "multipart: parts and an object result");
        Device *d;
        int rc = get_device(&d);
        if (rc) return rc;
        // digest bytes per part, and the device result words per part
        const size_t dsz = alg == AWS_CRT_AMD_XXH3_128 ? 16 : (alg == AWS_CRT_AMD_CRC32 || alg == AWS_CRT_AMD_CRC32C) ? 4 : 8;
        std::vector<uint8_t> h(count * dsz);
        if (count) {
            hipStream_t s = (hipStream_t)hip_stream;
            void *d_out = nullptr;
            HIP_TRY(hipMallocAsync(&d_out, count * dsz, s));
            rc = list_impl(d, alg, d_parts, lens, count, nullptr, d_out, s);
            hipError_t e = rc ? hipSuccess : hipMemcpyAsync(h.data(), d_out, h.size(), hipMemcpyDeviceToHost, s);
            const hipError_t f = hipFreeAsync(d_out, s);
            if (!e) e = hipStreamSynchronize(s);
            if (rc) return rc;
            if (e || f) return fail(AWS_CRT_AMD_ERR_HIP, "multipart: result copy failed");
        }
        // the part digests as values, then big-endian bytes (XXH3-128: high word, then low word)
        std::vector<uint8_t> cat(count * dsz);
        for (size_t i = 0; i < count; ++i) {
            uint64_t v[2] = {0, 0};
            if (dsz == 4) v[0] = ((const uint32_t *)h.data())[i];
            else if (dsz == 8) v[0] = ((const uint64_t *)h.data())[i];
            else v[0] = ((const uint64_t *)h.data())[2 * i], v[1] = ((const uint64_t *)h.data())[2 * i + 1];
            for (size_t b = 0; b < dsz; ++b) {
                const size_t word = b / 8, sh = dsz == 4 ? 8 * (3 - b) : 8 * (7 - (b & 7));
                cat[i * dsz + b] = (uint8_t)(v[word] >> sh);
            }
            if (h_part_out) std::memcpy((uint8_t *)h_part_out + i * dsz, dsz == 4 ? (const void *)((const uint32_t *)h.data() + i)
                                                                               : (const void *)(h.data() + i * dsz), dsz);
        }
        uint64_t obj[2] = {0, 0};
        switch (alg) {
            case AWS_CRT_AMD_CRC32: obj[0] = cpu::crc32(cat.data(), cat.size(), 0); break;
            case AWS_CRT_AMD_CRC32C: obj[0] = cpu::crc32c(cat.data(), cat.size(), 0); break;
            case AWS_CRT_AMD_CRC64NVME: obj[0] = cpu::crc64nvme(cat.data(), cat.size(), 0); break;
            case AWS_CRT_AMD_XXH64: obj[0] = cpu::xxh64(cat.data(), cat.size(), 0); break;
            case AWS_CRT_AMD_XXH3_64: obj[0] = cpu::xxh3_64(cat.data(), cat.size(), 0); break;
            default: cpu::xxh3_128(cat.data(), cat.size(), 0, obj); break;
        }
        if (dsz == 4) *(uint32_t *)h_object_out = (uint32_t)obj[0];
        else std::memcpy(h_object_out, obj, dsz);
        if (b64_out) {
            uint8_t be[16];
            for (size_t b = 0; b < dsz; ++b) be[b] = (uint8_t)(obj[b / 8] >> (dsz == 4 ? 8 * (3 - b) : 8 * (7 - (b & 7))));
            const std::string wire = wire_base64(be, dsz) + "-" + std::to_string(count);
            std::memcpy(b64_out, wire.c_str(), wire.size() + 1);
        }
        return 0;
    });
}

}  // extern "C"
