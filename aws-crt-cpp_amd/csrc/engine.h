// Internal structures shared by the HIP kernels (crc_kernels.hip) and the host engine (engine.cpp).
// Not part of the public C ABI (that is include/aws_crt_amd/checksums_batch.h).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "variant_guard.h"

namespace amdcrc {

// Work decomposition (DESIGN.md "Data layout"): every buffer is split into
//   head  [ptr, H)      H = ptr rounded up to 16      -- bytewise, folded into the first word
//   main  [H, E)        E = end rounded down to 16    -- the bulk, 16-byte vector loads
//   tail  [E, end)                                     -- bytewise after the main partial
// main is front-padded (virtually, with zeros: free for a raw CRC) to T*TILE bytes and cut into T
// tiles of TILE = 64 lanes * seg bytes.  One wavefront scans one tile; lane l scans the
// contiguous segment [l*seg, (l+1)*seg) of it.
constexpr int kWave = 64;
constexpr int kBlock = 1024;  // 16 waves: one workgroup per CU (the tables take 128 KiB of LDS)
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kGroupBytes = 64;  // bytes per lane per prefetch group (4 x 16-byte loads)
constexpr int kVecPerGroup = kGroupBytes / 16;

// crc64_stream4_kernel workgroup size, two per CU.  One 1024-thread workgroup per CU measured a 3 %
// shorter isolated C5 launch (95.8 vs 98.8 us) but 4-7 % less C5 throughput over three streams
// (launches of other streams no longer co-reside): 512.
#ifndef AMDCRC_W64_BLOCK  // compile-time only (geometry experiments)
#define AMDCRC_W64_BLOCK 512
#endif
constexpr int kW64StreamBlock = AMDCRC_W64_BLOCK;
// crc64_xcd_kernel: 4 KiB groups per chunk (a wave's contiguous piece of an XCD window)
#ifndef AMDCRC_XCD_CHUNK_GROUPS  // compile-time only (A/B builds)
#define AMDCRC_XCD_CHUNK_GROUPS 4
#endif
constexpr uint64_t kXcdChunkBytes = (uint64_t)AMDCRC_XCD_CHUNK_GROUPS * 4096;
#ifndef AMDCRC_XCD_BLOCK  // compile-time only (A/B builds): crc64_xcd_kernel workgroup size: 512 or 640 (two per CU) or 1024
#define AMDCRC_XCD_BLOCK 512
#endif
constexpr int kXcdBlock = AMDCRC_XCD_BLOCK;
#ifndef AMDCRC_XCD_BPC  // compile-time only (A/B builds): crc64_xcd_kernel workgroups per CU
#define AMDCRC_XCD_BPC (AMDCRC_XCD_BLOCK > 640 ? 1 : 2)
#endif
#ifndef AMDCRC_XCD_WPE  // compile-time only (A/B builds): crc64_xcd_kernel launch bound, waves per SIMD
#define AMDCRC_XCD_WPE 4
#endif
constexpr int kXcdBpc = AMDCRC_XCD_BPC;
constexpr int kMaxBatches = 32;  // batches per strided launch (kernel arguments, 768 bytes)
constexpr uint64_t kStreamLocalSlots = 128;  // crc32_stream_kernel: LDS slots for a workgroup's whole buffers

// The 16-byte-word CRC32 streaming scan (crc_kernels.hip Braid32W16: slice-by-16 rows, one
// global_load_dwordx4 per lane per row, one 1024-thread workgroup per CU) for launches of >= 256 MiB.
// Parity-green, but measured slower than the 8-byte-word scan on every shape, so
// the release build neither dispatches nor instantiates it; -DAMDCRC_STREAM_W16=1 builds it back.
#ifndef AMDCRC_STREAM_W16  // compile-time only (A/B builds)
#define AMDCRC_STREAM_W16 0
#endif

struct ScanParams {
    // ---- batch description: strided (base != 0) or list (d_ptrs != 0)
    uint64_t base;                 // strided: device address of buffer 0
    uint64_t stride;               // strided: bytes between buffer starts
    uint64_t len;                  // strided: uniform length
    uint64_t tiles_per_buf;        // strided: T (uniform)
    const uint64_t *d_ptrs;        // list: device addresses
    const uint64_t *d_lens;        // list: lengths
    const uint64_t *d_tile_prefix; // list: exclusive prefix of T_b (nbuf + 1 entries)
    const uint64_t *d_wave_buf;    // list: buffer index holding each wave's first tile (stream 4: each
                                   // wave's first buffer, nw + 1 entries; d_tile_prefix then holds its
                                   // first group in that buffer, nw + 1, and the group prefix, nw + 1)
    uint64_t nbuf;
    uint64_t ntiles;
    // ---- seeds (previous CRC, finalised) and results
    const void *d_seeds;           // u32/u64 per buffer, or null -> seed_all
    uint64_t seed_all;
    void *d_out;                   // u32/u64 per buffer
    // ---- geometry and constants
    uint32_t seg;                  // bytes per lane per tile (multiple of kGroupBytes)
    uint32_t list_mode;            // 1: d_ptrs/d_lens/d_tile_prefix/d_wave_buf describe the batch
    uint32_t stream;               // strided batch with main % TILE == 0: the streaming scan (crc32_stream_kernel /
                                   // crc64_stream4_kernel); W=32: 1 = 8-byte lane words (512-thread workgroups),
                                   // 2 = 16-byte lane words (one 1024-thread workgroup per CU); 3 = CRC64NVME
                                   // rows of 16 lanes (crc64_rows16_kernel); lists: 4 = crc32_list_stream_kernel;
                                   // 5 = CRC64NVME XCD-window chunks (crc64_xcd_kernel: tiles_per_buf = chunks
                                   // per buffer, ntiles = chunks, d_pcols = engine.cpp get_xcd_consts)
    const uint64_t *d_kvals;       // 64 x K_l = x^(8*seg*(63-l)) mod P
    const uint64_t *d_pcols;       // [tmax][W]: column j of x^(8*TILE*k) = x^(8*TILE*k) * x^j
    uint64_t pcols_tmax;
    // ---- cross-tile combine workspace (zero on entry, left zero on exit)
    unsigned long long *d_acc;     // per buffer
    unsigned int *d_cnt;           // per buffer (used when T > 32 or W = 64)
    unsigned long long *d_acc1;    // braided scans: per tile (slot of each 32-tile group)
    unsigned int *d_cnt1;          // W=64 braided scan: per tile (arrivals of each 32-tile group)
    // ---- strided launches over several batches (aws_crt_amd_checksum_batches): buffer b is buffer
    // i = b % bcount of batch j = b / bcount, at bbase[j] + i * stride, seed bseed[j][i] (bseed[j] == 0:
    // seed_all), result bout[j][i].  A plain strided launch is nbatch = 1.  All bases share their
    // alignment mod 16 (the host splits the launch otherwise).
    uint32_t nbatch;
    uint32_t xcd_pad;               // crc64_xcd_kernel: virtual zero bytes in front of every main region (< chunk)
    uint64_t bcount;
    uint64_t bbase[kMaxBatches], bout[kMaxBatches], bseed[kMaxBatches];
    // ---- dynamic tile pool (W=32 braided scan, strided batches): tiles [0, nstatic) are split
    // statically over the waves; tiles [nstatic, ntiles) are claimed at run time, per shard of
    // kShardBlocks workgroups, from d_claim[2 * shard] (claims) / [2 * shard + 1] (waves done)
    uint64_t nstatic;               // 0: no dynamic pool (every tile static)
    uint64_t dyn_chunk;             // pool tiles per shard
    unsigned int *d_claim;          // 2 words per shard, zero on entry, left zero on exit
    // ---- crc32_stream_kernel tile order (round 4): 0 = each wave a contiguous range of tiles; 1 = XCD
    // windows: the waves of XCD x (blockIdx mod 8) take tiles j, j + nwx, ... of the x-th eighth, a
    // buffer's T <= WAVES tiles falling to consecutive waves of one workgroup (combined in LDS)
    uint32_t xcd_order;
    uint32_t reserved0;
    // ---- round 5: the division-free prologue of crc32_stream_kernel.  Wave w of the launch's nw
    // waves takes tiles [w q + min(w, r), + q + (w < r)) (split_q = ntiles / nw, split_r = ntiles % nw,
    // set by the host once the grid is known).  tshift1 / bshift1: log2 + 1 of tiles_per_buf / bcount
    // when it is a power of two, else 0 (the kernels then divide), packed as tshift1 | bshift1 << 8.
    uint64_t split_q;
    uint32_t split_r;
    uint32_t shifts1;
};

// W=32 braided scan constants (engine.cpp get_braid_consts), u32 words:
//   [0, 2048)     K-matrix image: columns of K_l = x^(-32 l), [j/4][lane][j%4]
//   [2048, 3072)  T'_k[e] = e * x^(8(k+1) + 8*252): slice-by-4 step that also skips the other
//                 63 lanes' words of a 256-byte row
//   [3072, 3328)  T_0[e] = e * x^8: plain byte step for head / tail bytes
//   [3328, 5376)  K-matrix image of x^(-64 l) (the streaming scan's 8-byte words), same layout
//   [5376, 7424)  K-matrix image of x^(-128 l) (the streaming scan's 16-byte words), same layout
//   [7424, 7936)  columns (u64) of X^(-j), X = x^(8*512), j < 8: the list streaming scan's head-state
//                 entry (crc32_list_stream_kernel)
//   [7936, 9984)  columns (u64) of x^(8*4096*2^i), i < 32: the list streaming scan's part shifts
//   [9984, 14080) columns (u64) of x^(8*4096*m), m < 64: the same shifts in one product (round 4)
//   [14080, 27392) round 5: the same three matrix sets as nibble images (u32), 128 words per matrix,
//                 then [27392, 28416) the images of x^(-8 t), t < 8:
//                 word 16 i + v = the product of nibble i's value v (bits 31-4i .. 28-4i of the
//                 operand) -- a product is then 8 independent scalar loads, one round trip
//                 (crc_kernels.hip mul_nib), against 4 dependent rounds of 8 columns (mul_pcols)
constexpr int kShardBlocks = 8;        // workgroups per dynamic-pool shard (one per XCD under round-robin dispatch)
constexpr int kBraidRow = 256;        // bytes per row: 64 lanes x one 4-byte word
constexpr int kBraidRowsPerGroup = 16; // 4 KiB per wave per prefetch group
constexpr int kBraidConstWords = 28416;
constexpr int kBraidNibXneg8Word = 27392;   // nibble images of x^(-8 t), t < 8 (the list scans' masked edges)
constexpr int kBraidNibXinvWord = 14080;    // nibble images of the X^(-j) matrices, j < 8
constexpr int kBraidNibGshiftWord = 15104;  // nibble images of x^(8*4096*2^i), i < 32
constexpr int kBraidNibGmWord = 19200;      // nibble images of x^(8*4096*m), m < kBraidGmCount
constexpr int kBraidXinvWord = 7424;    // first word of the X^(-j) columns
constexpr int kBraidGshiftWord = 7936;  // first word of the x^(8*4096*2^i) columns
constexpr int kBraidGmWord = 9984;      // first word of the x^(8*4096*m) columns, m < kBraidGmCount
constexpr int kBraidGmCount = 64;
// crc64 constants (engine.cpp get_xcd_consts), u64 units: the column sets, then the nibble images of
// the list scan's three sets (crc_kernels.hip mul_nib64)
constexpr uint64_t kXcdNibXinvU64 = 256 + 40 * 64 + 4 * 256 * 64 + 32 * 64 + 40 * 64 + kBraidGmCount * 64;
constexpr uint64_t kXcdNibGshiftU64 = kXcdNibXinvU64 + 32 * 256;
constexpr uint64_t kXcdNibGmU64 = kXcdNibGshiftU64 + 40 * 256;
constexpr uint64_t kXcdNibXneg8U64 = kXcdNibGmU64 + kBraidGmCount * 256;
constexpr uint64_t kXcdConstU64 = kXcdNibXneg8U64 + 8 * 256;
constexpr int kBraidK64Word = 3328;   // first word of the x^(-64 l) K image
constexpr int kBraidK128Word = 5376;  // first word of the x^(-128 l) K image

struct XxhParams {
    const uint64_t *d_ptrs;  // device addresses (list) or null (strided)
    const uint64_t *d_lens;
    uint64_t base, stride, len;
    uint64_t nbuf;
    const uint64_t *d_seeds;
    uint64_t seed_all;
    uint64_t *d_out;
    uint64_t *d_sums;  // split XXH3 long path: 8 accumulator sums per full 1 KiB block, or null
};

struct CombineParams {
    const void *d_crc1;
    const void *d_crc2;
    const uint64_t *d_len2;
    uint64_t n;
    void *d_out;
    const uint64_t *d_xpow2;  // x^(8 * 2^i) mod P, i < 64
};

// Lane-per-buffer scan (crc_lanes_kernel): a ragged list of short buffers, or (d_ptrs == null) up to
// kMaxBatches strided batches of short uniform buffers -- buffer b of the launch is buffer b % bcount
// of batch b / bcount, at bbase[j] + i * stride, seeds / results per batch as in ScanParams
struct LaneParams {
    const uint64_t *d_ptrs;  // device addresses (list form)
    const uint64_t *d_lens;
    uint64_t nbuf;
    const void *d_seeds;  // u32/u64 per buffer, or null -> seed_all
    uint64_t seed_all;
    void *d_out;  // u32/u64 per buffer
    uint64_t stride, len, bcount;  // strided form
    uint64_t bbase[kMaxBatches], bout[kMaxBatches], bseed[kMaxBatches];
};

// Event-stream framing check (eventstream_kernel)
struct EventStreamParams {
    const uint8_t *base;
    const uint64_t *d_offsets;  // message starts, bytes from base
    uint64_t count, limit;      // limit: bytes readable from base
    uint32_t *d_prelude_crc, *d_message_crc, *d_status;
    const uint32_t *d_imgs;     // eventstream_flat_kernel's nibble images (engine.cpp get_es_images); null: lane kernel
};
// eventstream_flat_kernel's image buffer: x^(64 v 16^d), d < 4, v = 1..15 (image 15 d + v - 1), then
// x^(-8 t), t = 1..7 (image 60 + t - 1); 128 words each (nib_image)
constexpr int kEsImages = 67;

}  // namespace amdcrc

extern "C" {
int amdcrc_launch_eventstream(const amdcrc::EventStreamParams *p, void *stream, void *const *events);
int amdcrc_launch_lanes(int alg, const amdcrc::LaneParams *p, void *stream, void *const *events);
int amdcrc_launch_combine(int alg, const amdcrc::CombineParams *p, void *stream);
int amdcrc_launch_scan(int alg, const amdcrc::ScanParams *p, int nblocks, void *stream, void *const *events);
int amdcrc_launch_xxh64(const amdcrc::XxhParams *p, void *stream, void *const *events);
int amdcrc_launch_xxh3_blocksum(const amdcrc::XxhParams *p, void *stream, void *start_event);
int amdcrc_launch_xxh3(int bits, const amdcrc::XxhParams *p, void *stream, void *const *events);
int amdcrc_launch_xxh3_stream(const void *d_ptr, uint64_t nblocks, uint64_t seed, uint64_t *d_sums, uint64_t *d_acc, void *stream);
int amdcrc_launch_read_ceiling(const void *base, uint64_t bytes, uint32_t *sink, int nblocks, void *stream, void *const *events);
}
