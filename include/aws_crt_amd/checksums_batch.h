#pragma once
/*
 * MI355X batched checksum engine -- C ABI (the drop-in boundary below Aws::Crt::Checksum).
 *
 * Single-buffer entry points with aws-checksums' names and signatures live in
 * include/aws/checksums/crc.h and include/aws/checksums/xxhash.h.  This header adds the batched,
 * device-resident entry points that the reference has no counterpart for: the
 * reference computes one buffer per call on the calling CPU thread
 * (source/checksum/CRC.cpp:15-43 -> aws_checksums_*_ex).
 *
 * Conventions (identical to the reference per buffer):
 *   CRC32      reflected 0x04C11DB7, init/xorout ~0       (CRC.h:15-20)
 *   CRC32C     reflected 0x1EDC6F41, init/xorout ~0       (CRC.h:22-27)
 *   CRC64NVME  reflected 0xAD93D23594C93659, ~0           (CRC.h:29-36)
 *   XXH64      published xxHash64; raw 64-bit value here  (XXHash.h:21, digest byte order is the
 *              caller's business: the C++ wrapper writes it big-endian)
 *   seed       = the finalised CRC of the preceding bytes ("previousCRC", CRC.h:20,27,36), or the
 *                XXH64 seed.
 *
 * All pointers named d_* are device addresses on the current HIP device.  Results are written
 * to d_out (uint32_t per buffer for CRC32/CRC32C, uint64_t for CRC64NVME/XXH64/XXH3_64, two uint64_t
 * {high, low} for XXH3_128).  Calls are
 * asynchronous on `hip_stream` (a hipStream_t; NULL = the legacy default stream).  Inputs must stay
 * valid until the stream reaches the work.  Every call returns 0 on success or a negative
 * aws_crt_amd_status; aws_crt_amd_last_error() describes the last failure on the calling thread.
 * The device-pointer batch calls need a usable gfx950 device (AWS_CRT_AMD_ERR_NO_DEVICE otherwise);
 * the host-memory calls (aws_checksums_*, aws_xxhash_*, aws_crt_amd_checksum_host,
 * aws_crt_amd_cpu_batch) always complete, on the host path when there is no device.
 */
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(AWS_CRT_AMD_BUILD)
#    define AWS_CRT_AMD_API __attribute__((visibility("default")))
#else
#    define AWS_CRT_AMD_API
#endif

enum aws_crt_amd_algorithm {
    AWS_CRT_AMD_CRC32 = 0,
    AWS_CRT_AMD_CRC32C = 1,
    AWS_CRT_AMD_CRC64NVME = 2,
    AWS_CRT_AMD_XXH64 = 3,
    AWS_CRT_AMD_XXH3_64 = 4,
    AWS_CRT_AMD_XXH3_128 = 5, /* 16 bytes per buffer: high 64 bits, then low 64 bits */
};

enum aws_crt_amd_status {
    AWS_CRT_AMD_OK = 0,
    AWS_CRT_AMD_ERR_NO_DEVICE = -1,
    AWS_CRT_AMD_ERR_INVALID_ARG = -2,
    AWS_CRT_AMD_ERR_HIP = -3,
    AWS_CRT_AMD_ERR_OOM = -4,
    AWS_CRT_AMD_ERR_TICKET_EXPIRED = -5, /* queue_status: the ticket's record is gone (see below) */
};

/*
 * Where the single-buffer ABI (aws_checksums_*_ex, aws_xxhash*_compute) runs host-memory input.
 * Device-resident input always runs on the GPU.  The mode never changes the arithmetic, only the
 * processor: AUTO (default) = host path for host memory; CPU = host path; GPU = host memory is
 * staged through the gfx950 kernels.  A GPU failure falls back to the host path in every mode and
 * is counted by aws_crt_amd_fallback_count().  Initial value from the environment variable
 * AWS_CRT_AMD_DISPATCH=auto|cpu|gpu.
 * Memory kept: in GPU mode an xxHash of a host buffer stages the whole buffer in HBM; the staging
 * buffer is cached per device up to 64 MiB (larger hashes use a temporary allocation), so at most
 * 64 MiB of HBM per device stays allocated for the life of the process.
 */
enum aws_crt_amd_dispatch {
    AWS_CRT_AMD_DISPATCH_AUTO = 0,
    AWS_CRT_AMD_DISPATCH_CPU = 1,
    AWS_CRT_AMD_DISPATCH_GPU = 2,
};
AWS_CRT_AMD_API int aws_crt_amd_set_dispatch(int mode);
AWS_CRT_AMD_API int aws_crt_amd_get_dispatch(void);
AWS_CRT_AMD_API unsigned long long aws_crt_amd_fallback_count(void);
/* The host CRC tier chosen from CPUID: "avx512-vpclmulqdq", "pclmulqdq" or "slice-by-8". */
AWS_CRT_AMD_API const char *aws_crt_amd_cpu_tier(void);

/*
 * Host path over a batch of HOST buffers, `threads` std::threads (buffers round-robin).  out: one
 * uint64_t per buffer (CRC32/32C values zero-extended; XXH3_128: two words, high then low).
 * seeds: uint64_t per buffer or NULL.  Needs no device.
 */
AWS_CRT_AMD_API int aws_crt_amd_cpu_batch(
    int algorithm,
    const void *const *h_ptrs,
    const size_t *lens,
    size_t count,
    const uint64_t *seeds,
    uint64_t *out,
    int threads);

/* Bring up the engine on the current device (idempotent; called implicitly by every entry point). */
AWS_CRT_AMD_API int aws_crt_amd_init(void);
/* Number of visible HIP devices (0 when the runtime has none); never initialises a device. */
AWS_CRT_AMD_API int aws_crt_amd_device_count(void);
AWS_CRT_AMD_API const char *aws_crt_amd_last_error(void);

/*
 * Per-stream state.  Launches on one stream share engine scratch in stream order (cross-tile
 * workspace, descriptor staging, XXH3 block sums, multipart results), so the engine keeps that state
 * per stream.  At most 64 streams per device hold state: a new stream beyond that takes over the
 * state of the least recently used stream whose engine work has completed.  A caller that creates
 * streams per request should release each one (before hipStreamDestroy): its state goes back at once
 * and is reused once its last launch has completed -- release never waits and never frees, so device
 * and pinned memory stay bounded by the streams whose work is in flight.  aws_crt_amd_stream_states
 * reports the current device's live / spare / ever-created states.
 */
AWS_CRT_AMD_API int aws_crt_amd_stream_release(void *hip_stream);
AWS_CRT_AMD_API int aws_crt_amd_stream_states(size_t *live, size_t *spare, size_t *created);

/*
 * Uniform batch: buffer i = [d_base + i*stride, + len), i < count.  stride must be a multiple of
 * 16 (or count == 1).  d_seeds: device array of count seeds (uint32_t for CRC32/32C, uint64_t
 * otherwise) or NULL for seed 0.  This is the shape of BASELINE.json configs 2, 4 and 5.
 */
AWS_CRT_AMD_API int aws_crt_amd_checksum_strided(
    int algorithm,
    const void *d_base,
    size_t stride,
    size_t len,
    size_t count,
    const void *d_seeds,
    void *d_out,
    void *hip_stream);

/*
 * Several uniform batches of the same shape (stride, len, count), each with its own base, seeds and
 * results -- e.g. successive queued part batches.  CRC algorithms: up to 32 batches whose bases share
 * their alignment mod 16 go into ONE launch, so back-to-back batches do not each pay a launch's ramp
 * and tail; xxHash: one launch per batch.  Same per-buffer semantics as
 * aws_crt_amd_checksum_strided.  `batches` is a HOST array.
 */
struct aws_crt_amd_batch {
    const void *d_base;  /* buffer i = [d_base + i*stride, + len) */
    const void *d_seeds; /* count seeds, or NULL for seed 0 */
    void *d_out;         /* count results */
};
AWS_CRT_AMD_API int aws_crt_amd_checksum_batches(
    int algorithm,
    const struct aws_crt_amd_batch *batches,
    size_t nbatches,
    size_t stride,
    size_t len,
    size_t count,
    void *hip_stream);

/*
 * Prepared submission: the planning of aws_crt_amd_checksum_batches (runs of batches, kernel, tile
 * size, launch geometry, constant tables) done once for fixed batches; aws_crt_amd_plan_launch then
 * only launches, on any stream of the plan's device, as often as wanted (a producer that re-submits
 * the same resident buffers, e.g. a ring of part slots).  The batches' memory must stay valid while
 * the plan may be launched.  plan_launches = launches per plan_launch (hashes: one per batch).
 */
struct aws_crt_amd_plan;
AWS_CRT_AMD_API int aws_crt_amd_plan_create(
    int algorithm,
    const struct aws_crt_amd_batch *batches,
    size_t nbatches,
    size_t stride,
    size_t len,
    size_t count,
    struct aws_crt_amd_plan **out_plan);
AWS_CRT_AMD_API int aws_crt_amd_plan_launch(struct aws_crt_amd_plan *plan, void *hip_stream);
AWS_CRT_AMD_API size_t aws_crt_amd_plan_launches(const struct aws_crt_amd_plan *plan);
AWS_CRT_AMD_API void aws_crt_amd_plan_destroy(struct aws_crt_amd_plan *plan);

/*
 * Submission queue: a producer that gets one uniform batch at a time (aws-c-s3 checksumming parts as
 * they arrive, source/s3/S3.cpp:1133-1149) pushes each batch and the engine launches them together.
 * Default (eager) policy, round 6: a push that finds none of the queue's launches still running on its
 * stream launches at once, with every batch queued so far (once at least min_launch, default 2, are
 * queued); batches pushed while a launch runs coalesce
 * and go out with the first push that finds it done, at 32 queued batches, or at
 * aws_crt_amd_queue_flush / _wait / _destroy (or the age bound, below).  So the GPU is never left idle
 * while batches wait, and a busy GPU gets them in ever larger launches (one launch of up to 32, as
 * aws_crt_amd_checksum_batches).  The batched policy (options below) launches only at max_batches, the
 * age bound, flush, wait or destroy.  Work is on the stream only after the launch that holds it: a
 * caller that synchronises the stream, records an event on it or reads a result flushes first.  Every
 * batch of a queue has the queue's algorithm and shape (stride, len, count).  Push, flush, pending,
 * status and wait may be called from several threads; destroy must not overlap any other call on the
 * same queue.  A refused launch (e.g. a HIP error) drops the batches it held: the push or flush that
 * made it returns the error, and every dropped batch's ticket reports it (below).
 */
struct aws_crt_amd_queue;
AWS_CRT_AMD_API int aws_crt_amd_queue_create(
    int algorithm,
    size_t stride,
    size_t len,
    size_t count,
    void *hip_stream,
    struct aws_crt_amd_queue **out_queue);
AWS_CRT_AMD_API int aws_crt_amd_queue_push(struct aws_crt_amd_queue *queue, const void *d_base, const void *d_seeds, void *d_out);
AWS_CRT_AMD_API int aws_crt_amd_queue_flush(struct aws_crt_amd_queue *queue);
/* batches pushed and not yet launched */
AWS_CRT_AMD_API size_t aws_crt_amd_queue_pending(const struct aws_crt_amd_queue *queue);
/* flushes (and stops the age flusher), then frees the queue; returns the flush's status */
AWS_CRT_AMD_API int aws_crt_amd_queue_destroy(struct aws_crt_amd_queue *queue);

/*
 * Queue policy and per-push completion (round 4; policy and max_inflight round 6).
 *   max_batches  launch when this many batches are queued (1..32; 0 = 32)
 *   max_age_us   0 = no age bound; otherwise a flusher thread launches the queued batches once the
 *                oldest has waited this long, so no push waits for later pushes indefinitely
 *   policy       AWS_CRT_AMD_QUEUE_EAGER (0, the default) or AWS_CRT_AMD_QUEUE_BATCHED (1)
 *   max_inflight eager policy: a push launches while fewer than this many of the queue's launches
 *                are running (1..8; 0 = 1)
 *   min_launch   eager policy: a push launches only with at least this many batches queued (1..32;
 *                0 = the default, 2: a lone one-batch launch runs at about half the rate of a
 *                multi-batch one); fewer wait for a later push, flush, wait, destroy or the age bound
 * Each push_ex returns a ticket (1, 2, ... per queue).  queue_status(ticket):
 *   AWS_CRT_AMD_TICKET_QUEUED    pushed, not launched yet
 *   AWS_CRT_AMD_TICKET_LAUNCHED  on the stream, not complete
 *   0                            complete: the batch's results are written
 *   < 0                          the launch that held it was refused (that status): its results are
 *                                never written -- every batch of a refused launch reports it
 *   AWS_CRT_AMD_ERR_TICKET_EXPIRED  the queue no longer knows the ticket's outcome: it lies below the
 *                                oldest of more than 1024 separate refused ranges, whose records were
 *                                dropped (adjacent refused launches share one record).  Never
 *                                reported for a ticket whose outcome is still recorded.
 * queue_wait(ticket) launches the ticket's batch if it is still queued and waits for it; it returns 0
 * or the error.  queue_first_pending: the ticket of the oldest queued batch (every lower ticket has
 * been launched or refused).  Status and wait may be called from any thread.
 */
enum { AWS_CRT_AMD_TICKET_QUEUED = 1, AWS_CRT_AMD_TICKET_LAUNCHED = 2 };
enum { AWS_CRT_AMD_QUEUE_EAGER = 0, AWS_CRT_AMD_QUEUE_BATCHED = 1 };
struct aws_crt_amd_queue_options {
    size_t max_batches;
    uint64_t max_age_us;
    uint32_t policy;
    uint32_t max_inflight;
    uint32_t min_launch;
    uint32_t reserved; /* 0 */
};
AWS_CRT_AMD_API int aws_crt_amd_queue_create_ex(
    int algorithm,
    size_t stride,
    size_t len,
    size_t count,
    void *hip_stream,
    const struct aws_crt_amd_queue_options *options,
    struct aws_crt_amd_queue **out_queue);
AWS_CRT_AMD_API int aws_crt_amd_queue_push_ex(
    struct aws_crt_amd_queue *queue,
    const void *d_base,
    const void *d_seeds,
    void *d_out,
    uint64_t *ticket);
AWS_CRT_AMD_API int aws_crt_amd_queue_status(struct aws_crt_amd_queue *queue, uint64_t ticket);
AWS_CRT_AMD_API int aws_crt_amd_queue_wait(struct aws_crt_amd_queue *queue, uint64_t ticket);
AWS_CRT_AMD_API uint64_t aws_crt_amd_queue_first_pending(const struct aws_crt_amd_queue *queue);
/* launches the queue has made so far (refused ones included) */
AWS_CRT_AMD_API uint64_t aws_crt_amd_queue_launches(const struct aws_crt_amd_queue *queue);

/*
 * Ragged batch: buffer i = [d_ptrs[i], + lens[i]).  d_ptrs and lens are HOST arrays describing
 * device buffers (any alignment, any length including 0).  The engine uploads a compact
 * descriptor (16 B per buffer + tile prefix) per call.  d_seeds as above.
 */
AWS_CRT_AMD_API int aws_crt_amd_checksum_list(
    int algorithm,
    const void *const *d_ptrs,
    const size_t *lens,
    size_t count,
    const void *d_seeds,
    void *d_out,
    void *hip_stream);

/*
 * Event-stream framing check (aws-c-event-stream wire format; SURVEY.md 8(f) rank 4, initialised by
 * the reference at source/Api.cpp:51).  Message i starts at base + d_offsets[i] (d_offsets, and the
 * three outputs, are DEVICE arrays of count entries; base is device memory with `limit` readable
 * bytes).  Its prelude is total_length (u32 BE) | headers_length (u32 BE) | prelude_crc (u32 BE), its
 * last 4 bytes the message CRC (u32 BE) over bytes [0, total_length - 4).  Writes the computed
 * prelude and message CRC32s and d_status[i]: bit 0 = stored prelude CRC matches, bit 1 = stored
 * message CRC matches, bit 2 = malformed (total_length < 16 or past `limit`, or headers_length >
 * total_length - 16; nothing beyond the first 16 bytes is read then, and both CRCs are 0).  One lane per message: for many short
 * messages; a message of megabytes is better checked with aws_crt_amd_checksum_strided.
 */
AWS_CRT_AMD_API int aws_crt_amd_eventstream_crcs(
    const void *base,
    uint64_t limit,
    const uint64_t *d_offsets,
    size_t count,
    uint32_t *d_prelude_crc,
    uint32_t *d_message_crc,
    uint32_t *d_status,
    void *hip_stream);

/*
 * Device-side combine of running CRCs (CombineCRC32/32C/64NVME, CRC.h:41-51, over a batch):
 * d_out[i] = d_crc1[i] * x^(8*len2[i]) ^ d_crc2[i].  len2 is a HOST array.  For S3 multipart
 * composition of part CRCs into an object CRC.
 */
AWS_CRT_AMD_API int aws_crt_amd_crc_combine_batch(
    int algorithm,
    const void *d_crc1,
    const void *d_crc2,
    const uint64_t *len2,
    size_t count,
    void *d_out,
    void *hip_stream);

/*
 * Host-memory convenience: checksum `count` host buffers (pageable or pinned), staging them
 * through pinned memory and the GPU; results written to the HOST array h_out.  Synchronous.
 * This is the end-to-end (PCIe-inclusive) path DESIGN.md reports separately.
 */
AWS_CRT_AMD_API int aws_crt_amd_checksum_host(
    int algorithm,
    const void *const *h_ptrs,
    const size_t *lens,
    size_t count,
    const void *h_seeds,
    void *h_out);

/*
 * Host ingest (S3 part buffers, S3BufferTicket.h:20-30 / S3MetaRequest::Write,
 * S3.cpp:1133-1149).  Asynchronous: checksums `count` HOST buffers and writes one result per buffer
 * to the HOST array h_out (u32 CRC32/32C, u64 CRC64NVME/XXH64/XXH3_64, two u64 {high, low}
 * XXH3_128) once aws_crt_amd_job_wait(job) returns 0.  Buffers, seeds and h_out must stay valid
 * until then.  CRCs are split between the host threads of the process's CPU share and `ndevices`
 * GPUs (0 = all visible; by default only when the CPU share is under 12 threads -- on a larger share
 * the host path alone is faster than a PCIe lane plus the threads it displaces): both take runs of
 * pieces from one cursor over the job (work stealing).  Each device runs a three-slot pipeline (H2D on a
 * copy stream overlapping the scans; 32 MiB slots); buffers longer than a piece (8 MiB, or a slot
 * when no host thread takes part) are cut into pieces folded with Combine.  Registered / pinned
 * memory is DMA'd in place; pageable memory goes through pinned mirrors.  xxHash (a serial chain per
 * buffer), and every algorithm when no device is usable, run on the host path.  h_seeds: u32
 * (CRC32/32C) or u64 per buffer, or NULL.
 */
struct aws_crt_amd_job;
AWS_CRT_AMD_API int aws_crt_amd_host_submit(
    int algorithm,
    const void *const *h_ptrs,
    const size_t *lens,
    size_t count,
    const void *h_seeds,
    void *h_out,
    int ndevices,
    struct aws_crt_amd_job **job);
/*
 * aws_crt_amd_host_submit with options.  ndevices: 0 = every visible device (with host_threads -1:
 * only when the CPU share is under 12 threads), n > 0 = the first n, < 0 = none (the host path alone,
 * on the CPU share).  host_threads: -1 = the CPU share less four threads per device lane (the lane's
 * own and the HIP runtime's), 0 = devices only (the PCIe-bound pipeline), n = n host threads beside
 * the lanes.  device_bytes (optional): set by aws_crt_amd_job_wait to the bytes the devices
 * checksummed.  AWS_CRT_AMD_INGEST_TRACE=1 prints one JSON line per job to stderr (claims, when each
 * side ran out of work, the lanes' staging / issue / wait times, the NUMA node).  Host threads of a
 * job >= 16 MiB whose bytes sit on one NUMA node run on that node's CPUs (as do
 * aws_crt_amd_cpu_batch's); AWS_CRT_AMD_NUMA=0 turns that off.
 */
struct aws_crt_amd_ingest_options {
    int ndevices;
    int host_threads;
    uint64_t *device_bytes;
};
AWS_CRT_AMD_API int aws_crt_amd_host_submit_ex(
    int algorithm,
    const void *const *h_ptrs,
    const size_t *lens,
    size_t count,
    const void *h_seeds,
    void *h_out,
    const struct aws_crt_amd_ingest_options *options,
    struct aws_crt_amd_job **job);
/* Wait for a job and release it; returns its status (aws_crt_amd_job_last_error() on failure). */
AWS_CRT_AMD_API int aws_crt_amd_job_wait(struct aws_crt_amd_job *job);
AWS_CRT_AMD_API const char *aws_crt_amd_job_last_error(void);
/* Page-lock (hipHostRegister, portable to every device) / release a host range, e.g. a part-buffer
 * pool, so host jobs DMA from it directly. */
AWS_CRT_AMD_API int aws_crt_amd_register_host(void *p, size_t n);
AWS_CRT_AMD_API int aws_crt_amd_unregister_host(void *p);

/*
 * In-process multi-device fan-out (north_star: batches sharded over the node's GPUs, one HIP stream
 * per GPU, no collective).
 *   aws_crt_amd_checksum_list_devices: device buffers living on any visible devices (HOST arrays
 *     d_ptrs / lens); grouped by owning device, one thread + stream per device, results (and the
 *     optional HOST seeds) in caller order in HOST h_out.  Synchronous.
 *   aws_crt_amd_checksum_devices: one uniform batch per entry, each on its device, all devices at
 *     once (the entry's stream, or one the call creates); returns when every device is done.
 */
AWS_CRT_AMD_API int aws_crt_amd_checksum_list_devices(
    int algorithm,
    const void *const *d_ptrs,
    const size_t *lens,
    size_t count,
    const void *h_seeds,
    void *h_out);
struct aws_crt_amd_device_batch {
    int device;
    const void *d_base; /* buffer i = [d_base + i*stride, + len) on `device` */
    size_t stride, len, count;
    const void *d_seeds; /* on `device`, or NULL */
    void *d_out;         /* on `device` */
    void *hip_stream;    /* a stream of `device`, or NULL */
};
AWS_CRT_AMD_API int aws_crt_amd_checksum_devices(int algorithm, const struct aws_crt_amd_device_batch *batches, size_t n);

/*
 * S3 multipart checksum composition (the aws-c-s3 layer the reference's
 * S3ChecksumConfig selects, S3.cpp:380-428, default CRC64NVME at S3.cpp:31-36).
 *
 * `count` device-resident parts, in object order, are checksummed in one batched scan; the part
 * values are then folded with Combine (CRC.h:41-51) into the FULL_OBJECT checksum, i.e. the CRC of
 * the parts' concatenation.  Algorithms: CRC32, CRC32C, CRC64NVME.
 *   h_part_out    host array of `count` results (u32, or u64 for CRC64NVME); may be null
 *   h_object_out  host u32 / u64: the full-object checksum
 *   b64_out       optional (may be null): its S3 wire form, base64 of the big-endian bytes
 *                 (Types.h:70-75), NUL-terminated; needs 13 bytes of room.
 * Synchronous on hip_stream.  Returns 0 or a negative status.
 */
AWS_CRT_AMD_API int aws_crt_amd_multipart_crc(
    int algorithm,
    const void *const *d_parts,
    const size_t *lens,
    size_t count,
    void *h_part_out,
    void *h_object_out,
    char *b64_out,
    void *hip_stream);

/*
 * S3 multipart checksums for every algorithm of S3ChecksumAlgorithm except the SHAs (ref
 * include/aws/crt/s3/S3.h:69-81, source/s3/S3.cpp:392-424): the parts (device buffers, host arrays
 * of pointers / lengths, object order) are checksummed on the GPU, then
 *   AWS_CRT_AMD_MULTIPART_FULL_OBJECT  CRC32 / CRC32C / CRC64NVME only: as aws_crt_amd_multipart_crc;
 *   AWS_CRT_AMD_MULTIPART_COMPOSITE    any algorithm: the same algorithm over the concatenated
 *                                      big-endian part digests; b64_out = base64 + "-" + part count.
 * h_part_out: count digests as the batch API writes them (uint32 for CRC32/32C, uint64 otherwise,
 * two uint64 -- high, then low -- for XXH3-128); h_object_out: one such digest.  b64_out: at least
 * 48 bytes.  Synchronous on hip_stream.  COMPOSITE parity is unpinned: the reference has no fixture.
 */
enum { AWS_CRT_AMD_MULTIPART_FULL_OBJECT = 0, AWS_CRT_AMD_MULTIPART_COMPOSITE = 1 };
AWS_CRT_AMD_API int aws_crt_amd_multipart_checksum(
    int algorithm,
    int type,
    const void *const *d_parts,
    const size_t *lens,
    size_t count,
    void *h_part_out,
    void *h_object_out,
    char *b64_out,
    void *hip_stream);

#ifdef __cplusplus
}
#endif
