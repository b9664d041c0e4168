// Host-only build of the streaming XXH3 device path (tests/test_host_sanitizers.py
// ::test_device_stream_xxh3_split_logic): the engine stand-ins report g_fake_dev as device memory
// that a read-back can reach (memcpy), and amdcrc_gpu_xxh3_blocks -- the GPU block absorb -- is
// modelled by the host path with the same contract (whole 1 KiB blocks into the stream's
// accumulators), or fails when g_fail_blocks is set, so both the device path's host-side split
// logic (abi_single.cpp, cpu::xxh3_update_source) and its fallback run under ASan + UBSan.
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "../../aws-crt-cpp_amd/csrc/cpu/cpu_checksums.h"

extern "C" {
uint8_t g_fake_dev[(4u << 20) + 4096];
int g_fail_blocks = 0;
unsigned long long g_blocks_calls = 0, g_blocks_absorbed = 0;
}

static bool on_dev(const void *p, size_t n) {
    const uint8_t *q = (const uint8_t *)p;
    return q >= g_fake_dev && q + n <= g_fake_dev + sizeof(g_fake_dev);
}
extern "C" int amdcrc_gpu_usable(void) { return 1; }
extern "C" int amdcrc_is_device_ptr(const void *p) { return on_dev(p, 1) ? 1 : 0; }
extern "C" int amdcrc_gpu_single(int, const void *, size_t, uint64_t, uint64_t *) { return -1; }
extern "C" int amdcrc_copy_to_host(void *dst, const void *src, size_t n) {
    if (!on_dev(src, n)) return -1;
    memcpy(dst, src, n);
    return 0;
}
extern "C" int amdcrc_gpu_xxh3_blocks(const void *d_ptr, uint64_t nblocks, uint64_t seed, uint64_t acc[8]) {
    if (g_fail_blocks || !on_dev(d_ptr, 1024 * nblocks)) return -1;
    amdcrc::cpu::Xxh3State s;
    amdcrc::cpu::xxh3_reset(&s, seed);
    memcpy(s.acc, acc, 64);
    amdcrc::cpu::xxh3_consume(&s, (const uint8_t *)d_ptr, (size_t)(16 * nblocks));
    memcpy(acc, s.acc, 64);
    ++g_blocks_calls;
    g_blocks_absorbed += nblocks;
    return 0;
}
extern "C" const char *aws_crt_amd_last_error(void) { return "host-only build"; }
