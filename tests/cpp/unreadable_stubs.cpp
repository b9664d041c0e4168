// Host-only build with an unreadable "device" buffer (tests/test_host_sanitizers.py
// ::test_unreadable_device_buffer_raises): the engine stand-ins report g_unreadable as device
// memory that neither the GPU path nor a device-to-host read-back can serve -- the path where the
// value-only CRC ABI must raise an aws error instead of returning a plausible CRC silently.
#include <stddef.h>
#include <stdint.h>

extern "C" const uint8_t g_unreadable[256] = {0};

static bool unreadable(const void *p) {
    const uint8_t *q = (const uint8_t *)p;
    return q >= g_unreadable && q < g_unreadable + sizeof(g_unreadable);
}
extern "C" int amdcrc_gpu_usable(void) { return 1; }
extern "C" int amdcrc_is_device_ptr(const void *p) { return unreadable(p) ? 1 : 0; }
extern "C" int amdcrc_gpu_single(int, const void *, size_t, uint64_t, uint64_t *) { return -1; }
extern "C" int amdcrc_copy_to_host(void *, const void *, size_t) { return -1; }
extern "C" const char *aws_crt_amd_last_error(void) { return "injected: device buffer unreadable"; }
extern "C" int amdcrc_gpu_xxh3_blocks(const void *, uint64_t, uint64_t, uint64_t *) { return -1; }
