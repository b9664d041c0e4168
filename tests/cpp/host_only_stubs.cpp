// Host-only sanitizer builds (tests/test_host_sanitizers.py): the whole host side of the engine --
// the C++ surface, the aws-c-common shim, the single-buffer ABI with its dispatch (abi_single.cpp)
// and the host checksum path (csrc/cpu/) -- is compiled straight into the test binary under
// ASan + UBSan or TSan.  The HIP engine is not linked: these stand-ins report "no usable device",
// which is exactly the dispatch the host path takes on a machine without a gfx950 GPU.
#include <stddef.h>
#include <stdint.h>

extern "C" int amdcrc_gpu_usable(void) { return 0; }
extern "C" int amdcrc_is_device_ptr(const void *) { return 0; }
extern "C" int amdcrc_gpu_single(int, const void *, size_t, uint64_t, uint64_t *) { return -1; }
extern "C" int amdcrc_copy_to_host(void *, const void *, size_t) { return -1; }
extern "C" const char *aws_crt_amd_last_error(void) { return "no device (host-only build)"; }
extern "C" int amdcrc_gpu_xxh3_blocks(const void *, uint64_t, uint64_t, uint64_t *) { return -1; }
