// Host-only sanitizer build of the C++ surface (tests/test_host_sanitizers.py): the Types / Api /
// aws-c-common shim sources are compiled straight into the test binary under ASan + UBSan, without
// the HIP engine.  Api.cpp's ApiHandle calls the engine's library init / clean-up; these two no-ops
// stand in for them here only -- no checksum is computed in this binary.
#include <aws/checksums/crc.h>

extern "C" void aws_checksums_library_init(struct aws_allocator *) {}
extern "C" void aws_checksums_library_clean_up(void) {}
