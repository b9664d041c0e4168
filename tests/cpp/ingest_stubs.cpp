// Host-only sanitizer build of the host-ingest jobs (ingest_host_test.cpp): the device engine's batch
// entry points report "no device"; the jobs under test run on the host path (ndevices < 0) and never
// reach them.
#include <aws_crt_amd/checksums_batch.h>

extern "C" AWS_CRT_AMD_API int aws_crt_amd_checksum_strided(int, const void *, size_t, size_t, size_t, const void *, void *, void *)
{
    return AWS_CRT_AMD_ERR_NO_DEVICE;
}
extern "C" AWS_CRT_AMD_API int aws_crt_amd_checksum_list(int, const void *const *, const size_t *, size_t, const void *, void *, void *)
{
    return AWS_CRT_AMD_ERR_NO_DEVICE;
}
