// Exceptions never cross the C ABI.  Host-side containers and std::thread can throw (std::bad_alloc,
// std::system_error); every exported entry that uses them runs its body under guarded(), which turns
// them into the ABI's error codes and records a message through `sink` (itself non-throwing).
#pragma once

#include <exception>
#include <new>

#include <aws_crt_amd/checksums_batch.h>

namespace amdcrc {

template <class Sink, class F>
int guarded(Sink &&sink, F &&body) noexcept {
    try {
        return body();
    } catch (const std::bad_alloc &) {
        sink("out of host memory");
        return AWS_CRT_AMD_ERR_OOM;
    } catch (const std::exception &e) {
        sink(e.what());
        return AWS_CRT_AMD_ERR_HIP;
    } catch (...) {
        sink("internal error");
        return AWS_CRT_AMD_ERR_HIP;
    }
}

}  // namespace amdcrc
