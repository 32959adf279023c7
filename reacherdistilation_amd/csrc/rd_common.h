// Shared host helpers for the C ABI (error strings, HIP error mapping).
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

namespace rd {

inline char* last_error_buf() {
    static thread_local char buf[512] = "";
    return buf;
}

inline int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(last_error_buf(), 512, fmt, ap);
    va_end(ap);
    return code;
}

inline int hip_fail(hipError_t e, const char* what) {
    return set_error(-(int)e, "%s: %s", what, hipGetErrorString(e));
}

// Make `device` current for the duration of an API call.
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int device) {
        err = hipGetDevice(&prev);
        if (err == hipSuccess && prev != device) err = hipSetDevice(device);
    }
    ~DeviceGuard() {
        int cur;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

}  // namespace rd

#define RD_HIP(call, what)                                \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return rd::hip_fail(e_, what); \
    } while (0)
