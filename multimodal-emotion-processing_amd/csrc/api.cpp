// Error plumbing and ABI metadata of libmep_hip.so.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/mep.h"

namespace {
thread_local std::string g_last_error;

}

extern "C" void mep_set_error(const char* msg) { g_last_error = msg ? msg : ""; }

int mep_check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) return 0;
    char buf[256];
    std::snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
    g_last_error = buf;
    return -(int)e;
}

extern "C" int mep_abi_version(void) { return MEP_ABI_VERSION; }

extern "C" int mep_last_error(char* buf, size_t len) {
    if (!buf || len == 0) return (int)g_last_error.size();
    const size_t n = g_last_error.size() < len - 1 ? g_last_error.size() : len - 1;
    std::memcpy(buf, g_last_error.data(), n);
    buf[n] = 0;
    return (int)n;
}

extern "C" int mep_device_sync(void) {
    const hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) return 0;
    g_last_error = std::string("hipDeviceSynchronize: ") + hipGetErrorString(e);
    return -(int)e;
}

