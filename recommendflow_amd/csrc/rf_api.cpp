// rf_api.cpp — error state and version of the librf.so C ABI (include/rf_api.h).
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

#include "rf_common.h"

namespace {
thread_local char g_err[1024] = "";
}

int rf_set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int rf_check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rf_set_error(RF_EHIP, "%s: %s", what, hipGetErrorString(e));
    return RF_OK;
}

extern "C" int32_t rf_abi_version(void) { return RF_ABI_VERSION; }

extern "C" const char* rf_last_error(void) { return g_err; }
