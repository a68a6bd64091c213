// Host-side plumbing of the C ABI: version, thread-local error string, launch checks.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "trlx_t5_amd.h"

namespace trlx {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return TRLX_ERR_LAUNCH;
    }
    return TRLX_OK;
}

}  // namespace trlx

extern "C" int trlx_abi_version(void) { return TRLX_ABI_VERSION; }
extern "C" const char* trlx_last_error(void) { return trlx::g_err; }
