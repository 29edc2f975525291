// C-ABI plumbing of libnfx.so: version, thread-local error string, launch checks.
#include <stdarg.h>
#include <stdio.h>

#include "nfx_common.h"

namespace nfx {

static thread_local char g_err[512] = "";

int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(NFX_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
    return NFX_OK;
}

int num_cus() {
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cache[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            n <= 0)
            n = 256;
        cache[dev] = n;
    }
    return cache[dev];
}

}  // namespace nfx

extern "C" int nfx_abi_version(void) { return NFX_ABI_VERSION; }
extern "C" const char* nfx_last_error(void) { return nfx::g_err; }
