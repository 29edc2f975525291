// C-ABI plumbing of libnfx.so: version, thread-local error string, launch checks.
#include <stdarg.h>
#include <stdio.h>

#include "nfx_common.h"

namespace nfx {

static thread_local char g_err[512] = "";
static thread_local const char* g_last_kernel = "";  // (string literals of the launch sites)

int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char* what) {
    g_last_kernel = what;
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
extern "C" const char* nfx_last_kernel(void) { return nfx::g_last_kernel; }

// Test hook: fill the whole LDS of every CU with the 32-bit pattern `bits` (one 160 KiB workgroup
// per CU, several rounds), so a kernel that read LDS it never wrote would see that pattern
// instead of whatever the previous kernel left behind. No effect on any later result.
__global__ __launch_bounds__(256) void nfx_fill_lds_kernel(uint32_t bits, int nwords) {
    extern __shared__ uint32_t fill[];
    for (int i = threadIdx.x; i < nwords; i += 256) fill[i] = bits;
    __syncthreads();
}

extern "C" int nfx_debug_fill_lds(uint32_t bits, void* stream) {
    const int bytes = 160 * 1024;
    int rc = nfx::prepare_lds((const void*)nfx_fill_lds_kernel, bytes);
    if (rc) return rc;
    nfx_fill_lds_kernel<<<8 * nfx::num_cus(), 256, bytes, (hipStream_t)stream>>>(bits, bytes / 4);
    return nfx::check_launch("nfx_fill_lds_kernel");
}
