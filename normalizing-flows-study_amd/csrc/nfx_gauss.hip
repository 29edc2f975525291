// Gaussian base log-density and NLL partial sums (the log_prob glue of the reference callers).
//
// Reference: Flow.log_prob src/flows/flow/flow.py:56-73 and the inline callers README.md:113-114,
// src/utils.py:39-55, plots/_common.py:201-202:
//   log_p = MultivariateNormal(0, I).log_prob(z) + log_det,   loss = -log_p.mean()
// torch's MVN log_prob with identity scale_tril reduces to -0.5*(fp32(d*log 2pi) + sum_j z_j^2)
// (bit-exact). The mean is accumulated in float64 (NLL parity at 1M-4M
// samples needs it) with a deterministic two-pass block reduction.
#include <math.h>

#include "nfx_common.h"

namespace nfx {

constexpr int kGaussThreads = 256;
constexpr int kGaussMaxBlocks = 1024;
static_assert(kGaussMaxBlocks <= kMaxPartials, "partials capacity");

__device__ __forceinline__ double block_sum_f64(double v) { return block_sum_f64<kGaussThreads>(v); }

__global__ __launch_bounds__(kGaussThreads) void gauss_logprob_kernel(
    const float* __restrict__ z, const float* __restrict__ ld, float* __restrict__ logp,
    double* __restrict__ partials, double* __restrict__ sums, int64_t B, int d, float c) {
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kGaussThreads + threadIdx.x; i < B;
         i += (int64_t)gridDim.x * kGaussThreads) {
        const float* zr = z + i * d;
        float m = gauss_sq0(zr[0]);
        for (int j = 1; j < d; ++j) m = gauss_sq(m, zr[j]);
        const float lp = gauss_lp(m, c, ld[i]);
        if (logp) logp[i] = lp;
        acc += (double)lp;
    }
    logp_commit<kGaussThreads>(acc, partials, sums, B);
}

// d > 8: a thread-per-sample walk over [B, d] rows is uncoalesced (64 lanes hit 64 lines per
// load) and thrashes L2 at d = 63 (measured 6x the algorithmic bytes). Instead each wave stages
// its 64-sample tile through LDS in 32-dimension chunks with coalesced 128-byte row segments,
// then every lane sums its own row from LDS (stride-33 rows: conflict-free).
__global__ __launch_bounds__(kGaussThreads) void gauss_logprob_tiled_kernel(
    const float* __restrict__ z, const float* __restrict__ ld, float* __restrict__ logp,
    double* __restrict__ partials, double* __restrict__ sums, int64_t B, int d, float c) {
    __shared__ float stage[kGaussThreads / 64][64 * 33];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float* st = stage[wave];
    double acc = 0.0;
    const int64_t ntiles = (B + 63) / 64;
    for (int64_t t = (int64_t)blockIdx.x * (kGaussThreads / 64) + wave; t < ntiles;
         t += (int64_t)gridDim.x * (kGaussThreads / 64)) {
        const int64_t base = t * 64;
        float m = 0.f;
        for (int dim0 = 0; dim0 < d; dim0 += 32) {
#pragma unroll 8
            for (int i = 0; i < 32; ++i) {
                const int idx = i * 64 + lane, s = idx >> 5, dd = idx & 31;
                const int64_t row = base + s;
                st[s * 33 + dd] = (row < B && dim0 + dd < d) ? z[row * d + dim0 + dd] : 0.f;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const int n = (d - dim0) < 32 ? (d - dim0) : 32;
            for (int j = 0; j < n; ++j) {
                const float v = st[lane * 33 + j];
                m = (dim0 == 0 && j == 0) ? gauss_sq0(v) : gauss_sq(m, v);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        const int64_t i = base + lane;
        if (i < B) {
            const float lp = gauss_lp(m, c, ld[i]);
            if (logp) logp[i] = lp;
            acc += (double)lp;
        }
    }
    logp_commit<kGaussThreads>(acc, partials, sums, B);
}

__global__ __launch_bounds__(kGaussThreads) void gauss_finish_kernel(const double* __restrict__ partials,
                                                                     int n, double* __restrict__ sums,
                                                                     int64_t B) {
    double acc = 0.0;
    for (int i = threadIdx.x; i < n; i += kGaussThreads) acc += partials[i];
    const double t = block_sum_f64(acc);
    if (threadIdx.x == 0) {
        sums[0] = t;
        sums[1] = (double)B;
    }
}

int gauss_finish(const double* partials, int n, double* sums, int64_t B, hipStream_t s) {
    gauss_finish_kernel<<<1, kGaussThreads, 0, s>>>(partials, n, sums, B);
    return check_launch("gauss_finish_kernel");
}

// Its adjoint under autograd: grad_z[i, j] = -z[i, j] * g[i] (torch's pow backward, 2 z times
// the sum's -0.5 g: both exact scalings, one rounding), grad_log_det[i] = g[i].
template <bool WIDE>
__global__ __launch_bounds__(256) void gauss_logprob_bwd_kernel(const float* __restrict__ z, const float* __restrict__ g,
                                                                float* __restrict__ gz, float* __restrict__ gld,
                                                                int64_t B, int d) {
    const int64_t n = B * d, stride = (int64_t)gridDim.x * 256;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += stride) {
        const int64_t i = WIDE ? e / d : (int64_t)((uint32_t)e / (uint32_t)d);
        gz[e] = -(z[e] * g[i]);
    }
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < B; i += stride) gld[i] = g[i];
}

}  // namespace nfx

using namespace nfx;

extern "C" int nfx_gauss_logprob_backward(const float* z, const float* grad_logp, float* grad_z, float* grad_log_det,
                                          int64_t B, int d, void* stream) {
    if (B < 0 || d <= 0) return set_error(NFX_EINVAL, "gauss_logprob_backward: bad shape B=%lld d=%d", (long long)B, d);
    if (B == 0) return NFX_OK;
    if (!z || !grad_logp || !grad_z || !grad_log_det) return set_error(NFX_EINVAL, "gauss_logprob_backward: null pointer");
    const int64_t n = B * d;
    int64_t blocks = (n + 255) / 256;
    const int64_t cap = (int64_t)num_cus() * 8;
    if (blocks > cap) blocks = cap;
    if (n < ((int64_t)1 << 31))
        gauss_logprob_bwd_kernel<false><<<(int)blocks, 256, 0, (hipStream_t)stream>>>(z, grad_logp, grad_z, grad_log_det, B, d);
    else
        gauss_logprob_bwd_kernel<true><<<(int)blocks, 256, 0, (hipStream_t)stream>>>(z, grad_logp, grad_z, grad_log_det, B, d);
    return check_launch("gauss_logprob_bwd_kernel");
}

namespace nfx {
__global__ void gauss_workspace_init_kernel(double* partials) {
    *reinterpret_cast<uint64_t*>(partials + kMaxPartials) = kLogpClean;
}
}  // namespace nfx

extern "C" int nfx_gauss_workspace_init(void* workspace, void* stream) {
    if (!workspace) return set_error(NFX_EINVAL, "gauss_workspace_init: null workspace");
    gauss_workspace_init_kernel<<<1, 1, 0, (hipStream_t)stream>>>(reinterpret_cast<double*>(workspace));
    return check_launch("gauss_workspace_init_kernel");
}

extern "C" size_t nfx_gauss_workspace_bytes(int64_t B) {
    (void)B;
    return (size_t)(kMaxPartials + 1) * sizeof(double);  // partials + logp_commit's arrival counter
}

extern "C" int nfx_gauss_logprob(const float* z, const float* log_det, float* logp, double* sums,
                                 void* workspace, int64_t B, int d, void* stream) {
    if (B < 0 || d <= 0) return set_error(NFX_EINVAL, "gauss_logprob: bad shape B=%lld d=%d", (long long)B, d);
    if (!sums || !workspace) return set_error(NFX_EINVAL, "gauss_logprob: null sums/workspace");
    if (B > 0 && (!z || !log_det)) return set_error(NFX_EINVAL, "gauss_logprob: null z/log_det");
    hipStream_t s = (hipStream_t)stream;
    int blocks = (int)((B + kGaussThreads - 1) / kGaussThreads);
    if (blocks > kGaussMaxBlocks) blocks = kGaussMaxBlocks;
    if (blocks < 1) blocks = 1;
    const float c = gauss_const(d);
    double* partials = reinterpret_cast<double*>(workspace);
    if (B > 0 && d > 8) {
        int64_t tb = ((B + 63) / 64 + 3) / 4;
        blocks = (int)(tb < kGaussMaxBlocks ? tb : kGaussMaxBlocks);
        gauss_logprob_tiled_kernel<<<blocks, kGaussThreads, 0, s>>>(z, log_det, logp, partials, sums, B, d, c);
        int rc = check_launch("gauss_logprob_tiled_kernel");
        if (rc) return rc;
    } else if (B > 0) {
        gauss_logprob_kernel<<<blocks, kGaussThreads, 0, s>>>(z, log_det, logp, partials, sums, B, d, c);
        int rc = check_launch("gauss_logprob_kernel");
        if (rc) return rc;
    } else {
        return gauss_finish(partials, 0, sums, B, s);
    }
    return NFX_OK;  // the kernels' last workgroup wrote sums (logp_commit)
}
