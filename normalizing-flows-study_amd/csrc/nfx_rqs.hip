// Unit-interval rational-quadratic spline, elementwise (rational_quadratic_spline).
//
// Reference: src/flows/spline/rational_quadratic_spline.py:4-104. Differences from the
// coupling layer's spline that this kernel keeps: epsilon forced to 1e-6 (:19), knots on
// [0, 1] without pinning (:36-37), softplus(d) + min_d (:32), no tails, no zero-denominator
// guard in the inverse root (:79: 0/0 -> NaN propagates through the clamp like torch.clamp).
//
// One thread per input; the N x (3K-1) parameter rows are read once (HBM-bound:
// (3K+2)*4 bytes per element at K bins).
#include "nfx_rqs_unit.h"

namespace nfx {

template <int K, bool INV>
__global__ __launch_bounds__(256) void rqs_unit_kernel(
    const float* __restrict__ in, const float* __restrict__ uw, const float* __restrict__ uh,
    const float* __restrict__ ud, float* __restrict__ out, float* __restrict__ logdet, int64_t N,
    float min_w, float cw, float min_h, float ch, float min_d) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N; i += (int64_t)gridDim.x * 256) {
        float w[K], h[K], dv[K - 1];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            w[k] = uw[i * K + k];
            h[k] = uh[i * K + k];
        }
#pragma unroll
        for (int k = 0; k < K - 1; ++k) dv[k] = ud[i * (K - 1) + k];
        float o, l;
        rqs_unit_eval<K, INV>(in[i], w, h, dv, min_w, cw, min_h, ch, min_d, o, l);
        out[i] = o;
        logdet[i] = l;
    }
}

// The adjoint (rqs_unit_adjoint): per element the upstream gradients of the output and the
// log-det in, dL/dx and dL/d(unnormalised widths, heights, inner derivatives) out — one pass,
// (3K + 4) * 4 bytes read and (3K) * 4 written per element.
template <int K, bool INV>
__global__ __launch_bounds__(256) void rqs_unit_bwd_kernel(
    const float* __restrict__ in, const float* __restrict__ uw, const float* __restrict__ uh,
    const float* __restrict__ ud, const float* __restrict__ gout, const float* __restrict__ gld,
    float* __restrict__ gin, float* __restrict__ gw, float* __restrict__ gh, float* __restrict__ gd, int64_t N,
    float min_w, float cw, float min_h, float ch, float min_d) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N; i += (int64_t)gridDim.x * 256) {
        float w[K], h[K], dv[K - 1], tw[K], th[K], td[K - 1];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            w[k] = uw[i * K + k];
            h[k] = uh[i * K + k];
        }
#pragma unroll
        for (int k = 0; k < K - 1; ++k) dv[k] = ud[i * (K - 1) + k];
        float o, l, gx;
        rqs_unit_adjoint<K, INV>(in[i], w, h, dv, min_w, cw, min_h, ch, min_d, gout[i], gld[i], o, l, gx, tw, th, td);
        gin[i] = gx;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            gw[i * K + k] = tw[k];
            gh[i * K + k] = th[k];
        }
#pragma unroll
        for (int k = 0; k < K - 1; ++k) gd[i * (K - 1) + k] = td[k];
    }
}

typedef void (*rqs_bwd_kernel_t)(const float*, const float*, const float*, const float*, const float*, const float*,
                                 float*, float*, float*, float*, int64_t, float, float, float, float, float);

typedef void (*rqs_kernel_t)(const float*, const float*, const float*, const float*, float*, float*,
                             int64_t, float, float, float, float, float);

template <int K>
static rqs_kernel_t rqs_dir(int inv) {
    return inv ? rqs_unit_kernel<K, true> : rqs_unit_kernel<K, false>;
}

template <int K>
static rqs_bwd_kernel_t rqs_bwd_dir(int inv) {
    return inv ? rqs_unit_bwd_kernel<K, true> : rqs_unit_bwd_kernel<K, false>;
}

static rqs_bwd_kernel_t pick_rqs_bwd(int K, int inv) {
    switch (K) {
        case 2: return rqs_bwd_dir<2>(inv);
        case 3: return rqs_bwd_dir<3>(inv);
        case 4: return rqs_bwd_dir<4>(inv);
        case 5: return rqs_bwd_dir<5>(inv);
        case 6: return rqs_bwd_dir<6>(inv);
        case 7: return rqs_bwd_dir<7>(inv);
        case 8: return rqs_bwd_dir<8>(inv);
        case 9: return rqs_bwd_dir<9>(inv);
        case 10: return rqs_bwd_dir<10>(inv);
        case 11: return rqs_bwd_dir<11>(inv);
        case 12: return rqs_bwd_dir<12>(inv);
        case 13: return rqs_bwd_dir<13>(inv);
        case 14: return rqs_bwd_dir<14>(inv);
        case 15: return rqs_bwd_dir<15>(inv);
        case 16: return rqs_bwd_dir<16>(inv);
        default: return nullptr;
    }
}

static rqs_kernel_t pick_rqs(int K, int inv) {
    switch (K) {
        case 2: return rqs_dir<2>(inv);
        case 3: return rqs_dir<3>(inv);
        case 4: return rqs_dir<4>(inv);
        case 5: return rqs_dir<5>(inv);
        case 6: return rqs_dir<6>(inv);
        case 7: return rqs_dir<7>(inv);
        case 8: return rqs_dir<8>(inv);
        case 9: return rqs_dir<9>(inv);
        case 10: return rqs_dir<10>(inv);
        case 11: return rqs_dir<11>(inv);
        case 12: return rqs_dir<12>(inv);
        case 13: return rqs_dir<13>(inv);
        case 14: return rqs_dir<14>(inv);
        case 15: return rqs_dir<15>(inv);
        case 16: return rqs_dir<16>(inv);
        default: return nullptr;
    }
}

}  // namespace nfx

using namespace nfx;

extern "C" int nfx_rqs_unit(const float* in, const float* widths, const float* heights,
                            const float* derivatives, float* out, float* log_det, int64_t N, int K,
                            float min_bin_width, float min_bin_height, float min_derivative,
                            int inverse, void* stream) {
    if (N < 0 || K < 2) return set_error(NFX_EINVAL, "rqs_unit: bad shape N=%lld K=%d", (long long)N, K);
    rqs_kernel_t k = pick_rqs(K, inverse ? 1 : 0);
    if (!k) return set_error(NFX_EUNSUPPORTED, "rqs_unit: K=%d outside 2..16", K);
    if (N == 0) return NFX_OK;
    if (!in || !widths || !heights || !derivatives || !out || !log_det)
        return set_error(NFX_EINVAL, "rqs_unit: null pointer");
    const float cw = (float)(1.0 - (double)min_bin_width * K);
    const float ch = (float)(1.0 - (double)min_bin_height * K);
    int64_t blocks = (N + 255) / 256;
    const int64_t cap = (int64_t)num_cus() * 16;
    if (blocks > cap) blocks = cap;
    k<<<(int)blocks, 256, 0, (hipStream_t)stream>>>(in, widths, heights, derivatives, out, log_det, N,
                                                     min_bin_width, cw, min_bin_height, ch, min_derivative);
    return check_launch("rqs_unit_kernel");
}

extern "C" int nfx_rqs_unit_backward(const float* in, const float* widths, const float* heights,
                                     const float* derivatives, const float* grad_out, const float* grad_log_det,
                                     float* grad_in, float* grad_widths, float* grad_heights,
                                     float* grad_derivatives, int64_t N, int K, float min_bin_width,
                                     float min_bin_height, float min_derivative, int inverse, void* stream) {
    if (N < 0 || K < 2) return set_error(NFX_EINVAL, "rqs_unit_backward: bad shape N=%lld K=%d", (long long)N, K);
    rqs_bwd_kernel_t k = pick_rqs_bwd(K, inverse ? 1 : 0);
    if (!k) return set_error(NFX_EUNSUPPORTED, "rqs_unit_backward: K=%d outside 2..16", K);
    if (N == 0) return NFX_OK;
    if (!in || !widths || !heights || !derivatives || !grad_out || !grad_log_det || !grad_in || !grad_widths ||
        !grad_heights || !grad_derivatives)
        return set_error(NFX_EINVAL, "rqs_unit_backward: null pointer");
    const float cw = (float)(1.0 - (double)min_bin_width * K);
    const float ch = (float)(1.0 - (double)min_bin_height * K);
    int64_t blocks = (N + 255) / 256;
    const int64_t cap = (int64_t)num_cus() * 16;
    if (blocks > cap) blocks = cap;
    k<<<(int)blocks, 256, 0, (hipStream_t)stream>>>(in, widths, heights, derivatives, grad_out, grad_log_det, grad_in,
                                                     grad_widths, grad_heights, grad_derivatives, N, min_bin_width, cw,
                                                     min_bin_height, ch, min_derivative);
    return check_launch("rqs_unit_bwd_kernel");
}
