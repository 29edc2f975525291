// Unit-interval rational-quadratic spline, elementwise (rational_quadratic_spline).
//
// Reference: src/flows/spline/rational_quadratic_spline.py:4-104. Differences from the
// coupling layer's spline that this kernel keeps: epsilon forced to 1e-6 (:19), knots on
// [0, 1] without pinning (:36-37), softplus(d) + min_d (:32), no tails, no zero-denominator
// guard in the inverse root (:79: 0/0 -> NaN propagates through the clamp like torch.clamp).
//
// One thread per input; the N x (3K-1) parameter rows are read once (HBM-bound:
// (3K+2)*4 bytes per element at K bins).
#include "nfx_common.h"

namespace nfx {

template <int K, bool INV>
__global__ __launch_bounds__(256) void rqs_unit_kernel(
    const float* __restrict__ in, const float* __restrict__ uw, const float* __restrict__ uh,
    const float* __restrict__ ud, float* __restrict__ out, float* __restrict__ logdet, int64_t N,
    float min_w, float cw, float min_h, float ch, float min_d) {
#pragma clang fp contract(off)
    const float eps = 1e-6f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N; i += (int64_t)gridDim.x * 256) {
        const float x = in[i];
        float w[K], h[K], xk[K + 1], yk[K + 1], dv[K + 1];
        float mw = uw[i * K], mh = uh[i * K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            w[k] = uw[i * K + k];
            h[k] = uh[i * K + k];
            mw = tmax(mw, w[k]);
            mh = tmax(mh, h[k]);
        }
        float sw = 0.f, sh = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            w[k] = expf(w[k] - mw);
            sw = sw + w[k];
            h[k] = expf(h[k] - mh);
            sh = sh + h[k];
        }
        const float iw = 1.f / sw, ih = 1.f / sh;
        double aw = 0.0, ah = 0.0;
        xk[0] = 0.f;
        yk[0] = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            w[k] = tclamp_min(min_w + cw * (w[k] * iw), eps);
            h[k] = tclamp_min(min_h + ch * (h[k] * ih), eps);
            aw += (double)w[k];  // ATen CPU cumsum: float accumulated in double (:36-37)
            ah += (double)h[k];
            xk[k + 1] = (float)aw;
            yk[k + 1] = (float)ah;
        }
        dv[0] = 1.f;
        dv[K] = 1.f;
#pragma unroll
        for (int k = 0; k < K - 1; ++k) {
            const float u = ud[i * (K - 1) + k];
            const float sp = u > 20.f ? u : log1pf(expf(u));
            dv[k + 1] = tclamp_min(sp + min_d, eps);
        }
        int cnt = 0;
#pragma unroll
        for (int k = 0; k <= K; ++k) cnt += ((INV ? yk[k] : xk[k]) <= x) ? 1 : 0;
        int bin = cnt - 1;
        bin = bin < 0 ? 0 : (bin > K - 1 ? K - 1 : bin);
        float w_k = w[0], x_k = xk[0], h_k = h[0], y_k = yk[0], d_k = dv[0], d_k1 = dv[1];
#pragma unroll
        for (int k = 1; k < K; ++k) {
            const bool s = (k == bin);
            w_k = s ? w[k] : w_k;
            x_k = s ? xk[k] : x_k;
            h_k = s ? h[k] : h_k;
            y_k = s ? yk[k] : y_k;
            d_k = s ? dv[k] : d_k;
            d_k1 = s ? dv[k + 1] : d_k1;
        }
        const float s_k = h_k / tclamp_min(w_k, eps);
        float o, l;
        if constexpr (INV) {
            const float dy = x - y_k;
            const float t1 = dy * (d_k + d_k1 - 2.f * s_k);
            const float a = h_k * (s_k - d_k) + t1;
            const float b = h_k * d_k - t1;
            const float c = -s_k * dy;
            const float disc = tclamp_min(b * b - 4.f * a * c, 0.f);
            const float th = tclamp((2.f * c) / (-b - sqrtf(disc)), 0.f, 1.f);
            o = th * w_k + x_k;
            const float tt = th * (1.f - th);
            const float om = 1.f - th;
            const float nom = (s_k * s_k) * (d_k1 * (th * th) + 2.f * s_k * tt + d_k * (om * om));
            const float dd = s_k + (d_k + d_k1 - 2.f * s_k) * tt;
            l = -logf(tclamp_min(nom / tclamp_min(dd * dd, eps), eps));
        } else {
            const float th = tclamp((x - x_k) / tclamp_min(w_k, eps), 0.f, 1.f);
            const float tt = th * (1.f - th);
            const float om = 1.f - th;
            const float nom = h_k * (s_k * (th * th) + d_k * tt);
            const float den = s_k + (d_k + d_k1 - 2.f * s_k) * tt;
            o = y_k + nom / tclamp_min(den, eps);
            const float nd = (s_k * s_k) * (d_k1 * (th * th) + 2.f * s_k * tt + d_k * (om * om));
            l = logf(tclamp_min(nd / tclamp_min(den * den, eps), eps));
        }
        out[i] = o;
        logdet[i] = l;
    }
}

typedef void (*rqs_kernel_t)(const float*, const float*, const float*, const float*, float*, float*,
                             int64_t, float, float, float, float, float);

template <int K>
static rqs_kernel_t rqs_dir(int inv) {
    return inv ? rqs_unit_kernel<K, true> : rqs_unit_kernel<K, false>;
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
