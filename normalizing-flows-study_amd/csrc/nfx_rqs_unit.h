// Unit-interval rational-quadratic spline of one element (rational_quadratic_spline,
// src/flows/spline/rational_quadratic_spline.py:4-104), shared by the elementwise kernel
// (nfx_rqs.hip) and the ARQS kernel (nfx_arqs_kernel.h).
#pragma once
#include "nfx_common.h"

namespace nfx {

// uw, uh: unnormalised widths/heights [K]; ud: unnormalised inner derivatives [K-1].
// cw = fp32(1 - min_w*K), ch = fp32(1 - min_h*K) (computed in double on the host, :27-28).
template <int K, bool INV>
__device__ __forceinline__ void rqs_unit_eval(float x, const float (&uw)[K], const float (&uh)[K],
                                              const float (&ud)[K - 1], float min_w, float cw,
                                              float min_h, float ch, float min_d, float& o, float& l) {
#pragma clang fp contract(off)
    const float eps = 1e-6f;  // forced (:19)
    float w[K], h[K], xk[K + 1], yk[K + 1], dv[K + 1];
    float mw = uw[0], mh = uh[0];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        mw = tmax(mw, uw[k]);
        mh = tmax(mh, uh[k]);
    }
    float sw = 0.f, sh = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        w[k] = expf(uw[k] - mw);
        sw = sw + w[k];
        h[k] = expf(uh[k] - mh);
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
        const float u = ud[k];
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
}

}  // namespace nfx
