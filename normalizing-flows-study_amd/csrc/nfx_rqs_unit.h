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

namespace nfx {

// Adjoint of rqs_unit_eval (autograd of rational_quadratic_spline.py:4-104, torch semantics:
// clamp passes the gradient on [min, max] inclusive, softplus above threshold 20 passes it
// through, searchsorted/bin selection carries none). Given the upstream gradients go (output)
// and gl (log-det): o, l as rqs_unit_eval; gx = dL/dx; guw, guh, gud = dL/d(unnormalised
// widths, heights, inner derivatives).
template <int K, bool INV>
__device__ __forceinline__ void rqs_unit_adjoint(float x, const float (&uw)[K], const float (&uh)[K],
                                                 const float (&ud)[K - 1], float min_w, float cw, float min_h,
                                                 float ch, float min_d, float go, float gl, float& o, float& l,
                                                 float& gx, float (&guw)[K], float (&guh)[K], float (&gud)[K - 1]) {
#pragma clang fp contract(off)
    const float eps = 1e-6f;
    float smw[K], smh[K], w[K], h[K], pw[K], ph[K], xk[K + 1], yk[K + 1], dv[K + 1], spr[K + 1];
    float mw = uw[0], mh = uh[0];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        mw = tmax(mw, uw[k]);
        mh = tmax(mh, uh[k]);
    }
    float sw = 0.f, sh = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        smw[k] = expf(uw[k] - mw);
        sw = sw + smw[k];
        smh[k] = expf(uh[k] - mh);
        sh = sh + smh[k];
    }
    const float iw = 1.f / sw, ih = 1.f / sh;
    double aw = 0.0, ah = 0.0;
    xk[0] = 0.f;
    yk[0] = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        smw[k] = smw[k] * iw;
        smh[k] = smh[k] * ih;
        pw[k] = min_w + cw * smw[k];
        ph[k] = min_h + ch * smh[k];
        w[k] = tclamp_min(pw[k], eps);
        h[k] = tclamp_min(ph[k], eps);
        aw += (double)w[k];
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
        spr[k + 1] = sp + min_d;
        dv[k + 1] = tclamp_min(spr[k + 1], eps);
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
    const float W = tclamp_min(w_k, eps);
    const float s_k = h_k / W;
    const float A = d_k + d_k1 - 2.f * s_k;
    float g_s = 0.f, g_h = 0.f, g_w = 0.f, g_xk = 0.f, g_yk = 0.f, g_dk = 0.f, g_dk1 = 0.f, g_A = 0.f;
    gx = 0.f;
    if constexpr (INV) {
        const float dy = x - y_k;
        const float t1 = dy * A;
        const float a = h_k * (s_k - d_k) + t1;
        const float b = h_k * d_k - t1;
        const float c = -s_k * dy;
        const float discr = b * b - 4.f * a * c;
        const float disc = tclamp_min(discr, 0.f);
        const float q = sqrtf(disc);
        const float Den = -b - q;
        const float thr = (2.f * c) / Den;
        const float th = tclamp(thr, 0.f, 1.f);
        o = th * w_k + x_k;
        const float tt = th * (1.f - th);
        const float om = 1.f - th;
        const float R = d_k1 * (th * th) + 2.f * s_k * tt + d_k * (om * om);
        const float nom = (s_k * s_k) * R;
        const float E = s_k + A * tt;
        const float den = E * E;
        const float Dc = tclamp_min(den, eps);
        const float der = nom / Dc;
        const float derc = tclamp_min(der, eps);
        l = -logf(derc);
        // reverse
        const float g_der = der >= eps ? -gl / derc : 0.f;
        const float g_nom = g_der / Dc;
        const float g_den = den >= eps ? -g_der * der / Dc : 0.f;
        const float g_E = g_den * 2.f * E;
        float g_tt = g_E * A;
        g_s += g_E;
        g_A += g_E * tt;
        g_s += g_nom * R * 2.f * s_k;
        const float g_R = g_nom * (s_k * s_k);
        g_dk1 += g_R * (th * th);
        float g_th = g_R * d_k1 * 2.f * th;
        g_s += g_R * 2.f * tt;
        g_tt += g_R * 2.f * s_k;
        g_dk += g_R * (om * om);
        g_th -= g_R * d_k * 2.f * om;
        g_th += go * w_k;
        g_w += go * th;
        g_xk += go;
        g_th += g_tt * (1.f - 2.f * th);
        const float g_thr = (thr >= 0.f && thr <= 1.f) ? g_th : 0.f;
        float g_c = g_thr * 2.f / Den;
        const float g_Den = -g_thr * thr / Den;
        float g_b = -g_Den;
        const float g_q = -g_Den;
        const float g_disc = g_q / (2.f * q);
        const float g_discr = discr >= 0.f ? g_disc : 0.f;
        g_b += g_discr * 2.f * b;
        const float g_a = -4.f * c * g_discr;
        g_c += -4.f * a * g_discr;
        g_s += -dy * g_c;
        float g_dy = -s_k * g_c;
        g_h += d_k * g_b;
        g_dk += h_k * g_b;
        float g_t1 = -g_b;
        g_h += (s_k - d_k) * g_a;
        g_s += h_k * g_a;
        g_dk += -h_k * g_a;
        g_t1 += g_a;
        g_dy += A * g_t1;
        g_A += dy * g_t1;
        gx += g_dy;
        g_yk += -g_dy;
    } else {
        const float thr = (x - x_k) / W;
        const float th = tclamp(thr, 0.f, 1.f);
        const float tt = th * (1.f - th);
        const float om = 1.f - th;
        const float Q = s_k * (th * th) + d_k * tt;
        const float nom = h_k * Q;
        const float den = s_k + A * tt;
        const float Dc = tclamp_min(den, eps);
        o = y_k + nom / Dc;
        const float R = d_k1 * (th * th) + 2.f * s_k * tt + d_k * (om * om);
        const float nd = (s_k * s_k) * R;
        const float den2 = den * den;
        const float D2c = tclamp_min(den2, eps);
        const float der = nd / D2c;
        const float derc = tclamp_min(der, eps);
        l = logf(derc);
        // reverse
        const float g_der = der >= eps ? gl / derc : 0.f;
        const float g_nd = g_der / D2c;
        float g_den = den2 >= eps ? -g_der * der / D2c * 2.f * den : 0.f;
        const float g_nom = go / Dc;
        g_den += den >= eps ? -go * (nom / Dc) / Dc : 0.f;
        g_yk += go;
        g_h += g_nom * Q;
        const float g_Q = g_nom * h_k;
        g_s += g_Q * (th * th);
        float g_th = g_Q * s_k * 2.f * th;
        g_dk += g_Q * tt;
        float g_tt = g_Q * d_k;
        g_s += g_nd * R * 2.f * s_k;
        const float g_R = g_nd * (s_k * s_k);
        g_dk1 += g_R * (th * th);
        g_th += g_R * d_k1 * 2.f * th;
        g_s += g_R * 2.f * tt;
        g_tt += g_R * 2.f * s_k;
        g_dk += g_R * (om * om);
        g_th -= g_R * d_k * 2.f * om;
        g_s += g_den;
        g_A += g_den * tt;
        g_tt += g_den * A;
        g_th += g_tt * (1.f - 2.f * th);
        const float g_thr = (thr >= 0.f && thr <= 1.f) ? g_th : 0.f;
        gx += g_thr / W;
        g_xk -= g_thr / W;
        g_w += -g_thr * thr / W;  // through W = max(w_k, eps)
    }
    g_dk += g_A;
    g_dk1 += g_A;
    g_s += -2.f * g_A;
    g_h += g_s / W;
    const float g_W = -g_s * s_k / W;
    g_w += w_k >= eps ? g_W : 0.f;  // s_k = h_k / max(w_k, eps) (INV: theta * w_k uses w_k itself)
    // scatter the selected bin's gradients; knots are prefix sums (xk[k+1] = sum_{j<=k} w_j)
    float gwa[K], gha[K], gdv[K + 1];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        gwa[k] = k == bin ? g_w : 0.f;
        gha[k] = k == bin ? g_h : 0.f;
    }
#pragma unroll
    for (int k = 0; k <= K; ++k) gdv[k] = (k == bin ? g_dk : 0.f) + (k == bin + 1 ? g_dk1 : 0.f);
    // g_xk, g_yk belong to knot index `bin` (knot 0 is the pad: no gradient); knot k >= 1 is the
    // prefix sum through w_{k-1}, so it feeds every w_j with j <= k - 1 < bin
#pragma unroll
    for (int j = 0; j < K; ++j) {
        if (j < bin) {
            gwa[j] += g_xk;
            gha[j] += g_yk;
        }
    }
    // clamp(min_w + cw * softmax, eps), then the softmax backward
    float dw = 0.f, dh = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        gwa[k] = pw[k] >= eps ? gwa[k] * cw : 0.f;
        gha[k] = ph[k] >= eps ? gha[k] * ch : 0.f;
        dw += gwa[k] * smw[k];
        dh += gha[k] * smh[k];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        guw[k] = smw[k] * (gwa[k] - dw);
        guh[k] = smh[k] * (gha[k] - dh);
    }
#pragma unroll
    for (int k = 0; k < K - 1; ++k) {
        const float u = ud[k];
        const float g = spr[k + 1] >= eps ? gdv[k + 1] : 0.f;
        if (u > 20.f) {
            gud[k] = g;
        } else {
            const float z = expf(u);
            gud[k] = g * z / (z + 1.f);
        }
    }
}

}  // namespace nfx
