// Backward of the rational-quadratic-spline coupling layer (SplineCouplingLayer) for gfx950:
// SURVEY.md §8(f) item 1. See nfx_spline_bwd.hip for the entry points.
//
// One kernel per layer call: per 64-sample chunk (a wave; lane l <-> sample l) it recomputes
// the param MLP on fp32 MFMA exactly like spline_coupling_kernel, runs the spline FORWARD and
// its hand-written adjoint per transformed element (rq_spline_adjoint below: softmax, min-width
// affine, knot cumsum with the pinned ends, softplus derivatives, bin gather and the RQ map or
// its citardauq inverse, every torch.clamp / torch.where guard with autograd's semantics), then
// the data-gradient chain back through the MLP on MFMA with transposed weight tiles and the
// weight gradients as MFMA contractions over the sample dimension (per-wave LDS transposes, as
// in nfx_affine_train_kernel.h). Reference: src/flows/spline/spline_coupling_layer.py:96-309.
#pragma once
#ifndef NFX_SBWD_EXPT
#define NFX_SBWD_EXPT 0
#endif
#include "nfx_affine_train_kernel.h"  // transpose_tile, kTS
#include "nfx_spline_kernel.h"        // SplineConsts, tsoftplus, crow/mfma helpers

namespace nfx {

// Backward pack: [forward spline pack with output-tile capacity NTMAX] then
//   w2t [HT][HT][4][64][4]   A operand of W2^T (output tile = layer-2 input tile)
//   w3t [HT][NTMAX][4][64][4] A operand of W3_t^T: A[i = hidden 32kt + i][k = param row of tile t]
//   w1c [8][HT][32]           W1[row][j] in accumulator order
struct SplineBwdLayout {
    SplineLayout F;
    int w2t, w3t, w1c, total;
};

__host__ __device__ constexpr SplineBwdLayout spline_bwd_layout(int HT, int NTMAX) {
    SplineBwdLayout L{};
    L.F = spline_layout(HT, NTMAX);
    int o = L.F.total;
    L.w2t = o; o += HT * HT * 1024;
    L.w3t = o; o += HT * NTMAX * 1024;
    L.w1c = o; o += 8 * HT * 32;
    L.total = (o + 3) & ~3;
    return L;
}

// Per-workgroup partial (floats): dW1 [8][Hp] (j-major) | db1 [Hp] | dW2 [Hp][Hp] | db2 [Hp] |
// dW3 [NTMAX][32][Hp] | db3 [NTMAX][32]
struct SplineGrad {
    int w1, b1, w2, b2, w3, b3, total;
};
__host__ __device__ constexpr SplineGrad spline_grad_layout(int HT, int NTMAX) {
    SplineGrad g{};
    const int Hp = 32 * HT;
    int o = 0;
    g.w1 = o; o += 8 * Hp;
    g.b1 = o; o += Hp;
    g.w2 = o; o += Hp * Hp;
    g.b2 = o; o += Hp;
    g.w3 = o; o += NTMAX * 32 * Hp;
    g.b3 = o; o += NTMAX * 32;
    g.total = o;
    return g;
}

// Spline forward + adjoint for one element (the reference's _rational_quadratic_spline per
// element and its autograd), split over the two lane halves that hold the same sample: lane half
// h owns one SIDE of the spline — h = 0 the bin widths, h = 1 the bin heights (softmax, min-width
// affine and clamp, knot cumsum, knot differences, and all of their backward) — and the
// derivative logits of parity h (softplus forward and backward). The gathered bin quantities and
// the searched side's bin index are exchanged with one v_permlane32_swap each; the scalar RQ map
// and its adjoint run on both halves (same data, same instructions). Every value goes through
// exactly the operations of the unsplit formulation, so the results are bit-identical to it.
// Given the input v, the 3K-1 raw parameters p[] (all of them, on both halves), the upstream
// gradients go (output) and gl (log-det): out = the spline output (after the spline-level guard),
// gv = dL/dv, gs[k] = dL/dp[h*K + k] (this half's side), gd[t] = dL/dp[2K + 2t + h].
template <int K, bool INV>
__device__ __forceinline__ void rq_spline_adjoint(float v, const float (&p)[32], const SplineConsts C,
                                                  float go, float gl, float& out, float (&gs)[K],
                                                  float (&gd)[K / 2], float& gv) {
#pragma clang fp contract(off)
    constexpr int ND = K / 2;  // derivative logits per half: k = 2t + h < K - 1
    const float eps = 1e-8f;
    const float B = C.bound;
    const bool hi = (threadIdx.x & 32) != 0;
#pragma unroll
    for (int k = 0; k < K; ++k) gs[k] = 0.f;
#pragma unroll
    for (int t = 0; t < ND; ++t) gd[t] = 0.f;
    out = v;
    gv = go;  // identity outside [-B, B] (and the spline-level guard's fallback)
    if (!(v >= -B && v <= B)) return;
    // per-half selects between two parameters: the operands pass through an empty asm first, so
    // the select stays a select of VALUES (a select between two elements of an array would
    // otherwise become a select of addresses and send the array to scratch)
    auto pick = [&](int i0, int i1) -> float {
        float a = p[i0], b = p[i1];
        asm volatile("" : "+v"(a), "+v"(b));
        return hi ? b : a;
    };

    // ---- this half's side, forward (same arithmetic as rq_spline_elem) ----
    float sm[K], pre[K], val[K], knot[K + 1], wd[K];
    {
        float u[K];
#pragma unroll
        for (int k = 0; k < K; ++k) u[k] = pick(k, K + k);
        const float mins = hi ? C.min_h : C.min_w, cs = hi ? C.ch : C.cw;
        float m = u[0];
#pragma unroll
        for (int k = 1; k < K; ++k) m = tmax(m, u[k]);
        float ssum = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) { sm[k] = exp_safe(u[k] - m); ssum = ssum + sm[k]; }
        const float inv = 1.f / ssum;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            sm[k] = sm[k] * inv;
            pre[k] = mins + cs * sm[k];
            val[k] = tclamp_min(pre[k], eps);
        }
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            acc += (double)val[k];
            knot[k + 1] = C.two_bound * (float)acc + (-B);
        }
        knot[0] = -B;
        knot[K] = B;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            wd[k] = knot[k + 1] - knot[k];
            val[k] = tclamp_min(wd[k], eps);
        }
    }
    // ---- derivatives: this half computes k = 2t + h, then both halves hold all of them ----
    float dpre[ND], dk[K + 1];
    dk[0] = 1.f;
    dk[K] = 1.f;
#pragma unroll
    for (int t = 0; t < ND; ++t) {
        const int k0 = 2 * t, k1 = 2 * t + 1;  // this half's k is k0 (h = 0) or k1 (h = 1)
        const float uu = pick(2 * K + k0, 2 * K + (k1 < K - 1 ? k1 : k0));
        dpre[t] = C.min_d + tsoftplus(uu);
        const float mine = tclamp_min(dpre[t], eps);
        const float other = halves_other(mine, mine);
        dk[k0 + 1] = hi ? other : mine;
        if (k1 < K - 1) dk[k1 + 1] = hi ? mine : other;
    }
    // ---- bin: counted on the searched side's knots (heights when inverting) ----
    int cnt = 0;
#pragma unroll
    for (int k = 0; k <= K; ++k) cnt += (knot[k] <= v) ? 1 : 0;
    {
        const int cnt_other = __float_as_int(halves_other(__int_as_float(cnt), __int_as_float(cnt)));
        cnt = (hi == INV) ? cnt : cnt_other;
    }
    int bin = cnt - 1;
    bin = bin < 0 ? 0 : (bin > K - 1 ? K - 1 : bin);
    float vb = val[0], kb = knot[0], d_k = dk[0], d_k1 = dk[1];
#pragma unroll
    for (int k = 1; k < K; ++k) {
        const bool s = (k == bin);
        vb = s ? val[k] : vb;
        kb = s ? knot[k] : kb;
        d_k = s ? dk[k] : d_k;
        d_k1 = s ? dk[k + 1] : d_k1;
    }
    const float vo = halves_other(vb, vb), ko = halves_other(kb, kb);
    const float w_k = hi ? vo : vb, x_k = hi ? ko : kb;
    const float h_k = hi ? vb : vo, y_k = hi ? kb : ko;
    const float wc = tclamp_min(w_k, eps);
    const float s_k = h_k / wc;

    // ---- the element's forward value and the gradients of the gathered quantities ----
    float o, l;
    float g_w = 0.f, g_x = 0.f, g_h = 0.f, g_y = 0.f, g_d0 = 0.f, g_d1 = 0.f, g_s = 0.f, g_v = 0.f;
    if constexpr (INV) {
        const float dy = v - y_k;
        const float T = d_k + d_k1 - 2.f * s_k;
        const float a = dy * T + h_k * (s_k - d_k);
        const float b = h_k * d_k - dy * T;
        const float c = -s_k * dy;
        const float dpr = b * b - 4.f * a * c;
        const float disc = tclamp_min(dpr, 0.f);
        const float sq = sqrtf(disc);
        const float den0 = -b - sq;
        const bool small = fabsf(den0) < eps;
        const float den = small ? eps : den0;
        const float xp = (2.f * c) / den;
        const float xi = tclamp(xp, 0.f, 1.f);
        o = xi * w_k + x_k;
        const float omx = 1.f - xi;
        const float A = xi * omx;
        const float T2 = d_k1 + d_k - 2.f * s_k;
        const float dld = s_k + T2 * A;
        const float Q = d_k1 * (xi * xi) + 2.f * s_k * A + d_k * (omx * omx);
        const float nld = (s_k * s_k) * Q;
        l = -logf(tclamp_min(nld, eps)) + 2.f * logf(tclamp_min(dld, eps));
        // spline-level guards (:306-307): non-finite out -> input (grad to v), lad -> 0
        const bool fo = !nonfinite(o), fl = !nonfinite(l);
        const float gO = fo ? go : 0.f;
        const float gL = fl ? gl : 0.f;
        g_v = fo ? 0.f : go;
        float g_xi = gO * w_k;
        g_w += gO * xi;
        g_x += gO;
        const float g_nld = nld >= eps ? -gL / nld : 0.f;
        const float g_dld = dld >= eps ? (2.f * gL) / dld : 0.f;
        // dld = s + T2 A
        g_s += g_dld;
        float g_T2 = g_dld * A;
        float g_A = g_dld * T2;
        // nld = s^2 Q
        g_s += g_nld * Q * (2.f * s_k);
        const float g_Q = g_nld * (s_k * s_k);
        g_d1 += g_Q * (xi * xi);
        g_xi += g_Q * d_k1 * (2.f * xi);
        g_s += g_Q * (2.f * A);
        g_A += g_Q * (2.f * s_k);
        g_d0 += g_Q * (omx * omx);
        float g_omx = g_Q * d_k * (2.f * omx);
        g_xi += g_A * omx;
        g_omx += g_A * xi;
        g_xi -= g_omx;
        g_d1 += g_T2;
        g_d0 += g_T2;
        g_s -= 2.f * g_T2;
        const float g_xp = (xp >= 0.f && xp <= 1.f) ? g_xi : 0.f;
        if (!small && dpr > 0.f) {
            // Away from the den/discriminant guards the quadratic formula's root xi solves
            // G(xi) = h N(xi)/D(xi) - dy = 0 (N = s xi^2 + d0 A, D = s + T A): differentiate that
            // implicitly, dxi/dth = -(dG/dth)/(dG/dxi) with dG/dxi = h s Q / D^2. Exactly what
            // autograd through -2c/(b + sqrt(b^2 - 4ac)) computes, without the cancellation in
            // b^2 - 4ac that makes the explicit chain lose digits on flat stretches of the map.
            const float Nn = s_k * (xi * xi) + d_k * A;
            const float D = s_k + T * A;
            const float iD = 1.f / D;
            const float R = Nn * iD;
            const float hD = h_k * iD;
            const float lam = g_xp / (hD * s_k * Q * iD);
            g_v += lam;
            g_y -= lam;
            g_h -= lam * R;
            g_s -= lam * hD * (xi * xi - R * (1.f - 2.f * A));
            g_d0 -= lam * hD * A * (1.f - R);
            g_d1 += lam * hD * R * A;
        } else {
            // xp = 2c / den
            float g_c = g_xp * 2.f / den;
            const float g_den = -g_xp * (2.f * c) / (den * den);
            const float g_den0 = small ? 0.f : g_den;
            float g_b = -g_den0;
            const float g_sq = -g_den0;
            const float g_disc = g_sq / (2.f * sq);
            const float g_dpr = dpr >= 0.f ? g_disc : 0.f;
            g_b += g_dpr * (2.f * b);
            const float g_a = -4.f * c * g_dpr;
            g_c += -4.f * a * g_dpr;
            // c = -s dy ; b = h d0 - dy T ; a = dy T + h (s - d0)
            g_s += -g_c * dy;
            float g_dy = -g_c * s_k;
            g_h += g_b * d_k;
            g_d0 += g_b * h_k;
            g_dy -= g_b * T;
            float g_T = -g_b * dy;
            g_dy += g_a * T;
            g_T += g_a * dy;
            g_h += g_a * (s_k - d_k);
            g_s += g_a * h_k;
            g_d0 -= g_a * h_k;
            g_d0 += g_T;
            g_d1 += g_T;
            g_s -= 2.f * g_T;
            g_v += g_dy;
            g_y -= g_dy;
        }
    } else {
        const float xp = (v - x_k) / wc;
        const float xi = tclamp(xp, 0.f, 1.f);
        const float omx = 1.f - xi;
        const float A = xi * omx;
        const float T = d_k1 + d_k - 2.f * s_k;
        const float denp = s_k + T * A;
        const float den = tclamp_min(denp, eps);
        const float P = s_k * (xi * xi) + d_k * A;
        const float num = h_k * P;
        o = y_k + num / den;
        const float Q = d_k1 * (xi * xi) + 2.f * s_k * A + d_k * (omx * omx);
        const float nd = (s_k * s_k) * Q;
        const float den2 = den * den;
        const float den2c = tclamp_min(den2, eps);
        const float q = nd / den2c;
        l = logf(tclamp_min(q, eps));
        const bool fo = !nonfinite(o), fl = !nonfinite(l);
        const float gO = fo ? go : 0.f;
        const float gL = fl ? gl : 0.f;
        g_v = fo ? 0.f : go;
        const float g_q = q >= eps ? gL / q : 0.f;
        const float g_nd = g_q / den2c;
        const float g_den2 = den2 >= eps ? -g_q * nd / (den2c * den2c) : 0.f;
        float g_den = g_den2 * (2.f * den);
        g_y += gO;
        const float g_num = gO / den;
        g_den += -gO * num / (den * den);
        const float g_denp = denp >= eps ? g_den : 0.f;
        g_s += g_denp;
        const float g_T = g_denp * A;
        float g_A = g_denp * T;
        g_d1 += g_T;
        g_d0 += g_T;
        g_s -= 2.f * g_T;
        g_h += g_num * P;
        const float g_P = g_num * h_k;
        g_s += g_P * (xi * xi);
        float g_xi = g_P * s_k * (2.f * xi);
        g_d0 += g_P * A;
        g_A += g_P * d_k;
        g_s += g_nd * Q * (2.f * s_k);
        const float g_Q = g_nd * (s_k * s_k);
        g_d1 += g_Q * (xi * xi);
        g_xi += g_Q * d_k1 * (2.f * xi);
        g_s += g_Q * (2.f * A);
        g_A += g_Q * (2.f * s_k);
        g_d0 += g_Q * (omx * omx);
        float g_omx = g_Q * d_k * (2.f * omx);
        g_xi += g_A * omx;
        g_omx += g_A * xi;
        g_xi -= g_omx;
        const float g_xp = (xp >= 0.f && xp <= 1.f) ? g_xi : 0.f;
        g_v += g_xp / wc;
        g_x -= g_xp / wc;
        g_w -= g_xp * (v - x_k) / (wc * wc);
    }
    // s = h / clamp(w, eps)
    g_h += g_s / wc;
    g_w -= g_s * h_k / (wc * wc);
    out = nonfinite(o) ? v : o;
    gv = g_v;

    // ---- this half's side: scatter to the bin arrays, knot differences, cumsum, softmax ----
    const float g_val = hi ? g_h : g_w, g_knot = hi ? g_y : g_x;
    float gval[K], gc[K + 1];
#pragma unroll
    for (int k = 0; k <= K; ++k) {
        const bool s0 = (k == bin);
        if (k < K) gval[k] = s0 ? g_val : 0.f;
        gc[k] = s0 ? g_knot : 0.f;
    }
    // val = clamp(diff(knot), eps): the knot differences
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const float a = wd[k] >= eps ? gval[k] : 0.f;
        gc[k + 1] += a;
        gc[k] -= a;
    }
    // knots 0 and K are pinned (in-place assignment): no gradient. knot_j = 2B cumsum_{i<j} val'_i - B.
    float gpv[K];
    {
        float a = 0.f;
#pragma unroll
        for (int i = K - 1; i >= 0; --i) {
            gpv[i] = a;
            if (i >= 1) a += C.two_bound * gc[i];
        }
    }
    // val' = clamp(min + c * softmax(u), eps) -> softmax backward
    {
        const float cs = hi ? C.ch : C.cw;
        float dot = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            gpv[k] = pre[k] >= eps ? gpv[k] * cs : 0.f;
            dot += gpv[k] * sm[k];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) gs[k] = sm[k] * (gpv[k] - dot);
    }
    // derivatives: d_{k+1} = clamp(min_d + softplus(u_k), eps); ends padded with 1 (no gradient)
#pragma unroll
    for (int t = 0; t < ND; ++t) {
        const int k0 = 2 * t, k1 = 2 * t + 1;
        const int k = hi ? k1 : k0;
        if (hi && k1 >= K - 1) continue;
        const float u = pick(2 * K + k0, 2 * K + (k1 < K - 1 ? k1 : k0));
        const float z = exp_safe(u);
        const float sp = u > 20.f ? 1.f : z / (z + 1.f);
        const float gdk = (k + 1 == bin) ? g_d0 : ((k + 1 == bin + 1) ? g_d1 : 0.f);
        gd[t] = dpre[t] >= eps ? gdk * sp : 0.f;
    }
}

// delta3 of a parameter tile in accumulator layout from the split adjoint: lane (col, h),
// register r needs row R = crow(r, h) of sample col. Rows < K are held by the h = 0 half (widths),
// K..2K-1 by h = 1 (heights), derivative row 2K + k by half k & 1; each lane sends the partner the
// rows it holds that the partner needs (one v_permlane32_swap per register).
template <int K>
__device__ __forceinline__ void split_grads_to_tile(const float (&gs)[K], const float (&gd)[K / 2], f32x16& e) {
    const bool hi = (threadIdx.x & 32) != 0;
    auto held = [&](int R, bool as_hi) -> float {  // value this lane holds for row R (0 if none)
        if (R < K) return as_hi ? 0.f : gs[R];
        if (R < 2 * K) return as_hi ? gs[R - K] : 0.f;
        if (R < 3 * K - 1) {
            const int k = R - 2 * K;
            return ((k & 1) == (as_hi ? 1 : 0)) ? gd[k >> 1] : 0.f;
        }
        return 0.f;
    };
    auto owns = [&](int R, bool as_hi) -> bool {
        if (R < K) return !as_hi;
        if (R < 2 * K) return as_hi;
        if (R < 3 * K - 1) return ((R - 2 * K) & 1) == (as_hi ? 1 : 0);
        return true;  // padding rows: zero, no exchange needed
    };
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int R0 = crow(r, 0), R1 = crow(r, 1);
        // the partner (other half) needs its row for r: R1 if I am h = 0, R0 if I am h = 1
        const float send = hi ? held(R0, true) : held(R1, false);
        const float recv = halves_other(send, send);
        const float mine = hi ? held(R1, true) : held(R0, false);
        const bool own = hi ? owns(R1, true) : owns(R0, false);
        e[r] = own ? mine : recv;
    }
}

template <int HT, int K, int NTMAX, bool INV>
__global__ __launch_bounds__(256) void spline_bwd_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, const float* __restrict__ gy,
    const float* __restrict__ gld, float* __restrict__ gx, float* __restrict__ part, int64_t B, int d,
    SplineConsts C, int64_t ntiles) {
#pragma clang fp contract(off)
    constexpr SplineBwdLayout BL = spline_bwd_layout(HT, NTMAX);
    constexpr SplineLayout L = BL.F;
    constexpr SplineGrad GL = spline_grad_layout(HT, NTMAX);
    constexpr int Hp = 32 * HT;
    static_assert(GL.total <= BL.total, "reduction buffer must fit the pack region");
    extern __shared__ f32x4 lds4[];
    float* sm = reinterpret_cast<float*>(lds4);
    float* tbuf_all = sm + BL.total;            // 4 x 32 x kTS
    float* xbuf_all = tbuf_all + 4 * 32 * kTS;  // 4 x 32 x 8  (xa rows of the tile)
    {
        const f32x4* src = reinterpret_cast<const f32x4*>(packed);
        for (int i = threadIdx.x; i < BL.total / 4; i += 256) lds4[i] = src[i];
    }
    __syncthreads();
    const int lane = lane_id(), h = lane >> 5, col = lane & 31, wave = threadIdx.x >> 6;
    float* tbuf = tbuf_all + wave * 32 * kTS;
    float* xbuf = xbuf_all + wave * 32 * 8;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    const int KS1 = (d + 1) / 2;
    const int NT = (int)sm[L.meta];
    float mk[8], mkb[4];
#pragma unroll
    for (int j = 0; j < 8; ++j) mk[j] = j < d ? sm[L.mask + j] : 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) mkb[ks] = (2 * ks + h < d) ? sm[L.mask + 2 * ks + h] : 0.f;

    // the tile's sample row per lane (both lane halves hold sample `col` of the tile)
    struct Fetch {
        float xr[8];
        float gyr[8];
        float gl;
    };
    auto fetch = [&](int64_t t, Fetch& f) {
        const int64_t s = t * 32 + col;
        const bool ok = t < ntiles && s < B;
        const int64_t sc = ok ? s : 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float a = j < d ? in[sc * d + j] : 0.f;
            const float b = j < d ? gy[sc * d + j] : 0.f;
            f.xr[j] = ok ? a : 0.f;
            f.gyr[j] = ok ? b : 0.f;
        }
        const float g = gld[sc];
        f.gl = ok ? g : 0.f;
    };

    // weight-gradient accumulators (per lane, over the wave's tiles)
    f32x16 a_w3[NTMAX][HT], a_w2[HT][HT];
    float a_b3[NTMAX], a_b2[HT], a_b1[HT], a_w1[HT][8];
#pragma unroll
    for (int ht = 0; ht < HT; ++ht) {
        a_b2[ht] = a_b1[ht] = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) a_w1[ht][j] = 0.f;
#pragma unroll
        for (int kt = 0; kt < HT; ++kt)
#pragma unroll
            for (int r = 0; r < 16; ++r) a_w2[ht][kt][r] = 0.f;
#pragma unroll
        for (int t = 0; t < NTMAX; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) a_w3[t][ht][r] = 0.f;
    }
#pragma unroll
    for (int t = 0; t < NTMAX; ++t) a_b3[t] = 0.f;

    int64_t tile = (int64_t)blockIdx.x * 4 + wave;
    Fetch cur;
    fetch(tile, cur);
    for (; tile < ntiles; tile += nwaves) {
        const int64_t so = tile * 32 + col;
        const float* P = sm + opaque_zero();
        Fetch nxt;
        fetch(tile + nwaves, nxt);
        float xb[4];  // layer-1 B operand xa[sample col][2ks + h]
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const float v0 = cur.xr[2 * ks], v1 = cur.xr[2 * ks + 1];
            xb[ks] = (h ? v1 : v0) * mkb[ks];
        }
        if (h == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) xbuf[col * 8 + j] = cur.xr[j] * mk[j];
        }

        f32x16 h1[HT], h2[HT];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
            f32x16 a = load_bias16(P + L.b1 + ht * 32, h);
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
                if (ks < KS1) a = mfma32(P[L.w1 + (ht * 4 + ks) * 64 + lane], xb[ks], a);
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = trelu(a[r]);
            h1[ht] = a;
        }
#pragma unroll
        for (int hto = 0; hto < HT; ++hto) {
            f32x16 a = load_bias16(P + L.b2 + hto * 32, h);
#pragma unroll
            for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) {
                    const f32x4 w = *reinterpret_cast<const f32x4*>(P + L.w2 + (((hto * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) a = mfma32(w[rr], h1[kt][4 * rq + rr], a);
                }
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = trelu(a[r]);
            h2[hto] = a;
        }

        // the layer guard z = where(nonfinite(z), 0, z) needs z: conditioning dims pass x through
        float zr[8], gvx[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            zr[j] = cur.xr[j];
            gvx[j] = 0.f;
        }
        f32x16 g2[HT];  // dL/dh2
#pragma unroll
        for (int kt = 0; kt < HT; ++kt)
#pragma unroll
            for (int r = 0; r < 16; ++r) g2[kt][r] = 0.f;

#pragma unroll
        for (int t = 0; t < NTMAX; ++t) {
            if (t < NT) {
                f32x16 a = load_bias16(P + L.b3 + t * 32, h);
#pragma unroll
                for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                    for (int rq = 0; rq < 4; ++rq) {
                        const f32x4 w = *reinterpret_cast<const f32x4*>(P + L.w3 + (((t * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) a = mfma32(w[rr], h2[kt][4 * rq + rr], a);
                    }
                // every lane gathers all 32 parameter rows of sample `col` (halves redundant)
                float prm[32];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float o = halves_other(a[r], a[r]);
                    prm[crow(r, 0)] = h ? o : a[r];
                    prm[crow(r, 1)] = h ? a[r] : o;
                }
                const int dt = (int)P[L.tdim + t];
                float v = 0.f, go = 0.f;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    v = (j == dt) ? cur.xr[j] : v;
                    go = (j == dt) ? cur.gyr[j] : go;
                }
                float o, gs[K], gd[K / 2], gvs;
                // z_dt is non-finite only when the spline fell back to a non-finite input: the
                // layer guard then blocks the output gradient
                rq_spline_adjoint<K, INV>(v, prm, C, nonfinite(v) ? 0.f : go, cur.gl, o, gs, gd, gvs);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    zr[j] = (j == dt) ? o : zr[j];
                    gvx[j] = (j == dt) ? gvs : gvx[j];
                }
                f32x16 e;  // delta3 of tile t in accumulator layout
                split_grads_to_tile<K>(gs, gd, e);
                const f32x4* wt = reinterpret_cast<const f32x4*>(P + BL.w3t) + lane;
#pragma unroll
                for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                    for (int rq = 0; rq < 4; ++rq) {
                        const f32x4 w = wt[((kt * NTMAX + t) * 4 + rq) * 64];
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) g2[kt] = mfma32(w[rr], e[4 * rq + rr], g2[kt]);
                    }
                float Te[16];
                transpose_tile(tbuf, e, Te);
                float sb = 0.f;
#pragma unroll
                for (int q = 0; q < 16; ++q) sb += Te[q];
                a_b3[t] += sb;
#if NFX_SBWD_EXPT != 2
#pragma unroll
                for (int kt = 0; kt < HT; ++kt) {
                    float Th[16];
                    transpose_tile(tbuf, h2[kt], Th);
#pragma unroll
                    for (int q = 0; q < 16; ++q) a_w3[t][kt] = mfma32(Te[q], Th[q], a_w3[t][kt]);
                }
#endif
            }
        }
        // layer 2: delta2 = relu'(h2) g2; dW2 += delta2 h1^T; dL/dh1 = W2^T delta2
        float Te2[HT][16];
#pragma unroll
        for (int o2 = 0; o2 < HT; ++o2) {
#pragma unroll
            for (int r = 0; r < 16; ++r) g2[o2][r] = h2[o2][r] > 0.f ? g2[o2][r] : 0.f;
            transpose_tile(tbuf, g2[o2], Te2[o2]);
            float sb = 0.f;
#pragma unroll
            for (int q = 0; q < 16; ++q) sb += Te2[o2][q];
            a_b2[o2] += sb;
        }
#if NFX_SBWD_EXPT != 2
#pragma unroll
        for (int kt = 0; kt < HT; ++kt) {
            float Th[16];
            transpose_tile(tbuf, h1[kt], Th);
#pragma unroll
            for (int o2 = 0; o2 < HT; ++o2)
#pragma unroll
                for (int q = 0; q < 16; ++q) a_w2[o2][kt] = mfma32(Te2[o2][q], Th[q], a_w2[o2][kt]);
        }
#endif
        float gxp[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) gxp[j] = 0.f;
        {
            const f32x4* wt = reinterpret_cast<const f32x4*>(P + BL.w2t) + lane;
#pragma unroll
            for (int kt = 0; kt < HT; ++kt) {
                f32x16 g1;
#pragma unroll
                for (int r = 0; r < 16; ++r) g1[r] = 0.f;
#pragma unroll
                for (int o2 = 0; o2 < HT; ++o2)
#pragma unroll
                    for (int rq = 0; rq < 4; ++rq) {
                        const f32x4 w = wt[((kt * HT + o2) * 4 + rq) * 64];
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) g1 = mfma32(w[rr], g2[o2][4 * rq + rr], g1);
                    }
                // layer 1: delta1 = relu'(h1) g1; dW1 += delta1 xa^T; dL/dxa = W1^T delta1
#pragma unroll
                for (int r = 0; r < 16; ++r) g1[r] = h1[kt][r] > 0.f ? g1[r] : 0.f;
                float Te[16];
                transpose_tile(tbuf, g1, Te);
                float sb = 0.f;
#pragma unroll
                for (int q = 0; q < 16; ++q) sb += Te[q];
                a_b1[kt] += sb;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (j < d) {
                        float w = 0.f;
#pragma unroll
                        for (int q = 0; q < 16; ++q) w = fmaf(xbuf[(16 * h + q) * 8 + j], Te[q], w);
                        a_w1[kt][j] += w;
                        const f32x16 wc = load_bias16(P + BL.w1c + (j * HT + kt) * 32, h);
#pragma unroll
                        for (int r = 0; r < 16; ++r) gxp[j] = fmaf(wc[r], g1[r], gxp[j]);
                    }
                }
            }
        }
        float ga[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) ga[j] = halves_sum(gxp[j], gxp[j]);  // both halves: sample col
        if (h == 0 && so < B) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < d) {
                    const bool zfin = !nonfinite(zr[j]);
                    // conditioning dims: z_j = x_j (clone) + the param-net path x_a = x * mask;
                    // transformed dims: the spline input gradient
                    const float direct = mk[j] != 0.f ? (zfin ? cur.gyr[j] : 0.f) : gvx[j];
                    gx[so * d + j] = direct + mk[j] * ga[j];
                }
            }
        }
        cur = nxt;
    }

    // ---- workgroup combine (wave order) into LDS, one partial per workgroup ----
    __syncthreads();
    float* red = sm;
    for (int rnd = 0; rnd < 4; ++rnd) {
        if (wave == rnd) {
            auto put = [&](int idx, float v) { red[idx] = rnd ? red[idx] + v : v; };
#pragma unroll
            for (int ht = 0; ht < HT; ++ht) {
                const float b1 = halves_sum(a_b1[ht], a_b1[ht]);
                const float b2 = halves_sum(a_b2[ht], a_b2[ht]);
                if (h == 0) {
                    put(GL.b1 + 32 * ht + col, b1);
                    put(GL.b2 + 32 * ht + col, b2);
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float w = halves_sum(a_w1[ht][j], a_w1[ht][j]);
                    if (h == 0) put(GL.w1 + j * Hp + 32 * ht + col, w);
                }
#pragma unroll
                for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) put(GL.w2 + (32 * ht + crow(r, h)) * Hp + 32 * kt + col, a_w2[ht][kt][r]);
            }
#pragma unroll
            for (int t = 0; t < NTMAX; ++t) {
                const float b3 = halves_sum(a_b3[t], a_b3[t]);
                if (h == 0) put(GL.b3 + t * 32 + col, b3);
#pragma unroll
                for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) put(GL.w3 + (t * 32 + crow(r, h)) * Hp + 32 * kt + col, a_w3[t][kt][r]);
            }
        }
        __syncthreads();
    }
    float* pw = part + (int64_t)blockIdx.x * GL.total;
    for (int i = threadIdx.x; i < GL.total; i += 256) pw[i] = red[i];
}

typedef void (*spline_bwd_kernel_t)(const float*, const float*, const float*, const float*, float*, float*,
                                    int64_t, int, SplineConsts, int64_t);

template <int HT>
spline_bwd_kernel_t spline_bwd_pick_ht(int K, int inv);

// Transformed-dimension tiles one launch handles (their dW3 accumulators stay in registers).
constexpr int spline_bwd_ntmax(int HT) { return HT == 1 ? 2 : 1; }

__host__ __device__ constexpr size_t spline_bwd_lds(int HT) {
    return (size_t)(spline_bwd_layout(HT, spline_bwd_ntmax(HT)).total + 4 * 32 * kTS + 4 * 32 * 8) * sizeof(float);
}

}  // namespace nfx
