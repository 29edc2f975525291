// Fused rational-quadratic-spline coupling layer (SplineCouplingLayer) for gfx950.
//
// Reference: src/flows/spline/spline_coupling_layer.py
//   param_net Linear(d,H) ReLU Linear(H,H) ReLU Linear(H, d(3K-1))        :56-62
//   params.view(-1, d, 3K-1) split [K | K | K-1]                         :66-76
//   forward :96-137 / inverse :139-180, spline core :182-309, guards :130-135/:173-178/:306-307
//
// One kernel = one layer: the param MLP on fp32 MFMA (32x32x2; hidden activations stay in
// accumulator registers), the output layer on MFMA with ONE 32-row tile per transformed
// dimension (its 3K-1 <= 32 parameters), a v_permlane32_swap that leaves every lane holding
// all 32 parameter rows of its own sample, then the whole spline in registers: softmax,
// min-width/height affine, knots (cumsum accumulated in float64 exactly like ATen's CPU cumsum),
// pinned ends, softplus derivatives, bin search, gather-by-select, the RQ forward or the
// citardauq inverse, and the reference's three guard stages. HBM traffic per sample is the
// x row in, the y row out and the log-det read-modify-write (8d + 8 bytes).
#pragma once
#include <type_traits>

#include "nfx_common.h"

namespace nfx {

__host__ __device__ constexpr int sp_up4(int v) { return (v + 3) & ~3; }

// Packed image (floats):
//   w1 [HT][KS][64]        layer-1 A operand, KS = spline_ks1(d) k-steps (4, padded, for d <= 8)
//   b1 [HT][2][16]         (bias of accumulator register r, lane-half h)
//   w2 [HT][HT][4][64][4]
//   b2 [HT][2][16]
//   w3 [d][HT][4][64][4]   output tile t = t-th transformed dim: row i = parameter i
//   b3 [d][2][16]
//   mask [max(8,d)], tdim [max(8,d)] (indices of the transformed dims, as floats), meta [4]
//   (meta[0] = NT)
struct SplineLayout {
    int HT, NT;  // NT here = capacity (d); the live count is meta[0]
    int w1, b1, w2, b2, w3, b3, mask, tdim, meta, total;
};

// layer-1 k-steps of the packed image: 4 (d <= 8, padded) or ceil(d/2) (wide kernel)
__host__ __device__ constexpr int spline_ks1(int d) { return d <= 8 ? 4 : (d + 1) / 2; }

__host__ __device__ constexpr SplineLayout spline_layout(int HT, int d) {
    SplineLayout L{};
    const int NT = d;
    L.HT = HT;
    L.NT = NT;
    int o = 0;
    L.w1 = o; o += HT * spline_ks1(d) * 64;
    L.b1 = o; o += HT * 32;
    L.w2 = o; o += HT * HT * 16 * 64;
    L.b2 = o; o += HT * 32;
    L.w3 = o; o += NT * HT * 16 * 64;
    L.b3 = o; o += NT * 32;
    L.mask = o; o += sp_up4(d > 8 ? d : 8);
    L.tdim = o; o += sp_up4(d > 8 ? d : 8);
    L.meta = o; o += 4;
    L.total = o;
    return L;
}

struct SplineConsts {
    float bound;        // B (:18)
    float two_bound;    // 2*B
    float min_w, cw;    // min_bin_width, (1 - min_bin_width*K) (:205)
    float min_h, ch;    // min_bin_height, (1 - min_bin_height*K) (:218)
    float min_d;        // min_derivative (:230)
    int rescale;        // data_min/data_max given (:78-94)
    float rs_to_scale, rs_lo;   // 2B/(hi-lo), lo
    float rs_from_scale;        // (hi-lo)/(2B)
};

// Scalars exactly as the reference's Python-float expressions round them into fp32 ops.
inline SplineConsts spline_consts(int K, float bound, float min_bin_width, float min_bin_height, float min_derivative,
                                  int rescale, float data_min, float data_max) {
    SplineConsts C;
    C.bound = bound;
    C.two_bound = (float)(2.0 * (double)bound);
    C.min_w = min_bin_width;
    C.cw = (float)(1.0 - (double)min_bin_width * K);
    C.min_h = min_bin_height;
    C.ch = (float)(1.0 - (double)min_bin_height * K);
    C.min_d = min_derivative;
    C.rescale = rescale ? 1 : 0;
    C.rs_lo = data_min;
    C.rs_to_scale = rescale ? (float)((2.0 * bound) / ((double)data_max - (double)data_min)) : 1.f;
    C.rs_from_scale = rescale ? (float)(((double)data_max - (double)data_min) / (2.0 * bound)) : 1.f;
    return C;
}

// torch softplus (beta=1, threshold=20): x > 20 ? x : log1p(exp(x)).
// log1p(u) = log(w) * u / (w - 1) with w = fl(1 + u) (exact u when w == 1): the rounding error
// of 1 + u cancels in the ratio, giving log1p to a few ulp for every u > 0 at ~1/6 the cost of
// the double-float log1pf (which dominated the spline's vector time).
__device__ __forceinline__ float tsoftplus(float x) {
#pragma clang fp contract(off)
    const float u = exp_safe(x);
    const float w = 1.f + u;
    const float wm1 = w - 1.f;
    const float l = wm1 == 0.f ? u : logf(w) * (u * __builtin_amdgcn_rcpf(wm1));
    return x > 20.f ? x : l;
}

// ---- VALU-lean helpers of the forward spline (the fp32 pipe is shared with the fp32 MFMAs, so
// every vector instruction here adds to the layer's time; DESIGN.md "roofline") ----
// a / b for b > 0 finite and a/b in the normal range (the spline's divisors are all clamped to
// >= eps): the hardware reciprocal plus one Newton correction of the quotient (Markstein),
// within 1 ulp of the correctly rounded quotient and usually equal to it — 4 instructions
// instead of the 10 of the IEEE division sequence (div_scale/div_fmas/div_fixup).
__device__ __forceinline__ float div_fast(float a, float b) {
    const float r = __builtin_amdgcn_rcpf(b);
    const float q = a * r;
    return __builtin_fmaf(__builtin_fmaf(-b, q, a), r, q);
}
// log(x) for normal x > 0 (the callers clamp to >= 1e-8 or pass 1 + u): hardware log2 * ln2,
// ~2 ulp.
__device__ __forceinline__ float log_fast(float x) { return __builtin_amdgcn_logf(x) * 0.693147182f; }

// exp_safe on a pair (widths, heights): the compensated exp2 of exp_fast with the arithmetic
// as packed fp32 (v_pk_mul/v_pk_fma), the two v_exp_f32 and the -inf clamp per element.
__device__ __forceinline__ f32x2 exp_safe2(f32x2 x) {
#ifdef NFX_SPLINE_SCALAR
    return f32x2{exp_safe(x.x), exp_safe(x.y)};
#else
    x = __builtin_elementwise_maximum(x, f32x2{-128.f, -128.f});
    const f32x2 c = {1.44269502f, 1.44269502f};
    const f32x2 t = x * c;
    const f32x2 e = __builtin_elementwise_fma(x, f32x2{1.9259629e-8f, 1.9259629e-8f},
                                              __builtin_elementwise_fma(x, c, -t));
    const f32x2 r = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
    return __builtin_elementwise_fma(r, e * f32x2{0.693147182f, 0.693147182f}, r);
#endif
}

// torch softplus (threshold 20) on a pair, log1p as in tsoftplus with the hardware log.
__device__ __forceinline__ f32x2 tsoftplus2(f32x2 x) {
#pragma clang fp contract(off)
    const f32x2 u = exp_safe2(x);
    const f32x2 w = u + f32x2{1.f, 1.f};
    const f32x2 wm1 = w - f32x2{1.f, 1.f};
    f32x2 l;
    l.x = wm1.x == 0.f ? u.x : log_fast(w.x) * (u.x * __builtin_amdgcn_rcpf(wm1.x));
    l.y = wm1.y == 0.f ? u.y : log_fast(w.y) * (u.y * __builtin_amdgcn_rcpf(wm1.y));
    return f32x2{x.x > 20.f ? x.x : l.x, x.y > 20.f ? x.y : l.y};
}

// One RQ spline evaluation of SplineCouplingLayer._rational_quadratic_spline for a single
// input v with its 3K-1 unnormalised parameters p[] (:182-309, per element).
// Returns the spline-level guarded output (NaN/Inf -> input, :306) and log|det| (-> 0, :307).
// Same operation order as the reference (contraction off); work the reference spends on bins
// the sample is not in is skipped: the widths/heights of every bin are needed for the knots,
// but only the selected bin's two derivatives go through softplus (the reference evaluates
// all K-1), and the knots of the bin (not the width array) are gathered by a select chain on
// the monotone comparisons `knot_k <= v` (= searchsorted(right=True) - 1, clamped).
template <int K, bool INV>
__device__ __forceinline__ void rq_spline_elem(float v, const float (&p)[32], const SplineConsts C,
                                               float& out, float& lad) {
#pragma clang fp contract(off)
    const float eps = 1e-8f;
    const float B = C.bound;
    out = v;
    lad = 0.f;
    if (v >= -B && v <= B) {
        // softmax of widths (.x) and heights (.y) together: max-subtracted exp, times the
        // reciprocal of the sum (ATen's vectorised softmax), then the min-width affine (:204-219)
        f32x2 m = {p[0], p[K]};
#pragma unroll
        for (int k = 1; k < K; ++k) m = __builtin_elementwise_maximum(m, f32x2{p[k], p[K + k]});
        f32x2 e[K];
        f32x2 s = {0.f, 0.f};
#pragma unroll
        for (int k = 0; k < K; ++k) {
#ifdef NFX_SPLINE_SCALAR
            e[k] = f32x2{exp_safe(p[k] - m.x), exp_safe(p[K + k] - m.y)};
            s.x = s.x + e[k].x;
            s.y = s.y + e[k].y;
#else
            e[k] = exp_safe2(f32x2{p[k], p[K + k]} - m);
            s = s + e[k];
#endif
        }
        const f32x2 inv = {div_fast(1.f, s.x), div_fast(1.f, s.y)};
        const f32x2 mins = {C.min_w, C.min_h}, scl = {C.cw, C.ch};
        // knots: ATen's CPU cumsum accumulates float in double and rounds each prefix (:208-213)
        float cwk[K + 1], chk[K + 1];
        {
            double aw = 0.0, ah = 0.0;
            const f32x2 tb = {C.two_bound, C.two_bound}, nb = {-B, -B};
#pragma unroll
            for (int k = 0; k < K; ++k) {
#ifdef NFX_SPLINE_SCALAR
                const float wx = tclamp_min(C.min_w + C.cw * (e[k].x * inv.x), eps);
                const float wy = tclamp_min(C.min_h + C.ch * (e[k].y * inv.y), eps);
                aw += (double)wx;
                ah += (double)wy;
                cwk[k + 1] = C.two_bound * (float)aw + (-B);
                chk[k + 1] = C.two_bound * (float)ah + (-B);
#else
                const f32x2 wv = __builtin_elementwise_maximum(mins + scl * (e[k] * inv), f32x2{eps, eps});
                aw += (double)wv.x;
                ah += (double)wv.y;
                const f32x2 kn = tb * f32x2{(float)aw, (float)ah} + nb;
                cwk[k + 1] = kn.x;
                chk[k + 1] = kn.y;
#endif
            }
            cwk[0] = -B; cwk[K] = B;
            chk[0] = -B; chk[K] = B;
        }
        // bin = last k in [0, K-1] with knot_k <= v (knots non-decreasing; the pinned knot_0 =
        // -B <= v): gather the bin's knots and the raw logits of its two derivatives
        float x_k = cwk[0], x_k1 = cwk[1], y_k = chk[0], y_k1 = chk[1];
        float ua = 0.f, ub = p[2 * K];
        bool in0 = true, inl = (K == 1);
#pragma unroll
        for (int k = 1; k < K; ++k) {
            const bool c = (INV ? chk[k] : cwk[k]) <= v;
            x_k = c ? cwk[k] : x_k;
            x_k1 = c ? cwk[k + 1] : x_k1;
            y_k = c ? chk[k] : y_k;
            y_k1 = c ? chk[k + 1] : y_k1;
            ua = c ? p[2 * K + k - 1] : ua;
            if (k < K - 1) ub = c ? p[2 * K + k] : ub;
            if (k == 1) in0 = !c;
            if (k == K - 1) inl = c;
        }
        // derivatives d_k, d_{k+1}: clamp(min_d + softplus(u), eps), pinned to 1 at both ends
        const f32x2 sp = tsoftplus2(f32x2{ua, ub});
        const float d_k = in0 ? 1.f : tclamp_min(C.min_d + sp.x, eps);
        const float d_k1 = inl ? 1.f : tclamp_min(C.min_d + sp.y, eps);
        const float w_k = tclamp_min(x_k1 - x_k, eps);   // :214-215 (w = diff of pinned knots)
        const float h_k = tclamp_min(y_k1 - y_k, eps);   // :227-228
        const float s_k = div_fast(h_k, w_k);            // (w_k >= eps already: the clamp at :260 is a no-op)
        float o, l;
        if constexpr (INV) {
            // citardauq root (:266-281)
            const float dy = v - y_k;
            const float t = d_k + d_k1 - 2.f * s_k;
            const float a = dy * t + h_k * (s_k - d_k);
            const float b = h_k * d_k - dy * t;
            const float c = -s_k * dy;
            const float disc = tclamp_min(b * b - 4.f * a * c, 0.f);
            float den = -b - __builtin_amdgcn_sqrtf(disc);
            den = fabsf(den) < eps ? eps : den;
            const float xi = tclamp((2.f * c) / den, 0.f, 1.f);
            o = xi * w_k + x_k;
            const float omx = 1.f - xi;
            const float dld = s_k + (d_k1 + d_k - 2.f * s_k) * xi * omx;
            const float nld = (s_k * s_k) * (d_k1 * (xi * xi) + 2.f * s_k * xi * omx + d_k * (omx * omx));
            l = -log_fast(tclamp_min(nld, eps)) + 2.f * log_fast(tclamp_min(dld, eps));
        } else {
            // forward (:283-293)
            const float xi = tclamp(div_fast(v - x_k, w_k), 0.f, 1.f);
            const float omx = 1.f - xi;
            const float den = tclamp_min(s_k + (d_k1 + d_k - 2.f * s_k) * xi * omx, eps);
            const float num = h_k * (s_k * (xi * xi) + d_k * xi * omx);
            o = y_k + div_fast(num, den);
            const float nd = (s_k * s_k) * (d_k1 * (xi * xi) + 2.f * s_k * xi * omx + d_k * (omx * omx));
            l = log_fast(tclamp_min(div_fast(nd, tclamp_min(den * den, eps)), eps));
        }
        out = o;
        lad = l;
    }
    if (nonfinite(out)) out = v;      // :306
    if (nonfinite(lad)) lad = 0.f;    // :307
}

// The layer's conditioner MLP and splines for one unit (TILES = 2: a 64-sample chunk, 1: a
// 32-sample half chunk) on the lane's own sample: xb = the layer-1 B operands (rescaled and
// masked), xr = the lane's raw row. Returns the layer output row before the layer-level guard
// (transformed dims replaced by the spline outputs, spline-guarded) and the spline log-det sum.
// The streaming chain's copy (nfx_spline_schain.hip) of spline_coupling_kernel's unit body, the
// same operations in the same order (bit-identical results); the per-layer kernel keeps its own
// inline body (factoring it out perturbed its register allocation: K = 8 spilled 15 VGPRs).
template <int HT, int K, int DIR, int DMAX, int TILES>
__device__ __forceinline__ void spline_unit_apply(const float* P, const SplineLayout& L,
                                                  const SplineConsts& C, int KS1, int NT, const float (&xb)[2][4],
                                                  const float (&xr)[DMAX], float (&y)[DMAX], float& ld) {
#pragma clang fp contract(off)
    const int lane = lane_id(), h = lane >> 5;
    // Layer 1 + ReLU
    f32x16 h1[HT][2];
#pragma unroll
    for (int ht = 0; ht < HT; ++ht) {
        f32x16 a0, a1;
        load_bias16_x2(P + L.b1 + ht * 32, h, a0, a1);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            if (ks < KS1) {
                const float w = P[L.w1 + (ht * 4 + ks) * 64 + lane];
                a0 = mfma32(w, xb[0][ks], a0);
                if constexpr (TILES == 2) a1 = mfma32(w, xb[1][ks], a1);
            }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            a0[r] = trelu(a0[r]);
            a1[r] = trelu(a1[r]);
        }
        h1[ht][0] = a0;
        h1[ht][1] = a1;
    }
    // Layer 2 + ReLU
    f32x16 h2[HT][2];
#pragma unroll
    for (int hto = 0; hto < HT; ++hto) {
        f32x16 a0, a1;
        load_bias16_x2(P + L.b2 + hto * 32, h, a0, a1);
#pragma unroll
        for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
            for (int rq = 0; rq < 4; ++rq) {
                const f32x4 w = *reinterpret_cast<const f32x4*>(
                    P + L.w2 + (((hto * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    a0 = mfma32(w[rr], h1[kt][0][4 * rq + rr], a0);
                    if constexpr (TILES == 2) a1 = mfma32(w[rr], h1[kt][1][4 * rq + rr], a1);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            a0[r] = trelu(a0[r]);
            a1[r] = trelu(a1[r]);
        }
        h2[hto][0] = a0;
        h2[hto][1] = a1;
    }

    #pragma unroll
    for (int j = 0; j < DMAX; ++j) y[j] = xr[j];
    ld = 0.f;
    for (int t = 0; t < NT; ++t) {
        // Layer 3, tile t: the 3K-1 parameters of transformed dim tdim[t].
        f32x16 a0, a1;
        load_bias16_x2(P + L.b3 + t * 32, h, a0, a1);
#pragma unroll
        for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
            for (int rq = 0; rq < 4; ++rq) {
                const f32x4 w = *reinterpret_cast<const f32x4*>(
                    P + L.w3 + (((t * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    a0 = mfma32(w[rr], h2[kt][0][4 * rq + rr], a0);
                    if constexpr (TILES == 2) a1 = mfma32(w[rr], h2[kt][1][4 * rq + rr], a1);
                }
            }
        }
        // Half-wave exchange: afterwards every lane holds rows 0..31 of its own sample.
        float prm[32];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(a0[r]), __float_as_uint(a1[r]),
                                                       false, false);
            prm[crow(r, 0)] = __uint_as_float(sw[0]);
            prm[crow(r, 1)] = __uint_as_float(sw[1]);
        }
        const int dt = (int)P[L.tdim + t];
        float v = 0.f;
#pragma unroll
        for (int j = 0; j < DMAX; ++j) v = (j == dt) ? xr[j] : v;
        if (C.rescale) v = C.rs_to_scale * (v - C.rs_lo) - C.bound;
        float o, l;
        rq_spline_elem<K, (DIR < 0)>(v, prm, C, o, l);
        if (C.rescale) o = (o + C.bound) * C.rs_from_scale + C.rs_lo;
#pragma unroll
        for (int j = 0; j < DMAX; ++j) y[j] = (j == dt) ? o : y[j];
        ld = (t == 0) ? l : ld + l;
    }
}

// spline_unit_apply with the two 32-sample tiles run one after the other through layers 1-3 (the
// same MFMAs on the same operands in the same order per tile, so bit-identical results): only one
// tile's hidden activations are live at a time (h1 + h2 of one tile, 64 VGPRs at H = 64, instead of
// both tiles' 128), which is what lets the 12-wave streaming chain (168 VGPRs per lane) hold its
// unit body without scratch spills. The layer weights are read from LDS once per tile.
template <int HT, int K, int DIR, int DMAX, int TILES>
__device__ __forceinline__ void spline_unit_apply_tseq(const float* P, const SplineLayout& L,
                                                       const SplineConsts& C, int KS1, int NT,
                                                       const float (&xb)[2][4], const float (&xr)[DMAX],
                                                       float (&y)[DMAX], float& ld) {
#pragma clang fp contract(off)
    const int lane = lane_id(), h = lane >> 5;
    f32x16 p3[2][DMAX];  // layer-3 outputs per tile and transformed-dim tile t < NT
#pragma unroll
    for (int tile = 0; tile < 2; ++tile) {
        if (tile == 1 && TILES == 1) {
            // (as spline_unit_apply: the absent tile's accumulators hold the bias)
#pragma unroll
            for (int t = 0; t < DMAX; ++t) p3[1][t] = load_bias16(P + L.b3 + t * 32 + opaque_zero(), h);
            break;
        }
        f32x16 h1[HT];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
            f32x16 a = load_bias16(P + L.b1 + ht * 32 + opaque_zero(), h);
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                if (ks < KS1) a = mfma32(P[L.w1 + (ht * 4 + ks) * 64 + lane], xb[tile][ks], a);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = trelu(a[r]);
            h1[ht] = a;
        }
        // (with one tile in flight a weight group feeds only 4 MFMAs, less than an LDS read's
        // latency: each group is read one group ahead)
        f32x16 h2[HT];
        auto w2at = [&](int q) {  // group q = (hto * HT + kt) * 4 + rq
            return *reinterpret_cast<const f32x4*>(P + L.w2 + (q * 64 + lane) * 4);
        };
        f32x4 wn = w2at(0);
#pragma unroll
        for (int hto = 0; hto < HT; ++hto) {
            f32x16 a = load_bias16(P + L.b2 + hto * 32 + opaque_zero(), h);
#pragma unroll
            for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) {
                    const int q = (hto * HT + kt) * 4 + rq;
                    const f32x4 w = wn;
                    if (q + 1 < HT * HT * 4) wn = w2at(q + 1);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) a = mfma32(w[rr], h1[kt][4 * rq + rr], a);
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = trelu(a[r]);
            h2[hto] = a;
        }
#pragma unroll
        for (int t = 0; t < DMAX; ++t) {
            if (t < NT) {
                f32x16 a = load_bias16(P + L.b3 + t * 32 + opaque_zero(), h);
                auto w3at = [&](int q) {  // group q = kt * 4 + rq of tile t
                    return *reinterpret_cast<const f32x4*>(P + L.w3 + ((t * HT * 4 + q) * 64 + lane) * 4);
                };
                f32x4 wn3 = w3at(0);
#pragma unroll
                for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
                    for (int rq = 0; rq < 4; ++rq) {
                        const int q = kt * 4 + rq;
                        const f32x4 w = wn3;
                        if (q + 1 < HT * 4) wn3 = w3at(q + 1);
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) a = mfma32(w[rr], h2[kt][4 * rq + rr], a);
                    }
                }
                p3[tile][t] = a;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < DMAX; ++j) y[j] = xr[j];
    ld = 0.f;
#pragma unroll
    for (int t = 0; t < DMAX; ++t) {
        if (t < NT) {
            // Half-wave exchange: afterwards every lane holds rows 0..31 of its own sample.
            float prm[32];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(p3[0][t][r]), __float_as_uint(p3[1][t][r]),
                                                           false, false);
                prm[crow(r, 0)] = __uint_as_float(sw[0]);
                prm[crow(r, 1)] = __uint_as_float(sw[1]);
            }
            const int dt = (int)P[L.tdim + t];
            float v = 0.f;
#pragma unroll
            for (int j = 0; j < DMAX; ++j) v = (j == dt) ? xr[j] : v;
            if (C.rescale) v = C.rs_to_scale * (v - C.rs_lo) - C.bound;
            float o, l;
            rq_spline_elem<K, (DIR < 0)>(v, prm, C, o, l);
            if (C.rescale) o = (o + C.bound) * C.rs_from_scale + C.rs_lo;
#pragma unroll
            for (int j = 0; j < DMAX; ++j) y[j] = (j == dt) ? o : y[j];
            ld = (t == 0) ? l : ld + l;
        }
    }
}

// spline_unit_apply's body in three parts (the same operations in the same order), for the stage
// clocks of the streaming chain's timing build (NFX_SCHAIN_TIMING): layers 1 and 2 (h2), layer 3's
// tile t with the half-wave exchange (the lane's 32 spline parameters), and dim t's spline. The
// product path keeps the single inline body (split, the allocation of the 8-wave chain kernel
// grew from 189 to 212 VGPRs).
template <int HT, int TILES>
__device__ __forceinline__ void spline_unit_hidden(const float* P, const SplineLayout& L, int KS1,
                                                   const float (&xb)[2][4], f32x16 (&h2)[HT][2]) {
#pragma clang fp contract(off)
    const int lane = lane_id(), h = lane >> 5;
    // Layer 1 + ReLU
    f32x16 h1[HT][2];
#pragma unroll
    for (int ht = 0; ht < HT; ++ht) {
        f32x16 a0, a1;
        load_bias16_x2(P + L.b1 + ht * 32, h, a0, a1);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            if (ks < KS1) {
                const float w = P[L.w1 + (ht * 4 + ks) * 64 + lane];
                a0 = mfma32(w, xb[0][ks], a0);
                if constexpr (TILES == 2) a1 = mfma32(w, xb[1][ks], a1);
            }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            a0[r] = trelu(a0[r]);
            a1[r] = trelu(a1[r]);
        }
        h1[ht][0] = a0;
        h1[ht][1] = a1;
    }
    // Layer 2 + ReLU
#pragma unroll
    for (int hto = 0; hto < HT; ++hto) {
        f32x16 a0, a1;
        load_bias16_x2(P + L.b2 + hto * 32, h, a0, a1);
#pragma unroll
        for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
            for (int rq = 0; rq < 4; ++rq) {
                const f32x4 w = *reinterpret_cast<const f32x4*>(
                    P + L.w2 + (((hto * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    a0 = mfma32(w[rr], h1[kt][0][4 * rq + rr], a0);
                    if constexpr (TILES == 2) a1 = mfma32(w[rr], h1[kt][1][4 * rq + rr], a1);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            a0[r] = trelu(a0[r]);
            a1[r] = trelu(a1[r]);
        }
        h2[hto][0] = a0;
        h2[hto][1] = a1;
    }
}

// Layer 3, tile t: the 3K-1 parameters of transformed dim tdim[t]; after the half-wave exchange
// every lane holds rows 0..31 of its own sample.
template <int HT, int TILES>
__device__ __forceinline__ void spline_unit_params(const float* P, const SplineLayout& L, const f32x16 (&h2)[HT][2],
                                                   int t, float (&prm)[32]) {
#pragma clang fp contract(off)
    const int lane = lane_id(), h = lane >> 5;
    f32x16 a0, a1;
    load_bias16_x2(P + L.b3 + t * 32, h, a0, a1);
#pragma unroll
    for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {
            const f32x4 w = *reinterpret_cast<const f32x4*>(P + L.w3 + (((t * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                a0 = mfma32(w[rr], h2[kt][0][4 * rq + rr], a0);
                if constexpr (TILES == 2) a1 = mfma32(w[rr], h2[kt][1][4 * rq + rr], a1);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(a0[r]), __float_as_uint(a1[r]), false, false);
        prm[crow(r, 0)] = __uint_as_float(sw[0]);
        prm[crow(r, 1)] = __uint_as_float(sw[1]);
    }
}

// Dim dt's spline on the lane's own sample: y[dt] and the log-det term (ld = l at t = 0, else +=).
template <int K, int DIR, int DMAX>
__device__ __forceinline__ void spline_unit_dim(const SplineConsts& C, int dt, int t, const float (&prm)[32],
                                                const float (&xr)[DMAX], float (&y)[DMAX], float& ld) {
#pragma clang fp contract(off)
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < DMAX; ++j) v = (j == dt) ? xr[j] : v;
    if (C.rescale) v = C.rs_to_scale * (v - C.rs_lo) - C.bound;
    float o, l;
    rq_spline_elem<K, (DIR < 0)>(v, prm, C, o, l);
    if (C.rescale) o = (o + C.bound) * C.rs_from_scale + C.rs_lo;
#pragma unroll
    for (int j = 0; j < DMAX; ++j) y[j] = (j == dt) ? o : y[j];
    ld = (t == 0) ? l : ld + l;
}

// DS = the data dimension when it is fixed at compile time (2: the two-moons-shaped BASELINE
// cfg3 / RealNVPSpline path), 0 = runtime d <= 8. With DS = 2 a lane's sample row is one
// 8-byte load and the layer-1 operands of the two sample tiles come out of one
// v_permlane32_swap of that row (no per-element loads or 64-bit address arithmetic), and every
// loop over the row is compile-time.
// Occupancy: the d = 2 kernels at H <= 64 fit 168 VGPRs without spilling, i.e. 3 waves per SIMD
// (3 workgroups per CU) instead of 2 — more MFMA/VALU interleaving across waves.
template <int HT, int K, int DIR, bool LOGP, int DS>
__global__ __launch_bounds__(256, (DS == 2 && HT <= 2) ? 3 : 1) void spline_coupling_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d_rt, SplineConsts C, int accumulate,
    int64_t nchunks, float* __restrict__ logp, double* __restrict__ partials, double* __restrict__ sums, float cgauss) {
#pragma clang fp contract(off)
    constexpr int DMAX = DS ? DS : 8;
    const int d = DS ? DS : d_rt;
    const SplineLayout L = spline_layout(HT, d);
    extern __shared__ f32x4 lds4[];
    {
        const f32x4* src = reinterpret_cast<const f32x4*>(packed);
        for (int i = threadIdx.x; i < L.total / 4; i += 256) lds4[i] = src[i];
    }
    __syncthreads();
    const float* sm = reinterpret_cast<const float*>(lds4);
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    const int KS1 = (d + 1) / 2;
    const int NT = (int)sm[L.meta];

    // Software pipeline: chunk c + nwaves's x rows and incoming log-det load while chunk c runs.
    struct Fetch {
        float xb[2][4];   // raw layer-1 operands x[sample base+32st+col][2ks+h] (DS = 0)
        float xr[DMAX];   // the lane's own sample row
        float ldin;
    };
    // Work split (as affine_coupling_kernel): every wave takes F = nchunks / nwaves whole 64-sample
    // chunks; the R leftover chunks go out as 2R 32-sample half chunks, one to each of the first
    // 2R waves (when 2R <= nwaves), so a SIMD's last round is half a chunk (1M samples: 15.26 chunks
    // per SIMD ran as 16 rounds, now 15.5).
    const int64_t wv = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t F = nchunks / nwaves, R = nchunks - F * nwaves;
    const bool split = 2 * R <= nwaves;
    const int64_t nfull = split ? F : F + (wv < R ? 1 : 0);
    const bool half = split && wv < 2 * R;
    const int64_t half_base = F * nwaves * 64 + wv * 32;
    auto unit_base = [&](int64_t u) { return u < nfull ? (wv + u * nwaves) * 64 : half_base; };
    auto fetch = [&](int64_t u, Fetch& f) {
        const int64_t base = unit_base(u);
        const int nsamp = u < nfull ? 64 : (u == nfull && half ? 32 : 0);
        const int64_t so = base + lane;
        const bool row = lane < nsamp && so < B;
        if constexpr (DS == 2) {
            const f32x2 v = row ? *reinterpret_cast<const f32x2*>(in + so * 2) : f32x2{0.f, 0.f};
            f.xr[0] = v.x;
            f.xr[1] = v.y;
        } else {
#pragma unroll
            for (int st = 0; st < 2; ++st) {
                const int64_t s = base + 32 * st + col;
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    const int k = 2 * ks + h;
                    f.xb[st][ks] = (32 * st + col < nsamp && ks < KS1 && k < d && s < B) ? in[s * d + k] : 0.f;
                }
            }
#pragma unroll
            for (int j = 0; j < DMAX; ++j) f.xr[j] = (row && j < d) ? in[so * d + j] : 0.f;
        }
        f.ldin = (row && accumulate) ? logdet[so] : 0.f;
    };
    float mkb[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) mkb[ks] = (2 * ks + h < d) ? sm[L.mask + 2 * ks + h] : 0.f;

    double lpacc = 0.0;
    // one unit: 2 sample tiles (TILES = 2) or the half chunk (TILES = 1: tile 1's MFMAs skipped,
    // lanes 32..63 compute unused values)
    auto unit = [&](auto tiles_c, int64_t base, const Fetch& cur) {
        constexpr int TILES = decltype(tiles_c)::value;
        const float* P = sm + opaque_zero();

        // Layer-1 B operands (x rescaled, times mask), k-steps padded to 4.
        float xraw[2][4];
        if constexpr (DS == 2) {
            // lanes 0..31 hold the rows of samples base+col, lanes 32..63 those of base+32+col;
            // operand (st, k = h) of lane (col, h) is x[base+32st+col][h]: one row swap
            const float other = halves_other(cur.xr[0], cur.xr[1]);
            xraw[0][0] = h ? other : cur.xr[0];
            xraw[1][0] = h ? cur.xr[1] : other;
#pragma unroll
            for (int ks = 1; ks < 4; ++ks) xraw[0][ks] = xraw[1][ks] = 0.f;
        } else {
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) xraw[st][ks] = cur.xb[st][ks];
        }
        float xb[2][4];
#pragma unroll
        for (int st = 0; st < 2; ++st) {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                float xv = xraw[st][ks];
                if (C.rescale) xv = C.rs_to_scale * (xv - C.rs_lo) - C.bound;
                xb[st][ks] = xv * mkb[ks];
            }
        }
        const int64_t so = base + lane;
        float xr[DMAX];
#pragma unroll
        for (int j = 0; j < DMAX; ++j) xr[j] = cur.xr[j];

        // Layer 1 + ReLU
        f32x16 h1[HT][2];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
            f32x16 a0, a1;
            load_bias16_x2(P + L.b1 + ht * 32, h, a0, a1);
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                if (ks < KS1) {
                    const float w = P[L.w1 + (ht * 4 + ks) * 64 + lane];
                    a0 = mfma32(w, xb[0][ks], a0);
                    if constexpr (TILES == 2) a1 = mfma32(w, xb[1][ks], a1);
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                a0[r] = trelu(a0[r]);
                a1[r] = trelu(a1[r]);
            }
            h1[ht][0] = a0;
            h1[ht][1] = a1;
        }
        // Layer 2 + ReLU
        f32x16 h2[HT][2];
#pragma unroll
        for (int hto = 0; hto < HT; ++hto) {
            f32x16 a0, a1;
            load_bias16_x2(P + L.b2 + hto * 32, h, a0, a1);
#pragma unroll
            for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) {
                    const f32x4 w = *reinterpret_cast<const f32x4*>(
                        P + L.w2 + (((hto * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        a0 = mfma32(w[rr], h1[kt][0][4 * rq + rr], a0);
                        if constexpr (TILES == 2) a1 = mfma32(w[rr], h1[kt][1][4 * rq + rr], a1);
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                a0[r] = trelu(a0[r]);
                a1[r] = trelu(a1[r]);
            }
            h2[hto][0] = a0;
            h2[hto][1] = a1;
        }

        float y[DMAX];
#pragma unroll
        for (int j = 0; j < DMAX; ++j) y[j] = xr[j];
        float ld = 0.f;
        for (int t = 0; t < NT; ++t) {
            // Layer 3, tile t: the 3K-1 parameters of transformed dim tdim[t].
            f32x16 a0, a1;
            load_bias16_x2(P + L.b3 + t * 32, h, a0, a1);
#pragma unroll
            for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) {
                    const f32x4 w = *reinterpret_cast<const f32x4*>(
                        P + L.w3 + (((t * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        a0 = mfma32(w[rr], h2[kt][0][4 * rq + rr], a0);
                        if constexpr (TILES == 2) a1 = mfma32(w[rr], h2[kt][1][4 * rq + rr], a1);
                    }
                }
            }
            // Half-wave exchange: afterwards every lane holds rows 0..31 of its own sample.
            float prm[32];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(a0[r]), __float_as_uint(a1[r]),
                                                           false, false);
                prm[crow(r, 0)] = __uint_as_float(sw[0]);
                prm[crow(r, 1)] = __uint_as_float(sw[1]);
            }
            const int dt = (int)P[L.tdim + t];
            float v = 0.f;
#pragma unroll
            for (int j = 0; j < DMAX; ++j) v = (j == dt) ? xr[j] : v;
            if (C.rescale) v = C.rs_to_scale * (v - C.rs_lo) - C.bound;
            float o, l;
            rq_spline_elem<K, (DIR < 0)>(v, prm, C, o, l);
            if (C.rescale) o = (o + C.bound) * C.rs_from_scale + C.rs_lo;
#pragma unroll
            for (int j = 0; j < DMAX; ++j) y[j] = (j == dt) ? o : y[j];
            ld = (t == 0) ? l : ld + l;
        }
        if (lane < 32 * TILES && so < B) {
            float m = 0.f;
            float yo[DMAX];
#pragma unroll
            for (int j = 0; j < DMAX; ++j) {
                const float v = nonfinite(y[j]) ? 0.f : y[j];
                yo[j] = v;
                if (j < d) m = (j == 0) ? gauss_sq0(v) : gauss_sq(m, v);
            }
            if constexpr (DS == 2) {
                *reinterpret_cast<f32x2*>(out + so * 2) = f32x2{yo[0], yo[1]};
            } else {
#pragma unroll
                for (int j = 0; j < DMAX; ++j)
                    if (j < d) out[so * d + j] = yo[j];
            }
            if (nonfinite(ld)) ld = 0.f;
            const float ldt = accumulate ? cur.ldin + ld : ld;
            logdet[so] = ldt;
            if constexpr (LOGP) {
                const float lp = gauss_lp(m, cgauss, ldt);
                logp[so] = lp;
                lpacc += (double)lp;
            }
        }
    };

    Fetch cur;
    fetch(0, cur);
    for (int64_t u = 0; u < nfull; ++u) {
        Fetch nxt;
        fetch(u + 1, nxt);
        unit(std::integral_constant<int, 2>{}, unit_base(u), cur);
        cur = nxt;
    }
    if (half) unit(std::integral_constant<int, 1>{}, half_base, cur);
    if constexpr (LOGP) {
        logp_commit<256>(lpacc, partials, sums, B);
    }
}

typedef void (*spline_kernel_t)(const float*, const float*, float*, float*, int64_t, int,
                                SplineConsts, int, int64_t, float*, double*, double*, float);

// DS = 0: runtime d <= 8; DS = 2: the d = 2 specialisation (nfx_spline_d2_h*.hip)
template <int HT, int DS>
spline_kernel_t spline_pick_ht(int K, int dir, bool logp);


// ---- wide spline coupling layers (8 < d <= 64) -----------------------------------------------
// A wave owns a 32-sample tile whose [32 x d] x block sits in a wave-private LDS tile (odd row
// stride), loaded/stored with coalesced row accesses. The param MLP runs as in the narrow kernel
// (weights from L2: the d(3K-1)-row output layer outgrows LDS); the output layer produces the
// tiles of two transformed dims (t, t+1) for the same 32 samples, and one v_permlane32_swap per
// register leaves lanes 0..31 holding all parameters of dim t and lanes 32..63 those of dim t+1
// for sample `col` — both lane halves run a spline, none is duplicated. Outputs go back into the
// tile in place (each spline reads only its own dimension).
constexpr int kSplineWideWaves = 4;

template <int HT, int K, int DIR, bool LOGP>
__global__ __launch_bounds__(64 * kSplineWideWaves) void spline_wide_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d, SplineConsts C, int accumulate, int64_t ntiles,
    float* __restrict__ logp, double* __restrict__ partials, double* __restrict__ sums, float cgauss) {
#pragma clang fp contract(off)
    const SplineLayout L = spline_layout(HT, d);
    const int KS = spline_ks1(d);
    const int S = d | 1;
    extern __shared__ f32x4 lds4[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float* xt = reinterpret_cast<float*>(lds4) + wave * 32 * S;
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    const int NT = (int)packed[L.meta];
    double lpacc = 0.0;
    for (int64_t t = (int64_t)blockIdx.x * kSplineWideWaves + wave; t < ntiles;
         t += (int64_t)gridDim.x * kSplineWideWaves) {
        const int64_t base = t * 32;
        const int rows = (int)(B - base < 32 ? B - base : 32);
        const float* src = in + base * d;
        for (int i = lane; i < 32 * d; i += 64) {
            const int r = i / d, c = i - r * d;
            xt[r * S + c] = r < rows ? src[i] : 0.f;
        }
        const float ldin = (accumulate && lane < rows) ? logdet[base + lane] : 0.f;
        wave_lds_sync();
        const float* P = packed + opaque_zero();
        // layer 1 (x rescaled, times mask) + ReLU
        f32x16 h1[HT];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) h1[ht] = load_bias16(P + L.b1 + ht * 32, h);
        for (int ks = 0; ks < KS; ++ks) {
            const int k = 2 * ks + h;
            float xv = 0.f;
            if (k < d) {
                xv = xt[col * S + k];
                if (C.rescale) xv = C.rs_to_scale * (xv - C.rs_lo) - C.bound;
                xv = xv * P[L.mask + k];
            }
#pragma unroll
            for (int ht = 0; ht < HT; ++ht) h1[ht] = mfma32(P[L.w1 + (ht * KS + ks) * 64 + lane], xv, h1[ht]);
        }
#pragma unroll
        for (int ht = 0; ht < HT; ++ht)
#pragma unroll
            for (int r = 0; r < 16; ++r) h1[ht][r] = trelu(h1[ht][r]);
        f32x16 h2[HT];
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
        float ldp = 0.f;
        for (int tt = 0; tt < NT; tt += 2) {
            const bool two = tt + 1 < NT;
            f32x16 a0 = load_bias16(P + L.b3 + tt * 32, h);
            f32x16 a1 = two ? load_bias16(P + L.b3 + (tt + 1) * 32, h) : f32x16{};
#pragma unroll
            for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) {
                    const f32x4 w0 = *reinterpret_cast<const f32x4*>(P + L.w3 + (((tt * HT + kt) * 4 + rq) * 64 + lane) * 4);
                    const f32x4 w1 = two ? *reinterpret_cast<const f32x4*>(
                                               P + L.w3 + ((((tt + 1) * HT + kt) * 4 + rq) * 64 + lane) * 4)
                                         : f32x4{};
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        a0 = mfma32(w0[rr], h2[kt][4 * rq + rr], a0);
                        a1 = mfma32(w1[rr], h2[kt][4 * rq + rr], a1);
                    }
                }
            float prm[32];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(a0[r]), __float_as_uint(a1[r]), false, false);
                prm[crow(r, 0)] = __uint_as_float(sw[0]);
                prm[crow(r, 1)] = __uint_as_float(sw[1]);
            }
            if (h == 0 || two) {
                const int dt = (int)P[L.tdim + tt + h];
                float* px = xt + col * S + dt;
                float v = *px;
                if (C.rescale) v = C.rs_to_scale * (v - C.rs_lo) - C.bound;
                float o, l;
                rq_spline_elem<K, (DIR < 0)>(v, prm, C, o, l);
                if (C.rescale) o = (o + C.bound) * C.rs_from_scale + C.rs_lo;
                *px = o;
                ldp = ldp + l;
            }
        }
        float ld = halves_sum(ldp, ldp);
        if (nonfinite(ld)) ld = 0.f;
        wave_lds_sync();
        float* dst = out + base * d;
        for (int i = lane; i < rows * d; i += 64) {
            const int r = i / d, c = i - r * d;
            const float v = xt[r * S + c];
            dst[i] = nonfinite(v) ? 0.f : v;
        }
        if (lane < rows) {
            const float ldt = accumulate ? ldin + ld : ld;
            logdet[base + lane] = ldt;
            if constexpr (LOGP) {
                float m = 0.f;
                for (int c = 0; c < d; ++c) {
                    float v = xt[lane * S + c];
                    v = nonfinite(v) ? 0.f : v;
                    m = c == 0 ? gauss_sq0(v) : gauss_sq(m, v);
                }
                const float lp = gauss_lp(m, cgauss, ldt);
                logp[base + lane] = lp;
                lpacc += (double)lp;
            }
        }
        wave_lds_sync();
    }
    if constexpr (LOGP) {
        logp_commit<64 * kSplineWideWaves>(lpacc, partials, sums, B);
    }
}

// wide kernels (8 < d <= 64), one TU per HT (nfx_spline_w_h*.hip)
template <int HT>
spline_kernel_t spline_wide_pick_ht(int K, int dir, bool logp);

}  // namespace nfx
