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
#include "nfx_common.h"

namespace nfx {

__host__ __device__ constexpr int sp_up4(int v) { return (v + 3) & ~3; }

// Packed image (floats):
//   w1 [HT][4][64]         layer-1 A operand, k-steps padded to 4 (d <= 8)
//   b1 [HT][2][16]         (bias of accumulator register r, lane-half h)
//   w2 [HT][HT][4][64][4]
//   b2 [HT][2][16]
//   w3 [d][HT][4][64][4]   output tile t = t-th transformed dim: row i = parameter i
//   b3 [d][2][16]
//   mask [8], tdim [8] (indices of the transformed dims, as floats), meta [4] (meta[0] = NT)
struct SplineLayout {
    int HT, NT;  // NT here = capacity (d); the live count is meta[0]
    int w1, b1, w2, b2, w3, b3, mask, tdim, meta, total;
};

__host__ __device__ constexpr SplineLayout spline_layout(int HT, int d) {
    SplineLayout L{};
    const int NT = d;
    L.HT = HT;
    L.NT = NT;
    int o = 0;
    L.w1 = o; o += HT * 4 * 64;
    L.b1 = o; o += HT * 32;
    L.w2 = o; o += HT * HT * 16 * 64;
    L.b2 = o; o += HT * 32;
    L.w3 = o; o += NT * HT * 16 * 64;
    L.b3 = o; o += NT * 32;
    L.mask = o; o += 8;
    L.tdim = o; o += 8;
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

// One RQ spline evaluation of SplineCouplingLayer._rational_quadratic_spline for a single
// input v with its 3K-1 unnormalised parameters p[] (:182-309, per element).
// Returns the spline-level guarded output (NaN/Inf -> input, :306) and log|det| (-> 0, :307).
template <int K, bool INV>
__device__ __forceinline__ void rq_spline_elem(float v, const float (&p)[32], const SplineConsts& C,
                                               float& out, float& lad) {
#pragma clang fp contract(off)
    const float eps = 1e-8f;
    const float B = C.bound;
    out = v;
    lad = 0.f;
    if (v >= -B && v <= B) {
        float w[K], h[K], cwk[K + 1], chk[K + 1], dk[K + 1];
        // softmax (max-subtracted exp, times the reciprocal of the sum) then min-width affine
        {
            float m = p[0];
#pragma unroll
            for (int k = 1; k < K; ++k) m = tmax(m, p[k]);
            float s = 0.f;
#pragma unroll
            for (int k = 0; k < K; ++k) { w[k] = exp_safe(p[k] - m); s = s + w[k]; }
            const float inv = 1.f / s;
#pragma unroll
            for (int k = 0; k < K; ++k) w[k] = tclamp_min(C.min_w + C.cw * (w[k] * inv), eps);
        }
        {
            float m = p[K];
#pragma unroll
            for (int k = 1; k < K; ++k) m = tmax(m, p[K + k]);
            float s = 0.f;
#pragma unroll
            for (int k = 0; k < K; ++k) { h[k] = exp_safe(p[K + k] - m); s = s + h[k]; }
            const float inv = 1.f / s;
#pragma unroll
            for (int k = 0; k < K; ++k) h[k] = tclamp_min(C.min_h + C.ch * (h[k] * inv), eps);
        }
        // knots: ATen's CPU cumsum accumulates float in double and rounds each prefix (:208-213)
        {
            double aw = 0.0, ah = 0.0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                aw += (double)w[k];
                ah += (double)h[k];
                cwk[k + 1] = C.two_bound * (float)aw + (-B);
                chk[k + 1] = C.two_bound * (float)ah + (-B);
            }
            cwk[0] = -B; cwk[K] = B;
            chk[0] = -B; chk[K] = B;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                w[k] = tclamp_min(cwk[k + 1] - cwk[k], eps);
                h[k] = tclamp_min(chk[k + 1] - chk[k], eps);
            }
        }
        dk[0] = 1.f;
        dk[K] = 1.f;
#pragma unroll
        for (int k = 0; k < K - 1; ++k) dk[k + 1] = tclamp_min(C.min_d + tsoftplus(p[2 * K + k]), eps);

        // searchsorted(knots, v, right=True) - 1, clamped to [0, K-1]  (:241-244)
        int cnt = 0;
#pragma unroll
        for (int k = 0; k <= K; ++k) cnt += ((INV ? chk[k] : cwk[k]) <= v) ? 1 : 0;
        int bin = cnt - 1;
        bin = bin < 0 ? 0 : (bin > K - 1 ? K - 1 : bin);
        // gather by select (keeps every array in registers)
        float w_k = w[0], x_k = cwk[0], h_k = h[0], y_k = chk[0], d_k = dk[0], d_k1 = dk[1];
#pragma unroll
        for (int k = 1; k < K; ++k) {
            const bool s = (k == bin);
            w_k = s ? w[k] : w_k;
            x_k = s ? cwk[k] : x_k;
            h_k = s ? h[k] : h_k;
            y_k = s ? chk[k] : y_k;
            d_k = s ? dk[k] : d_k;
            d_k1 = s ? dk[k + 1] : d_k1;
        }
        const float s_k = h_k / tclamp_min(w_k, eps);
        float o, l;
        if constexpr (INV) {
            // citardauq root (:266-281)
            const float dy = v - y_k;
            const float t = d_k + d_k1 - 2.f * s_k;
            const float a = dy * t + h_k * (s_k - d_k);
            const float b = h_k * d_k - dy * t;
            const float c = -s_k * dy;
            const float disc = tclamp_min(b * b - 4.f * a * c, 0.f);
            float den = -b - sqrtf(disc);
            den = fabsf(den) < eps ? eps : den;
            const float xi = tclamp((2.f * c) / den, 0.f, 1.f);
            o = xi * w_k + x_k;
            const float omx = 1.f - xi;
            const float dld = s_k + (d_k1 + d_k - 2.f * s_k) * xi * omx;
            const float nld = (s_k * s_k) * (d_k1 * (xi * xi) + 2.f * s_k * xi * omx + d_k * (omx * omx));
            l = -logf(tclamp_min(nld, eps)) + 2.f * logf(tclamp_min(dld, eps));
        } else {
            // forward (:283-293)
            const float xi = tclamp((v - x_k) / tclamp_min(w_k, eps), 0.f, 1.f);
            const float omx = 1.f - xi;
            const float den = tclamp_min(s_k + (d_k1 + d_k - 2.f * s_k) * xi * omx, eps);
            const float num = h_k * (s_k * (xi * xi) + d_k * xi * omx);
            o = y_k + num / den;
            const float nd = (s_k * s_k) * (d_k1 * (xi * xi) + 2.f * s_k * xi * omx + d_k * (omx * omx));
            l = logf(tclamp_min(nd / tclamp_min(den * den, eps), eps));
        }
        out = o;
        lad = l;
    }
    if (nonfinite(out)) out = v;      // :306
    if (nonfinite(lad)) lad = 0.f;    // :307
}

template <int HT, int K, int DIR, bool LOGP>
__global__ __launch_bounds__(256) void spline_coupling_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d, SplineConsts C, int accumulate,
    int64_t nchunks, float* __restrict__ logp, double* __restrict__ partials, float cgauss) {
#pragma clang fp contract(off)
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
        float xb[2][4];  // raw layer-1 operands x[sample base+32st+col][2ks+h]
        float xr[8];     // the lane's own sample row
        float ldin;
    };
    auto fetch = [&](int64_t c, Fetch& f) {
        const int64_t base = c * 64;
        const bool live = c < nchunks;
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            const int64_t s = base + 32 * st + col;
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const int k = 2 * ks + h;
                f.xb[st][ks] = (live && ks < KS1 && k < d && s < B) ? in[s * d + k] : 0.f;
            }
        }
        const int64_t so = base + lane;
        const bool row = live && so < B;
#pragma unroll
        for (int j = 0; j < 8; ++j) f.xr[j] = (row && j < d) ? in[so * d + j] : 0.f;
        f.ldin = (row && accumulate) ? logdet[so] : 0.f;
    };
    float mkb[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) mkb[ks] = (2 * ks + h < d) ? sm[L.mask + 2 * ks + h] : 0.f;

    int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    Fetch cur;
    fetch(c, cur);
    double lpacc = 0.0;
    for (; c < nchunks; c += nwaves) {
        const int64_t base = c * 64;
        const float* P = sm + opaque_zero();
        Fetch nxt;
        fetch(c + nwaves, nxt);

        // Layer-1 B operands (x rescaled, times mask), k-steps padded to 4.
        float xb[2][4];
#pragma unroll
        for (int st = 0; st < 2; ++st) {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                float xv = cur.xb[st][ks];
                if (C.rescale) xv = C.rs_to_scale * (xv - C.rs_lo) - C.bound;
                xb[st][ks] = xv * mkb[ks];
            }
        }
        const int64_t so = base + lane;
        float xr[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) xr[j] = cur.xr[j];

        // Layer 1 + ReLU
        f32x16 h1[HT][2];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
            f32x16 a0, a1;
            a0 = a1 = load_bias16(P + L.b1 + ht * 32, h);
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                if (ks < KS1) {
                    const float w = P[L.w1 + (ht * 4 + ks) * 64 + lane];
                    a0 = mfma32(w, xb[0][ks], a0);
                    a1 = mfma32(w, xb[1][ks], a1);
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
            a0 = a1 = load_bias16(P + L.b2 + hto * 32, h);
#pragma unroll
            for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) {
                    const f32x4 w = *reinterpret_cast<const f32x4*>(
                        P + L.w2 + (((hto * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        a0 = mfma32(w[rr], h1[kt][0][4 * rq + rr], a0);
                        a1 = mfma32(w[rr], h1[kt][1][4 * rq + rr], a1);
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

        float y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = xr[j];
        float ld = 0.f;
        for (int t = 0; t < NT; ++t) {
            // Layer 3, tile t: the 3K-1 parameters of transformed dim tdim[t].
            f32x16 a0, a1;
            a0 = a1 = load_bias16(P + L.b3 + t * 32, h);
#pragma unroll
            for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) {
                    const f32x4 w = *reinterpret_cast<const f32x4*>(
                        P + L.w3 + (((t * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        a0 = mfma32(w[rr], h2[kt][0][4 * rq + rr], a0);
                        a1 = mfma32(w[rr], h2[kt][1][4 * rq + rr], a1);
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
            for (int j = 0; j < 8; ++j) v = (j == dt) ? xr[j] : v;
            if (C.rescale) v = C.rs_to_scale * (v - C.rs_lo) - C.bound;
            float o, l;
            rq_spline_elem<K, (DIR < 0)>(v, prm, C, o, l);
            if (C.rescale) o = (o + C.bound) * C.rs_from_scale + C.rs_lo;
#pragma unroll
            for (int j = 0; j < 8; ++j) y[j] = (j == dt) ? o : y[j];
            ld = (t == 0) ? l : ld + l;
        }
        if (so < B) {
            float m = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = nonfinite(y[j]) ? 0.f : y[j];
                if (j < d) {
                    out[so * d + j] = v;
                    m = (j == 0) ? gauss_sq0(v) : gauss_sq(m, v);
                }
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
        cur = nxt;
    }
    if constexpr (LOGP) {
        const double t = block_sum_f64<256>(lpacc);
        if (threadIdx.x == 0) partials[blockIdx.x] = t;
    }
}

typedef void (*spline_kernel_t)(const float*, const float*, float*, float*, int64_t, int,
                                SplineConsts, int, int64_t, float*, double*, float);

template <int HT>
spline_kernel_t spline_pick_ht(int K, int dir, bool logp);

}  // namespace nfx
