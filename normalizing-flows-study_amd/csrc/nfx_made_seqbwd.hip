// Backward (training) pass of the SEQUENTIAL MADE directions — InverseAutoregressiveFlow.inverse
// (inverse_autoregressive_flow.py:65-103, the IAF density direction) and
// MaskedAutoregressiveFlow.forward (masked_autoregressive_flow.py:46-78, MAF sampling) — under
// autograd. SURVEY.md §8(f) item 1.
//
// The reference runs d MADE calls on the partially filled vector z^(i) and autograd
// differentiates all of them. Output i of call i depends only on hidden units of degree < i,
// which depend only on inputs < i (already final), so every call's output i, every activation
// it uses and every weight it touches equal those of ONE MADE evaluation at the final vector zs.
// The adjoint is therefore a triangular system solved by a REVERSE sweep that mirrors the
// forward sweep of made_seq_kernel: with ḡ_j the total adjoint of zs_j,
//   ḡ_j = gzs_j + Σ_a W1m[a, j] · gh1_a            (units a of degree >= j)
//   (δμ_j, δα_j) = local derivatives of step j given ḡ_j (clamps, exp, guards)
//   G3 += W4m[j, :] δμ_j + W4m[d + j, :] δα_j       (rank-1: layer-3 output adjoints)
// and a hidden unit of degree m is complete (has received every output > m) at step j = m, when
// it goes through ReLU' and its rank-1 contribution moves one layer down (G3 -> G2 -> G1 -> gh1).
// Per sample this costs one MADE evaluation forward (recompute, as made_seq_kernel) plus one
// backward, instead of d of each. One lane = one sample; weights are wave-uniform scalar loads;
// per-lane state: pre-activations and layer-3 values/adjoints in registers, layer-1/2 values and
// adjoints in wave-private LDS rows.
//
// Outputs: grad_in [B, d] and the feature-major factors of nfx_made_backward_weights (rows of
// pitch nfx_made_factor_pitch(B) = B): D4 = (δμ | δα), D3/D2/D1 = the ReLU'-gated hidden
// adjoints, H3/H2/H1 = the hidden activations at zs, X1 = zs (the MADE input). The D4 rows hold
// the raw (μ, α) of the forward sweep until the reverse sweep overwrites them.
//
// Epilogues (torch semantics of the reference ops; gzs = finite(zs) ? gz : 0):
//   IAF inverse: αc = clamp(α,-2,2), μc = clamp(μ,-10,10), e = exp(-αc), zs = (x - μc) e;
//     out = finite ? zs : x; ld = clamp(finite(-Σαc) ? -Σαc : 0, -50, 50)
//     gx = ḡ e + [!finite(zs)] gz;  δμ = [|μ|<=10] (-ḡ e);  δα = [|α|<=2] (-ḡ (x - μc) e - gld0)
//   MAF forward: αc = clamp(α,-3,3), e = exp(αc), zs = x e + μ; out = finite ? zs : 0;
//     ld = clamp(finite(Σαc) ? Σαc : 0, -100, 100)
//     gx = ḡ e;  δμ = ḡ;  δα = [|α|<=3] (ḡ x e + gld0)
//   gld0 = gld · [Σ finite] · [ld1 inside the clamp].
// A non-finite step poisons the later MADE outputs exactly like the forward kernels (NaN); the
// gradients of such rows are NaN-contaminated as autograd's are, without claiming bit parity.
#include "nfx_made_kernel.h"

namespace nfx {

template <int HT>
__device__ __forceinline__ bool mask_bit(const uint32_t (&m)[2 * HT], int a) {
    uint32_t w = 0;
#pragma unroll
    for (int k = 0; k < 2 * HT; ++k) w = (k == (a >> 4)) ? m[k] : w;  // a is wave-uniform
    return (w >> (a & 15)) & 1u;
}

template <int HT, int VAR>
__global__ __launch_bounds__(64) void made_seq_bwd_kernel(const float* __restrict__ packed, const float* __restrict__ in,
                                                          const float* __restrict__ gout,
                                                          const float* __restrict__ gld_in, float* __restrict__ gin,
                                                          float* __restrict__ fac, int64_t B, int d, int H) {
    constexpr int Hp = 32 * HT;
    constexpr int RS = Hp + 4;  // LDS row stride (conflict-free ds_read_b128 across lanes)
    constexpr bool IAF = VAR == NFX_IAF_INVERSE;
    const MadeLayout L = made_layout(d, HT);
    extern __shared__ f32x4 lds4[];
    float* r0 = reinterpret_cast<float*>(lds4) + threadIdx.x * RS;  // h1 (forward) -> G2 (reverse)
    float* r1 = r0 + 64 * RS;                                       // h2 -> G1
    float* r2 = r1 + 64 * RS;                                       // gh1
    const int lane = threadIdx.x;
    const int64_t s = (int64_t)blockIdx.x * 64 + lane;
    const bool valid = s < B;
    const int64_t sv = valid ? s : 0;
    const float* P = packed;
    const int64_t Pt = B;  // factor row pitch (nfx_made_factor_pitch)
    float* D4 = fac;
    float* D3 = D4 + (int64_t)2 * d * Pt;
    float* D2 = D3 + (int64_t)H * Pt;
    float* D1 = D2 + (int64_t)H * Pt;
    float* H3 = D1 + (int64_t)H * Pt;
    float* H2 = H3 + (int64_t)(H + 1) * Pt;
    float* H1 = H2 + (int64_t)(H + 1) * Pt;
    float* X1 = H1 + (int64_t)(H + 1) * Pt;
    const float* ord = P + L.s_deg;

    // ---- forward sweep: zs, raw (mu, alpha), the hidden activations at zs ----
    float pre1[Hp], h3[Hp];
#pragma unroll
    for (int a = 0; a < Hp; ++a) {
        pre1[a] = P[L.s_b1 + a];
        h3[a] = 0.f;
        r0[a] = 0.f;
        r1[a] = 0.f;
        r2[a] = 0.f;
    }
    float ld0 = 0.f;
    bool poison = false;
    int p = 0;
    for (int i = 0; i < d; ++i) {
        float mu = 0.f, al = 0.f;
        const float* w_mu = P + L.s_w4 + (size_t)i * Hp;
        const float* w_al = P + L.s_w4 + (size_t)(d + i) * Hp;
#pragma unroll
        for (int a = 0; a < Hp; ++a) {
            mu = fmaf(w_mu[a], h3[a], mu);
            al = fmaf(w_al[a], h3[a], al);
        }
        mu = mu + P[L.s_b4 + i];
        al = al + P[L.s_b4 + d + i];
        if (poison) { mu = __builtin_nanf(""); al = mu; }
        const float xin = valid ? in[sv * d + i] : 0.f;
        float zi;
        {
#pragma clang fp contract(off)  // the forward kernels' roundings
            if constexpr (IAF) {
                const float a = tclamp(al, -2.f, 2.f);
                zi = (xin - tclamp(mu, -10.f, 10.f)) * exp_fast(-a);
                ld0 = ld0 - a;
            } else {
                const float a = tclamp(al, -3.f, 3.f);
                zi = xin * exp_fast(a) + mu;
                ld0 = ld0 + a;
            }
        }
        if (valid) {
            D4[(int64_t)i * Pt + s] = mu;
            D4[(int64_t)(d + i) * Pt + s] = al;
            X1[(int64_t)i * Pt + s] = zi;
        }
        if (nonfinite(zi)) poison = true;
        const float* w1c = P + L.s_w1t + (size_t)i * Hp;
#pragma unroll
        for (int a = 0; a < Hp; ++a) pre1[a] = fmaf(w1c[a], zi, pre1[a]);
        int q = p;
        while (q < H && (int)ord[Hp + q] == i) ++q;
        if (q > p) {
            for (int k = p; k < q; ++k) {
                const int a = (int)ord[2 * Hp + k];
                float v = 0.f;
#pragma unroll
                for (int b = 0; b < Hp; ++b) v = (b == a) ? pre1[b] : v;
                r0[a] = trelu(v);
            }
            for (int k = p; k < q; ++k) {
                const int a = (int)ord[2 * Hp + k];
                const float* w = P + L.s_w2 + (size_t)a * Hp;
                float v = 0.f;
#pragma unroll
                for (int b = 0; b < Hp; b += 4) {
                    const f32x4 hv = *reinterpret_cast<const f32x4*>(r0 + b);
                    v = fmaf(w[b], hv[0], v);
                    v = fmaf(w[b + 1], hv[1], v);
                    v = fmaf(w[b + 2], hv[2], v);
                    v = fmaf(w[b + 3], hv[3], v);
                }
                r1[a] = trelu(v + P[L.s_b2 + a]);
            }
            for (int k = p; k < q; ++k) {
                const int a = (int)ord[2 * Hp + k];
                const float* w = P + L.s_w3 + (size_t)a * Hp;
                float v = 0.f;
#pragma unroll
                for (int b = 0; b < Hp; b += 4) {
                    const f32x4 hv = *reinterpret_cast<const f32x4*>(r1 + b);
                    v = fmaf(w[b], hv[0], v);
                    v = fmaf(w[b + 1], hv[1], v);
                    v = fmaf(w[b + 2], hv[2], v);
                    v = fmaf(w[b + 3], hv[3], v);
                }
                v = trelu(v + P[L.s_b3 + a]);
#pragma unroll
                for (int b = 0; b < Hp; ++b) h3[b] = (b == a) ? v : h3[b];
            }
            p = q;
        }
    }
    // activations out (feature-major), ReLU' masks kept as bits, rows cleared for the adjoints
    uint32_t m1[2 * HT], m2[2 * HT], m3[2 * HT];
#pragma unroll
    for (int k = 0; k < 2 * HT; ++k) m1[k] = m2[k] = m3[k] = 0u;
#pragma unroll
    for (int a = 0; a < Hp; ++a) {
        const float v1 = r0[a], v2 = r1[a];
        m1[a >> 4] |= (v1 > 0.f ? 1u : 0u) << (a & 15);
        m2[a >> 4] |= (v2 > 0.f ? 1u : 0u) << (a & 15);
        m3[a >> 4] |= (h3[a] > 0.f ? 1u : 0u) << (a & 15);
        if (valid && a < H) {
            H1[(int64_t)a * Pt + s] = v1;
            H2[(int64_t)a * Pt + s] = v2;
            H3[(int64_t)a * Pt + s] = h3[a];
        }
        r0[a] = 0.f;
        r1[a] = 0.f;
    }

    // ---- reverse sweep ----
    float g3[Hp];
#pragma unroll
    for (int a = 0; a < Hp; ++a) g3[a] = 0.f;
    const float gld = valid ? gld_in[s] : 0.f;
    float gld0;
    {
        const float ld1 = nonfinite(ld0) ? 0.f : ld0;
        const float lim = IAF ? 50.f : 100.f;
        gld0 = (nonfinite(ld0) || !(ld1 >= -lim && ld1 <= lim)) ? 0.f : gld;
    }
    int q = H;  // completion order, walked backwards (degrees descending)
    for (int i = d - 1; i >= 0; --i) {
        int pe = q;
        while (pe > 0 && (int)ord[Hp + pe - 1] == i) --pe;
        if (pe < q) {
            // units of degree i have received every output > i: layer 3, then 2, then 1
            for (int k = pe; k < q; ++k) {
                const int a = (int)ord[2 * Hp + k];
                float v = 0.f;
#pragma unroll
                for (int b = 0; b < Hp; ++b) v = (b == a) ? g3[b] : v;
                const float gh = mask_bit<HT>(m3, a) ? v : 0.f;
                if (valid) D3[(int64_t)a * Pt + s] = gh;
                const float* w = P + L.s_w3 + (size_t)a * Hp;  // row a of W3m: G2 += W3m[a, :] gh
#pragma unroll
                for (int b = 0; b < Hp; b += 4) {
                    f32x4 g = *reinterpret_cast<f32x4*>(r0 + b);
                    g[0] = fmaf(w[b], gh, g[0]);
                    g[1] = fmaf(w[b + 1], gh, g[1]);
                    g[2] = fmaf(w[b + 2], gh, g[2]);
                    g[3] = fmaf(w[b + 3], gh, g[3]);
                    *reinterpret_cast<f32x4*>(r0 + b) = g;
                }
            }
            for (int k = pe; k < q; ++k) {
                const int a = (int)ord[2 * Hp + k];
                const float gh = mask_bit<HT>(m2, a) ? r0[a] : 0.f;
                if (valid) D2[(int64_t)a * Pt + s] = gh;
                const float* w = P + L.s_w2 + (size_t)a * Hp;
#pragma unroll
                for (int b = 0; b < Hp; b += 4) {
                    f32x4 g = *reinterpret_cast<f32x4*>(r1 + b);
                    g[0] = fmaf(w[b], gh, g[0]);
                    g[1] = fmaf(w[b + 1], gh, g[1]);
                    g[2] = fmaf(w[b + 2], gh, g[2]);
                    g[3] = fmaf(w[b + 3], gh, g[3]);
                    *reinterpret_cast<f32x4*>(r1 + b) = g;
                }
            }
            for (int k = pe; k < q; ++k) {
                const int a = (int)ord[2 * Hp + k];
                const float gh = mask_bit<HT>(m1, a) ? r1[a] : 0.f;
                if (valid) D1[(int64_t)a * Pt + s] = gh;
                r2[a] = gh;
            }
            q = pe;
        }
        // total adjoint of zs_i: the output gradient + the MADE path into input i
        const float* w1c = P + L.s_w1t + (size_t)i * Hp;
        float dot = 0.f;
#pragma unroll
        for (int b = 0; b < Hp; b += 4) {
            const f32x4 g = *reinterpret_cast<const f32x4*>(r2 + b);
            dot = fmaf(w1c[b], g[0], dot);
            dot = fmaf(w1c[b + 1], g[1], dot);
            dot = fmaf(w1c[b + 2], g[2], dot);
            dot = fmaf(w1c[b + 3], g[3], dot);
        }
        const float zi = valid ? X1[(int64_t)i * Pt + s] : 0.f;
        const float gz = valid ? gout[sv * d + i] : 0.f;
        const float xin = valid ? in[sv * d + i] : 0.f;
        const float mu = valid ? D4[(int64_t)i * Pt + s] : 0.f;
        const float al = valid ? D4[(int64_t)(d + i) * Pt + s] : 0.f;
        const bool bad = nonfinite(zi);
        const float gb = (bad ? 0.f : gz) + dot;
        float gx, dmu, dal;
        if constexpr (IAF) {
            const float ac = tclamp(al, -2.f, 2.f), mc = tclamp(mu, -10.f, 10.f);
            const float e = exp_fast(-ac);
            gx = gb * e + (bad ? gz : 0.f);
            dmu = (mu >= -10.f && mu <= 10.f) ? -(gb * e) : 0.f;
            dal = (al >= -2.f && al <= 2.f) ? -(gb * (xin - mc) * e) - gld0 : 0.f;
        } else {
            const float ac = tclamp(al, -3.f, 3.f);
            const float e = exp_fast(ac);
            gx = gb * e;
            dmu = gb;
            dal = (al >= -3.f && al <= 3.f) ? gb * xin * e + gld0 : 0.f;
        }
        if (valid) {
            gin[s * d + i] = gx;
            D4[(int64_t)i * Pt + s] = dmu;
            D4[(int64_t)(d + i) * Pt + s] = dal;
        }
        const float* w_mu = P + L.s_w4 + (size_t)i * Hp;
        const float* w_al = P + L.s_w4 + (size_t)(d + i) * Hp;
#pragma unroll
        for (int a = 0; a < Hp; ++a) g3[a] = fmaf(w_al[a], dal, fmaf(w_mu[a], dmu, g3[a]));
    }
}

typedef void (*made_seq_bwd_t)(const float*, const float*, const float*, const float*, float*, float*, int64_t, int,
                               int);

template <int VAR>
static made_seq_bwd_t seq_bwd_pick(int HT) {
    switch (HT) {
        case 1: return made_seq_bwd_kernel<1, VAR>;
        case 2: return made_seq_bwd_kernel<2, VAR>;
        case 3: return made_seq_bwd_kernel<3, VAR>;
        case 4: return made_seq_bwd_kernel<4, VAR>;
        default: return nullptr;
    }
}

bool made_seqw_bwd_supported(int d, int H);
int made_seqw_bwd_launch(const float* packed, const float* in, const float* gout, const float* gld, float* gin,
                         float* fac, int64_t B, int d, int H, int variant, hipStream_t s);
int made_seq_policy_get();

// Which sequential backward runs (nfx_made_seq_policy): SEGMENT = this file's lane-per-sample
// kernel, WAVE = made_seqw_bwd_kernel (a wave per sample, H <= 64, d <= 1024), AUTO = by a cost
// model of instruction issue per SIMD: the lane kernel runs ceil(B / 64 / SIMDs) rounds of a lane's
// serial sweeps (~ d*6Hp + 8Hp^2 VALU), the wave kernel ceil(B / SIMDs) samples per SIMD of
// ~ 80d + 30Hp instructions (reductions, rank-1 updates, the completions' broadcast FMAs).
static bool seq_bwd_use_wave(int64_t B, int d, int H) {
    if (!made_seqw_bwd_supported(d, H)) return false;
    const int pol = made_seq_policy_get();
    if (pol == NFX_MADE_SEQ_WAVE) return true;
    if (pol == NFX_MADE_SEQ_SEGMENT) return false;
    const int64_t simds = 4 * (int64_t)num_cus();
    const int64_t Hp = 32 * ((H + 31) / 32);
    const double lane = (double)((B + 64 * simds - 1) / (64 * simds)) * (double)(d * 6 * Hp + 8 * Hp * Hp);
    const double wave = (double)((B + simds - 1) / simds) * (double)(80 * d + 30 * Hp);
    return wave < lane;
}

}  // namespace nfx

using namespace nfx;

extern "C" int64_t nfx_made_backward_max_batch(int d, int H);

extern "C" int nfx_made_seq_backward(const float* packed, const float* in, const float* grad_out,
                                     const float* grad_log_det, float* grad_in, float* factors, int64_t B, int d, int H,
                                     int variant, void* stream) {
    if (variant != NFX_IAF_INVERSE && variant != NFX_MAF_FORWARD)
        return set_error(NFX_EUNSUPPORTED, "made_seq_backward: sequential directions only (NFX_IAF_INVERSE, "
                                           "NFX_MAF_FORWARD); the parallel ones are nfx_made_affine_backward");
    if (B < 0 || d <= 0 || H <= 0) return set_error(NFX_EINVAL, "made_seq_backward: bad shape");
    if (d > 4096 || H > 128)
        return set_error(NFX_EUNSUPPORTED, "made_seq_backward: d=%d H=%d outside d<=4096, H<=128", d, H);
    if (B > nfx_made_backward_max_batch(d, H))
        return set_error(NFX_EUNSUPPORTED, "made_seq_backward: B=%lld above nfx_made_backward_max_batch(%d, %d) = "
                                           "%lld (32-bit factor offsets); split the batch", (long long)B, d, H,
                         (long long)nfx_made_backward_max_batch(d, H));
    if (B == 0) return NFX_OK;
    if (!packed || !in || !grad_out || !grad_log_det || !grad_in || !factors)
        return set_error(NFX_EINVAL, "made_seq_backward: null pointer");
    if (seq_bwd_use_wave(B, d, H))
        return made_seqw_bwd_launch(packed, in, grad_out, grad_log_det, grad_in, factors, B, d, H, variant,
                                    (hipStream_t)stream);
    const int HT = (H + 31) / 32;
    made_seq_bwd_t k = variant == NFX_IAF_INVERSE ? seq_bwd_pick<NFX_IAF_INVERSE>(HT) : seq_bwd_pick<NFX_MAF_FORWARD>(HT);
    const size_t lds = (size_t)3 * 64 * (32 * HT + 4) * sizeof(float);
    int rc = prepare_lds((const void*)k, lds);
    if (rc) return rc;
    const int64_t grid = (B + 63) / 64;
    if (grid > 0x7fffffff) return set_error(NFX_EUNSUPPORTED, "made_seq_backward: batch too large");
    k<<<(unsigned)grid, 64, lds, (hipStream_t)stream>>>(packed, in, grad_out, grad_log_det, grad_in, factors, B, d, H);
    return check_launch("made_seq_bwd_kernel");
}
