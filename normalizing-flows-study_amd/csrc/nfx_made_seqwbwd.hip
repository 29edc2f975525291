// Backward of the SEQUENTIAL MADE directions with a WAVE per sample (H <= 64) — the small-batch
// counterpart of made_seq_bwd_kernel (nfx_made_seqbwd.hip; same math, results within tolerance:
// the recomputed mu/alpha sum by butterfly, not in the forward kernels' order):
// InverseAutoregressiveFlow.inverse (inverse_autoregressive_flow.py:65-103, the IAF density
// direction) and MaskedAutoregressiveFlow.forward (masked_autoregressive_flow.py:46-78) under
// autograd, e.g. the reference's 6x IAF(2, 64) figure model trained full-batch on 2,000 points
// (plots/_common.py:165-167,194-211).
//
// made_seq_bwd_kernel gives a sample one LANE, so 2,000 samples are 32 waves on 1,024 SIMDs, each
// lane walking both sweeps serially (~50k dependent VALU instructions at d = 2, H = 64: 310 us).
// Here lane a owns hidden unit a of ONE sample and the sweeps run across the wave:
//   forward: step i's (mu_i, alpha_i) are two wave reductions over the completed units' h3; the
//     layer-1 pre-activations take a rank-1 update (one FMA per lane); when the units of degree i
//     complete, their h1 is published in LDS and every lane adds W2m[lane, a] h1_a (incrementally:
//     a unit's layer-2 input sum is final once every unit of degree <= its own has completed, and
//     masked weights add exact zeros), then the same for layer 3;
//   reverse: when the units of degree i complete (every output > i has been seen), their ReLU'-gated
//     adjoints are published and every lane adds W3m[a, lane] gh3_a (then W2m), the total adjoint of
//     zs_i is the output gradient plus one wave reduction of W1m[:, i] gh1, and the local (dmu,
//     dalpha) of step i go into the layer-3 output adjoints with one FMA per lane.
// W2m and W3m sit in LDS once per workgroup, row stride Hp + 1 so both the row (reverse) and the
// column (forward) reads of a wave are bank-conflict-free; per wave a published row and the step
// values (zs, mu, alpha) of the sample. Outputs, feature-major factors and epilogue semantics are
// made_seq_bwd_kernel's (its header): grad_in, D4 = (dmu | dalpha), D3/D2/D1, H3/H2/H1, X1 = zs.
#include "nfx_made_kernel.h"

namespace nfx {

__device__ __forceinline__ float wave_sum64(float v) {
    // butterfly: every lane ends with the same (bitwise) sum
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

constexpr int kSeqwbMaxD = 1024;  // step values kept in LDS per wave

template <int VAR, int NWV>
__global__ __launch_bounds__(64 * NWV) void made_seqw_bwd_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, const float* __restrict__ gout,
    const float* __restrict__ gld_in, float* __restrict__ gin, float* __restrict__ fac, int64_t B, int d, int H,
    int HT) {
    constexpr bool IAF = VAR == NFX_IAF_INVERSE;
    const MadeLayout L = made_layout(d, HT);
    const int Hp = L.Hp, RS = Hp + 1;
    extern __shared__ float lds[];
    float* w2 = lds;               // W2m [Hp][Hp + 1]
    float* w3 = w2 + Hp * RS;      // W3m [Hp][Hp + 1]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float* pub = w3 + Hp * RS + wave * (2 * 64 + 3 * d);  // [2][64] published rows
    float* zrow = pub + 128;       // [d] zs
    float* murow = zrow + d;       // [d] raw mu
    float* alrow = murow + d;      // [d] raw alpha
    const float* P = packed;
    for (int e = threadIdx.x; e < Hp * Hp; e += 64 * NWV) {
        const int r = e / Hp, c = e - r * Hp;
        w2[r * RS + c] = P[L.s_w2 + e];
        w3[r * RS + c] = P[L.s_w3 + e];
    }
    __syncthreads();

    const int64_t Pt = B;
    float* D4 = fac;
    float* D3 = D4 + (int64_t)2 * d * Pt;
    float* D2 = D3 + (int64_t)H * Pt;
    float* D1 = D2 + (int64_t)H * Pt;
    float* H3 = D1 + (int64_t)H * Pt;
    float* H2 = H3 + (int64_t)(H + 1) * Pt;
    float* H1 = H2 + (int64_t)(H + 1) * Pt;
    float* X1 = H1 + (int64_t)(H + 1) * Pt;
    const float* ord = P + L.s_deg;
    const bool ul = lane < Hp;                        // lane holds a (possibly padded) unit
    const float mydeg = ul ? ord[lane] : 1e30f;       // padded units: 1e9 (never complete)
    const float b1 = ul ? P[L.s_b1 + lane] : 0.f;
    const float b2 = ul ? P[L.s_b2 + lane] : 0.f;
    const float b3 = ul ? P[L.s_b3 + lane] : 0.f;

    for (int64_t s = (int64_t)blockIdx.x * NWV + wave; s < B; s += (int64_t)gridDim.x * NWV) {
        // ---- forward sweep ----
        float pre1 = b1, acc2 = 0.f, acc3 = 0.f, h1 = 0.f, h2 = 0.f, h3 = 0.f;
        float ld0 = 0.f;
        bool poison = false;
        int p = 0;
        for (int i = 0; i < d; ++i) {
            const float wm = ul ? P[L.s_w4 + (size_t)i * Hp + lane] : 0.f;
            const float wa = ul ? P[L.s_w4 + (size_t)(d + i) * Hp + lane] : 0.f;
            float mu = wave_sum64(wm * h3) + P[L.s_b4 + i];
            float al = wave_sum64(wa * h3) + P[L.s_b4 + d + i];
            if (poison) { mu = __builtin_nanf(""); al = mu; }
            const float xin = in[s * d + i];
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
            if (lane == 0) {
                zrow[i] = zi;
                murow[i] = mu;
                alrow[i] = al;
                X1[(int64_t)i * Pt + s] = zi;
            }
            if (nonfinite(zi)) poison = true;
            if (ul) pre1 = fmaf(P[L.s_w1t + (size_t)i * Hp + lane], zi, pre1);
            int q = p;
            while (q < H && (int)ord[Hp + q] == i) ++q;
            if (q > p) {
                const bool mine = mydeg == (float)i;
                if (mine) h1 = trelu(pre1);
                pub[lane] = h1;
                wave_lds_sync();
                for (int k = p; k < q; ++k) {
                    const int a = (int)ord[2 * Hp + k];
                    if (ul) acc2 = fmaf(w2[lane * RS + a], pub[a], acc2);
                }
                if (mine) h2 = trelu(acc2 + b2);
                pub[64 + lane] = h2;
                wave_lds_sync();
                for (int k = p; k < q; ++k) {
                    const int a = (int)ord[2 * Hp + k];
                    if (ul) acc3 = fmaf(w3[lane * RS + a], pub[64 + a], acc3);
                }
                if (mine) h3 = trelu(acc3 + b3);
                p = q;
            }
        }
        if (lane < H) {
            H1[(int64_t)lane * Pt + s] = h1;
            H2[(int64_t)lane * Pt + s] = h2;
            H3[(int64_t)lane * Pt + s] = h3;
        }

        // ---- reverse sweep ----
        float g3 = 0.f, G2 = 0.f, G1 = 0.f, gh1 = 0.f;
        const float gld = gld_in[s];
        float gld0;
        {
            const float ld1 = nonfinite(ld0) ? 0.f : ld0;
            const float lim = IAF ? 50.f : 100.f;
            gld0 = (nonfinite(ld0) || !(ld1 >= -lim && ld1 <= lim)) ? 0.f : gld;
        }
        int q = H;
        for (int i = d - 1; i >= 0; --i) {
            int pe = q;
            while (pe > 0 && (int)ord[Hp + pe - 1] == i) --pe;
            if (pe < q) {
                const bool mine = mydeg == (float)i;
                wave_lds_sync();  // the previous reads of pub are done
                const float gh3 = (mine && h3 > 0.f) ? g3 : 0.f;
                if (mine && lane < H) D3[(int64_t)lane * Pt + s] = gh3;
                pub[lane] = gh3;
                wave_lds_sync();
                for (int k = pe; k < q; ++k) {
                    const int a = (int)ord[2 * Hp + k];
                    if (ul) G2 = fmaf(w3[a * RS + lane], pub[a], G2);
                }
                const float gh2 = (mine && h2 > 0.f) ? G2 : 0.f;
                if (mine && lane < H) D2[(int64_t)lane * Pt + s] = gh2;
                pub[64 + lane] = gh2;
                wave_lds_sync();
                for (int k = pe; k < q; ++k) {
                    const int a = (int)ord[2 * Hp + k];
                    if (ul) G1 = fmaf(w2[a * RS + lane], pub[64 + a], G1);
                }
                if (mine) {
                    gh1 = h1 > 0.f ? G1 : 0.f;
                    if (lane < H) D1[(int64_t)lane * Pt + s] = gh1;
                }
                q = pe;
            }
            const float w1 = ul ? P[L.s_w1t + (size_t)i * Hp + lane] : 0.f;
            const float dot = wave_sum64(w1 * gh1);
            const float zi = zrow[i], mu = murow[i], al = alrow[i];
            const float gz = gout[s * d + i];
            const float xin = in[s * d + i];
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
            if (lane == 0) {
                gin[s * d + i] = gx;
                D4[(int64_t)i * Pt + s] = dmu;
                D4[(int64_t)(d + i) * Pt + s] = dal;
            }
            if (ul) {
                const float wm = P[L.s_w4 + (size_t)i * Hp + lane];
                const float wa = P[L.s_w4 + (size_t)(d + i) * Hp + lane];
                g3 = fmaf(wa, dal, fmaf(wm, dmu, g3));
            }
        }
        wave_lds_sync();  // this sample's LDS reads are done before the next sample's writes
    }
}

typedef void (*made_seqw_bwd_t)(const float*, const float*, const float*, const float*, float*, float*, int64_t, int,
                                int, int);

// LDS: both matrices + per wave 2 published rows and 3 step rows of d floats.
static size_t seqw_bwd_lds(int d, int HT, int nwv) {
    const int Hp = 32 * HT;
    return (size_t)(2 * Hp * (Hp + 1) + nwv * (128 + 3 * d)) * sizeof(float);
}

bool made_seqw_bwd_supported(int d, int H) { return H <= 64 && d <= kSeqwbMaxD; }

// Launch with 16 waves per workgroup where the LDS allows and the batch still fills every CU,
// else 4.
int made_seqw_bwd_launch(const float* packed, const float* in, const float* gout, const float* gld, float* gin,
                         float* fac, int64_t B, int d, int H, int variant, hipStream_t s) {
    const int HT = (H + 31) / 32;
    const bool wide = seqw_bwd_lds(d, HT, 16) <= 160 * 1024 && B >= 16 * (int64_t)num_cus();
    const int nwv = wide ? 16 : 4;
    made_seqw_bwd_t k = variant == NFX_IAF_INVERSE
                            ? (wide ? made_seqw_bwd_kernel<NFX_IAF_INVERSE, 16> : made_seqw_bwd_kernel<NFX_IAF_INVERSE, 4>)
                            : (wide ? made_seqw_bwd_kernel<NFX_MAF_FORWARD, 16> : made_seqw_bwd_kernel<NFX_MAF_FORWARD, 4>);
    const size_t lds = seqw_bwd_lds(d, HT, nwv);
    int rc = prepare_lds((const void*)k, lds);
    if (rc) return rc;
    int64_t grid = (B + nwv - 1) / nwv;
    const int64_t cap = 8 * (int64_t)num_cus();
    if (grid > cap) grid = cap;
    k<<<(unsigned)grid, 64 * nwv, lds, s>>>(packed, in, gout, gld, gin, fac, B, d, H, HT);
    return check_launch("made_seqw_bwd_kernel");
}

}  // namespace nfx
