// Affine-coupling kernel template (see nfx_affine.hip for the design notes).
#pragma once
#include <type_traits>

#include "nfx_common.h"

namespace nfx {

__host__ __device__ constexpr int up4(int v) { return (v + 3) & ~3; }

// Packed weight image (floats). Per net (s_net = 0, b_net = 1):
//   w1 [HT][KS1][64]        A operand of layer 1 (BN folded)
//   b1 [HT][2][16]          bias of layer 1 at accumulator register r of half h (BN folded)
//   w2 [HT][HT][4][64][4]   A operand of layer 2: [out tile][k tile][r/4][lane][r%4]
//   b2 [HT][2][16]
//   w3 [d][HT][2][16]       output layer, by (j, k tile, half, r) for the VALU dot
//   b3 [up4(d)]
// then mask [up4(d)].
struct AffineLayout {
    int d, HT, KS1;
    int w1, b1, w2, b2, w3, b3, net, mask, total;
};

__host__ __device__ constexpr AffineLayout affine_layout(int d, int HT) {
    AffineLayout L{};
    L.d = d;
    L.HT = HT;
    L.KS1 = (d + 1) / 2;
    int o = 0;
    L.w1 = o; o += HT * L.KS1 * 64;
    L.b1 = o; o += HT * 32;
    L.w2 = o; o += HT * HT * 16 * 64;
    L.b2 = o; o += HT * 32;
    L.w3 = o; o += d * HT * 32;
    L.b3 = o; o += up4(d);
    L.net = o;
    L.mask = 2 * o;
    L.total = 2 * o + up4(d);
    return L;
}

template <int D>
__device__ __forceinline__ void load_row(const float* __restrict__ p, float (&v)[D]) {
    if constexpr (D == 2) {
        float2 t = *reinterpret_cast<const float2*>(p);
        v[0] = t.x; v[1] = t.y;
    } else if constexpr (D == 4) {
        float4 t = *reinterpret_cast<const float4*>(p);
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else {
#pragma unroll
        for (int j = 0; j < D; ++j) v[j] = p[j];
    }
}

template <int D>
__device__ __forceinline__ void store_row(float* __restrict__ p, const float (&v)[D]) {
    if constexpr (D == 2) {
        *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
    } else if constexpr (D == 4) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
        for (int j = 0; j < D; ++j) p[j] = v[j];
    }
}

// Conditioner MLP of one net for a 64-sample chunk; returns clamp(net(x*m), -10, 10)[j] for the
// lane's own sample (lane l <-> sample chunk*64 + l). TILES = 1: a 32-sample half chunk (sample
// tile 1 is skipped; lanes 32..63 return unused values).
template <int HT, int D, int TILES = 2>
__device__ __forceinline__ void affine_net(const float* __restrict__ P, const AffineLayout& L,
                                           const float (&xb)[2][(D + 1) / 2], float (&res)[D]) {
    constexpr int KS1 = (D + 1) / 2;
    const int lane = lane_id(), h = lane >> 5;

    // Layer 1: [H x d] * [d x 32] per sample tile, bias-initialised accumulators, ReLU.
    f32x16 h1[HT][2];
#pragma unroll
    for (int ht = 0; ht < HT; ++ht) {
        f32x16 a0, a1;
        load_bias16_x2(P + L.b1 + ht * 32, h, a0, a1);
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks) {
            const float w = P[L.w1 + (ht * KS1 + ks) * 64 + lane];
            a0 = mfma32(w, xb[0][ks], a0);
            if constexpr (TILES == 2) a1 = mfma32(w, xb[1][ks], a1);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            a0[r] = trelu(a0[r]);
            if constexpr (TILES == 2) a1[r] = trelu(a1[r]);
        }
        h1[ht][0] = a0;
        h1[ht][1] = a1;
    }

    // Layer 2 (H x H) tile by tile; each finished tile is ReLU'd and folded into the
    // output-layer partial dot products right away (keeps one tile of h2 live).
    float part[D][2];
#pragma unroll
    for (int j = 0; j < D; ++j) part[j][0] = part[j][1] = 0.f;
    const f32x4* wg = reinterpret_cast<const f32x4*>(P + L.w2) + lane;
#pragma unroll
    for (int hto = 0; hto < HT; ++hto) {
        f32x16 a0, a1;
        load_bias16_x2(P + L.b2 + hto * 32, h, a0, a1);
#pragma unroll
        for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
            for (int rq = 0; rq < 4; ++rq) {
                // (a one-group-ahead weight prefetch here measured 5% slower: the compiler
                // then interleaves both nets at 217 VGPRs = 2 waves/SIMD instead of 3)
                const f32x4 w = wg[((hto * HT + kt) * 4 + rq) * 64];
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    a0 = mfma32(w[rr], h1[kt][0][4 * rq + rr], a0);
                    if constexpr (TILES == 2) a1 = mfma32(w[rr], h1[kt][1][4 * rq + rr], a1);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const f32x16 w3 = load_bias16(P + L.w3 + (j * HT + hto) * 32, h);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                part[j][0] = fmaf(w3[r], trelu(a0[r]), part[j][0]);
                if constexpr (TILES == 2) part[j][1] = fmaf(w3[r], trelu(a1[r]), part[j][1]);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < D; ++j)
        res[j] = tclamp(halves_sum(part[j][0], part[j][1]) + P[L.b3 + j], -10.f, 10.f);
}

// LOGP: fused log_prob epilogue for the last layer of an inverse chain — logp = -0.5*(c +
// sum_j z_j^2) + total log-det per sample, and one float64 partial sum per workgroup.
template <int HT, int D, int DIR, bool LOGP>
__global__ __launch_bounds__(256) void affine_coupling_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int accumulate, int64_t nchunks,
    float* __restrict__ logp, double* __restrict__ partials, float cgauss) {
    constexpr AffineLayout L = affine_layout(D, HT);
    constexpr int KS1 = L.KS1;
    extern __shared__ f32x4 lds4[];
    {
        const f32x4* src = reinterpret_cast<const f32x4*>(packed);
        for (int i = threadIdx.x; i < L.total / 4; i += 256) lds4[i] = src[i];
    }
    __syncthreads();
    const float* sm = reinterpret_cast<const float*>(lds4);

    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    float mk[D], mkb[KS1];
#pragma unroll
    for (int j = 0; j < D; ++j) mk[j] = sm[L.mask + j];
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) mkb[ks] = (2 * ks + h < D) ? sm[L.mask + 2 * ks + h] : 0.f;

    // Work split: every wave takes F = nchunks / nwaves whole 64-sample chunks (grid-stride); the
    // R leftover chunks go out as 2R 32-sample half chunks, one to each of the first 2R waves
    // (when 2R <= nwaves), so a SIMD's last round is half a chunk instead of a whole one: at
    // B = 1M, 15.26 chunks per SIMD ran as 16, now as 15.5. (Otherwise the first R waves take
    // one more whole chunk.)
    const int64_t wv = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t F = nchunks / nwaves, R = nchunks - F * nwaves;
    const bool split = 2 * R <= nwaves;
    const int64_t nfull = split ? F : F + (wv < R ? 1 : 0);
    const bool half = split && wv < 2 * R;
    const int64_t half_base = F * nwaves * 64 + wv * 32;

    // Software pipeline: the x rows (both layouts) and the incoming log-det of the next unit are
    // loaded while the current one computes, so HBM latency never sits in front of the MFMAs.
    struct Fetch {
        float xb[2][KS1];  // layer-1 B operands x[base+32st+col][2ks+h] (unmasked)
        float xr[D];       // the lane's own sample row
        float ldin;        // log-det accumulated so far (accumulate = 1)
    };
    // unit u < nfull: chunk wv + u nwaves (64 samples); u == nfull: the half chunk, if any
    auto fetch = [&](int64_t u, Fetch& f) {
        const int64_t base = u < nfull ? (wv + u * nwaves) * 64 : half_base;
        const int nsamp = u < nfull ? 64 : (u == nfull && half ? 32 : 0);
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            const int64_t s = base + 32 * st + col;
#pragma unroll
            for (int ks = 0; ks < KS1; ++ks) {
                const int k = 2 * ks + h;
                f.xb[st][ks] = (32 * st + col < nsamp && k < D && s < B) ? in[s * D + k] : 0.f;
            }
        }
        const int64_t so = base + lane;
        if (lane < nsamp && so < B) {
            load_row<D>(in + so * D, f.xr);
            f.ldin = accumulate ? logdet[so] : 0.f;
        } else {
#pragma unroll
            for (int j = 0; j < D; ++j) f.xr[j] = 0.f;
            f.ldin = 0.f;
        }
    };

    double lpacc = 0.0;
    // one unit: 2 sample tiles (TILES = 2) or the half chunk (TILES = 1, lanes 0..31)
    auto unit = [&](auto tiles_c, int64_t base, const Fetch& cur) {
        constexpr int TILES = decltype(tiles_c)::value;
        const float* smi = sm + opaque_zero();
        float xb[2][KS1];
#pragma unroll
        for (int st = 0; st < 2; ++st) {
#pragma unroll
            for (int ks = 0; ks < KS1; ++ks) xb[st][ks] = cur.xb[st][ks] * mkb[ks];
        }

        float sv[D], bv[D];
        affine_net<HT, D, TILES>(smi, L, xb, sv);
        affine_net<HT, D, TILES>(smi + L.net, L, xb, bv);

        const int64_t so = base + lane;
        if (lane < 32 * TILES && so < B) {
#pragma clang fp contract(off)  // separate mul/add roundings, as the reference's torch ops
            float y[D];
            float ld = 0.f;
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const float m = mk[j], om = 1.f - m;
                const float xa = cur.xr[j] * m;
                float t;
                if constexpr (DIR < 0) {
                    t = (cur.xr[j] - bv[j]) * exp_fast(-sv[j]);
                    ld = ld + om * (-sv[j]);
                } else {
                    t = cur.xr[j] * exp_fast(sv[j]) + bv[j];
                    ld = ld + om * sv[j];
                }
                const float v = xa + om * t;
                y[j] = nonfinite(v) ? 0.f : v;
            }
            if (nonfinite(ld)) ld = 0.f;
            store_row<D>(out + so * D, y);
            const float ldt = accumulate ? cur.ldin + ld : ld;
            logdet[so] = ldt;
            if constexpr (LOGP) {
                float m = gauss_sq0(y[0]);
#pragma unroll
                for (int j = 1; j < D; ++j) m = gauss_sq(m, y[j]);
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
        unit(std::integral_constant<int, 2>{}, (wv + u * nwaves) * 64, cur);
        cur = nxt;
    }
    if (half) unit(std::integral_constant<int, 1>{}, half_base, cur);
    if constexpr (LOGP) {
        const double t = block_sum_f64<256>(lpacc);
        if (threadIdx.x == 0) partials[blockIdx.x] = t;
    }
}

typedef void (*affine_kernel_t)(const float*, const float*, float*, float*, int64_t, int, int64_t,
                                float*, double*, float);

template <int HT>
affine_kernel_t affine_pick_ht(int d, int dir, bool logp);

}  // namespace nfx
