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
//   w3 [d][HT][2][16]       output layer, by (j, k tile, half, r) for the VALU dot    (d <= 8)
//   b3 [up4(d)]
//   w3 [NJ][HT][4][64][4]   output layer as MFMA A-operand tiles, NJ = ceil(d/32)     (d > 8)
//   b3 [NJ][2][16]          its bias in accumulator order
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
    if (d <= 8) {  // VALU output layer (affine_coupling_kernel)
        L.w3 = o; o += d * HT * 32;
        L.b3 = o; o += up4(d);
    } else {       // MFMA output layer (affine_wide_kernel): A-operand tiles + accumulator-order bias
        const int NJ = (d + 31) / 32;
        L.w3 = o; o += NJ * HT * 1024;
        L.b3 = o; o += NJ * 32;
    }
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
    float* __restrict__ logp, double* __restrict__ partials, double* __restrict__ sums, float cgauss) {
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
        logp_commit<256>(lpacc, partials, sums, B);
    }
}


// ---- wide coupling layers (8 < d <= 64, e.g. UCI-shaped RealNVP d = 43 / 63) -------------------
// A wave owns a 32-sample tile whose [32 x d] x block sits in a wave-private LDS tile (odd row
// stride, conflict-free column reads), loaded and stored row by row with coalesced accesses.
// Layer 1 (K = d) reads its B operands (x * mask) from the tile, layers 2 and 3 (H -> d, one
// 32-row MFMA tile per 32 output dims) keep activations in accumulator registers, and the
// affine epilogue runs in accumulator layout on the tile in place. Weights (both nets) are
// read from L2 (up to ~260 KB at H = 128, beyond LDS).
constexpr int kWideWaves = 4;

template <int HT>
__device__ __forceinline__ void wide_net(const float* __restrict__ P, const AffineLayout& L, const float* xt, int S,
                                         const float* __restrict__ mask, int d, f32x16 (&res)[2]) {
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    f32x16 h1[HT];
#pragma unroll
    for (int ht = 0; ht < HT; ++ht) h1[ht] = load_bias16(P + L.b1 + ht * 32, h);
    for (int ks = 0; ks < L.KS1; ++ks) {
        const int k = 2 * ks + h;
        const float xb = k < d ? xt[col * S + k] * mask[k] : 0.f;
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) h1[ht] = mfma32(P[L.w1 + (ht * L.KS1 + ks) * 64 + lane], xb, h1[ht]);
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
    const int NJ = (d + 31) / 32;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (j < NJ) {
            f32x16 a = load_bias16(P + L.b3 + j * 32, h);
#pragma unroll
            for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) {
                    const f32x4 w = *reinterpret_cast<const f32x4*>(P + L.w3 + (((j * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) a = mfma32(w[rr], h2[kt][4 * rq + rr], a);
                }
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = tclamp(a[r], -10.f, 10.f);
            res[j] = a;
        } else {
            res[j] = f32x16{};
        }
    }
}

template <int HT, int DIR, bool LOGP>
__global__ __launch_bounds__(64 * kWideWaves) void affine_wide_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d, int accumulate, int64_t ntiles,
    float* __restrict__ logp, double* __restrict__ partials, double* __restrict__ sums, float cgauss) {
    const AffineLayout L = affine_layout(d, HT);
    const int S = d | 1;
    extern __shared__ f32x4 lds4[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float* xt = reinterpret_cast<float*>(lds4) + wave * 32 * S;
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    const float* mask = packed + L.mask;
    double lpacc = 0.0;
    for (int64_t t = (int64_t)blockIdx.x * kWideWaves + wave; t < ntiles; t += (int64_t)gridDim.x * kWideWaves) {
        const int64_t base = t * 32;
        const int rows = (int)(B - base < 32 ? B - base : 32);
        const float* src = in + base * d;
        for (int i = lane; i < 32 * d; i += 64) {
            const int r = i / d, c = i - r * d;
            xt[r * S + c] = r < rows ? src[i] : 0.f;
        }
        const float ldin = (accumulate && lane < rows) ? logdet[base + lane] : 0.f;
        wave_lds_sync();
        const float* Pw = packed + opaque_zero();
        f32x16 sv[2], bv[2];
        wide_net<HT>(Pw, L, xt, S, mask, d, sv);
        wide_net<HT>(Pw + L.net, L, xt, S, mask, d, bv);
        float ldp = 0.f;
        {
#pragma clang fp contract(off)  // separate mul/add roundings, as the reference's torch ops
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int dim = 32 * j + crow(r, h);
                    if (dim < d) {
                        float* px = xt + col * S + dim;
                        const float xv = *px, m = mask[dim], om = 1.f - m;
                        float tv;
                        if constexpr (DIR < 0) {
                            tv = (xv - bv[j][r]) * exp_fast(-sv[j][r]);
                            ldp = ldp + om * (-sv[j][r]);
                        } else {
                            tv = xv * exp_fast(sv[j][r]) + bv[j][r];
                            ldp = ldp + om * sv[j][r];
                        }
                        const float v = xv * m + om * tv;
                        *px = nonfinite(v) ? 0.f : v;
                    }
                }
        }
        float ld = halves_sum(ldp, ldp);  // lanes 0..31: sample col
        if (nonfinite(ld)) ld = 0.f;
        wave_lds_sync();
        float* dst = out + base * d;
        for (int i = lane; i < rows * d; i += 64) {
            const int r = i / d, c = i - r * d;
            dst[i] = xt[r * S + c];
        }
        if (lane < rows) {
            const float ldt = accumulate ? ldin + ld : ld;
            logdet[base + lane] = ldt;
            if constexpr (LOGP) {
                float m = gauss_sq0(xt[lane * S]);
                for (int c = 1; c < d; ++c) m = gauss_sq(m, xt[lane * S + c]);
                const float lp = gauss_lp(m, cgauss, ldt);
                logp[base + lane] = lp;
                lpacc += (double)lp;
            }
        }
        wave_lds_sync();
    }
    if constexpr (LOGP) {
        logp_commit<64 * kWideWaves>(lpacc, partials, sums, B);
    }
}

typedef void (*affine_kernel_t)(const float*, const float*, float*, float*, int64_t, int, int64_t,
                                float*, double*, double*, float);

template <int HT>
affine_kernel_t affine_pick_ht(int d, int dir, bool logp);

}  // namespace nfx
