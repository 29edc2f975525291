// Train-mode affine coupling with WIDE hidden layers (64 < H <= 128: HT = 3, 4 tiles of 32) and
// its backward, for gfx950 — the reference's benchmark-figure model RealNVP(2, 10, 128)
// (plots/_common.py:161, trained by :194-211) and every CouplingLayer(d <= 8, H <= 128).
// Same math, pack (train_layout) and float64 gradient-sum layout (train_grad_layout) as
// nfx_affine_train_kernel.h; what changes is how the work is split, because at HT = 4 one
// wave can no longer hold a whole tile's layer-2 recompute, both nets and the dW2 accumulators
// (2 x 16 x 16 registers), and both nets' W2 (2 x 64 KB) plus its transpose do not fit LDS:
//
//  * one NET per workgroup (blockIdx.y) for the W2-heavy passes; its W2 image is LDS-resident;
//  * a workgroup runs kTWGroups tile groups; a tile group is HT waves that work on the SAME
//    32-sample tile, wave o owning hidden tile o: layer 1 is recomputed whole by every wave
//    (K = d: HT * ceil(d/2) MFMAs) and gives the B operands of layer 2, but each wave computes
//    only its layer-2 output tile (16 HT MFMAs), its statistics / BatchNorm-backward sums and
//    its rows of dW2 (HT accumulator tiles, summed over the wave's tiles in registers);
//  * the output layer's partial dot products meet in LDS (OUT pass: raw net outputs written to
//    a [2][B][D] workspace, so the epilogue backward of either net sees both s and b);
//  * g_a1 = (diag(r2) W2)^T e2 needs every e2 tile: the group's e2 tiles are exchanged through
//    LDS and wave o forms tile o of g_a1 with the transposed weight tiles read from the packed
//    image in global memory (64 KB per net, L2-resident);
//  * BWD3 (layer 1 only) runs both nets in one workgroup (2 HT waves on one tile) so the two
//    nets' dL/dx contributions meet in LDS and are added to dL/dx by one lane in a fixed order.
// Passes: STATS1, STATS2 (per net) -> fold + eval kernel (y, log_det) -> OUT, BWD1, BWD2 (per
// net), BWD3 (both nets). BWD2 also produces the BN1-backward sums (g_a1 is final there).
#pragma once
#include "nfx_affine_train_kernel.h"

namespace nfx {

enum TrainWStage { TW_STATS1 = 0, TW_STATS2 = 1, TW_OUT = 2, TW_BWD1 = 3, TW_BWD2 = 4, TW_BWD3 = 5 };
constexpr int kTWGroups = 2;  // tile groups per workgroup (per-net passes)

__host__ __device__ constexpr bool trainw_both_nets(int stage) { return stage == TW_BWD3; }
__host__ __device__ constexpr int trainw_waves(int HT, int stage) {
    return trainw_both_nets(stage) ? 2 * HT : kTWGroups * HT;
}

// LDS layout. Per-net passes: the net's pack floats [0, w2t) (w1 .. b3, with w2) at their pack
// offsets, then w1c, then the mask. BWD3: per net [0, w2) (w1, c1, g1, e1) + w1c at net * SN.
// Largest image: BWD2 at HT = 4, D = 8: 151.6 KB (fits the 160 KB of a CU; one workgroup).
struct TrainWLds {
    int SN;         // floats per net image
    int w1c;        // offset of w1c inside a net image
    int mask;       // offset of the mask
    int tbuf;       // per-wave 32 x kTS transpose buffers
    int sbuf;       // per-wave [32][2 D] per-sample scratch
    int kc;         // BatchNorm-backward constants [nets][2][Hp]
    int ex;         // e2 exchange [groups][HT][16][64] (BWD2) / output partials (OUT)
    int total;      // floats
};

__host__ __device__ constexpr TrainWLds trainw_lds(int D, int HT, int stage) {
    const TrainLayout L = train_layout(D, HT);
    const bool both = trainw_both_nets(stage);
    const int nw = trainw_waves(HT, stage);
    TrainWLds s{};
    const int base = both ? L.w2 : L.w2t;
    s.SN = (base + D * HT * 32 + 3) & ~3;
    s.w1c = base;
    int o = (both ? 2 : 1) * s.SN;
    s.mask = o; o += (D + 3) & ~3;
    s.tbuf = o; o += nw * 32 * kTS;
    s.sbuf = o;  // per-sample scratch: only BWD1 (delta3) and BWD3 (xa) use it
    if (stage == TW_BWD1 || stage == TW_BWD3) o += nw * 32 * 2 * D;
    s.kc = o; o += (both ? 2 : 1) * 2 * 32 * HT;
    s.ex = o;
    if (stage == TW_BWD2) o += kTWGroups * HT * 16 * 64;
    else if (stage == TW_OUT) o += kTWGroups * HT * 32 * D;
    else if (stage == TW_BWD3) o += 2 * HT * 32 * D;
    s.total = (o + 3) & ~3;
    return s;
}

// Per-net compact partial of one workgroup (floats), and where element i of net n lands in G:
//   BWD1: [Σg_y2 | Σg_y2 x^2] (2 Hp) then dW3 [D][Hp], db3 [D]        -> g1s / g1w blocks
//   BWD2: [Σg_y1 | Σg_y1 x^1] (2 Hp) then Σ e2 a1^T [Hp][Hp], Σ e2 [Hp] -> g2s / g2w blocks
__host__ __device__ constexpr int trainw_len(int D, int HT, int stage) {
    const int Hp = 32 * HT;
    return stage == TW_BWD1 ? 2 * Hp + D * Hp + D : (stage == TW_BWD2 ? 2 * Hp + Hp * Hp + Hp : 0);
}

template <int HT, int D, int STAGE>
__global__ __launch_bounds__(kTWGroups * 4 * 64) void affine_trainw_kernel(
    const float* __restrict__ pack, const float* __restrict__ x, const float* __restrict__ gy,
    const float* __restrict__ gld, float* __restrict__ gx, float* __restrict__ gbuf, float* __restrict__ obuf,
    const double* __restrict__ G, const double* __restrict__ stats2, void* __restrict__ part, int64_t B, int d,
    int dir, int64_t ntiles) {
    constexpr TrainLayout L = train_layout(D, HT);
    constexpr TrainGrad GL = train_grad_layout(D, HT);
    constexpr TrainWLds S = trainw_lds(D, HT, STAGE);
    constexpr bool BOTH = trainw_both_nets(STAGE);
    constexpr int NW = trainw_waves(HT, STAGE);
    constexpr int TG = BOTH ? 1 : kTWGroups;
    constexpr int KS1 = L.KS1;
    constexpr int Hp = 32 * HT;
    extern __shared__ f32x4 lds4[];
    float* sm = reinterpret_cast<float*>(lds4);
    const int net_wg = BOTH ? 0 : (int)blockIdx.y;
    // ---- stage the weight image(s) ----
    for (int nn = 0; nn < (BOTH ? 2 : 1); ++nn) {
        const int n = BOTH ? nn : net_wg;
        const float* src = pack + (size_t)n * L.net;
        float* dst = sm + nn * S.SN;
        const int n0 = BOTH ? L.w2 : L.w2t;  // [0, n0) then w1c
        for (int i = threadIdx.x; i < n0; i += NW * 64) dst[i] = src[i];
        for (int i = threadIdx.x; i < D * HT * 32; i += NW * 64) dst[S.w1c + i] = src[L.w1c + i];
    }
    for (int i = threadIdx.x; i < D; i += NW * 64) sm[S.mask + i] = pack[L.mask + i];
    if constexpr (STAGE == TW_BWD2 || STAGE == TW_BWD3) {
        // k1 = Σg / N, k2 = Σg x^ / N in accumulator order (N < 0: running statistics -> 0)
        const double N = stats2[0];
        const double* Sg = G + (STAGE == TW_BWD2 ? GL.g1s : GL.g2s);
        const int nn_cnt = BOTH ? 2 : 1;
        for (int i = threadIdx.x; i < nn_cnt * 2 * Hp; i += NW * 64) {
            const int nn = i / (2 * Hp), q = (i / Hp) & 1, a = i % Hp;
            const int n = BOTH ? nn : net_wg;
            const int ht = a >> 5, hh = (a >> 4) & 1, r = a & 15;
            const int row = 32 * ht + crow(r, hh);
            sm[S.kc + i] = N > 0.0 ? (float)(Sg[(n * 2 + q) * Hp + row] / N) : 0.f;
        }
    }
    __syncthreads();

    const int lane = lane_id(), h = lane >> 5, col = lane & 31, wave = threadIdx.x >> 6;
    const int grp = BOTH ? 0 : wave / HT;
    const int o = wave % HT;                       // this wave's hidden tile
    const int n = BOTH ? wave / HT : net_wg;        // this wave's net
    const float* P = sm + (BOTH ? n * S.SN : 0);    // net image (pack offsets for w1 .. b3)
    const float* Pg = pack + (size_t)n * L.net;     // the net's packed image in global memory
    float* tbuf = sm + S.tbuf + wave * 32 * kTS;
    float* sbuf = sm + S.sbuf + wave * 32 * 2 * D;
    const float* kcn = sm + S.kc + (BOTH ? n * 2 * Hp : 0);

    float mk[D];
#pragma unroll
    for (int j = 0; j < D; ++j) mk[j] = sm[S.mask + j];

    // ---- per-lane accumulators (transposed layout: lane <-> feature 32 o + col) ----
    float st_c = 0.f;
    double st_s1 = 0.0, st_s2 = 0.0, st_n = 0.0;
    float ac_s1 = 0.f, ac_s2 = 0.f, ac_db = 0.f;
    float ac_w[D], ac_b[D];
    f32x16 ac_dw[HT];
#pragma unroll
    for (int j = 0; j < D; ++j) ac_w[j] = ac_b[j] = 0.f;
    if constexpr (STAGE == TW_BWD2) {
#pragma unroll
        for (int kt = 0; kt < HT; ++kt)
#pragma unroll
            for (int r = 0; r < 16; ++r) ac_dw[kt][r] = 0.f;
    }
    bool first = true;

    // uniform round loop: every wave of the workgroup runs the same number of rounds (barriers)
    const int64_t ngroups = (ntiles + TG - 1) / TG;
    for (int64_t rnd = blockIdx.x; rnd < ngroups; rnd += gridDim.x) {
        const int64_t tile = rnd * TG + grp;
        const bool tile_ok = tile < ntiles;
        const int64_t base = tile * 32;
        const int64_t s = base + col;
        const bool valid = tile_ok && s < B;
        const int64_t sc = valid ? s : 0;
        const float* Pi = P + opaque_zero();
        float xr[D];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const float v = j < d ? x[sc * d + j] : 0.f;
            xr[j] = valid ? v : 0.f;
        }
        float xb[KS1];
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks) {
            const float v0 = xr[2 * ks] * mk[2 * ks];
            const float v1 = (2 * ks + 1 < D) ? xr[2 * ks + 1] * mk[2 * ks + 1] : 0.f;
            xb[ks] = h ? v1 : v0;
        }
        const int64_t rem = tile_ok ? B - base - 16 * h : 0;
        const int nvh = rem <= 0 ? 0 : (rem >= 16 ? 16 : (int)rem);

        auto layer1_tile = [&](int kt) {
            f32x16 a = load_bias16(Pi + L.c1 + kt * 32, h);
#pragma unroll
            for (int ks = 0; ks < KS1; ++ks) a = mfma32(Pi[L.w1 + (kt * KS1 + ks) * 64 + lane], xb[ks], a);
            return a;
        };
        auto bn_relu_tile = [&](int goff, int eoff, int kt, const f32x16& xh) {
            const f32x16 g = load_bias16(Pi + goff + kt * 32, h), e = load_bias16(Pi + eoff + kt * 32, h);
            f32x16 a;
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = trelu(fmaf(g[r], xh[r], e[r]));
            return a;
        };
        auto stats_tile = [&](const f32x16& X) {
            float T[16];
            transpose_tile(tbuf, X, T);
            if (first) st_c = T[0];
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const float v = t < nvh ? T[t] - st_c : 0.f;
                s1 += v;
                s2 = fmaf(v, v, s2);
            }
            st_s1 += (double)s1;
            st_s2 += (double)s2;
        };

        if constexpr (STAGE == TW_STATS1) {
            stats_tile(layer1_tile(o));
            st_n += (double)nvh;
        } else if constexpr (STAGE == TW_BWD3) {
            // ---- layer 1 backward (both nets): e1 = gamma1 (g_y1 - k1 - x^1 k2) ----
            if (h == 0) {
#pragma unroll
                for (int j = 0; j < D; ++j) sbuf[col * 2 * D + j] = xr[j] * mk[j];
            }
            const f32x16 xh1 = layer1_tile(o);
            const f32x16 g = load_bias16(Pi + L.g1 + o * 32, h);
            const f32x16 k1 = load_bias16(kcn + o * 32, h), k2 = load_bias16(kcn + Hp + o * 32, h);
            const int64_t tcl = tile_ok ? tile : 0;
            const float* gq = gbuf + (((tcl * 2 + n) * HT + o) * 16) * 64 + lane;
            f32x16 e1;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float v = g[r] * ((gq[r * 64] - k1[r]) - xh1[r] * k2[r]);
                e1[r] = valid ? v : 0.f;
            }
            float Te[16];
            transpose_tile(tbuf, e1, Te);
            float sb = 0.f;
#pragma unroll
            for (int t = 0; t < 16; ++t) sb += Te[t];
            ac_s1 += sb;
            float gp[D];
#pragma unroll
            for (int j = 0; j < D; ++j) {
                float w = 0.f;
#pragma unroll
                for (int t = 0; t < 16; ++t) w = fmaf(sbuf[(16 * h + t) * 2 * D + j], Te[t], w);
                ac_w[j] += w;
                const f32x16 wc = load_bias16(Pi + S.w1c + (j * HT + o) * 32, h);
                float p = 0.f;
#pragma unroll
                for (int r = 0; r < 16; ++r) p = fmaf(wc[r], e1[r], p);
                gp[j] = halves_sum(p, p);
            }
            // the 2 HT partial dot products meet in LDS; one lane per sample adds them in order
            float* gxx = sm + S.ex;
            if (h == 0) {
#pragma unroll
                for (int j = 0; j < D; ++j) gxx[(wave * 32 + col) * D + j] = gp[j];
            }
            __syncthreads();
            if (wave == 0 && h == 0 && valid) {
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    if (j < d) {
                        float a = 0.f;
                        for (int w = 0; w < NW; ++w) a += gxx[(w * 32 + col) * D + j];
                        gx[s * d + j] = gx[s * d + j] + mk[j] * a;
                    }
                }
            }
            __syncthreads();
        } else {
            // ---- layer 1 (all tiles: layer 2's B operands), layer 2 tile o ----
            f32x16 a1[HT];
#pragma unroll
            for (int kt = 0; kt < HT; ++kt) a1[kt] = bn_relu_tile(L.g1, L.e1, kt, layer1_tile(kt));
            f32x16 xh2;
            {
                const f32x4* wg = reinterpret_cast<const f32x4*>(Pi + L.w2) + lane;
                f32x16 a = load_bias16(Pi + L.c2 + o * 32, h);
#pragma unroll
                for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                    for (int rq = 0; rq < 4; ++rq) {
                        const f32x4 w = wg[((o * HT + kt) * 4 + rq) * 64];
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) a = mfma32(w[rr], a1[kt][4 * rq + rr], a);
                    }
                xh2 = a;
            }
            if constexpr (STAGE == TW_STATS2) {
                stats_tile(xh2);
                st_n += (double)nvh;
            } else if constexpr (STAGE == TW_OUT) {
                // output layer: partial dot products of tile o's rows, summed over the HT waves
                const f32x16 a2 = bn_relu_tile(L.g2, L.e2, o, xh2);
                float* ox = sm + S.ex + grp * HT * 32 * D;
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    const f32x16 w3 = load_bias16(Pi + L.w3 + (j * HT + o) * 32, h);
                    float p = 0.f;
#pragma unroll
                    for (int r = 0; r < 16; ++r) p = fmaf(w3[r], a2[r], p);
                    p = halves_sum(p, p);
                    if (h == 0) ox[(o * 32 + col) * D + j] = p;
                }
                __syncthreads();
                if (o == 0 && h == 0 && valid) {
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        float a = 0.f;
#pragma unroll
                        for (int w = 0; w < HT; ++w) a += ox[(w * 32 + col) * D + j];
                        obuf[((int64_t)n * B + s) * D + j] = a + Pi[L.b3 + j];
                    }
                }
                __syncthreads();
            } else {
                // ---- epilogue backward (coupling_layer.py:40-96 under autograd) from the raw net
                // outputs of both nets (OUT pass) ----
                float outv[2][D], gyr[D];
#pragma unroll
                for (int nn = 0; nn < 2; ++nn)
#pragma unroll
                    for (int j = 0; j < D; ++j) outv[nn][j] = obuf[((int64_t)nn * B + sc) * D + j];
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    const float v = j < d ? gy[sc * d + j] : 0.f;
                    gyr[j] = valid ? v : 0.f;
                }
                const float gl_in = valid ? gld[sc] : 0.f;
                float dl[D], gxd[D];
                {
#pragma clang fp contract(off)
                    float ld = 0.f;
                    float ev[D], sv[D], bv[D];
                    bool fy[D];
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        sv[j] = tclamp(outv[0][j], -10.f, 10.f);
                        bv[j] = tclamp(outv[1][j], -10.f, 10.f);
                        const float m = mk[j], om = 1.f - m;
                        float t;
                        if (dir < 0) {
                            ev[j] = exp_fast(-sv[j]);
                            t = (xr[j] - bv[j]) * ev[j];
                            ld = ld + om * (-sv[j]);
                        } else {
                            ev[j] = exp_fast(sv[j]);
                            t = xr[j] * ev[j] + bv[j];
                            ld = ld + om * sv[j];
                        }
                        fy[j] = !nonfinite(xr[j] * m + om * t);
                    }
                    const float gl = nonfinite(ld) ? 0.f : gl_in;
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        const float m = mk[j], om = 1.f - m;
                        const float gv = (fy[j] && j < d) ? gyr[j] : 0.f;
                        const float gt = gv * om;
                        float gs, gb;
                        if (dir < 0) {
                            gs = (gt * (xr[j] - bv[j])) * (-ev[j]) + gl * (-om);
                            gb = -(gt * ev[j]);
                        } else {
                            gs = (gt * xr[j]) * ev[j] + gl * om;
                            gb = gt;
                        }
                        gxd[j] = gv * m + gt * ev[j];
                        if (j >= d) gs = gb = 0.f;
                        const float g_own = n == 0 ? gs : gb;
                        const float raw = outv[n][j];
                        dl[j] = (raw >= -10.f && raw <= 10.f) ? g_own : 0.f;
                    }
                }
                // g_y2 of tile o = relu'(y2) W3[:, tile o]^T delta3
                const f32x16 g2 = load_bias16(Pi + L.g2 + o * 32, h), e2c = load_bias16(Pi + L.e2 + o * 32, h);
                f32x16 gy2, a2;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    a2[r] = trelu(fmaf(g2[r], xh2[r], e2c[r]));
                    gy2[r] = 0.f;
                }
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    const f32x16 w3 = load_bias16(Pi + L.w3 + (j * HT + o) * 32, h);
#pragma unroll
                    for (int r = 0; r < 16; ++r) gy2[r] = fmaf(w3[r], dl[j], gy2[r]);
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) gy2[r] = a2[r] > 0.f ? gy2[r] : 0.f;
                if constexpr (STAGE == TW_BWD1) {
                    if (n == 0 && o == 0 && h == 0 && valid) {
#pragma unroll
                        for (int j = 0; j < D; ++j)
                            if (j < d) gx[s * d + j] = gxd[j];
                    }
                    if (h == 0) {
#pragma unroll
                        for (int j = 0; j < D; ++j) sbuf[col * 2 * D + j] = dl[j];
                    }
                    if (o == 0) {
#pragma unroll
                        for (int j = 0; j < D; ++j) ac_b[j] += h == 0 ? dl[j] : 0.f;
                    }
                    float Tg[16], Tx[16], Ta[16];
                    transpose_tile(tbuf, gy2, Tg);
                    transpose_tile(tbuf, xh2, Tx);
                    transpose_tile(tbuf, a2, Ta);
                    float s1 = 0.f, s2 = 0.f;
#pragma unroll
                    for (int t = 0; t < 16; ++t) {
                        s1 += Tg[t];
                        s2 = fmaf(Tg[t], Tx[t], s2);
                    }
                    ac_s1 += s1;
                    ac_s2 += s2;
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        float w = 0.f;
#pragma unroll
                        for (int t = 0; t < 16; ++t) w = fmaf(sbuf[(16 * h + t) * 2 * D + j], Ta[t], w);
                        ac_w[j] += w;
                    }
                } else {  // TW_BWD2
                    // e2 = gamma2 (g_y2 - k1 - x^2 k2)
                    f32x16 e2;
                    {
                        const f32x16 k1 = load_bias16(kcn + o * 32, h), k2 = load_bias16(kcn + Hp + o * 32, h);
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const float v = g2[r] * ((gy2[r] - k1[r]) - xh2[r] * k2[r]);
                            e2[r] = valid ? v : 0.f;
                        }
                    }
                    {
                        float Te[16];
                        transpose_tile(tbuf, e2, Te);
                        float sb = 0.f;
#pragma unroll
                        for (int t = 0; t < 16; ++t) sb += Te[t];
                        ac_db += sb;
#pragma unroll
                        for (int kt = 0; kt < HT; ++kt) {
                            float Ta[16];
                            transpose_tile(tbuf, a1[kt], Ta);
#pragma unroll
                            for (int t = 0; t < 16; ++t) ac_dw[kt] = mfma32(Te[t], Ta[t], ac_dw[kt]);
                        }
                    }
                    // exchange the group's e2 tiles; wave o forms g_a1 tile o = sum_o' W2r[o', o]^T e2[o']
                    float* ex = sm + S.ex + grp * HT * 1024;
#pragma unroll
                    for (int r = 0; r < 16; ++r) ex[(o * 16 + r) * 64 + lane] = e2[r];
                    __syncthreads();
                    f32x16 ga;
#pragma unroll
                    for (int r = 0; r < 16; ++r) ga[r] = 0.f;
                    const f32x4* wt = reinterpret_cast<const f32x4*>(Pg + L.w2t) + lane;
#pragma unroll
                    for (int op = 0; op < HT; ++op) {
                        f32x4 w[4];
#pragma unroll
                        for (int rq = 0; rq < 4; ++rq) w[rq] = wt[((o * HT + op) * 4 + rq) * 64];
#pragma unroll
                        for (int rq = 0; rq < 4; ++rq)
#pragma unroll
                            for (int rr = 0; rr < 4; ++rr)
                                ga = mfma32(w[rq][rr], ex[(op * 16 + 4 * rq + rr) * 64 + lane], ga);
                    }
                    __syncthreads();  // the exchange buffer is rewritten next round
#pragma unroll
                    for (int r = 0; r < 16; ++r) ga[r] = a1[o][r] > 0.f ? ga[r] : 0.f;
                    const int64_t tcl = tile_ok ? tile : 0;
                    float* gp = gbuf + (((tcl * 2 + n) * HT + o) * 16) * 64 + lane;
                    if (tile_ok) {
#pragma unroll
                        for (int r = 0; r < 16; ++r) gp[r * 64] = ga[r];
                    }
                    const f32x16 xh1 = layer1_tile(o);
                    float Tg[16], Tx[16];
                    transpose_tile(tbuf, ga, Tg);
                    transpose_tile(tbuf, xh1, Tx);
                    float s1 = 0.f, s2 = 0.f;
#pragma unroll
                    for (int t = 0; t < 16; ++t) {
                        s1 += Tg[t];
                        s2 = fmaf(Tg[t], Tx[t], s2);
                    }
                    ac_s1 += s1;
                    ac_s2 += s2;
                }
            }
        }
        first = false;
    }

    // ---- workgroup combine: tile groups in order, into LDS (the weight region is free now) ----
    __syncthreads();
    float* red = sm;
    double* redd = reinterpret_cast<double*>(sm);
    constexpr int LEN = trainw_len(D, HT, STAGE);
    static_assert(LEN <= S.SN + (BOTH ? S.SN : 0) || STAGE == TW_OUT || STAGE == TW_STATS1 || STAGE == TW_STATS2 ||
                      STAGE == TW_BWD3,
                  "reduction buffer must fit the weight region");
    static_assert(2 * Hp * 3 * 2 <= S.total, "statistics triples must fit LDS");
    static_assert(GL.len3 <= S.total, "BWD3 block must fit LDS");
    if constexpr (STAGE == TW_STATS1 || STAGE == TW_STATS2) {
        // triples [2 nets][Hp][3]; this workgroup's net only (the other net's rows stay zero: n = 0
        // triples are skipped by the merge)
        for (int i = threadIdx.x; i < 2 * Hp * 3; i += NW * 64) redd[i] = 0.0;
        __syncthreads();
        for (int g = 0; g < TG; ++g) {
            if (grp == g) {
                double cnt = st_n, mean = 0.0, m2 = 0.0;
                if (cnt > 0.0) {
                    mean = (double)st_c + st_s1 / cnt;
                    m2 = st_s2 - st_s1 * st_s1 / cnt;
                    if (m2 < 0.0) m2 = 0.0;
                }
                const double nb = __shfl_xor(cnt, 32, 64), mb = __shfl_xor(mean, 32, 64), qb = __shfl_xor(m2, 32, 64);
                if (h == 0) {
                    if (cnt == 0.0) {
                        cnt = nb; mean = mb; m2 = qb;
                    } else {
                        chan_merge(cnt, mean, m2, nb, mb, qb);
                    }
                    double* q = redd + (n * Hp + 32 * o + col) * 3;
                    if (q[0] == 0.0) {
                        q[0] = cnt; q[1] = mean; q[2] = m2;
                    } else {
                        double a = q[0], b = q[1], c = q[2];
                        chan_merge(a, b, c, cnt, mean, m2);
                        q[0] = a; q[1] = b; q[2] = c;
                    }
                }
            }
            __syncthreads();
        }
        double* pw = reinterpret_cast<double*>(part) + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * (2 * Hp * 3);
        for (int i = threadIdx.x; i < 2 * Hp * 3; i += NW * 64) pw[i] = redd[i];
    } else if constexpr (STAGE == TW_BWD1 || STAGE == TW_BWD2) {
        for (int g = 0; g < TG; ++g) {
            if (grp == g) {
                auto put = [&](int idx, float v) { red[idx] = g ? red[idx] + v : v; };
                const float a = halves_sum(ac_s1, ac_s1), b = halves_sum(ac_s2, ac_s2);
                if (h == 0) {
                    put(32 * o + col, a);
                    put(Hp + 32 * o + col, b);
                }
                if constexpr (STAGE == TW_BWD1) {
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        const float w = halves_sum(ac_w[j], ac_w[j]);
                        if (h == 0) put(2 * Hp + j * Hp + 32 * o + col, w);
                    }
                    if (o == 0) {
#pragma unroll
                        for (int j = 0; j < D; ++j) {
                            float v = ac_b[j];
#pragma unroll
                            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
                            if (lane == 0) put(2 * Hp + D * Hp + j, v);
                        }
                    }
                } else {
                    const float c = halves_sum(ac_db, ac_db);
                    if (h == 0) put(2 * Hp + Hp * Hp + 32 * o + col, c);
#pragma unroll
                    for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                        for (int r = 0; r < 16; ++r) put(2 * Hp + (32 * o + crow(r, h)) * Hp + 32 * kt + col, ac_dw[kt][r]);
                }
            }
            __syncthreads();
        }
        float* pw = reinterpret_cast<float*>(part) + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * LEN;
        for (int i = threadIdx.x; i < LEN; i += NW * 64) pw[i] = red[i];
    } else if constexpr (STAGE == TW_BWD3) {
        // g3w block [2 nets][D*Hp + Hp]: dW1 sums [D][Hp], db1 sums [Hp]
        const float c = halves_sum(ac_s1, ac_s1);
        if (h == 0) red[n * (D * Hp + Hp) + D * Hp + 32 * o + col] = c;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const float w = halves_sum(ac_w[j], ac_w[j]);
            if (h == 0) red[n * (D * Hp + Hp) + j * Hp + 32 * o + col] = w;
        }
        __syncthreads();
        float* pw = reinterpret_cast<float*>(part) + (int64_t)blockIdx.x * GL.len3;
        for (int i = threadIdx.x; i < GL.len3; i += NW * 64) pw[i] = red[i];
    }
}

typedef void (*affine_trainw_kernel_t)(const float*, const float*, const float*, const float*, float*, float*, float*,
                                       const double*, const double*, void*, int64_t, int, int, int64_t);

template <int HT>
affine_trainw_kernel_t affine_trainw_pick_ht(int D, int stage);

}  // namespace nfx
