// Small-batch affine-coupling kernel: one workgroup per 32 samples, the conditioner spread over
// 2*HT waves (one per (net, hidden output tile)).
//
// The streaming kernel (nfx_affine_kernel.h) gives each wave whole 64-sample chunks: at a few
// thousand samples (the reference's own throughput runs use n = 4000, plots/_common.py:264-274,
// and a strong-scaled shard is small too) only tens of waves exist and each runs its chunk's
// entire MFMA chain alone — the layer takes as long as one wave's 2*HT^2*32 dependent MFMAs.
// Here wave w of a workgroup computes net w / HT, layer-2 output tile w % HT for ONE 32-sample
// tile: layer 1 (K = d, a handful of MFMAs) is recomputed by each wave, layer 2 is HT*16 MFMAs
// per wave, the output layer's dot products are partial per tile and meet in LDS, where the
// first 32 threads finish the affine transform, guards and log-det of their sample. A wave's
// weight operands (its layer-2 row tile, 16*HT floats per lane, and layer 1) are loaded once
// into registers and reused for every tile it grid-strides over; biases, the output layer and
// the mask sit in LDS. (A first version re-read them from L2 per tile: the compiler spread the
// loads through the MFMA chain, ~16 dependent L2 round trips, 23 us per layer at n = 4000.) Same math and guards as the streaming kernel;
// the output-layer sums are associated per hidden tile (a different fp32 rounding order, well
// inside the parity tolerance).
#pragma once
#include "nfx_affine_kernel.h"

namespace nfx {

template <int HT, int D, int DIR, bool LOGP>
__global__ __launch_bounds__(128 * HT) void affine_small_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int accumulate, int64_t ntiles,
    float* __restrict__ logp, double* __restrict__ partials, double* __restrict__ sums, float cgauss) {
    constexpr AffineLayout L = affine_layout(D, HT);
    constexpr int KS1 = L.KS1;
    constexpr int NB1 = HT * 32;            // b1 of one net
    constexpr int NTAIL = L.net - L.b2;     // b2, w3, b3 of one net (contiguous in the image)
    constexpr int NPN = NB1 + NTAIL;
    constexpr int NTHR = 128 * HT;
    // Small per-net pieces (biases, output layer, mask) in LDS; the output-layer partials are
    // double-buffered so one barrier per tile suffices.
    __shared__ __attribute__((aligned(16))) float sw[2 * NPN + up4(D)];
    __shared__ float part[2][2][HT][D][32];
    for (int i = threadIdx.x; i < 2 * NPN + up4(D); i += NTHR) {
        float v;
        if (i >= 2 * NPN) {
            v = packed[L.mask + i - 2 * NPN];
        } else {
            const int net = i / NPN, o = i - net * NPN;
            v = packed[net * L.net + (o < NB1 ? L.b1 + o : L.b2 + o - NB1)];
        }
        sw[i] = v;
    }

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int net = wave / HT, hto = wave % HT;
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    // The wave's weight operands never change across tiles: layer-1 A operand and its
    // layer-2 output row tile stay in registers for the whole grid-stride loop.
    const float* P = packed + net * L.net;
    float w1r[HT][KS1];
#pragma unroll
    for (int ht = 0; ht < HT; ++ht)
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks) w1r[ht][ks] = P[L.w1 + (ht * KS1 + ks) * 64 + lane];
    f32x4 w2r[HT][4];
    {
        const f32x4* wg = reinterpret_cast<const f32x4*>(P + L.w2) + lane;
#pragma unroll
        for (int kt = 0; kt < HT; ++kt)
#pragma unroll
            for (int rq = 0; rq < 4; ++rq) w2r[kt][rq] = wg[((hto * HT + kt) * 4 + rq) * 64];
    }
    __syncthreads();
    const float* sb1 = sw + net * NPN;
    const float* sb2 = sb1 + NB1;                  // [HT][2][16]
    const float* sw3 = sb2 + (L.w3 - L.b2);        // [D][HT][2][16]
    float mkb[KS1];
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) mkb[ks] = (2 * ks + h < D) ? sw[2 * NPN + 2 * ks + h] : 0.f;
    double lpacc = 0.0;

    auto fetch = [&](int64_t t, float (&xb)[KS1]) {
        const int64_t s = t * 32 + col;
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks) {
            const int k = 2 * ks + h;
            xb[ks] = (t < ntiles && k < D && s < B) ? in[s * D + k] : 0.f;
        }
    };
    int64_t t = blockIdx.x;
    float xcur[KS1];
    fetch(t, xcur);
    for (int buf = 0; t < ntiles; t += gridDim.x, buf ^= 1) {
        const int64_t s = t * 32 + col;
        float xnxt[KS1];
        fetch(t + gridDim.x, xnxt);
        // the lane's own sample row for the epilogue (wave 0, lanes 0..31)
        float xr[D];
        const bool fin = wave == 0 && lane < 32 && s < B;
#pragma unroll
        for (int j = 0; j < D; ++j) xr[j] = fin ? in[s * D + j] : 0.f;
        const float ldin = (fin && accumulate) ? logdet[s] : 0.f;

        // layer 1 (K = d), every hidden tile
        f32x16 h1[HT];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
            f32x16 a = load_bias16(sb1 + ht * 32, h);
#pragma unroll
            for (int ks = 0; ks < KS1; ++ks) a = mfma32(w1r[ht][ks], xcur[ks] * mkb[ks], a);
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = trelu(a[r]);
            h1[ht] = a;
        }
        // layer 2, this wave's output tile
        f32x16 a = load_bias16(sb2 + hto * 32, h);
#pragma unroll
        for (int kt = 0; kt < HT; ++kt)
#pragma unroll
            for (int rq = 0; rq < 4; ++rq)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) a = mfma32(w2r[kt][rq][rr], h1[kt][4 * rq + rr], a);
        // output-layer partial dots over this tile's 32 hidden units
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const f32x16 w3 = load_bias16(sw3 + (j * HT + hto) * 32, h);
            float p = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) p = fmaf(w3[r], trelu(a[r]), p);
            p = halves_sum(p, p);  // rows crow(r, 0) + rows crow(r, 1) of sample col
            if (lane < 32) part[buf][net][hto][j][col] = p;
        }
        __syncthreads();
        if (fin) {
#pragma clang fp contract(off)  // separate mul/add roundings, as the reference's torch ops
            const float* sb3s = sw + NB1 + (L.b3 - L.b2);  // net 0 b3 (per net: b1 | b2 w3 b3)
            const float* sb3b = sb3s + NPN;                 // net 1 b3
            float y[D];
            float ld = 0.f;
#pragma unroll
            for (int j = 0; j < D; ++j) {
                float ps = part[buf][0][0][j][col], pb = part[buf][1][0][j][col];
#pragma unroll
                for (int ht = 1; ht < HT; ++ht) {
                    ps = ps + part[buf][0][ht][j][col];
                    pb = pb + part[buf][1][ht][j][col];
                }
                const float sv = tclamp(ps + sb3s[j], -10.f, 10.f);
                const float bv = tclamp(pb + sb3b[j], -10.f, 10.f);
                const float m = sw[2 * NPN + j], om = 1.f - m;
                const float xa = xr[j] * m;
                float tv;
                if constexpr (DIR < 0) {
                    tv = (xr[j] - bv) * exp_fast(-sv);
                    ld = ld + om * (-sv);
                } else {
                    tv = xr[j] * exp_fast(sv) + bv;
                    ld = ld + om * sv;
                }
                const float v = xa + om * tv;
                y[j] = nonfinite(v) ? 0.f : v;
            }
#pragma unroll
            for (int j = 0; j < D; ++j) out[s * D + j] = y[j];
            if (nonfinite(ld)) ld = 0.f;
            const float ldt = accumulate ? ldin + ld : ld;
            logdet[s] = ldt;
            if constexpr (LOGP) {
                float m = gauss_sq0(y[0]);
#pragma unroll
                for (int j = 1; j < D; ++j) m = gauss_sq(m, y[j]);
                const float lp = gauss_lp(m, cgauss, ldt);
                logp[s] = lp;
                lpacc += (double)lp;
            }
        }
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks) xcur[ks] = xnxt[ks];
    }
    if constexpr (LOGP) {
        logp_commit<NTHR>(lpacc, partials, sums, B);
    }
}

template <int HT>
affine_kernel_t affine_small_pick_ht(int d, int dir, bool logp);

}  // namespace nfx
