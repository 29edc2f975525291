// Train-mode affine coupling (RealNVP CouplingLayer with batch-statistics BatchNorm) and its
// backward, for gfx950. See nfx_affine_train.hip for the pass structure and the math.
//
// Every kernel here walks the batch in 32-sample tiles, one tile per wave per iteration
// (grid-stride), with the conditioner MLPs on fp32 MFMA exactly like the eval kernel: hidden
// activations in accumulator layout, "hidden-unit rows x sample columns" (nfx_common.h).
// Reductions over the SAMPLE dimension (BatchNorm statistics, weight and BN-parameter
// gradients) need the sample index off the lane: a per-wave LDS transpose turns an
// accumulator tile into lane l <-> feature (l & 31), samples 16*(l >> 5) + t (t = 0..15).
// In that layout the per-feature sums are lane-local adds, and a weight gradient
// dW = sum_s P[:, s] Q[:, s]^T is an MFMA whose k dimension runs over samples
// (A = P^T-tile, B = Q^T-tile, both in the transposed layout).
#pragma once
#include "nfx_common.h"

namespace nfx {

// TS_BWD1K / TS_BWD2K: BWD1 / BWD2 reading the layer-2 pre-activations STATS2 kept in HBM
// (`keep`, 512 B per sample at H = 64) instead of recomputing layers 1-2 of both nets.
// TS_OUTK: the layer's forward output (y, log-det) from the kept pre-activations.
enum TrainStage {
    TS_STATS1 = 0, TS_STATS2 = 1, TS_BWD1 = 2, TS_BWD2 = 3, TS_BWD3 = 4, TS_BWD1K = 5, TS_BWD2K = 6, TS_OUTK = 7
};

constexpr int kTS = 36;  // row stride (floats) of a per-wave 32 x 32 transpose buffer

// Train pack, per net (floats). BatchNorm enters as x^ = (h - mu) * r, r = 1/sqrt(var + eps)
// folded into the linear layer ("identity fold": mu = 0, r = 1 when the statistics of that layer
// are not known yet), then y = gamma * x^ + beta on the VALU:
//   w1  [HT][KS1][64]       A operand of diag(r1) W1          (columns = inputs)
//   c1  [HT][32]            r1 (b1 - mu1)                       accumulator order [tile][half][16]
//   g1  [HT][32], e1 [HT][32]   gamma1, beta1                   accumulator order
//   w2  [HT][HT][4][64][4]  A operand of diag(r2) W2            [out tile][k tile][r/4][lane][r%4]
//   c2, g2, e2 [HT][32]
//   w3  [D][HT][32]         W3[j][row]                          accumulator order
//   b3  [D]
//   w2t [HT][HT][4][64][4]  A operand of (diag(r2) W2)^T         [in tile][out tile][..]
//   w1c [D][HT][32]         (diag(r1) W1)[row][j]              accumulator order
//   m2, r2 [HT][32]         mu2, r2 of BN2 (float)              accumulator order  (K stages)
// then mask [D] (padding columns j >= d: mask 1, zero weights).
struct TrainLayout {
    int D, HT, KS1;
    int w1, c1, g1, e1, w2, c2, g2, e2, w3, b3, w2t, w1c, m2, r2, net, mask, total;
};

__host__ __device__ constexpr TrainLayout train_layout(int D, int HT) {
    TrainLayout L{};
    L.D = D;
    L.HT = HT;
    L.KS1 = (D + 1) / 2;
    int o = 0;
    L.w1 = o; o += HT * L.KS1 * 64;
    L.c1 = o; o += HT * 32;
    L.g1 = o; o += HT * 32;
    L.e1 = o; o += HT * 32;
    L.w2 = o; o += HT * HT * 1024;
    L.c2 = o; o += HT * 32;
    L.g2 = o; o += HT * 32;
    L.e2 = o; o += HT * 32;
    L.w3 = o; o += D * HT * 32;
    L.b3 = o; o += (D + 3) & ~3;
    L.w2t = o; o += HT * HT * 1024;
    L.w1c = o; o += D * HT * 32;
    L.m2 = o; o += HT * 32;
    L.r2 = o; o += HT * 32;
    L.net = o;
    L.mask = 2 * o;
    L.total = 2 * o + ((D + 3) & ~3);
    return L;
}

// The pack's LDS image in a pass: the layer-2 transpose w2t only where BWD2 reads it, so every
// other pass fits two workgroups per CU (H = 64, d = 2: 94 -> 62 KB of LDS per workgroup);
// BWD2K (one net per workgroup) holds only its net's image.
__host__ __device__ constexpr bool train_stage_w2t(int stage) { return stage == TS_BWD2 || stage == TS_BWD2K; }
#ifndef NFX_TRAIN_NET1
#define NFX_TRAIN_NET1 1
#endif
__host__ __device__ constexpr int train_stage_nets(int stage) { return (stage == TS_BWD2K && NFX_TRAIN_NET1) ? 1 : 2; }

// OUTK reads only the layer-2 BatchNorm / output-layer block [c2, w2t) and m2, r2 of each net
// (3.6 KB at H = 64, d = 2): occupancy is then set by the registers alone.
__host__ __device__ constexpr TrainLayout train_lds_layout_out(int D, int HT) {
    TrainLayout L = train_layout(D, HT);
    const int cut = L.c2, piece = L.w2t - L.c2;
    L.w1 = L.c1 = L.g1 = L.e1 = L.w2 = L.w2t = L.w1c = -1;
    L.c2 -= cut;
    L.g2 -= cut;
    L.e2 -= cut;
    L.w3 -= cut;
    L.b3 -= cut;
    L.m2 = piece;
    L.r2 = piece + HT * 32;
    L.net = piece + 2 * HT * 32;
    L.mask = 2 * L.net;
    L.total = 2 * L.net + ((D + 3) & ~3);
    return L;
}

__host__ __device__ constexpr TrainLayout train_lds_layout(int D, int HT, bool w2t, int nets) {
    TrainLayout L = train_layout(D, HT);
    const int cut = w2t ? 0 : HT * HT * 1024;
    if (!w2t) L.w2t = -1;
    L.w1c -= cut;
    L.m2 -= cut;
    L.r2 -= cut;
    L.net -= cut;
    L.mask = nets * L.net;
    L.total = nets * L.net + ((D + 3) & ~3);
    return L;
}

// Per-wave partial lengths (floats, doubles for the statistics) and the layout of the float64
// gradient-sum vector G (one per layer; a stage's partials have exactly its G block's layout):
//   g1s [2 nets][2][Hp]        BWD1: sum g_y2, sum g_y2 * x^2     (BN2 backward sums)
//   g1w [2 nets][D*Hp + D]     BWD1: dW3 [D][Hp], db3 [D]
//   g2s [2 nets][2][Hp]        BWD2: sum g_y1, sum g_y1 * x^1     (BN1 backward sums)
//   g2w [2 nets][Hp*Hp + Hp]   BWD2: sum e2 a1^T [Hp][Hp], sum e2 [Hp]   (dW2 = diag(r2) .)
//   g3w [2 nets][D*Hp + Hp]    BWD3: sum e1 xa^T stored [D][Hp], sum e1 [Hp]  (dW1 = diag(r1) .)
struct TrainGrad {
    int Hp, D;
    int g1s, g1w, g2s, g2w, g3w, total;
    int len1, len2, len3;  // per-stage block lengths (contiguous from g1s, g2s, g3w)
};

__host__ __device__ constexpr TrainGrad train_grad_layout(int D, int HT) {
    TrainGrad g{};
    const int Hp = 32 * HT;
    g.Hp = Hp;
    g.D = D;
    int o = 0;
    g.g1s = o; o += 4 * Hp;
    g.g1w = o; o += 2 * (D * Hp + D);
    g.g2s = o; o += 4 * Hp;
    g.g2w = o; o += 2 * (Hp * Hp + Hp);
    g.g3w = o; o += 2 * (D * Hp + Hp);
    g.total = o;
    g.len1 = g.g2s - g.g1s;
    g.len2 = g.g3w - g.g2s;
    g.len3 = g.total - g.g3w;
    return g;
}

// Accumulator tile X (lane l, reg r = X[crow(r, h)][l & 31]) -> T[t] = X[l & 31][16h + t].
// buf: this wave's 32 x kTS LDS region. A wave's LDS instructions execute in order, so the
// write -> read (other lanes) and read -> next write sequences need no barrier.
__device__ __forceinline__ void transpose_tile(float* buf, const f32x16& X, float (&T)[16]) {
    const int l = lane_id(), h = l >> 5, c = l & 31;
    f32x4* wp = reinterpret_cast<f32x4*>(buf + c * kTS + 4 * h);
#pragma unroll
    for (int q = 0; q < 4; ++q) wp[2 * q] = f32x4{X[4 * q], X[4 * q + 1], X[4 * q + 2], X[4 * q + 3]};
    __builtin_amdgcn_wave_barrier();
    const float* rp = buf + (16 * h) * kTS + c;
#pragma unroll
    for (int t = 0; t < 16; ++t) T[t] = rp[t * kTS];
    __builtin_amdgcn_wave_barrier();
}

// Chan et al. pairwise combination of (count, mean, M2) — the stable parallel variance.
__device__ __forceinline__ void chan_merge(double& n, double& mean, double& m2, double nb, double meanb,
                                           double m2b) {
    const double nt = n + nb;
    if (nb == 0.0) return;
    const double dl = meanb - mean;
    mean = mean + dl * (nb / nt);
    m2 = m2 + m2b + dl * dl * (n * nb / nt);
    n = nt;
}

template <int D>
struct TrainRow {
    float v[D];
};

// keep: the raw layer-2 pre-activations h2 = W2 a1 + b2 of both nets, [tile][net][HT][4][64 lanes]
// of 16-byte vectors (accumulator registers 4q..4q+3 of a lane together): written by STATS2 when
// non-null, read by the K stages. The g_y1 tiles BWD2 hands to BWD3 (gbuf) use the same layout.
// (Lane-contiguous single floats measured 2.4 % slower on the train step: 4x the memory
// instructions; a register-major [q][tile][lane] order measured slower still.)
// Passes whose register use is held to 256 (2 waves per SIMD; the LDS image admits 2
// workgroups per CU) at the cost of a few scratch spills.
#ifndef NFX_TRAIN_W2_MASK
#define NFX_TRAIN_W2_MASK ((1 << TS_BWD1K) | (1 << TS_BWD2K))
#endif
__host__ __device__ constexpr int train_waves_per_eu(int stage, int D) {
    // OUTK at d <= 2: 128 registers without spills (4 waves per SIMD)
    return stage == TS_OUTK ? (D <= 2 ? 4 : 2) : (((NFX_TRAIN_W2_MASK) >> stage) & 1 ? 2 : 1);
}

template <int HT, int D, int TSTAGE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(train_waves_per_eu(TSTAGE, D)))) void affine_train_kernel(
    const float* __restrict__ pack, const float* __restrict__ x, const float* __restrict__ gy,
    const float* __restrict__ gld, float* __restrict__ gx, float* __restrict__ gbuf,
    const double* __restrict__ G, const double* __restrict__ stats2, void* __restrict__ part,
    float* __restrict__ keep, float* __restrict__ dlb, int64_t B, int d, int dir, int64_t ntiles) {
    constexpr bool KEEP = TSTAGE == TS_BWD1K || TSTAGE == TS_BWD2K || TSTAGE == TS_OUTK;
    constexpr bool NET1 = train_stage_nets(TSTAGE) == 1;  // one net per workgroup: net = blockIdx.y
    constexpr int STAGE = TSTAGE == TS_BWD1K ? TS_BWD1 : (TSTAGE == TS_BWD2K ? TS_BWD2 : TSTAGE);
    constexpr TrainLayout PL = train_layout(D, HT);                          // the pack in HBM
    constexpr TrainLayout L = TSTAGE == TS_OUTK ? train_lds_layout_out(D, HT)  // LDS image
                                                : train_lds_layout(D, HT, train_stage_w2t(TSTAGE), train_stage_nets(TSTAGE));
    const int net = NET1 ? (int)blockIdx.y : 0;
    constexpr TrainGrad GL = train_grad_layout(D, HT);
    constexpr int KS1 = L.KS1;
    constexpr int Hp = 32 * HT;
    constexpr int PACKF = (L.total + 3) & ~3;
    static_assert(L.net % 4 == 0 && L.m2 % 4 == 0 && (L.w1c % 4 == 0 || TSTAGE == TS_OUTK) && PL.w1c % 4 == 0 &&
                      PL.net % 4 == 0 && PL.c2 % 4 == 0 && PL.m2 % 4 == 0,
                  "16-byte pack pieces");
    extern __shared__ f32x4 lds4[];
    float* sm = reinterpret_cast<float*>(lds4);
    float* tbuf_all = sm + PACKF;                        // 4 x 32 x kTS
    float* sbuf_all = tbuf_all + 4 * 32 * kTS;           // 4 x 32 x (2D)  per-sample scratch
    float* kc = sbuf_all + 4 * 32 * 2 * D;               // [2 nets][2][Hp] BN-backward constants
    {
        for (int i = threadIdx.x; i < PACKF / 4; i += 256) {
            const int f = 4 * i;  // LDS float index -> pack float index (w2t skipped unless kept)
            int src;
            if (f >= L.mask) {
                src = PL.mask + (f - L.mask);
            } else {
                const int n = NET1 ? 0 : (f >= L.net), o = f - n * L.net;
                if constexpr (TSTAGE == TS_OUTK)
                    src = n * PL.net + (o < L.m2 ? PL.c2 + o : PL.m2 + (o - L.m2));
                else
                    src = (NET1 ? net : n) * PL.net + (o < L.w1c ? o : o + (PL.w1c - L.w1c));
            }
            lds4[i] = *reinterpret_cast<const f32x4*>(pack + src);
        }
    }
    if constexpr (STAGE == TS_BWD2 || STAGE == TS_BWD3) {
        // k1 = sum g / N, k2 = sum g x^ / N in accumulator order, N = the batch the statistics
        // were taken over (all ranks under SyncBN); N < 0 marks running statistics (eval-mode
        // BatchNorm): the normalisation does not depend on the batch, k1 = k2 = 0
        const double N = stats2[0];
        const double* S = G + (STAGE == TS_BWD2 ? GL.g1s : GL.g2s);
        for (int i = threadIdx.x; i < 4 * Hp; i += 256) {
            const int n = i / (2 * Hp), q = (i / Hp) & 1, a = i % Hp;  // a: accumulator index
            const int ht = a >> 5, hh = (a >> 4) & 1, r = a & 15;
            const int row = 32 * ht + crow(r, hh);
            kc[i] = N > 0.0 ? (float)(S[(n * 2 + q) * Hp + row] / N) : 0.f;  // N < 0: running stats
        }
    }
    __syncthreads();

    const int lane = lane_id(), h = lane >> 5, col = lane & 31, wave = threadIdx.x >> 6;
    float* tbuf = tbuf_all + wave * 32 * kTS;
    float* sbuf = sbuf_all + wave * 32 * 2 * D;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    const int64_t wid = (int64_t)blockIdx.x * 4 + wave;

    float mk[D];
#pragma unroll
    for (int j = 0; j < D; ++j) mk[j] = sm[L.mask + j];

    // ---- per-lane accumulators ------------------------------------------------------------
    // statistics: shift, sum, sum of squares per (net, tile) in the transposed layout
    float st_c[2][HT];
    double st_s1[2][HT], st_s2[2][HT];
    double st_n = 0.0;
    // backward sums (transposed layout unless noted)
    float ac_s1[2][HT], ac_s2[2][HT];   // BWD1/BWD2: sum g, sum g x^;  BWD3: sum e1 (ac_s1)
    float ac_w[2][HT][D];               // BWD1: dW3 (per j);  BWD3: dW1 (per j)
    float ac_b[2][D];                   // BWD1: db3 (epilogue layout, half 0)
    float ac_db[2][HT];                 // BWD2: sum e2
    f32x16 ac_dw[2][HT][HT];            // BWD2: sum e2 a1^T (accumulator layout)
#pragma unroll
    for (int n = 0; n < 2; ++n) {
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
            st_c[n][ht] = 0.f;
            st_s1[n][ht] = st_s2[n][ht] = 0.0;
            ac_s1[n][ht] = ac_s2[n][ht] = ac_db[n][ht] = 0.f;
#pragma unroll
            for (int j = 0; j < D; ++j) ac_w[n][ht][j] = 0.f;
            if constexpr (STAGE == TS_BWD2) {
#pragma unroll
                for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) ac_dw[n][ht][kt][r] = 0.f;
            }
        }
#pragma unroll
        for (int j = 0; j < D; ++j) ac_b[n][j] = 0.f;
    }

    // Software pipeline: the next tile's per-sample inputs (x row, upstream gradients, and in
    // BWD3 the g_y1 tiles) are loaded while the current tile computes. Out-of-range lanes load
    // a clamped valid address and zero the value.
    constexpr bool GRADS = STAGE == TS_BWD1 || (STAGE == TS_BWD2 && !NET1);
    // NET1 loads its kept tile at the top of the iteration (a register double buffer pushed it
    // to 1 wave per SIMD and measured ~2x slower); BWD3 with or without the prefetch measured equal
    constexpr bool QPRE = !NET1 && (KEEP || STAGE == TS_BWD3);
    constexpr int NGQ = QPRE ? 2 * HT * 16 : 1;
    struct Fetch {
        float xr[D];
        float gyr[D];
        float gl;
        float gq[NGQ];
        float dl[D];  // NET1: the net's delta3 row from BWD1K
    };
    auto fetch = [&](int64_t tile, Fetch& f) {
        const int64_t s = tile * 32 + col;
        const bool ok = tile < ntiles && s < B;
        const int64_t sc = ok ? s : 0;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const float v = j < d ? x[sc * d + j] : 0.f;
            f.xr[j] = ok ? v : 0.f;
        }
        if constexpr (GRADS) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const float v = j < d ? gy[sc * d + j] : 0.f;
                f.gyr[j] = ok ? v : 0.f;
            }
            const float v = gld[sc];
            f.gl = ok ? v : 0.f;
        }
        if constexpr (QPRE) {  // g_y1 tiles (BWD3) / kept h2 tiles
            const int64_t tc = tile < ntiles ? tile : 0;
            const f32x4* gq = reinterpret_cast<const f32x4*>((KEEP ? keep : gbuf) + ((tc * 2 + net) * HT * 16) * 64) + lane;
#pragma unroll
            for (int q4 = 0; q4 < NGQ / 4; ++q4) {
                const f32x4 v = gq[q4 * 64];
#pragma unroll
                for (int c = 0; c < 4; ++c) f.gq[4 * q4 + c] = v[c];
            }
        }
        if constexpr (NET1) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const float v = dlb[(sc * 2 + net) * D + j];
                f.dl[j] = ok ? v : 0.f;
            }
        }
    };

    bool first = true;
    Fetch cur;
    fetch(wid, cur);
    for (int64_t tile = wid; tile < ntiles; tile += nwaves) {
        const int64_t base = tile * 32;
        const int64_t s = base + col;
        const bool valid = s < B;
        const float* smi = sm + opaque_zero();
        const float* kci = kc + opaque_zero();  // keeps the BN constants in LDS, not in VGPRs
        Fetch nxt;
        fetch(tile + nwaves, nxt);
        // the lane's sample row (both lane halves hold the same sample)
        float xr[D];
#pragma unroll
        for (int j = 0; j < D; ++j) xr[j] = cur.xr[j];
        float xb[KS1];  // layer-1 B operand: xa[sample col][2ks + h]
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks) {
            const float v0 = xr[2 * ks] * mk[2 * ks];
            const float v1 = (2 * ks + 1 < D) ? xr[2 * ks + 1] * mk[2 * ks + 1] : 0.f;
            xb[ks] = h ? v1 : v0;
        }
        // samples of this tile in the lane's transposed half: 16h + t valid for t < nvh
        const int64_t rem = B - base - 16 * h;
        const int nvh = rem <= 0 ? 0 : (rem >= 16 ? 16 : (int)rem);

        auto layer1 = [&](const float* P, f32x16 (&acc)[HT]) {
#pragma unroll
            for (int ht = 0; ht < HT; ++ht) {
                f32x16 a = load_bias16(P + L.c1 + ht * 32, h);
#pragma unroll
                for (int ks = 0; ks < KS1; ++ks) a = mfma32(P[L.w1 + (ht * KS1 + ks) * 64 + lane], xb[ks], a);
                acc[ht] = a;
            }
        };
        // a1 = relu(gamma1 x^1 + beta1) in place (keeps x^1 in xh, writes a1 into act)
        auto bn_relu = [&](const float* gp, const float* ep, const f32x16 (&xh)[HT], f32x16 (&act)[HT]) {
#pragma unroll
            for (int ht = 0; ht < HT; ++ht) {
                const f32x16 g = load_bias16(gp + ht * 32, h), e = load_bias16(ep + ht * 32, h);
#pragma unroll
                for (int r = 0; r < 16; ++r) act[ht][r] = trelu(fmaf(g[r], xh[ht][r], e[r]));
            }
        };
        auto layer2 = [&](const float* P, const f32x16 (&act)[HT], f32x16 (&acc)[HT]) {
            const f32x4* wg = reinterpret_cast<const f32x4*>(P + L.w2) + lane;
#pragma unroll
            for (int o = 0; o < HT; ++o) {
                f32x16 a = load_bias16(P + L.c2 + o * 32, h);
#pragma unroll
                for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                    for (int rq = 0; rq < 4; ++rq) {
                        const f32x4 w = wg[((o * HT + kt) * 4 + rq) * 64];
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) a = mfma32(w[rr], act[kt][4 * rq + rr], a);
                    }
                acc[o] = a;
            }
        };
        // statistics of an accumulator tile (transposed; invalid samples excluded)
        auto stats_tile = [&](int n, int ht, const f32x16& X) {
            float T[16];
            transpose_tile(tbuf, X, T);
            if (first) st_c[n][ht] = T[0];
            const float c = st_c[n][ht];
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const float v = t < nvh ? T[t] - c : 0.f;
                s1 += v;
                s2 = fmaf(v, v, s2);
            }
            st_s1[n][ht] += (double)s1;
            st_s2[n][ht] += (double)s2;
        };

        // BWD2 after e2 of net n: a1 of the net again (layer 1 is K = d: cheap) and its
        // pre-activation for the ReLU, db2 / dW2 sums into accumulator slot sl, g_a1 = (diag(r2)
        // W2)^T e2 -> relu backward -> the g_y1 tiles to HBM, BN1 sums.
        auto bwd2_tail = [&](const float* P, int n, int sl, const f32x16 (&e2t)[HT]) {
            f32x16 xh1[HT], a1[HT];
            layer1(P, xh1);
            bn_relu(P + L.g1, P + L.e1, xh1, a1);
            float Te[HT][16];
#pragma unroll
            for (int o = 0; o < HT; ++o) {
                transpose_tile(tbuf, e2t[o], Te[o]);
                float sb = 0.f;
#pragma unroll
                for (int t = 0; t < 16; ++t) sb += Te[o][t];
                ac_db[sl][o] += sb;
            }
#pragma unroll
            for (int kt = 0; kt < HT; ++kt) {
                float Ta[16];
                transpose_tile(tbuf, a1[kt], Ta);
#pragma unroll
                for (int o = 0; o < HT; ++o)
#pragma unroll
                    for (int t = 0; t < 16; ++t) ac_dw[sl][o][kt] = mfma32(Te[o][t], Ta[t], ac_dw[sl][o][kt]);
            }
            // g_a1 = (diag(r2) W2)^T e2, relu backward, BN1 sums, g_y1 to HBM
            const f32x4* wt = reinterpret_cast<const f32x4*>(P + L.w2t) + lane;
#pragma unroll
            for (int kt = 0; kt < HT; ++kt) {
                f32x16 ga;
#pragma unroll
                for (int r = 0; r < 16; ++r) ga[r] = 0.f;
#pragma unroll
                for (int o = 0; o < HT; ++o)
#pragma unroll
                    for (int rq = 0; rq < 4; ++rq) {
                        const f32x4 w = wt[((kt * HT + o) * 4 + rq) * 64];
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) ga = mfma32(w[rr], e2t[o][4 * rq + rr], ga);
                    }
#pragma unroll
                for (int r = 0; r < 16; ++r) ga[r] = a1[kt][r] > 0.f ? ga[r] : 0.f;
                f32x4* gp = reinterpret_cast<f32x4*>(gbuf + (((tile * 2 + n) * HT + kt) * 16) * 64) + lane;
#pragma unroll
                for (int rq = 0; rq < 4; ++rq)
                    gp[rq * 64] = f32x4{ga[4 * rq], ga[4 * rq + 1], ga[4 * rq + 2], ga[4 * rq + 3]};
                float Tg[16], Tx[16];
                transpose_tile(tbuf, ga, Tg);
                transpose_tile(tbuf, xh1[kt], Tx);
                float s1 = 0.f, s2 = 0.f;
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    s1 += Tg[t];
                    s2 = fmaf(Tg[t], Tx[t], s2);
                }
                ac_s1[sl][kt] += s1;
                ac_s2[sl][kt] += s2;
            }
        };

        if constexpr (STAGE == TS_STATS1 || STAGE == TS_STATS2) {
#pragma unroll
            for (int n = 0; n < 2; ++n) {
                const float* P = smi + n * L.net;
                f32x16 xh1[HT];
                layer1(P, xh1);
                if constexpr (STAGE == TS_STATS1) {
#pragma unroll
                    for (int ht = 0; ht < HT; ++ht) stats_tile(n, ht, xh1[ht]);
                } else {
                    f32x16 a1[HT], h2[HT];
                    bn_relu(P + L.g1, P + L.e1, xh1, a1);
                    layer2(P, a1, h2);
                    if (keep) {  // (the pack folds no layer-2 statistics here: h2 is raw)
#pragma unroll
                        for (int ht = 0; ht < HT; ++ht) {
                            f32x4* kp = reinterpret_cast<f32x4*>(keep + (((tile * 2 + n) * HT + ht) * 16) * 64) + lane;
#pragma unroll
                            for (int rq = 0; rq < 4; ++rq)
                                kp[rq * 64] = f32x4{h2[ht][4 * rq], h2[ht][4 * rq + 1], h2[ht][4 * rq + 2], h2[ht][4 * rq + 3]};
                        }
                    }
#pragma unroll
                    for (int ht = 0; ht < HT; ++ht) stats_tile(n, ht, h2[ht]);
                }
            }
            st_n += (double)nvh;
        } else if constexpr (TSTAGE == TS_OUTK) {
            // ---- forward output from the kept h2 (OUTK: gx = y, dlb = log-det), with the
            // epilogue of the streaming eval kernel (nfx_affine_kernel.h) ----------------------
            float outv[2][D];
#pragma unroll
            for (int n = 0; n < 2; ++n) {
                const float* P = smi + n * L.net;
                float pj[D];
#pragma unroll
                for (int j = 0; j < D; ++j) pj[j] = 0.f;
#pragma unroll
                for (int o = 0; o < HT; ++o) {
                    const f32x16 m = load_bias16(P + L.m2 + o * 32, h), rs = load_bias16(P + L.r2 + o * 32, h);
                    const f32x16 g = load_bias16(P + L.g2 + o * 32, h), e = load_bias16(P + L.e2 + o * 32, h);
                    f32x16 a2;
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        a2[r] = trelu(fmaf(g[r], (cur.gq[(n * HT + o) * 16 + r] - m[r]) * rs[r], e[r]));
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        const f32x16 w3 = load_bias16(P + L.w3 + (j * HT + o) * 32, h);
#pragma unroll
                        for (int r = 0; r < 16; ++r) pj[j] = fmaf(w3[r], a2[r], pj[j]);
                    }
                }
#pragma unroll
                for (int j = 0; j < D; ++j) outv[n][j] = halves_sum(pj[j], pj[j]) + P[L.b3 + j];
            }
            if (h == 0 && valid) {
#pragma clang fp contract(off)  // separate mul/add roundings, as the reference's torch ops
                float ld = 0.f, yv[D];
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    const float sv = tclamp(outv[0][j], -10.f, 10.f), bv = tclamp(outv[1][j], -10.f, 10.f);
                    const float m = mk[j], om = 1.f - m;
                    const float xa = xr[j] * m;
                    float t;
                    if (dir < 0) {
                        t = (xr[j] - bv) * exp_fast(-sv);
                        ld = ld + om * (-sv);
                    } else {
                        t = xr[j] * exp_fast(sv) + bv;
                        ld = ld + om * sv;
                    }
                    const float v = xa + om * t;
                    yv[j] = nonfinite(v) ? 0.f : v;
                }
                if (nonfinite(ld)) ld = 0.f;
#pragma unroll
                for (int j = 0; j < D; ++j)
                    if (j < d) gx[s * d + j] = yv[j];
                dlb[s] = ld;
            }
        } else if constexpr (NET1) {
            // ---- BWD2, net `net` only: x^2 from the kept h2, delta3 from BWD1K -------------
            const float* P = smi;
            float kq[HT * 16];  // the net's kept h2 tile (loaded here: no register double buffer)
            {
                const f32x4* q = reinterpret_cast<const f32x4*>(keep + ((tile * 2 + net) * HT * 16) * 64) + lane;
#pragma unroll
                for (int i4 = 0; i4 < HT * 4; ++i4) {
                    const f32x4 v = q[i4 * 64];
#pragma unroll
                    for (int c = 0; c < 4; ++c) kq[4 * i4 + c] = v[c];
                }
            }
            f32x16 e2t[HT];
#pragma unroll
            for (int o = 0; o < HT; ++o) {
                const f32x16 m = load_bias16(P + L.m2 + o * 32, h), rs = load_bias16(P + L.r2 + o * 32, h);
                const f32x16 g = load_bias16(P + L.g2 + o * 32, h), e = load_bias16(P + L.e2 + o * 32, h);
                f32x16 xh2, gy2, a2;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    xh2[r] = (kq[o * 16 + r] - m[r]) * rs[r];
                    a2[r] = trelu(fmaf(g[r], xh2[r], e[r]));
                    gy2[r] = 0.f;
                }
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    const f32x16 w3 = load_bias16(P + L.w3 + (j * HT + o) * 32, h);
#pragma unroll
                    for (int r = 0; r < 16; ++r) gy2[r] = fmaf(w3[r], cur.dl[j], gy2[r]);
                }
                const f32x16 k1 = load_bias16(kci + (net * 2 + 0) * Hp + o * 32, h);
                const f32x16 k2 = load_bias16(kci + (net * 2 + 1) * Hp + o * 32, h);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float gr = a2[r] > 0.f ? gy2[r] : 0.f;  // relu backward
                    const float v = g[r] * ((gr - k1[r]) - xh2[r] * k2[r]);
                    e2t[o][r] = valid ? v : 0.f;
                }
            }
            bwd2_tail(P, net, 0, e2t);
        } else if constexpr (STAGE == TS_BWD1 || STAGE == TS_BWD2) {
            // ---- recompute the forward of both nets (layer-2 x^2 kept for both) ----------
            f32x16 xh2[2][HT];
            float outv[2][D];
#pragma unroll
            for (int n = 0; n < 2; ++n) {
                const float* P = smi + n * L.net;
                if constexpr (KEEP) {
                    // x^2 = (h2 - mu2) r2 from the kept pre-activations
#pragma unroll
                    for (int o = 0; o < HT; ++o) {
                        const f32x16 m = load_bias16(P + L.m2 + o * 32, h), rs = load_bias16(P + L.r2 + o * 32, h);
#pragma unroll
                        for (int r = 0; r < 16; ++r) xh2[n][o][r] = (cur.gq[(n * HT + o) * 16 + r] - m[r]) * rs[r];
                    }
                } else {
                    f32x16 xh1[HT], a1[HT];
                    layer1(P, xh1);
                    bn_relu(P + L.g1, P + L.e1, xh1, a1);
                    layer2(P, a1, xh2[n]);
                }
                float pj[D];
#pragma unroll
                for (int j = 0; j < D; ++j) pj[j] = 0.f;
#pragma unroll
                for (int o = 0; o < HT; ++o) {
                    const f32x16 g = load_bias16(P + L.g2 + o * 32, h), e = load_bias16(P + L.e2 + o * 32, h);
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        const f32x16 w3 = load_bias16(P + L.w3 + (j * HT + o) * 32, h);
#pragma unroll
                        for (int r = 0; r < 16; ++r)
                            pj[j] = fmaf(w3[r], trelu(fmaf(g[r], xh2[n][o][r], e[r])), pj[j]);
                    }
                }
#pragma unroll
                for (int j = 0; j < D; ++j) outv[n][j] = halves_sum(pj[j], pj[j]) + P[L.b3 + j];
            }
            // ---- epilogue backward (coupling_layer.py:40-96 under autograd) ---------------
            const float gl_in = cur.gl;
            float gyr[D];
#pragma unroll
            for (int j = 0; j < D; ++j) gyr[j] = cur.gyr[j];
            float dl[2][D], gxd[D];
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
                    const float gt = gv * om;  // d v / d t = (1 - m)
                    float gs, gb;
                    if (dir < 0) {  // t = (x - b) * exp(-s); ld = sum (1-m)(-s)
                        gs = (gt * (xr[j] - bv[j])) * (-ev[j]) + gl * (-om);
                        gb = -(gt * ev[j]);
                    } else {        // t = x * exp(s) + b;  ld = sum (1-m) s
                        gs = (gt * xr[j]) * ev[j] + gl * om;
                        gb = gt;
                    }
                    gxd[j] = gv * m + gt * ev[j];
                    if (j >= d) gs = gb = 0.f;
                    // torch.clamp backward: gradient where min <= input <= max
                    dl[0][j] = (outv[0][j] >= -10.f && outv[0][j] <= 10.f) ? gs : 0.f;
                    dl[1][j] = (outv[1][j] >= -10.f && outv[1][j] <= 10.f) ? gb : 0.f;
                }
            }
            if constexpr (STAGE == TS_BWD1) {
                if (h == 0 && valid) {
#pragma unroll
                    for (int j = 0; j < D; ++j)
                        if (j < d) gx[s * d + j] = gxd[j];
                    if constexpr (KEEP) {  // delta3 of both nets for BWD2K
#pragma unroll
                        for (int n = 0; n < 2; ++n)
#pragma unroll
                            for (int j = 0; j < D; ++j) dlb[(s * 2 + n) * D + j] = dl[n][j];
                    }
                }
                // per-sample delta3 of both nets for the transposed dW3 sums
                if (h == 0) {
#pragma unroll
                    for (int n = 0; n < 2; ++n)
#pragma unroll
                        for (int j = 0; j < D; ++j) sbuf[col * 2 * D + n * D + j] = dl[n][j];
                }
#pragma unroll
                for (int n = 0; n < 2; ++n)
#pragma unroll
                    for (int j = 0; j < D; ++j) ac_b[n][j] += h == 0 ? dl[n][j] : 0.f;
            }
#pragma unroll
            for (int n = 0; n < 2; ++n) {
                const float* P = smi + n * L.net;
                f32x16 e2t[HT];  // BWD2: e2 of net n (accumulator layout)
#pragma unroll
                for (int o = 0; o < HT; ++o) {
                    const f32x16 g = load_bias16(P + L.g2 + o * 32, h), e = load_bias16(P + L.e2 + o * 32, h);
                    f32x16 gy2, a2;
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float y2 = fmaf(g[r], xh2[n][o][r], e[r]);
                        a2[r] = trelu(y2);
                        gy2[r] = 0.f;
                    }
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        const f32x16 w3 = load_bias16(P + L.w3 + (j * HT + o) * 32, h);
#pragma unroll
                        for (int r = 0; r < 16; ++r) gy2[r] = fmaf(w3[r], dl[n][j], gy2[r]);
                    }
#pragma unroll
                    for (int r = 0; r < 16; ++r) gy2[r] = a2[r] > 0.f ? gy2[r] : 0.f;  // relu backward
                    if constexpr (STAGE == TS_BWD1) {
                        float Tg[16], Tx[16], Ta[16];
                        transpose_tile(tbuf, gy2, Tg);
                        transpose_tile(tbuf, xh2[n][o], Tx);
                        transpose_tile(tbuf, a2, Ta);
                        float s1 = 0.f, s2 = 0.f;
#pragma unroll
                        for (int t = 0; t < 16; ++t) {
                            s1 += Tg[t];
                            s2 = fmaf(Tg[t], Tx[t], s2);
                        }
                        ac_s1[n][o] += s1;
                        ac_s2[n][o] += s2;
#pragma unroll
                        for (int j = 0; j < D; ++j) {
                            float w = 0.f;
#pragma unroll
                            for (int t = 0; t < 16; ++t) w = fmaf(sbuf[(16 * h + t) * 2 * D + n * D + j], Ta[t], w);
                            ac_w[n][o][j] += w;
                        }
                    } else {
                        // e2 = gamma2 (g_y2 - k1 - x^2 k2)  (BatchNorm backward with batch statistics)
                        const f32x16 k1 = load_bias16(kci + (n * 2 + 0) * Hp + o * 32, h);
                        const f32x16 k2 = load_bias16(kci + (n * 2 + 1) * Hp + o * 32, h);
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const float v = g[r] * ((gy2[r] - k1[r]) - xh2[n][o][r] * k2[r]);
                            e2t[o][r] = valid ? v : 0.f;
                        }
                    }
                }
                if constexpr (STAGE == TS_BWD2) bwd2_tail(P, n, n, e2t);
            }
        } else {  // TS_BWD3: layer 1 only
            if (h == 0) {
#pragma unroll
                for (int j = 0; j < D; ++j) sbuf[col * 2 * D + j] = xr[j] * mk[j];
            }
            float gp[D];
#pragma unroll
            for (int j = 0; j < D; ++j) gp[j] = 0.f;
#pragma unroll
            for (int n = 0; n < 2; ++n) {
                const float* P = smi + n * L.net;
                f32x16 xh1[HT];
                layer1(P, xh1);
#pragma unroll
                for (int kt = 0; kt < HT; ++kt) {
                    const f32x16 g = load_bias16(P + L.g1 + kt * 32, h);
                    const f32x16 k1 = load_bias16(kci + (n * 2 + 0) * Hp + kt * 32, h);
                    const f32x16 k2 = load_bias16(kci + (n * 2 + 1) * Hp + kt * 32, h);
                    f32x16 e1;
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float v = g[r] * ((cur.gq[(n * HT + kt) * 16 + r] - k1[r]) - xh1[kt][r] * k2[r]);
                        e1[r] = valid ? v : 0.f;
                    }
                    float Te[16];
                    transpose_tile(tbuf, e1, Te);
                    float sb = 0.f;
#pragma unroll
                    for (int t = 0; t < 16; ++t) sb += Te[t];
                    ac_s1[n][kt] += sb;
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        float w = 0.f;
#pragma unroll
                        for (int t = 0; t < 16; ++t) w = fmaf(sbuf[(16 * h + t) * 2 * D + j], Te[t], w);
                        ac_w[n][kt][j] += w;
                        const f32x16 wc = load_bias16(P + L.w1c + (j * HT + kt) * 32, h);
#pragma unroll
                        for (int r = 0; r < 16; ++r) gp[j] = fmaf(wc[r], e1[r], gp[j]);
                    }
                }
            }
            float gxa[D];
#pragma unroll
            for (int j = 0; j < D; ++j) gxa[j] = halves_sum(gp[j], gp[j]);
            if (h == 0 && valid) {
#pragma unroll
                for (int j = 0; j < D; ++j)
                    if (j < d) gx[s * d + j] = gx[s * d + j] + mk[j] * gxa[j];
            }
        }
        first = false;
        cur = nxt;
    }

    // ---- workgroup combine: the 4 waves add (merge) their partials into LDS in wave order,
    // then the workgroup writes one partial; the finish kernels reduce workgroups in order ----
    static_assert(TSTAGE == TS_OUTK || (GL.len1 <= PACKF && GL.len2 <= PACKF && GL.len3 <= PACKF && 12 * Hp <= PACKF),
                  "reduction buffer must fit the pack region");
    __syncthreads();  // every wave is done with the weight pack: reuse its LDS
    float* red = sm;
    double* redd = reinterpret_cast<double*>(sm);
    constexpr int LEN = STAGE == TS_BWD1 ? GL.len1 : (STAGE == TS_BWD2 ? GL.len2 : (STAGE == TS_BWD3 ? GL.len3 : 0));
    if constexpr (NET1) {  // the other net's entries of this workgroup's partial stay zero
        for (int i = threadIdx.x; i < LEN; i += 256) red[i] = 0.f;
        __syncthreads();
    }
    for (int rnd = 0; rnd < 4; ++rnd) {
        if (wave == rnd) {
            auto put = [&](int idx, float v) { red[idx] = (rnd || NET1) ? red[idx] + v : v; };
            if constexpr (STAGE == TS_STATS1 || STAGE == TS_STATS2) {
                // per lane (n, mean, M2) of its half's samples; merge the halves (same features)
#pragma unroll
                for (int n = 0; n < 2; ++n)
#pragma unroll
                    for (int ht = 0; ht < HT; ++ht) {
                        double cnt = st_n, mean = 0.0, m2 = 0.0;
                        if (cnt > 0.0) {
                            mean = (double)st_c[n][ht] + st_s1[n][ht] / cnt;
                            m2 = st_s2[n][ht] - st_s1[n][ht] * st_s1[n][ht] / cnt;
                            if (m2 < 0.0) m2 = 0.0;
                        }
                        const double nb = __shfl_xor(cnt, 32, 64), mb = __shfl_xor(mean, 32, 64),
                                     qb = __shfl_xor(m2, 32, 64);
                        if (h == 0) {
                            if (cnt == 0.0) {
                                cnt = nb; mean = mb; m2 = qb;
                            } else {
                                chan_merge(cnt, mean, m2, nb, mb, qb);
                            }
                            double* q = redd + (n * Hp + 32 * ht + col) * 3;
                            if (rnd == 0 || q[0] == 0.0) {
                                q[0] = cnt; q[1] = mean; q[2] = m2;
                            } else {
                                double a = q[0], b = q[1], c = q[2];
                                chan_merge(a, b, c, cnt, mean, m2);
                                q[0] = a; q[1] = b; q[2] = c;
                            }
                        }
                    }
            } else if constexpr (STAGE == TS_BWD1) {
#pragma unroll
                for (int n = 0; n < 2; ++n)
#pragma unroll
                    for (int ht = 0; ht < HT; ++ht) {
                        const float a = halves_sum(ac_s1[n][ht], ac_s1[n][ht]);
                        const float b = halves_sum(ac_s2[n][ht], ac_s2[n][ht]);
                        if (h == 0) {
                            put((n * 2 + 0) * Hp + 32 * ht + col, a);
                            put((n * 2 + 1) * Hp + 32 * ht + col, b);
                        }
#pragma unroll
                        for (int j = 0; j < D; ++j) {
                            const float w = halves_sum(ac_w[n][ht][j], ac_w[n][ht][j]);
                            if (h == 0) put(4 * Hp + n * (D * Hp + D) + j * Hp + 32 * ht + col, w);
                        }
                    }
#pragma unroll
                for (int n = 0; n < 2; ++n)
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        float v = ac_b[n][j];
#pragma unroll
                        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
                        if (lane == 0) put(4 * Hp + n * (D * Hp + D) + D * Hp + j, v);
                    }
            } else if constexpr (STAGE == TS_BWD2) {
#pragma unroll
                for (int n = 0; n < (NET1 ? 1 : 2); ++n) {
                    const int nd = NET1 ? net : n;  // the net whose G block slot n holds
#pragma unroll
                    for (int ht = 0; ht < HT; ++ht) {
                        const float a = halves_sum(ac_s1[n][ht], ac_s1[n][ht]);
                        const float b = halves_sum(ac_s2[n][ht], ac_s2[n][ht]);
                        const float c = halves_sum(ac_db[n][ht], ac_db[n][ht]);
                        if (h == 0) {
                            put((nd * 2 + 0) * Hp + 32 * ht + col, a);
                            put((nd * 2 + 1) * Hp + 32 * ht + col, b);
                            put(4 * Hp + nd * (Hp * Hp + Hp) + Hp * Hp + 32 * ht + col, c);
                        }
                    }
                    const int pdw = 4 * Hp + nd * (Hp * Hp + Hp);
#pragma unroll
                    for (int o = 0; o < HT; ++o)
#pragma unroll
                        for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                            for (int r = 0; r < 16; ++r)
                                put(pdw + (32 * o + crow(r, h)) * Hp + 32 * kt + col, ac_dw[n][o][kt][r]);
                }
            } else if constexpr (STAGE == TS_BWD3) {
#pragma unroll
                for (int n = 0; n < 2; ++n)
#pragma unroll
                    for (int ht = 0; ht < HT; ++ht) {
                        const float c = halves_sum(ac_s1[n][ht], ac_s1[n][ht]);
                        if (h == 0) put(n * (D * Hp + Hp) + D * Hp + 32 * ht + col, c);
#pragma unroll
                        for (int j = 0; j < D; ++j) {
                            const float w = halves_sum(ac_w[n][ht][j], ac_w[n][ht][j]);
                            if (h == 0) put(n * (D * Hp + Hp) + j * Hp + 32 * ht + col, w);
                        }
                    }
            }
        }
        __syncthreads();
    }
    if constexpr (STAGE == TS_STATS1 || STAGE == TS_STATS2) {
        double* pw = reinterpret_cast<double*>(part) + (int64_t)blockIdx.x * (2 * Hp * 3);
        for (int i = threadIdx.x; i < 2 * Hp * 3; i += 256) pw[i] = redd[i];
    } else {
        float* pw = reinterpret_cast<float*>(part) + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * LEN;
        for (int i = threadIdx.x; i < LEN; i += 256) pw[i] = red[i];
    }
}

typedef void (*affine_train_kernel_t)(const float*, const float*, const float*, const float*, float*, float*,
                                      const double*, const double*, void*, float*, float*, int64_t, int, int,
                                      int64_t);

template <int HT>
affine_train_kernel_t affine_train_pick_ht(int D, int stage);

// LDS bytes of affine_train_kernel<HT, D, stage>
__host__ __device__ constexpr size_t affine_train_lds(int D, int HT, int stage) {
    if (stage == TS_OUTK) return (size_t)(((train_lds_layout_out(D, HT).total + 3) & ~3) + 4 * 32 * kTS +
                                          4 * 32 * 2 * D + 4 * 32 * HT) * sizeof(float);
    return (size_t)(((train_lds_layout(D, HT, train_stage_w2t(stage), train_stage_nets(stage)).total + 3) & ~3) +
                    4 * 32 * kTS +
                    4 * 32 * 2 * D + 4 * 32 * HT) *
           sizeof(float);
}

}  // namespace nfx
