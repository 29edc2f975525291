// MADE-masked autoregressive affine flows (MAF / IAF) for gfx950.
//
// Reference: src/flows/autoregressive/made.py:81-140 (4 MaskedLinear, ReLU between, output
// order [mu_0..mu_{d-1} | alpha_0..alpha_{d-1}]), masked_linear.py:14-18 (W * mask),
// masked_autoregressive_flow.py:18-78, inverse_autoregressive_flow.py:30-103.
//
// Parallel directions (MAF.inverse = density, IAF.forward = sampling): the dense masked MADE
// is a genuine GEMM chain under a static mask (W*M folded once at pack time — bit-identical to
// the per-call weight*mask because the mask is 0/1). One wave owns 64 samples (two 32-column
// MFMA tiles); hidden activations stay in accumulator registers between layers; the input layer
// streams x through a wave-private LDS tile in 32-dimension chunks (coalesced 128-byte rows in,
// conflict-free stride-33 column reads out); the output layer is produced in (mu, alpha) tile
// pairs so mu_i and alpha_i land in the same lane/register, and the affine epilogue runs on the
// same LDS tile before a coalesced store. Weights are read by A-operand-ordered 16-byte loads
// from LDS when the whole image fits (small d, e.g. the d=63 MAF of BASELINE cfg4) and from
// global/L2 otherwise (e.g. d=784 IAF).
#pragma once
#include "nfx_common.h"

namespace nfx {

// Packed image (floats), A-operand order, 4 consecutive k-steps per lane as one float4:
//   w1 [HT][G1][64][4]    G1 = 4 * NKC k-step groups, NKC = ceil(d/32) input chunks
//   b1 [HT][2][16]        bias at accumulator register r of lane-half h (row crow(r, h))
//   w2 [HT][HT][4][64][4], b2 [HT][2][16], w3 (same), b3
//   w4 [NJ][2][HT][4][64][4]  NJ = ceil(d/32) output tile pairs (0 = mu rows, 1 = alpha rows)
//   b4 [NJ][2][2][16]
// then, for the sequential kernels, plain row-major copies (Hp = 32*HT):
//   s_w1t [d][Hp]  (W1m transposed: column i = the inputs' contributions of x_i)
//   s_b1 [Hp], s_w2 [Hp][Hp], s_b2 [Hp], s_w3 [Hp][Hp], s_b3 [Hp]
//   s_w4 [2d][Hp], s_b4 [2d(up4)],
//   s_deg [3][Hp]: unit degree (padded units 1e9) | degrees in completion order | unit index in
//   completion order (units sorted by degree, stable)
// then the structural-zero extents of the parallel image (int32, written by made_live_kernel):
// per output tile, 1 + the index of its last k-block holding a nonzero weight (every later
// k-block of that tile's rows is exactly zero under the MADE masks)
//   nk1 [HT]  in 32-input chunks (layer 1)      nk2 [HT], nk3 [HT]  in 32-unit tiles
//   nk4 [NJ]  in 32-unit tiles (mu and alpha rows of output tile pair j)
//   tsafe (float): inputs with max|x| <= tsafe cannot overflow any layer (made_live_kernel)
// then the transposed A-operand images of the backward data path (made_bwd_pack_kernel,
// same [out tile][k tile][r/4][lane][r%4] order; row = out index, col = k index):
//   t4 [HT][2*NJ][4][64][4]   W4mᵀ: hidden rows x (mu|alpha block) k tiles
//   t3 [HT][HT]..., t2 [HT][HT]...  W3mᵀ, W2mᵀ
//   t1 [NKC][HT]...           W1mᵀ: input rows x hidden k tiles
// then (HT <= 2) the rank-ordered image made_seqs_kernel copies into LDS as its prologue
// (made_seqs_image_kernel; layout = the first S.blk floats of seqs_lds).
struct MadeLayout {
    int d, HT, Hp, NKC, NJ;
    int w1, b1, w2, b2, w3, b3, w4, b4;  // parallel image
    int par_total;                       // floats of the parallel image (LDS-resident prefix)
    int s_w1t, s_b1, s_w2, s_b2, s_w3, s_b3, s_w4, s_b4, s_deg;
    int nk1, nk2, nk3, nk4, tsafe;
    int t4, t3, t2, t1;
    int rimg;  // made_seqs_kernel's LDS prologue image (HT <= 2): [w2 | w3 by rank][b1 | b2 | b3 | deg | gend]
    int sw1, sw4, sb4;  // made_seqs_kernel's block-ready step rows (HT <= 2), d + kSeqsPadRows rows each
    int ctab;           // the sequential kernels' chunk schedule (HT <= 2): seqs_max_chunks x 8 words
    // made_seqp_kernel (HT <= 2, d <= 1024; 0-sized otherwise), units by completion rank g, steps
    // in 64-step slots s (lane l = step 64 s + l):
    //   pw4 [Hp][ceil(ps/2)][64][4]  unit g's (mu, alpha) output weights of step 64 s + l, slots
    //                                 2j and 2j + 1 in one 16-byte piece per lane
    //   pw1 [Hp][ceil(ps/4)][64][4]  its W1 row, slots 4j .. 4j + 3 per piece
    //   pb4 [ps][64][2]      (mu, alpha) biases per step
    //   pw23 [Hp][Hp][2]     row g, lane p = (W2, W3)[rank p][rank g] (unit g's outgoing weights)
    //   ptb [4][Hp]          b1 | b2 | b3 by rank, degree by rank      ptab: the chunk schedule
    int ps, pw4, pw1, pb4, pw23, ptb, ptab;
    int total;
};

__host__ __device__ constexpr int made_up4(int v) { return (v + 3) & ~3; }

// made_seqs_kernel's staged step rows: W4 (mu, alpha) pairs by completion rank + 4 pad floats
// (bank-conflict-free column reads of 16 consecutive rows), and the zero rows past d that let a
// 64-step block always be copied whole.
__host__ __device__ constexpr int seqs_w4_stride(int Hp) { return 2 * Hp + 4; }
constexpr int kSeqsPadRows = 64;
// Chunks of the sequential schedule: each ends at 16 steps (<= d/16), at a completion (<= Hp) or
// at a staged block's end (<= d/64 + Hp + 1); + 1 sentinel entry.
__host__ __device__ constexpr int seqs_max_chunks(int d, int Hp) { return d / 8 + 2 * Hp + 8; }
// made_seqp_kernel: 64-step slots (0 = not built: HT > 2 or d > 1024); chunks end at a completion
// (<= Hp; a group of m units of one degree takes 3m chunks), a slot end (<= slots) or the last
// step; + 1 sentinel entry
constexpr int kSeqpMaxS = 16;
__host__ __device__ constexpr int seqp_slots(int d, int HT) {
    return (HT <= 2 && d <= 64 * kSeqpMaxS) ? (d + 63) / 64 : 0;
}
__host__ __device__ constexpr int seqp_max_chunks(int d, int Hp) { return (d + 63) / 64 + 3 * Hp + 4; }

__host__ __device__ constexpr MadeLayout made_layout(int d, int HT) {
    MadeLayout L{};
    L.d = d;
    L.HT = HT;
    L.Hp = 32 * HT;
    L.NKC = (d + 31) / 32;
    L.NJ = (d + 31) / 32;
    int o = 0;
    L.w1 = o; o += HT * 4 * L.NKC * 256;
    L.b1 = o; o += HT * 32;
    L.w2 = o; o += HT * HT * 1024;
    L.b2 = o; o += HT * 32;
    L.w3 = o; o += HT * HT * 1024;
    L.b3 = o; o += HT * 32;
    L.w4 = o; o += L.NJ * 2 * HT * 1024;
    L.b4 = o; o += L.NJ * 2 * 32;
    L.par_total = o;
    L.s_w1t = o; o += made_up4(d * L.Hp);
    L.s_b1 = o; o += L.Hp;
    L.s_w2 = o; o += L.Hp * L.Hp;
    L.s_b2 = o; o += L.Hp;
    L.s_w3 = o; o += L.Hp * L.Hp;
    L.s_b3 = o; o += L.Hp;
    L.s_w4 = o; o += made_up4(2 * d * L.Hp);
    L.s_b4 = o; o += made_up4(2 * d);
    L.s_deg = o; o += 3 * L.Hp;
    L.nk1 = o; o += HT;
    L.nk2 = o; o += HT;
    L.nk3 = o; o += HT;
    L.nk4 = o; o += L.NJ;
    L.tsafe = o; o += 1;
    o = made_up4(o);
    L.t4 = o; o += HT * 2 * L.NJ * 1024;
    L.t3 = o; o += HT * HT * 1024;
    L.t2 = o; o += HT * HT * 1024;
    L.t1 = o; o += L.NKC * HT * 1024;
    L.rimg = o; o += HT <= 2 ? 2 * L.Hp * L.Hp + 5 * L.Hp : 0;
    o = made_up4(o);
    const int rows = HT <= 2 ? d + kSeqsPadRows : 0;
    L.sw1 = o; o += made_up4(rows * L.Hp);
    L.sw4 = o; o += made_up4(rows * seqs_w4_stride(L.Hp));
    L.sb4 = o; o += made_up4(2 * rows);
    L.ctab = o; o += HT <= 2 ? 8 * seqs_max_chunks(d, L.Hp) : 0;
    // made_seqp_kernel's images (HT <= 2, d <= 1024; nfx_made_seqp_kernel.h)
    const int PS = seqp_slots(d, HT);
    L.ps = PS;
    L.pw4 = o; o += L.Hp * ((PS + 1) / 2) * 256;
    L.pw1 = o; o += L.Hp * ((PS + 3) / 4) * 256;
    L.pb4 = o; o += PS * 128;
    L.pw23 = o; o += PS ? 2 * L.Hp * L.Hp : 0;
    L.ptb = o; o += PS ? 4 * L.Hp : 0;
    L.ptab = o; o += PS ? 16 * seqp_max_chunks(d, L.Hp) : 0;
    L.total = o;
    return L;
}

constexpr int kStageStride = 33;              // wave-private x tile [64][33] (conflict-free)
constexpr int kTileStride = 65;               // made_tile_kernel x tile [32][65] (d <= 64)
constexpr int kStageFloats = 64 * kStageStride;

// Affine epilogues (exact reference op order and clamps). The reference's second clamp of the
// scale exponent (clamp(-alpha, -5, 5) after alpha in [-3, 3]; clamp(alpha, -3, 3) after alpha in
// [-2, 2]) is the identity on that range, NaN included, and is not repeated here.
template <int VAR>
__device__ __forceinline__ float made_affine(float xv, float mu, float al, float& acc) {
#pragma clang fp contract(off)  // separate mul/add roundings, as the reference's torch ops
    if constexpr (VAR == NFX_MAF_INVERSE) {
        // masked_autoregressive_flow.py:25-31: alpha = clamp(alpha,-3,3);
        // z = (x - mu) * exp(clamp(-alpha, -5, 5)); guard z -> 0 (:35)
        const float a = tclamp(al, -3.f, 3.f);
        acc = acc + a;
        const float z = (xv - mu) * exp_fast(-a);
        return nonfinite(z) ? 0.f : z;
    } else {
        // inverse_autoregressive_flow.py:40-53: alpha = clamp(alpha,-2,2); mu = clamp(mu,-10,10);
        // x = z * exp(clamp(alpha,-3,3)) + mu; guard x -> z
        const float a = tclamp(al, -2.f, 2.f);
        const float m = tclamp(mu, -10.f, 10.f);
        acc = acc + a;
        const float y = xv * exp_fast(a) + m;
        return nonfinite(y) ? xv : y;
    }
}

// Stage x[64 samples][32 dims] (dims dim0..dim0+31) of a chunk into the wave's LDS tile.
__device__ __forceinline__ void stage_in(const float* __restrict__ in, int64_t base, int d, int64_t B,
                                         int dim0, float* st) {
    const int lane = lane_id();
#pragma unroll 8
    for (int i = 0; i < 32; ++i) {
        const int idx = i * 64 + lane;
        const int s = idx >> 5, dd = idx & 31;
        const int64_t row = base + s;
        const int dim = dim0 + dd;
        st[s * kStageStride + dd] = (row < B && dim < d) ? in[row * d + dim] : 0.f;
    }
}

__device__ __forceinline__ void stage_out(float* __restrict__ out, int64_t base, int d, int64_t B,
                                          int dim0, const float* st) {
    const int lane = lane_id();
#pragma unroll 8
    for (int i = 0; i < 32; ++i) {
        const int idx = i * 64 + lane;
        const int s = idx >> 5, dd = idx & 31;
        const int64_t row = base + s;
        const int dim = dim0 + dd;
        if (row < B && dim < d) out[row * d + dim] = st[s * kStageStride + dd];
    }
}


template <int HT>
__device__ __forceinline__ void made_hidden(const float* __restrict__ W, int woff, int boff,
                                            const f32x16 (&hin)[HT][2], f32x16 (&hout)[HT][2]) {
    const int lane = lane_id(), h = lane >> 5;
#pragma unroll
    for (int hto = 0; hto < HT; ++hto) {
        f32x16 a0, a1;
        load_bias16_x2(W + boff + hto * 32, h, a0, a1);
#pragma unroll
        for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
            for (int rq = 0; rq < 4; ++rq) {
                const f32x4 w = *reinterpret_cast<const f32x4*>(W + woff + (((hto * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    a0 = mfma32(w[rr], hin[kt][0][4 * rq + rr], a0);
                    a1 = mfma32(w[rr], hin[kt][1][4 * rq + rr], a1);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            a0[r] = trelu(a0[r]);
            a1[r] = trelu(a1[r]);
        }
        hout[hto][0] = a0;
        hout[hto][1] = a1;
    }
}

template <int HT, bool WLDS, int VAR>
__global__ __launch_bounds__(WLDS ? 512 : 256) void made_parallel_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d, int accumulate, int64_t nchunks,
    float* __restrict__ /*logp*/, double* __restrict__ /*partials*/, double* __restrict__ /*sums*/,
    float /*cgauss*/) {
    constexpr int NWAVE = WLDS ? 8 : 4;
    const MadeLayout L = made_layout(d, HT);
    extern __shared__ f32x4 lds4[];
    float* lds = reinterpret_cast<float*>(lds4);
    const int wave = threadIdx.x >> 6;
    float* stg;
    if constexpr (WLDS) {
        const f32x4* src = reinterpret_cast<const f32x4*>(packed);
        for (int i = threadIdx.x; i < L.par_total / 4; i += NWAVE * 64) lds4[i] = src[i];
        stg = lds + L.par_total + wave * kStageFloats;
        __syncthreads();
    } else {
        stg = lds + wave * kStageFloats;
    }
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    const int64_t nwaves = (int64_t)gridDim.x * NWAVE;

    for (int64_t c = (int64_t)blockIdx.x * NWAVE + wave; c < nchunks; c += nwaves) {
        const int64_t base = c * 64;
        const float* W = (WLDS ? lds : packed) + opaque_zero();

        // ---- layer 1: h1 = relu(W1m x + b1), K streamed in 32-dim chunks through LDS ----
        f32x16 h1[HT][2];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) load_bias16_x2(W + L.b1 + ht * 32, h, h1[ht][0], h1[ht][1]);
        for (int kc = 0; kc < L.NKC; ++kc) {
            stage_in(in, base, d, B, 32 * kc, stg);
            wave_lds_sync();
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                f32x4 w[HT];
#pragma unroll
                for (int ht = 0; ht < HT; ++ht)
                    w[ht] = *reinterpret_cast<const f32x4*>(W + L.w1 + ((ht * 4 * L.NKC + kc * 4 + g) * 64 + lane) * 4);
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int k = 8 * g + 2 * rr + h;
                    const float b0 = stg[col * kStageStride + k];
                    const float b1 = stg[(32 + col) * kStageStride + k];
#pragma unroll
                    for (int ht = 0; ht < HT; ++ht) {
                        h1[ht][0] = mfma32(w[ht][rr], b0, h1[ht][0]);
                        h1[ht][1] = mfma32(w[ht][rr], b1, h1[ht][1]);
                    }
                }
            }
            wave_lds_sync();
        }
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                h1[ht][0][r] = trelu(h1[ht][0][r]);
                h1[ht][1][r] = trelu(h1[ht][1][r]);
            }
        }
        // ---- layers 2, 3 ----
        f32x16 h2[HT][2];
        made_hidden<HT>(W, L.w2, L.b2, h1, h2);
        made_hidden<HT>(W, L.w3, L.b3, h2, h1);  // h3 -> h1 registers

        // ---- layer 4 in (mu, alpha) tile pairs + affine epilogue ----
        float acc0 = 0.f, acc1 = 0.f;
        for (int j = 0; j < L.NJ; ++j) {
            f32x16 mu0, mu1, al0, al1;
            load_bias16_x2(W + L.b4 + (j * 2 + 0) * 32, h, mu0, mu1);
            load_bias16_x2(W + L.b4 + (j * 2 + 1) * 32, h, al0, al1);
#pragma unroll
            for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) {
                    const f32x4 wm = *reinterpret_cast<const f32x4*>(
                        W + L.w4 + ((((j * 2 + 0) * HT + kt) * 4 + rq) * 64 + lane) * 4);
                    const f32x4 wa = *reinterpret_cast<const f32x4*>(
                        W + L.w4 + ((((j * 2 + 1) * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const float b0 = h1[kt][0][4 * rq + rr], b1 = h1[kt][1][4 * rq + rr];
                        mu0 = mfma32(wm[rr], b0, mu0);
                        mu1 = mfma32(wm[rr], b1, mu1);
                        al0 = mfma32(wa[rr], b0, al0);
                        al1 = mfma32(wa[rr], b1, al1);
                    }
                }
            }
            stage_in(in, base, d, B, 32 * j, stg);
            wave_lds_sync();
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = crow(r, h);
                if (32 * j + row < d) {
                    float* p0 = stg + col * kStageStride + row;
                    float* p1 = stg + (32 + col) * kStageStride + row;
                    *p0 = made_affine<VAR>(*p0, mu0[r], al0[r], acc0);
                    *p1 = made_affine<VAR>(*p1, mu1[r], al1[r], acc1);
                }
            }
            wave_lds_sync();
            stage_out(out, base, d, B, 32 * j, stg);
            wave_lds_sync();
        }
        // per-sample alpha sum: lane l <-> sample base + l
        float s = halves_sum(acc0, acc1);
        const int64_t so = base + lane;
        if (so < B) {
            float ld;
            if constexpr (VAR == NFX_MAF_INVERSE) {
                ld = -s;
                if (nonfinite(ld)) ld = 0.f;
                ld = tclamp(ld, -100.f, 100.f);
            } else {
                ld = s;
                if (nonfinite(ld)) ld = 0.f;
                ld = tclamp(ld, -50.f, 50.f);
            }
            logdet[so] = accumulate ? logdet[so] + ld : ld;
        }
    }
}


// Sequential directions (MAF.forward = sampling, IAF.inverse = density): the reference runs d
// full MADE evaluations on the partially filled vector (masked_autoregressive_flow.py:55-67,
// inverse_autoregressive_flow.py:74-90). Output i only depends on hidden units of degree < i,
// and a hidden unit of degree m only on inputs 0..m, so with the masked weights multiplying
// exact zeros every MADE output equals its value on the final vector: this kernel computes each
// hidden unit ONCE, as soon as the input of its degree is known, and each output once — one
// MADE evaluation per sample instead of d. Layer-1 pre-activations are accumulated by a rank-1
// update per step (register-resident), completed units go through layers 2-3 (dots over the
// wave-private LDS rows of h1/h2), outputs are dots over the register-resident h3. Weights are
// wave-uniform (scalar loads). One lane = one sample.
// The reference's NaN contamination is reproduced: once an x_j is non-finite, every later MADE
// call sees 0*inf = NaN through the masked weights, so all later (mu, alpha) are NaN (`poison`).
template <int HT, int VAR>
__global__ __launch_bounds__(64) void made_seq_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d, int H, int accumulate) {
    constexpr int Hp = 32 * HT;
    constexpr int RS = Hp + 4;  // LDS row stride (conflict-free ds_read_b128 across lanes)
    const MadeLayout L = made_layout(d, HT);
    extern __shared__ f32x4 lds4[];
    float* h1s = reinterpret_cast<float*>(lds4);
    float* h2s = h1s + 64 * RS;
    const int lane = threadIdx.x;
    const int64_t s = (int64_t)blockIdx.x * 64 + lane;
    const bool valid = s < B;
    const float* P = packed;

    float pre1[Hp], h3[Hp];
#pragma unroll
    for (int a = 0; a < Hp; ++a) {
        pre1[a] = P[L.s_b1 + a];
        h3[a] = 0.f;
        h1s[lane * RS + a] = 0.f;
        h2s[lane * RS + a] = 0.f;
    }
    float ld = 0.f;
    bool poison = false;
    int p = 0;  // next unit (in degree order) to complete
    const float* ord = P + L.s_deg;  // s_deg holds [unit degree] ; order is implicit below

    for (int i = 0; i < d; ++i) {
        // output i from units of degree < i (incomplete units hold h3 = 0 and masked weights)
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
        const float xin = valid ? in[s * d + i] : 0.f;
        float xi;
        if constexpr (VAR == NFX_MAF_FORWARD) {
            // masked_autoregressive_flow.py:57-65
            const float a = tclamp(al, -3.f, 3.f);
            xi = xin * exp_fast(a) + mu;
            ld = ld + a;
            if (valid) out[s * d + i] = nonfinite(xi) ? 0.f : xi;
        } else {
            // inverse_autoregressive_flow.py:79-88
            const float a = tclamp(al, -2.f, 2.f);
            const float m = tclamp(mu, -10.f, 10.f);
            xi = (xin - m) * exp_fast(-a);
            ld = ld - a;
            if (valid) out[s * d + i] = nonfinite(xi) ? xin : xi;
        }
        if (nonfinite(xi)) poison = true;
        // rank-1 update of the layer-1 pre-activations with the new input x_i
        const float* w1c = P + L.s_w1t + (size_t)i * Hp;
#pragma unroll
        for (int a = 0; a < Hp; ++a) pre1[a] = fmaf(w1c[a], xi, pre1[a]);
        // hidden units of degree i are now complete: layer 1, then 2, then 3 of the level
        int q = p;
        while (q < H && (int)ord[Hp + q] == i) ++q;  // ord[Hp + k] = degree of k-th unit in order
        if (q > p) {
            for (int k = p; k < q; ++k) {
                const int a = (int)ord[2 * Hp + k];   // unit index of the k-th completion
                float v = 0.f;
#pragma unroll
                for (int b = 0; b < Hp; ++b) v = (b == a) ? pre1[b] : v;
                h1s[lane * RS + a] = trelu(v);
            }
            for (int k = p; k < q; ++k) {
                const int a = (int)ord[2 * Hp + k];
                const float* w = P + L.s_w2 + (size_t)a * Hp;
                float v = 0.f;
#pragma unroll
                for (int b = 0; b < Hp; b += 4) {
                    const f32x4 hv = *reinterpret_cast<const f32x4*>(h1s + lane * RS + b);
                    v = fmaf(w[b], hv[0], v);
                    v = fmaf(w[b + 1], hv[1], v);
                    v = fmaf(w[b + 2], hv[2], v);
                    v = fmaf(w[b + 3], hv[3], v);
                }
                h2s[lane * RS + a] = trelu(v + P[L.s_b2 + a]);
            }
            for (int k = p; k < q; ++k) {
                const int a = (int)ord[2 * Hp + k];
                const float* w = P + L.s_w3 + (size_t)a * Hp;
                float v = 0.f;
#pragma unroll
                for (int b = 0; b < Hp; b += 4) {
                    const f32x4 hv = *reinterpret_cast<const f32x4*>(h2s + lane * RS + b);
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
    if (valid) {
        if (nonfinite(ld)) ld = 0.f;
        ld = (VAR == NFX_MAF_FORWARD) ? tclamp(ld, -100.f, 100.f) : tclamp(ld, -50.f, 50.f);
        logdet[s] = accumulate ? logdet[s] + ld : ld;
    }
}

typedef void (*made_seq_kernel_t)(const float*, const float*, float*, float*, int64_t, int, int, int);


// Small-d parallel kernel (d <= 64, e.g. the UCI-shaped d=63 MAF of cfg4). One wave owns a
// 32-sample tile: its whole [32 x d] x block sits in a wave-private LDS tile (row stride d|1,
// conflict-free column reads), loaded row by row with coalesced <=256-byte loads — and the NEXT
// tile's rows are prefetched into registers while layer 4 runs, so HBM latency hides behind
// MFMA work. Layer 1 reads its B operands from the tile, the epilogue reads x and writes z in
// place, the tile is stored row by row. Weights in LDS (512-thread workgroups, 1 per CU) when
// they fit beside the eight tiles, otherwise read from L2.
template <int HT>
__device__ __forceinline__ void made_hidden1(const float* __restrict__ W, int woff, int boff,
                                             const f32x16 (&hin)[HT], f32x16 (&hout)[HT]) {
    // All HT output tiles advance together: HT independent MFMA accumulator chains per k-step.
    const int lane = lane_id(), h = lane >> 5;
    f32x16 a[HT];
#pragma unroll
    for (int hto = 0; hto < HT; ++hto) {
        a[hto] = load_bias16(W + boff + hto * 32, h);
    }
#pragma unroll
    for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {
            f32x4 w[HT];
#pragma unroll
            for (int hto = 0; hto < HT; ++hto)
                w[hto] = *reinterpret_cast<const f32x4*>(W + woff + (((hto * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
#pragma unroll
                for (int hto = 0; hto < HT; ++hto) a[hto] = mfma32(w[hto][rr], hin[kt][4 * rq + rr], a[hto]);
            }
        }
    }
#pragma unroll
    for (int hto = 0; hto < HT; ++hto) {
#pragma unroll
        for (int r = 0; r < 16; ++r) a[hto][r] = trelu(a[hto][r]);
        hout[hto] = a[hto];
    }
}

// One output tile of a hidden layer over its first NK input tiles only (bias, MFMA chain, relu)
// — the structurally-zero trailing blocks of a MADE mask are skipped.
template <int HT, int NK>
__device__ __forceinline__ f32x16 hidden_tile(const float* __restrict__ W, int woff, int boff, int hto,
                                              const f32x16 (&hin)[HT]) {
    const int lane = lane_id(), h = lane >> 5;
    f32x16 a = load_bias16(W + boff + hto * 32, h);
#pragma unroll
    for (int kt = 0; kt < NK; ++kt) {
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {
            const f32x4 w = *reinterpret_cast<const f32x4*>(W + woff + (((hto * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) a = mfma32(w[rr], hin[kt][4 * rq + rr], a);
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) a[r] = trelu(a[r]);
    return a;
}

// hidden_tile<HT, n> for a wave-uniform runtime n in [0, N].
template <int HT, int N>
__device__ __forceinline__ f32x16 hidden_tile_n(int n, const float* __restrict__ W, int woff, int boff,
                                                int hto, const f32x16 (&hin)[HT]) {
    if constexpr (N == 0) {
        return hidden_tile<HT, 0>(W, woff, boff, hto, hin);
    } else {
        if (n >= N) return hidden_tile<HT, N>(W, woff, boff, hto, hin);
        return hidden_tile_n<HT, N - 1>(n, W, woff, boff, hto, hin);
    }
}

// Hidden layer with per-output-tile k extents nk (all HT: the interleaved dense form).
template <int HT>
__device__ __forceinline__ void made_hidden_nk(const float* __restrict__ W, int woff, int boff,
                                               const f32x16 (&hin)[HT], f32x16 (&hout)[HT],
                                               const int (&nk)[HT], bool full) {
    if (full) {
        made_hidden1<HT>(W, woff, boff, hin, hout);
        return;
    }
#pragma unroll
    for (int hto = 0; hto < HT; ++hto) hout[hto] = hidden_tile_n<HT, HT>(nk[hto], W, woff, boff, hto, hin);
}

// Layer-4 tile pair j (mu rows, alpha rows) over its first NK hidden tiles.
template <int HT, int NK>
__device__ __forceinline__ void out_pair(const float* __restrict__ W, const MadeLayout& L, int j,
                                         const f32x16 (&hin)[HT], f32x16& mu, f32x16& al) {
    const int lane = lane_id(), h = lane >> 5;
    mu = load_bias16(W + L.b4 + (j * 2 + 0) * 32, h);
    al = load_bias16(W + L.b4 + (j * 2 + 1) * 32, h);
#pragma unroll
    for (int kt = 0; kt < NK; ++kt) {
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {
            const f32x4 wm = *reinterpret_cast<const f32x4*>(
                W + L.w4 + ((((j * 2 + 0) * HT + kt) * 4 + rq) * 64 + lane) * 4);
            const f32x4 wa = *reinterpret_cast<const f32x4*>(
                W + L.w4 + ((((j * 2 + 1) * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                mu = mfma32(wm[rr], hin[kt][4 * rq + rr], mu);
                al = mfma32(wa[rr], hin[kt][4 * rq + rr], al);
            }
        }
    }
}

template <int HT, int N>
__device__ __forceinline__ void out_pair_n(int n, const float* __restrict__ W, const MadeLayout& L, int j,
                                           const f32x16 (&hin)[HT], f32x16& mu, f32x16& al) {
    if constexpr (N == 0) {
        out_pair<HT, 0>(W, L, j, hin, mu, al);
    } else {
        if (n >= N) {
            out_pair<HT, N>(W, L, j, hin, mu, al);
            return;
        }
        out_pair_n<HT, N - 1>(n, W, L, j, hin, mu, al);
    }
}

template <int HT, bool WLDS, int VAR, bool LOGP>
__global__ __launch_bounds__(512) void made_tile_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d, int accumulate, int64_t ntiles,
    float* __restrict__ logp, double* __restrict__ partials, double* __restrict__ sums, float cgauss) {
    const MadeLayout L = made_layout(d, HT);
    constexpr int S = kTileStride;
    extern __shared__ f32x4 lds4[];
    float* lds = reinterpret_cast<float*>(lds4);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // waves per workgroup: 8, or fewer (no fused log_prob) to spread a small batch over more CUs
    const int nwg = LOGP ? 8 : (int)(blockDim.x >> 6);
    if constexpr (WLDS) {
        const f32x4* src = reinterpret_cast<const f32x4*>(packed);
        for (int i = threadIdx.x; i < L.par_total / 4; i += 64 * nwg) lds4[i] = src[i];
    }
    float* xt = lds + (WLDS ? L.par_total : 0) + wave * 32 * S;
    if constexpr (WLDS) __syncthreads();
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    const int64_t nwaves = (int64_t)gridDim.x * nwg;
    // Rows move through raw buffer loads/stores: the per-tile descriptor's range check returns 0
    // for (and drops stores to) lanes >= d and rows >= B, so no per-row branches or 64-bit
    // address arithmetic; the row offset r*d*4 rides in the scalar soffset.
    const int voff = lane < d ? lane * 4 : (1 << 30);
    const int rowb = d * 4;
    // Structural-zero extents (wave-uniform scalar loads) and the overflow-safe input bound.
    const int* nkp = reinterpret_cast<const int*>(packed);
    int nk1[HT], nk2[HT], nk3[HT];
    bool full2 = true, full3 = true;
#pragma unroll
    for (int i = 0; i < HT; ++i) {
        nk1[i] = nkp[L.nk1 + i];
        nk2[i] = nkp[L.nk2 + i];
        nk3[i] = nkp[L.nk3 + i];
        full2 = full2 && nk2[i] >= HT;
        full3 = full3 && nk3[i] >= HT;
    }
    const float tsafe = packed[L.tsafe];

    int64_t t = (int64_t)blockIdx.x * nwg + wave;
    double lpacc = 0.0;
    float pf[32];
    float ldpf = 0.f;  // incoming log-det of the lane's sample (accumulate), prefetched too
    {
        if (accumulate && t < ntiles && lane < 32 && t * 32 + col < B) ldpf = logdet[t * 32 + col];
        const int64_t rows = t < ntiles ? (B - t * 32 < 32 ? B - t * 32 : 32) : 0;
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in) + (t < ntiles ? t * 32 * d : 0), 0,
                                                          (int)(rows * rowb), 0x00020000);
#pragma unroll
        for (int r = 0; r < 32; ++r)
            pf[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, r * rowb, 0));
    }
    for (; t < ntiles; t += nwaves) {
        const int64_t base = t * 32;
        const int rows = (int)(B - base < 32 ? B - base : 32);
        const float* W = (WLDS ? lds : packed) + opaque_zero();
        // Skip the structurally-zero blocks only when every input of the tile is finite and
        // within the overflow-safe bound (bit-identical then); the dense product otherwise.
        float xmax = 0.f;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            xt[r * S + lane] = pf[r];
            xmax = tmax(xmax, fabsf(pf[r]));  // NaN-propagating: a NaN fails the test
        }
        const bool dense = __builtin_amdgcn_ballot_w64(!(xmax <= tsafe)) != 0;
        wave_lds_sync();

        f32x16 h1[HT];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
            f32x16 a = load_bias16(W + L.b1 + ht * 32, h);
            const int nkc = dense ? L.NKC : nk1[ht];
            for (int kc = 0; kc < nkc; ++kc) {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x4 w =
                        *reinterpret_cast<const f32x4*>(W + L.w1 + ((ht * 4 * L.NKC + kc * 4 + g) * 64 + lane) * 4);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) a = mfma32(w[rr], xt[col * S + 32 * kc + 8 * g + 2 * rr + h], a);
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = trelu(a[r]);
            h1[ht] = a;
        }
        f32x16 h2[HT];
        made_hidden_nk<HT>(W, L.w2, L.b2, h1, h2, nk2, dense || full2);
        made_hidden_nk<HT>(W, L.w3, L.b3, h2, h1, nk3, dense || full3);  // h3 -> h1

        // prefetch the next tile's rows (and incoming log-det) while layer 4 runs
        const float ldin = ldpf;
        {
            const int64_t tn = t + nwaves;
            ldpf = (accumulate && tn < ntiles && lane < 32 && tn * 32 + col < B) ? logdet[tn * 32 + col] : 0.f;
            const int64_t rn = tn < ntiles ? (B - tn * 32 < 32 ? B - tn * 32 : 32) : 0;
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in) + (tn < ntiles ? tn * 32 * d : 0), 0,
                                                              (int)(rn * rowb), 0x00020000);
#pragma unroll
            for (int r = 0; r < 32; ++r)
                pf[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, r * rowb, 0));
        }

        // Layer 4 + affine epilogue. Padded output rows (dim >= d) have zero weights and bias:
        // their alpha is 0 (adds nothing to the log-det) and their z lands in the tile padding.
        float acc = 0.f;
        for (int j = 0; j < L.NJ; ++j) {
            f32x16 mu, al;
            out_pair_n<HT, HT>(dense ? HT : nkp[L.nk4 + j], W, L, j, h1, mu, al);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float* p = xt + col * S + 32 * j + crow(r, h);
                *p = made_affine<VAR>(*p, mu[r], al[r], acc);
            }
        }
        const float ssum = halves_sum(acc, acc);  // both halves of sample `col`
        wave_lds_sync();
        float zsq = 0.f;  // fused log_prob: sum_j z_j^2 of sample `col`, in dimension order
        if constexpr (LOGP) {
            if (lane < 32) {
                for (int jd = 0; jd < d; ++jd) {
                    const float v = xt[col * S + jd];
                    zsq = (jd == 0) ? gauss_sq0(v) : gauss_sq(zsq, v);
                }
            }
        }
        {
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(out + base * d, 0, rows * rowb, 0x00020000);
#pragma unroll
            for (int r = 0; r < 32; ++r)
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xt[r * S + lane]), rs, voff, r * rowb, 0);
        }
        if (lane < 32 && col < rows) {
            float ldv;
            if constexpr (VAR == NFX_MAF_INVERSE) {
                ldv = -ssum;
                if (nonfinite(ldv)) ldv = 0.f;
                ldv = tclamp(ldv, -100.f, 100.f);
            } else {
                ldv = ssum;
                if (nonfinite(ldv)) ldv = 0.f;
                ldv = tclamp(ldv, -50.f, 50.f);
            }
            const int64_t so = base + col;
            const float ldt = accumulate ? ldin + ldv : ldv;
            logdet[so] = ldt;
            if constexpr (LOGP) {
                const float lp = gauss_lp(zsq, cgauss, ldt);
                logp[so] = lp;
                lpacc += (double)lp;
            }
        }
        wave_lds_sync();
    }
    if constexpr (LOGP) {
        logp_commit<512>(lpacc, partials, sums, B);
    }
}

typedef void (*made_par_kernel_t)(const float*, const float*, float*, float*, int64_t, int, int, int64_t,
                                  float*, double*, double*, float);

template <int HT>
made_par_kernel_t made_pick_ht(bool wlds, int variant);
template <int HT>
made_par_kernel_t made_tile_pick_ht(bool wlds, int variant, bool logp);
template <int HT>
made_seq_kernel_t made_seq_pick_ht(int variant);

}  // namespace nfx
