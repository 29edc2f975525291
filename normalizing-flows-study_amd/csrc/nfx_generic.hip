// Any-shape path for the conditioner MLPs and the spline coupling element math (gfx950).
//
// The fused layer kernels (nfx_spline*.hip, nfx_affine*.hip, nfx_made*.hip) hold a whole
// conditioner in registers and LDS and therefore cover bounded shape families. Shapes beyond
// them — e.g. SplineCouplingLayer with H = 128 or several transformed dims under autograd, or
// d > 64 — run the same math as a short sequence of launches over HBM-resident activations:
//
//   nfx_linear_forward        Y = act((X o s_k) W^T + b)          one nn.Linear (+ ReLU)
//   nfx_linear_backward_data  G = ((D W) o s_k) [relu'(A)] (+ G)   dL/dinput of one nn.Linear
//   nfx_linear_backward_weight dW = D^T (X o s_k), db = sum_rows D  split-K, fixed-order reduce
//   nfx_spline_elem_forward   the coupling's RQ spline per (sample, transformed dim), guards,
//                             log-det sum (spline_coupling_layer.py:96-180, :182-309)
//   nfx_spline_elem_backward  its adjoint: dL/dparams, the direct dL/dx term
//
// GEMM: one kernel template for the three operand layouts an nn.Linear needs (NT forward, NN
// data gradient, TN weight gradient), fp32 v_mfma_f32_32x32x2_f32 (exact fp32 products, fp32
// accumulation), 64 x 64 output tile per 256-thread workgroup (2 x 2 waves of 32 x 32), K staged
// through LDS 32 at a time with the next K tile's global loads in flight during the current
// tile's MFMAs. The weight gradient contracts over the batch: split-K over workgroups into a
// [split][M][N] float workspace summed in a fixed order (deterministic, no atomics).
#include <cstdlib>
#include <type_traits>

#include "nfx_common.h"
#include "nfx_rqs_unit.h"           // rqs_unit_eval, rqs_unit_adjoint (ARQS)
#include "nfx_spline_bwd_kernel.h"  // rq_spline_adjoint
#include "nfx_spline_kernel.h"      // rq_spline_elem, SplineConsts

namespace nfx {

constexpr int kGBM = 64, kGBN = 64, kGBK = 32;

struct GemmArgs {
    const float* a;          // A(m, k): TA = 0 -> a[m * lda + k], TA = 1 -> a[k * lda + m]
    const float* b;          // B(k, n): TB = 0 -> b[k * ldb + n], TB = 1 -> b[n * ldb + k]
    float* c;                // C(m, n) = c[m * ldc + n] (+ z * M * N for split-K partials)
    int64_t M, N, K, lda, ldb, ldc;
    const float* kscale;     // optional, length K: A(m, k) *= kscale[k]   (x * mask inputs)
    const float* bmask;      // optional, indexed like b: B(k, n) *= bmask (MaskedLinear weight * mask)
    const float* bias;       // optional, length N
    const float* pscale;     // optional, length N: C = C * pscale[n] + pshift[n] after the bias
    const float* pshift;     //   (an eval-mode BatchNorm1d folded per output feature)
    const float* act;        // optional [M][ldact]: keep C(m, n) where act(m, n) > 0 (ReLU backward)
    int64_t ldact;
    const float* nscale;     // optional, length N: C(m, n) *= nscale[n]
    int relu, accumulate;
    int64_t kchunk;          // split-K: workgroup z covers k in [z * kchunk, (z + 1) * kchunk)
    float* asum;             // optional (gemm2, TA = 1): asum[z * M + m] = sum over the z slice's k of A(m, k)
};

// VA / VB: the operand's contiguous index is 16-byte aligned (ld % 4 == 0, aligned base): tiles
// move as float4s (2 per thread per operand instead of 8 dword loads), edges component-wise.
template <int TA, int TB, bool VA, bool VB>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
    __shared__ float As[kGBM][kGBK + 1];
    __shared__ float Bs[kGBK][kGBN + 1];
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, h = lane >> 5, col = lane & 31;
    const int wm = wave >> 1, wn = wave & 1;
    const int64_t m0 = (int64_t)blockIdx.x * kGBM, n0 = (int64_t)blockIdx.y * kGBN;
    const int64_t kb = (int64_t)blockIdx.z * g.kchunk;
    const int64_t ke = kb + g.kchunk < g.K ? kb + g.kchunk : g.K;
    float ra[8], rb[8];
    // element (r, c) of a row-major operand p[r * ld + c] with c the contiguous index, 4 at a time
    auto vec4 = [](const float* p, const float* msk, int64_t r, int64_t c, int64_t ld, int64_t rmax, int64_t cmax,
                   float (&o)[4]) {
        if (r < rmax && c + 3 < cmax) {
            f32x4 v = *reinterpret_cast<const f32x4*>(p + r * ld + c);
            if (msk) v *= *reinterpret_cast<const f32x4*>(msk + r * ld + c);
            o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; o[3] = v[3];
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool ok = r < rmax && c + q < cmax;
                o[q] = ok ? p[r * ld + c + q] * (msk ? msk[r * ld + c + q] : 1.f) : 0.f;
            }
        }
    };
    // global -> registers for the K tile at k0 (coalesced along the contiguous index)
    auto load = [&](int64_t k0) {
        if constexpr (VA) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int q = e * 256 + t;
                float o[4];
                if (TA == 0) {  // k contiguous: row m, 4 k's
                    const int64_t m = m0 + (q >> 3), k = k0 + (q & 7) * 4;
                    vec4(g.a, nullptr, m, k, g.lda, g.M, ke, o);
                    if (g.kscale)
#pragma unroll
                        for (int c = 0; c < 4; ++c) o[c] *= (k + c < ke) ? g.kscale[k + c] : 0.f;
                } else {        // m contiguous: row k, 4 m's
                    const int64_t k = k0 + (q >> 4), m = m0 + (q & 15) * 4;
                    vec4(g.a, nullptr, k, m, g.lda, ke, g.M, o);
                    if (g.kscale && k < ke)
#pragma unroll
                        for (int c = 0; c < 4; ++c) o[c] *= g.kscale[k];
                }
#pragma unroll
                for (int c = 0; c < 4; ++c) ra[4 * e + c] = o[c];
            }
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int idx = e * 256 + t;
                int mi, ki;
                if (TA == 0) { mi = idx >> 5; ki = idx & 31; } else { ki = idx >> 6; mi = idx & 63; }
                const int64_t m = m0 + mi, k = k0 + ki;
                float v = 0.f;
                if (m < g.M && k < ke) {
                    v = TA == 0 ? g.a[m * g.lda + k] : g.a[k * g.lda + m];
                    if (g.kscale) v *= g.kscale[k];
                }
                ra[e] = v;
            }
        }
        if constexpr (VB) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int q = e * 256 + t;
                float o[4];
                if (TB == 0) {  // n contiguous: row k, 4 n's
                    vec4(g.b, g.bmask, k0 + (q >> 4), n0 + (q & 15) * 4, g.ldb, ke, g.N, o);
                } else {        // k contiguous: row n, 4 k's
                    vec4(g.b, g.bmask, n0 + (q >> 3), k0 + (q & 7) * 4, g.ldb, g.N, ke, o);
                }
#pragma unroll
                for (int c = 0; c < 4; ++c) rb[4 * e + c] = o[c];
            }
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int idx = e * 256 + t;
                int ni, kj;
                if (TB == 0) { kj = idx >> 6; ni = idx & 63; } else { ni = idx >> 5; kj = idx & 31; }
                const int64_t n = n0 + ni, k2 = k0 + kj;
                float w = 0.f;
                if (n < g.N && k2 < ke) {
                    const int64_t o = TB == 0 ? k2 * g.ldb + n : n * g.ldb + k2;
                    w = g.b[o];
                    if (g.bmask) w *= g.bmask[o];
                }
                rb[e] = w;
            }
        }
    };
    auto park = [&]() {
        if constexpr (VA) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int q = e * 256 + t;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    if (TA == 0) As[q >> 3][(q & 7) * 4 + c] = ra[4 * e + c];
                    else As[(q & 15) * 4 + c][q >> 4] = ra[4 * e + c];
                }
            }
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int idx = e * 256 + t;
                if (TA == 0) As[idx >> 5][idx & 31] = ra[e]; else As[idx & 63][idx >> 6] = ra[e];
            }
        }
        if constexpr (VB) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int q = e * 256 + t;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    if (TB == 0) Bs[q >> 4][(q & 15) * 4 + c] = rb[4 * e + c];
                    else Bs[(q & 7) * 4 + c][q >> 3] = rb[4 * e + c];
                }
            }
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int idx = e * 256 + t;
                if (TB == 0) Bs[idx >> 6][idx & 63] = rb[e]; else Bs[idx & 31][idx >> 5] = rb[e];
            }
        }
    };
    f32x16 acc = {};
    if (kb < ke) load(kb);
    for (int64_t k0 = kb; k0 < ke; k0 += kGBK) {
        __syncthreads();  // previous tile's readers are done
        park();
        __syncthreads();
        if (k0 + kGBK < ke) load(k0 + kGBK);  // in flight during this tile's MFMAs
#pragma unroll
        for (int s = 0; s < kGBK / 2; ++s)
            acc = mfma32(As[wm * 32 + col][2 * s + h], Bs[2 * s + h][wn * 32 + col], acc);
    }
    float* c = g.c + (int64_t)blockIdx.z * g.M * g.N;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm * 32 + crow(r, h), n = n0 + wn * 32 + col;
        if (m < g.M && n < g.N) {
            float v = acc[r];
            if (g.bias) v += g.bias[n];
            if (g.pscale) v = v * g.pscale[n] + g.pshift[n];
            if (g.relu) v = trelu(v);
            if (g.act) v = g.act[m * g.ldact + n] > 0.f ? v : 0.f;
            if (g.nscale) v *= g.nscale[n];
            float* p = c + m * g.ldc + n;
            if (g.accumulate) v += *p;
            *p = v;
        }
    }
}

// ---- large-tile GEMM (M >= 128, N >= 64) -------------------------------------------------------
// 128 x BN output tile per 256-thread workgroup, 2 x 2 waves of 64 x BN/2, i.e. 2 x BN/64
// independent 32 x 32 accumulators per wave. The K tile (16 = 8 MFMA k-steps) sits in LDS split by
// k parity, A as [h][m][s] and B as [h][n][s] (k = 2s + h, rows padded to 12 floats), so a lane's
// four k-steps of one 32-row operand are ONE ds_read_b128 (12-float rows: the 16 rows of a
// ds_read_b128 lane group land on 16 different 16-B bank slots) and a k-step feeds 2 x BN/64
// MFMAs from 2 + BN/64 fragments already in registers. Double-buffered: the next K tile's global
// loads are in flight during the current tile's MFMAs and are parked into the other buffer after
// them, one barrier per K tile. The k-steps run in increasing k like gemm_kernel's, so both produce
// the same sums.
constexpr int kG2M = 128, kG2K = 16, kG2RS = 8;
// LDS float offset of 16-byte chunk `ch` (0/1: s = 4 ch .. 4 ch + 3) of operand row `row`: rows of 8
// floats, chunks swapped on odd 8-row groups, so the 16 rows of a ds_read_b128 lane group
// ({0-3, 12-15, 20-27} + base) land on 16 different 16-byte bank slots
__device__ __forceinline__ int g2_off(int row, int ch) { return row * kG2RS + 4 * (ch ^ ((row >> 3) & 1)); }

template <int TA, int TB, bool VA, bool VB, int BN, bool EXTRA, int WPE = (TA == 0 && TB == 1) ? 4 : 3>
__global__ __launch_bounds__(256, WPE) void gemm2_kernel(GemmArgs g) {
    constexpr int NJ = BN / 64;                 // 32-column tiles per wave
    constexpr int ASZ = 2 * kG2M * kG2RS;       // floats of one A stage
    constexpr int BSZ = 2 * BN * kG2RS;
    __shared__ __attribute__((aligned(16))) float sm[2 * (ASZ + BSZ)];
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, h = lane >> 5, col = lane & 31;
    const int wm = wave >> 1, wn = wave & 1;
    // XCD-aware tile order: workgroup b runs on XCD b % 8, so the bijective remap gives each XCD a
    // contiguous run of tile ids, and tile ids walk the N tiles of one 128-row band first: the
    // workgroups that share an A band share that XCD's L2 (A is read once from HBM, not N/BN times).
    const int64_t gmt = (g.M + kG2M - 1) / kG2M, gnt = (g.N + BN - 1) / BN, nwg = gmt * gnt;
    const int64_t bx = blockIdx.x, xcd = bx % 8, q8 = nwg / 8, r8 = nwg % 8;
    const int64_t wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bx / 8;
    const int64_t m0 = (wgid / gnt) * kG2M, n0 = (wgid % gnt) * BN;
    const int64_t kb = (int64_t)blockIdx.z * g.kchunk;
    const int64_t ke = kb + g.kchunk < g.K ? kb + g.kchunk : g.K;
    // Operand tiles: 128 x 16 (A) and BN x 16 (B) floats per K tile. A k-contiguous operand (A with
    // TA = 0, B with TB = 1) is read as float4s along k by all 256 threads (2 resp. BN / 64 each) and
    // parked as float2 pairs. A k-major operand (A with TA = 1, B with TB = 0: rows are k) is read as
    // float4s along its row index by R threads (R = its tile rows), each taking the 4 same-parity
    // rows k = 8 sq + 2 j + h (j = 0..3) of one 4-wide column group: a 4 x 4 register transpose then
    // gives 4 consecutive s of one row, parked with ONE 16-byte store per row (the old per-element
    // transposed stores hit 4 banks per 32 lanes: 8-way conflicts on the weight-gradient's park).
    constexpr bool AKM = TA == 1, BKM = TB == 0;
    constexpr int NA = AKM ? 4 : 2, NB = BKM ? 4 : BN / 64;
    float ra[NA][4], rb_own[(AKM && BKM) ? 1 : NB][4];
    // both k-major: a thread stages A or B, never both, so they share one register set
    auto& rb = [&]() -> auto& {
        if constexpr (AKM && BKM) return ra;
        else return rb_own;
    }();
    // k-major roles: A on threads [0, 128), B on threads [128, 128 + BN) when both are k-major,
    // else the k-major operand on threads [0, R)
    constexpr int BKM0 = AKM ? 128 : 0;
    const bool a_role = !AKM || t < 128;
    const bool b_role = !BKM || (t >= BKM0 && t < BKM0 + BN);
    auto ld4 = [](const float* p, const float* msk, int64_t r, int64_t c, int64_t ld, int64_t rmax, int64_t cmax,
                  bool vec, float (&o)[4]) {
        if (vec && r < rmax && c + 3 < cmax) {
            f32x4 v = *reinterpret_cast<const f32x4*>(p + r * ld + c);
            if (EXTRA && msk) v *= *reinterpret_cast<const f32x4*>(msk + r * ld + c);
            o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; o[3] = v[3];
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool ok = r < rmax && c + q < cmax;
                o[q] = ok ? p[r * ld + c + q] * (EXTRA && msk ? msk[r * ld + c + q] : 1.f) : 0.f;
            }
        }
    };
    // unguarded float4 (interior tiles of a plain GEMM: no bounds, no scales, no branches)
    auto ldf = [](const float* p, int64_t r, int64_t c, int64_t ld, float (&o)[4]) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(p + r * ld + c);
        o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; o[3] = v[3];
    };
    auto load = [&](int64_t k0, auto fast) {
        constexpr bool F = decltype(fast)::value;
        if constexpr (AKM) {  // A(m, k) = a[k * lda + m]; thread u: column group mq, parity h, half sq
            if (a_role) {
                const int u = t, mq = u & 31, h2 = (u >> 5) & 1, sq = u >> 6;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int64_t k = k0 + 8 * sq + 2 * j + h2, m = m0 + 4 * mq;
                    if constexpr (F) {
                        ldf(g.a, k, m, g.lda, ra[j]);
                    } else {
                        ld4(g.a, nullptr, k, m, g.lda, ke, g.M, VA, ra[j]);
                        if (EXTRA && g.kscale && k < ke)
#pragma unroll
                            for (int c = 0; c < 4; ++c) ra[j][c] *= g.kscale[k];
                    }
                }
            }
        } else {  // thread q owns row m = q >> 2, k = 4 (q & 3) .. +3
#pragma unroll
            for (int e = 0; e < NA; ++e) {
                const int q = e * 256 + t;
                const int64_t m = m0 + (q >> 2), k = k0 + (q & 3) * 4;
                if constexpr (F) {
                    ldf(g.a, m, k, g.lda, ra[e]);
                } else {
                    ld4(g.a, nullptr, m, k, g.lda, g.M, ke, VA, ra[e]);
                    if (EXTRA && g.kscale)
#pragma unroll
                        for (int c = 0; c < 4; ++c) ra[e][c] *= (k + c < ke) ? g.kscale[k + c] : 0.f;
                }
            }
        }
        if constexpr (BKM) {  // B(k, n) = b[k * ldb + n]
            if (b_role) {
                const int u = t - BKM0, nq = u % (BN / 4), h2 = (u / (BN / 4)) & 1, sq = u / (BN / 2);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int64_t k = k0 + 8 * sq + 2 * j + h2, n = n0 + 4 * nq;
                    if constexpr (F) ldf(g.b, k, n, g.ldb, rb[j]);
                    else ld4(g.b, g.bmask, k, n, g.ldb, ke, g.N, VB, rb[j]);
                }
            }
        } else {  // k contiguous: row n, 4 k's
#pragma unroll
            for (int e = 0; e < NB; ++e) {
                const int q = e * 256 + t;
                if constexpr (F) ldf(g.b, n0 + (q >> 2), k0 + (q & 3) * 4, g.ldb, rb[e]);
                else ld4(g.b, g.bmask, n0 + (q >> 2), k0 + (q & 3) * 4, g.ldb, g.N, ke, VB, rb[e]);
            }
        }
    };
    float asv[4] = {0.f, 0.f, 0.f, 0.f};  // row sums of A (TA = 1, g.asum): columns m0 + 4 mq + c
    auto park = [&](int buf) {
        float* As = sm + buf * (ASZ + BSZ);
        float* Bs = As + ASZ;
        if constexpr (AKM) {
            if (a_role) {
                const int u = t, mq = u & 31, h2 = (u >> 5) & 1, sq = u >> 6;
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    *reinterpret_cast<f32x4*>(As + g2_off(h2 * kG2M + 4 * mq + c, sq)) =
                        f32x4{ra[0][c], ra[1][c], ra[2][c], ra[3][c]};
                if (g.asum)  // the bias gradient: this thread's 4 rows, in row order
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int c = 0; c < 4; ++c) asv[c] += ra[j][c];
            }
        } else {
#pragma unroll
            for (int e = 0; e < NA; ++e) {  // k = 4 (q & 3) + c -> (h = c & 1, s = 2 (q & 3) + (c >> 1))
                const int q = e * 256 + t;
                const int m = q >> 2, s0 = 2 * (q & 3);
                *reinterpret_cast<f32x2*>(As + g2_off(0 * kG2M + m, s0 >> 2) + (s0 & 3)) = f32x2{ra[e][0], ra[e][2]};
                *reinterpret_cast<f32x2*>(As + g2_off(1 * kG2M + m, s0 >> 2) + (s0 & 3)) = f32x2{ra[e][1], ra[e][3]};
            }
        }
        if constexpr (BKM) {
            if (b_role) {
                const int u = t - BKM0, nq = u % (BN / 4), h2 = (u / (BN / 4)) & 1, sq = u / (BN / 2);
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    *reinterpret_cast<f32x4*>(Bs + g2_off(h2 * BN + 4 * nq + c, sq)) =
                        f32x4{rb[0][c], rb[1][c], rb[2][c], rb[3][c]};
            }
        } else {
#pragma unroll
            for (int e = 0; e < NB; ++e) {
                const int q = e * 256 + t;
                const int n = q >> 2, s0 = 2 * (q & 3);
                *reinterpret_cast<f32x2*>(Bs + g2_off(0 * BN + n, s0 >> 2) + (s0 & 3)) = f32x2{rb[e][0], rb[e][2]};
                *reinterpret_cast<f32x2*>(Bs + g2_off(1 * BN + n, s0 >> 2) + (s0 & 3)) = f32x2{rb[e][1], rb[e][3]};
            }
        }
    };
    f32x16 acc[2][NJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x16{};
    auto kloop = [&](auto fast) {
        int buf = 0;
        if (kb < ke) {
            load(kb, fast);
            park(0);
        }
        __syncthreads();
        for (int64_t k0 = kb; k0 < ke; k0 += kG2K) {
            const bool more = k0 + kG2K < ke;
            if (more) load(k0 + kG2K, fast);  // in flight during this tile's MFMAs
            const float* As = sm + buf * (ASZ + BSZ);
            const float* Bs = As + ASZ;
#pragma unroll
            for (int sh = 0; sh < 2; ++sh) {  // k-steps 4 sh .. 4 sh + 3
                f32x4 fa[2], fb[NJ];
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    fa[i] = *reinterpret_cast<const f32x4*>(As + g2_off(h * kG2M + wm * 64 + i * 32 + col, sh));
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                    fb[j] = *reinterpret_cast<const f32x4*>(Bs + g2_off(h * BN + wn * (BN / 2) + j * 32 + col, sh));
#pragma unroll
                for (int ss = 0; ss < 4; ++ss)
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma32(fa[i][ss], fb[j][ss], acc[i][j]);
            }
            if (more) park(buf ^ 1);
            __syncthreads();
            buf ^= 1;
        }
    };
    // interior tile of a plain GEMM with whole K tiles: the branch-free loader
    const bool inner = VA && VB && !EXTRA && m0 + kG2M <= g.M && n0 + BN <= g.N && (ke - kb) % kG2K == 0;
    if (inner) kloop(std::true_type{});
    else kloop(std::false_type{});
    if constexpr (AKM) {
        // the A row sums of this K slice, once per 128-row band (the N-tile-0 workgroup): the 4
        // (parity, half) thread groups combined in a fixed order through LDS
        if (g.asum && n0 == 0) {
            float* red = sm;  // the last tile's barrier has retired every read of the stages
            if (a_role) {
                const int u = t, mq = u & 31, grp = u >> 5;
#pragma unroll
                for (int c = 0; c < 4; ++c) red[grp * kG2M + 4 * mq + c] = asv[c];
            }
            __syncthreads();
            if (t < kG2M && m0 + t < g.M) {
                // groups (h, sq) = 0: rows 8 sq + 2 j + h; summed in group order
                const float v = ((red[t] + red[kG2M + t]) + red[2 * kG2M + t]) + red[3 * kG2M + t];
                g.asum[(int64_t)blockIdx.z * g.M + m0 + t] = v;
            }
        }
    }
    float* c = g.c + (int64_t)blockIdx.z * g.M * g.N;
    // per-column epilogue constants, read once per column (the output stores could alias them, so
    // the compiler would re-read them after every store)
    float cb[NJ], cs[NJ], ch[NJ], cn[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int64_t n = n0 + wn * (BN / 2) + j * 32 + col;
        const bool ok = n < g.N;
        cb[j] = g.bias && ok ? g.bias[n] : 0.f;
        cs[j] = g.pscale && ok ? g.pscale[n] : 1.f;
        ch[j] = g.pshift && ok ? g.pshift[n] : 0.f;
        cn[j] = g.nscale && ok ? g.nscale[n] : 1.f;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t m = m0 + wm * 64 + i * 32 + crow(r, h), n = n0 + wn * (BN / 2) + j * 32 + col;
                if (m < g.M && n < g.N) {
                    float v = acc[i][j][r];
                    if (g.bias) v += cb[j];
                    if (g.pscale) v = v * cs[j] + ch[j];
                    if (g.relu) v = trelu(v);
                    if (g.act) v = g.act[m * g.ldact + n] > 0.f ? v : 0.f;
                    if (g.nscale) v *= cn[j];
                    float* p = c + m * g.ldc + n;
                    if (g.accumulate) v += *p;
                    *p = v;
                }
            }
}

// Which GEMM: the large-tile kernel where the output has at least one full 128-row tile and 64
// columns (the conditioner GEMMs over the batch, the weight gradients of H >= 64 layers);
// $NFX_GEMM_TILE=64 forces the 64 x 64 kernel (tests compare both).
static int gemm_tile_bn(int64_t M, int64_t N) {
    static const int force = [] {
        const char* e = getenv("NFX_GEMM_TILE");
        return e ? atoi(e) : 0;
    }();
    if (force == 64 || M < kG2M || N < 64) return 0;
    return N >= 128 ? 128 : 64;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <int TA, int TB, int BN, bool EXTRA>
static void gemm2_go(const GemmArgs& g, dim3 grid, bool va, bool vb, hipStream_t s) {
    // $NFX_GEMM_WPE=3: the forward layout at 3 waves per SIMD instead of 4 (A/B measurements)
    static const int wpe = [] {
        const char* e = getenv("NFX_GEMM_WPE");
        return e ? atoi(e) : 0;
    }();
    if constexpr (TA == 0 && TB == 1 && !EXTRA) {
        if (wpe == 3 && va && vb) {
            gemm2_kernel<TA, TB, true, true, BN, EXTRA, 3><<<grid, 256, 0, s>>>(g);
            return;
        }
    }
    if (va && vb) gemm2_kernel<TA, TB, true, true, BN, EXTRA><<<grid, 256, 0, s>>>(g);
    else if (va) gemm2_kernel<TA, TB, true, false, BN, EXTRA><<<grid, 256, 0, s>>>(g);
    else if (vb) gemm2_kernel<TA, TB, false, true, BN, EXTRA><<<grid, 256, 0, s>>>(g);
    else gemm2_kernel<TA, TB, false, false, BN, EXTRA><<<grid, 256, 0, s>>>(g);
}

template <int TA, int TB>
static void gemm_go(const GemmArgs& g, dim3 grid, int bn, hipStream_t s) {
    const bool va = g.lda % 4 == 0 && aligned16(g.a);
    const bool vb = g.ldb % 4 == 0 && aligned16(g.b) && (!g.bmask || aligned16(g.bmask));
    const bool extra = g.kscale || g.bmask;
    if (bn) {
        // one-dimensional grid of M x N tiles (the kernel orders them per XCD), split-K on z
        const int64_t tiles = ((g.M + kG2M - 1) / kG2M) * ((g.N + bn - 1) / bn);
        const dim3 g1((unsigned)tiles, 1, grid.z);
        if (bn == 128) {
            if (extra) gemm2_go<TA, TB, 128, true>(g, g1, va, vb, s);
            else gemm2_go<TA, TB, 128, false>(g, g1, va, vb, s);
        } else {
            if (extra) gemm2_go<TA, TB, 64, true>(g, g1, va, vb, s);
            else gemm2_go<TA, TB, 64, false>(g, g1, va, vb, s);
        }
        return;
    }
    if (va && vb) gemm_kernel<TA, TB, true, true><<<grid, 256, 0, s>>>(g);
    else if (va) gemm_kernel<TA, TB, true, false><<<grid, 256, 0, s>>>(g);
    else if (vb) gemm_kernel<TA, TB, false, true><<<grid, 256, 0, s>>>(g);
    else gemm_kernel<TA, TB, false, false><<<grid, 256, 0, s>>>(g);
}

static int gemm_launch(const GemmArgs& g, int ta, int tb, int64_t splits, hipStream_t s) {
    // M tiles on x (the batch: up to 2^31 - 1 tiles), N tiles and split-K slices on y / z (< 65536)
    const int bn = gemm_tile_bn(g.M, g.N);
    const int64_t tm = bn ? kG2M : kGBM, tn = bn ? bn : kGBN;
    const int64_t gm = (g.M + tm - 1) / tm, gn = (g.N + tn - 1) / tn;
    if (gm > 0x7fffffff || gn > 65535 || splits > 65535 || (bn && gm * gn > 0x7fffffff))
        return set_error(NFX_EUNSUPPORTED, "linear: grid %lld x %lld x %lld out of range", (long long)gm,
                         (long long)gn, (long long)splits);
    dim3 grid((unsigned)gm, (unsigned)gn, (unsigned)splits);
    if (ta == 0 && tb == 1) gemm_go<0, 1>(g, grid, bn, s);
    else if (ta == 0 && tb == 0) gemm_go<0, 0>(g, grid, bn, s);
    else if (ta == 1 && tb == 0) gemm_go<1, 0>(g, grid, bn, s);
    else return set_error(NFX_EINVAL, "linear: unsupported layout");
    return check_launch("gemm_kernel");
}

// out[i] (+)= (sum_z part[z * n + i], z = 0 .. nz-1 in order) * mask[i] (mask optional)
__global__ void split_reduce_kernel(const float* __restrict__ part, int64_t nz, int64_t n, float* __restrict__ out,
                                    int accumulate, const float* __restrict__ mask) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        float v = 0.f;
#pragma unroll 8
        for (int64_t z = 0; z < nz; ++z) v += part[z * n + i];
        if (mask) v *= mask[i];
        out[i] = accumulate ? out[i] + v : v;
    }
}

// Column sums of D [M][N] over row range z: part[z][n] (8 row groups x 32 columns per block,
// the 8 group sums combined in a fixed order). VEC: a lane sums 4 adjacent columns read as one
// float4 (128 columns per block, N % 4 == 0 and D 16-byte aligned), 4 rows in flight per lane.
template <bool VEC>
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ d, int64_t M, int64_t N,
                                                     int64_t rchunk, float* __restrict__ part) {
    constexpr int W = VEC ? 4 : 1;
    __shared__ float red[8][32 * W + 1];
    const int cx = threadIdx.x & 31, rg = threadIdx.x >> 5;
    const int64_t n = ((int64_t)blockIdx.x * 32 + cx) * W;
    const int64_t rb = (int64_t)blockIdx.y * rchunk, re = rb + rchunk < M ? rb + rchunk : M;
    float v[W];
#pragma unroll
    for (int c = 0; c < W; ++c) v[c] = 0.f;
    if (n < N) {
        if constexpr (VEC) {
            int64_t m = rb + rg;
            for (; m + 24 < re; m += 32) {  // 4 rows in flight, summed in row order
                f32x4 x[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) x[u] = *reinterpret_cast<const f32x4*>(d + (m + 8 * u) * N + n);
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int c = 0; c < 4; ++c) v[c] += x[u][c];
            }
            for (; m < re; m += 8) {
                const f32x4 x = *reinterpret_cast<const f32x4*>(d + m * N + n);
#pragma unroll
                for (int c = 0; c < 4; ++c) v[c] += x[c];
            }
        } else {
            for (int64_t m = rb + rg; m < re; m += 8) v[0] += d[m * N + n];
        }
    }
#pragma unroll
    for (int c = 0; c < W; ++c) red[rg][cx * W + c] = v[c];
    __syncthreads();
    if (rg == 0) {
#pragma unroll
        for (int c = 0; c < W; ++c) {
            if (n + c >= N) break;
            float acc = 0.f;
            for (int q = 0; q < 8; ++q) acc += red[q][cx * W + c];
            part[(int64_t)blockIdx.y * N + n + c] = acc;
        }
    }
}

// row chunks of the bias-gradient column sum: ~1024 rows each (>= 4 waves per SIMD at the
// batch sizes the generic path serves), at most 1024 chunks
static int64_t colsum_chunks(int64_t M) {
    const int64_t c = (M + 1023) / 1024;
    return c < 1 ? 1 : (c > 1024 ? 1024 : c);
}

static int64_t wgrad_splits(int64_t M, int64_t N, int64_t K) {
    const int bn = gemm_tile_bn(M, N);
    const int64_t tm = bn ? kG2M : kGBM, tn = bn ? bn : kGBN;
    const int64_t tiles = ((M + tm - 1) / tm) * ((N + tn - 1) / tn);
    // one full round of resident workgroups (gemm2: 3 per CU at BN = 128, 4 at BN = 64, by LDS and
    // VGPRs): a split count that leaves a partial second round idles most of the chip for it
    const int64_t slots = (bn == 128 ? 3 : 4) * (int64_t)num_cus();
    const int64_t want = tiles >= slots ? 1 : slots / tiles;
    const int64_t maxs = (K + 1023) / 1024;  // at least 1024 rows per split
    int64_t s = want < maxs ? want : maxs;
    if (s < 1) s = 1;
    if (s > 1024) s = 1024;
    return s;
}

// Thin weight gradient (min(N, K) <= 8: a coupling net's first layer at small d, a MADE output
// layer's few outputs): a 64x64 MFMA tile would waste up to 63/64 of its work, so this is a
// streaming reduction instead. The wide operand (gy's N columns when THIN_X, else x's K columns)
// goes one column per lane, coalesced rows; the thin one (KT <= 8 values per row) is a uniform
// broadcast. 4 waves interleave the rows of a split; fixed-order LDS merge, one partial per split
// (part_w[split][N][K] pre-scaled by in_scale[k] like the GEMM epilogue, part_b[split][N]).
template <int KT, bool THIN_X>
__global__ __launch_bounds__(256) void thin_wgrad_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                                                         const float* __restrict__ in_scale, int64_t M, int N, int K,
                                                         int64_t rchunk, float* __restrict__ part_w,
                                                         float* __restrict__ part_b) {
    __shared__ float red[4][64][KT + 2];
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const int C = THIN_X ? N : K;
    const float* wide = THIN_X ? gy : x;
    const float* thin = THIN_X ? x : gy;
    const int64_t c = (int64_t)blockIdx.x * 64 + lane;
    const int64_t rb = (int64_t)blockIdx.y * rchunk;
    const int64_t re = rb + rchunk < M ? rb + rchunk : M;
    float acc[KT], bw = 0.f, bl = 0.f;
#pragma unroll
    for (int q = 0; q < KT; ++q) acc[q] = 0.f;
#pragma unroll 4
    for (int64_t m = rb + wave; m < re; m += 4) {
        const float w = c < C ? wide[m * C + c] : 0.f;
        bw += w;
        // gy thin: lane q < KT keeps column q's sum (the bias gradient)
        if (!THIN_X) bl += lane < KT ? thin[m * KT + lane] : 0.f;
#pragma unroll
        for (int q = 0; q < KT; ++q) acc[q] += w * thin[m * KT + q];
    }
#pragma unroll
    for (int q = 0; q < KT; ++q) red[wave][lane][q] = acc[q];
    red[wave][lane][KT] = bw;
    red[wave][lane][KT + 1] = bl;
    __syncthreads();
    if (wave != 0) return;
    const int64_t NK = (int64_t)N * K;
    if (c < C) {
#pragma unroll
        for (int q = 0; q < KT; ++q) {
            const float v = ((red[0][lane][q] + red[1][lane][q]) + red[2][lane][q]) + red[3][lane][q];
            const int64_t k = THIN_X ? q : c, n = THIN_X ? c : q;
            part_w[blockIdx.y * NK + n * K + k] = in_scale ? v * in_scale[k] : v;
        }
        if (THIN_X) {
            const float v = ((red[0][lane][KT] + red[1][lane][KT]) + red[2][lane][KT]) + red[3][lane][KT];
            part_b[(int64_t)blockIdx.y * N + c] = v;
        }
    }
    // gy is the thin operand: its column sums (the bias gradient), per wave in lanes < KT
    if (!THIN_X && blockIdx.x == 0 && lane < KT) {
        const float v = ((red[0][lane][KT + 1] + red[1][lane][KT + 1]) + red[2][lane][KT + 1]) + red[3][lane][KT + 1];
        part_b[(int64_t)blockIdx.y * N + lane] = v;
    }
}

// ---- RQ spline coupling, element math ------------------------------------------------------
static SplineConsts spline_consts(int K, float bound, float min_w, float min_h, float min_d) {
    SplineConsts C{};
    C.bound = bound;
    C.two_bound = (float)(2.0 * (double)bound);
    C.min_w = min_w;
    C.cw = (float)(1.0 - (double)min_w * K);
    C.min_h = min_h;
    C.ch = (float)(1.0 - (double)min_h * K);
    C.min_d = min_d;
    C.rescale = 0;
    return C;
}

// one lane per sample: every dim in order, spline on the transformed ones (mask == 0), the
// layer guards (spline_coupling_layer.py:130-135 / :173-178) and the log-det (sum over the
// transformed dims in order, then accumulate)
template <int K, bool INV>
__global__ __launch_bounds__(256) void spline_elem_fwd_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ prm,
                                                              const float* __restrict__ mask, float* __restrict__ y,
                                                              float* __restrict__ log_det, int64_t B, int d,
                                                              int accumulate, const SplineConsts C,
                                                              const float* __restrict__ rs) {
#pragma clang fp contract(off)  // the reference's separate roundings of the rescale
    constexpr int P = 3 * K - 1;
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= B) return;
    float ld = 0.f;
    bool first = true;
    for (int j = 0; j < d; ++j) {
        const float v = x[s * d + j];
        float o = v;
        if (mask[j] == 0.f) {
            float p[32];
            const float* pr = prm + (s * d + j) * P;
#pragma unroll
            for (int i = 0; i < 32; ++i) p[i] = i < P ? pr[i] : 0.f;
            float lad;
            // rs = [lo | to | from][d]: data_min/data_max bounds (spline_coupling_layer.py:78-94)
            const float vr = rs ? rs[d + j] * (v - rs[j]) - C.bound : v;
            rq_spline_elem<K, INV>(vr, p, C, o, lad);
            if (rs) o = (o + C.bound) * rs[2 * d + j] + rs[j];
            ld = first ? lad : ld + lad;
            first = false;
        }
        y[s * d + j] = nonfinite(o) ? 0.f : o;
    }
    if (nonfinite(ld)) ld = 0.f;
    log_det[s] = accumulate ? log_det[s] + ld : ld;
}

// two lanes per (sample, dim) element — lane half h = 0 owns the width side, h = 1 the heights
// (rq_spline_adjoint); a wave covers 32 samples, walking the dims. gprm gets dL/dparams of every
// dim (zeros for conditioning dims), gx the direct dL/dx term (the spline's own input gradient
// for transformed dims, gy through the layer guard for conditioning dims).
template <int K, bool INV>
__global__ __launch_bounds__(256) void spline_elem_bwd_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ prm,
                                                              const float* __restrict__ mask,
                                                              const float* __restrict__ gy,
                                                              const float* __restrict__ gld,
                                                              float* __restrict__ gprm, float* __restrict__ gx,
                                                              int64_t B, int d, const SplineConsts C,
                                                              const float* __restrict__ rs) {
#pragma clang fp contract(off)
    constexpr int P = 3 * K - 1;
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    const int64_t s = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 32 + col;
    const bool ok = s < B;
    const int64_t sc = ok ? s : 0;
    const float gl = gld ? gld[sc] : 0.f;
    for (int j = 0; j < d; ++j) {
        const float v = x[sc * d + j];
        const float g = gy ? gy[sc * d + j] : 0.f;
        float* gp = gprm + (sc * d + j) * P;
        if (mask[j] == 0.f) {
            float p[32];
            const float* pr = prm + (sc * d + j) * P;
#pragma unroll
            for (int i = 0; i < 32; ++i) p[i] = i < P ? pr[i] : 0.f;
            float o, gs[K], gd[K / 2], gv;
            // the layer guard zeroes a non-finite output, which only a non-finite input gives;
            // with bounds y = (S(vr) + B) from + lo, vr = to (v - lo) - B: dL/dS = g from, dv = dvr to
            const float gg = nonfinite(v) ? 0.f : g;
            if (rs) {
                const float vr = rs[d + j] * (v - rs[j]) - C.bound;
                rq_spline_adjoint<K, INV>(vr, p, C, gg * rs[2 * d + j], gl, o, gs, gd, gv);
                gv = gv * rs[d + j];
            } else {
                rq_spline_adjoint<K, INV>(v, p, C, gg, gl, o, gs, gd, gv);
            }
            if (ok) {
#pragma unroll
                for (int k = 0; k < K; ++k) gp[h * K + k] = gs[k];
#pragma unroll
                for (int q = 0; q < K / 2; ++q)
                    if (2 * q + h < K - 1) gp[2 * K + 2 * q + h] = gd[q];
                if (h == 0) gx[s * d + j] = gv;
            }
        } else if (ok) {
            for (int i = h; i < P; i += 2) gp[i] = 0.f;
            if (h == 0) gx[s * d + j] = nonfinite(v) ? 0.f : g;
        }
    }
}

template <bool BWD>
static const void* spline_elem_pick(int K, bool inv) {
#define NFX_SE(k)                                                                                         \
    case k:                                                                                               \
        if (BWD) return inv ? (const void*)spline_elem_bwd_kernel<k, true> : (const void*)spline_elem_bwd_kernel<k, false>; \
        return inv ? (const void*)spline_elem_fwd_kernel<k, true> : (const void*)spline_elem_fwd_kernel<k, false>;
    switch (K) {
        NFX_SE(2) NFX_SE(3) NFX_SE(4) NFX_SE(5) NFX_SE(6) NFX_SE(7) NFX_SE(8) NFX_SE(9) NFX_SE(10) NFX_SE(11)
    }
#undef NFX_SE
    return nullptr;
}

// ---- MADE affine flows, element math -----------------------------------------------------
// params [B][2d] = the MADE output, mu = params[:, :d], alpha = params[:, d:] (chunk(2, dim=1)).
// Parallel directions (one thread per sample, dims in order, log-det summed in dim order):
//   MAF inverse  masked_autoregressive_flow.py:18-44   z = (x - mu) exp(clamp(-clamp(a,-3,3),-5,5))
//   IAF forward  inverse_autoregressive_flow.py:30-63  y = x exp(clamp(clamp(a,-2,2),-3,3)) + clamp(mu,-10,10)
// A wave per sample (grid-stride over samples), lanes over the dims: every row access is
// coalesced; the log-det is a fixed-order wave reduction (xor butterfly) of the lanes' partial
// sums — deterministic, summed in another order than the reference's left-to-right
// torch.sum (within fp32 rounding).
__device__ __forceinline__ float wave_sum_xor(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ __launch_bounds__(256) void made_elem_fwd_kernel(const float* __restrict__ x, const float* __restrict__ prm,
                                                            float* __restrict__ y, float* __restrict__ log_det,
                                                            int64_t B, int d, int variant, int accumulate) {
#pragma clang fp contract(off)
    const int lane = lane_id();
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    const bool maf = variant == NFX_MAF_INVERSE;
    for (int64_t s = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); s < B; s += nw) {
        const float* mu = prm + s * 2 * d;
        const float* al = mu + d;
        float part = 0.f;
        for (int j = lane; j < d; j += 64) {
            const float xv = x[s * d + j];
            if (maf) {
                const float a = tclamp(al[j], -3.f, 3.f);
                const float z = (xv - mu[j]) * exp_fast(tclamp(-a, -5.f, 5.f));
                y[s * d + j] = nonfinite(z) ? 0.f : z;
                part = part + a;
            } else {
                const float a = tclamp(al[j], -2.f, 2.f);
                const float v = xv * exp_fast(tclamp(a, -3.f, 3.f)) + tclamp(mu[j], -10.f, 10.f);
                y[s * d + j] = nonfinite(v) ? xv : v;
                part = part + a;
            }
        }
        const float tot = wave_sum_xor(part);
        if (lane == 0) {
            float ld = maf ? -tot : tot;
            ld = nonfinite(ld) ? 0.f : (maf ? tclamp(ld, -100.f, 100.f) : tclamp(ld, -50.f, 50.f));
            log_det[s] = accumulate ? log_det[s] + ld : ld;
        }
    }
}

// One step i of a sequential direction on the running vector w [B][d] (the conditioner input of
// the next step) and the running log-det ld [B] (starts at 0):
//   MAF forward  masked_autoregressive_flow.py:55-74   w_i = x_i exp(clamp(a_i,-5,5)) + mu_i, ld += a_i
//   IAF inverse  inverse_autoregressive_flow.py:80-99  w_i = (x_i - clamp(mu_i,-10,10)) exp(clamp(-a_i,-3,3)), ld -= a_i
__global__ __launch_bounds__(256) void made_elem_step_kernel(const float* __restrict__ x, const float* __restrict__ prm,
                                                             float* __restrict__ w, float* __restrict__ ld, int64_t B,
                                                             int d, int i, int variant) {
#pragma clang fp contract(off)
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= B) return;
    const float mu = prm[s * 2 * d + i], al = prm[s * 2 * d + d + i], xv = x[s * d + i];
    if (variant == NFX_MAF_FORWARD) {
        const float a = tclamp(al, -3.f, 3.f);
        w[s * d + i] = xv * exp_fast(tclamp(a, -5.f, 5.f)) + mu;
        ld[s] = ld[s] + a;
    } else {
        const float a = tclamp(al, -2.f, 2.f);
        w[s * d + i] = (xv - tclamp(mu, -10.f, 10.f)) * exp_fast(tclamp(-a, -3.f, 3.f));
        ld[s] = ld[s] - a;
    }
}

// The sequential directions' final guards (:75-77 / :100-102), then write or accumulate the log-det.
__global__ __launch_bounds__(256) void made_elem_finish_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                               const float* __restrict__ ldw, float* __restrict__ y,
                                                               float* __restrict__ log_det, int64_t B, int d, int variant,
                                                               int accumulate) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= B) return;
    const bool maf = variant == NFX_MAF_FORWARD;
    for (int j = 0; j < d; ++j) {
        const float v = w[s * d + j];
        y[s * d + j] = nonfinite(v) ? (maf ? 0.f : x[s * d + j]) : v;
    }
    float ld = ldw[s];
    ld = nonfinite(ld) ? 0.f : (maf ? tclamp(ld, -100.f, 100.f) : tclamp(ld, -50.f, 50.f));
    log_det[s] = accumulate ? log_det[s] + ld : ld;
}

// Adjoint of made_elem_fwd_kernel (autograd of the reference's ops, guards and clamps included):
// gprm [B][2d] = (dL/dmu, dL/dalpha), gx [B][d] = the direct dL/dx term. A wave per sample,
// lanes over the dims, as the forward.
__global__ __launch_bounds__(256) void made_elem_bwd_kernel(const float* __restrict__ x, const float* __restrict__ prm,
                                                            const float* __restrict__ gy, const float* __restrict__ gld,
                                                            float* __restrict__ gprm, float* __restrict__ gx, int64_t B,
                                                            int d, int variant) {
#pragma clang fp contract(off)
    const int lane = lane_id();
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    const bool maf = variant == NFX_MAF_INVERSE;
    const float lo = maf ? -3.f : -2.f, hi = maf ? 3.f : 2.f, lim = maf ? 100.f : 50.f;
    for (int64_t s = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); s < B; s += nw) {
        const float* mu = prm + s * 2 * d;
        const float* al = mu + d;
        float* gmu = gprm + s * 2 * d;
        float* gal = gmu + d;
        float part = 0.f;
        for (int j = lane; j < d; j += 64) part = part + tclamp(al[j], lo, hi);
        const float asum = wave_sum_xor(part);
        const float ldraw = maf ? -asum : asum;
        const float ld1 = nonfinite(ldraw) ? 0.f : ldraw;
        const float g0 = gld ? gld[s] : 0.f;
        const float gl = (nonfinite(ldraw) || !(ld1 >= -lim && ld1 <= lim)) ? 0.f : g0;
        for (int j = lane; j < d; j += 64) {
            const float xv = x[s * d + j], alpha = al[j], m = mu[j];
            const float g = gy ? gy[s * d + j] : 0.f;
            const float a = tclamp(alpha, lo, hi);
            const bool ain = alpha >= lo && alpha <= hi;
            if (maf) {
                const float e = exp_fast(tclamp(-a, -5.f, 5.f));
                const float xm = xv - m;
                const float gz = nonfinite(xm * e) ? 0.f : g;
                const float ge = gz * e;
                gx[s * d + j] = ge;
                gmu[j] = -ge;
                gal[j] = ain ? -(gz * xm * e) - gl : 0.f;
            } else {
                const float e = exp_fast(tclamp(a, -3.f, 3.f));
                const float yr = xv * e + tclamp(m, -10.f, 10.f);
                const bool bad = nonfinite(yr);
                const float gyr = bad ? 0.f : g;
                gx[s * d + j] = bad ? g : gyr * e;
                gmu[j] = (m >= -10.f && m <= 10.f) ? gyr : 0.f;
                gal[j] = ain ? gyr * xv * e + gl : 0.f;
            }
        }
    }
}

// Adjoint pieces of a sequential direction, differentiated at the finished vector w (the raw
// conditioner input after the last step; params = MADE(w): column i of it equals step i's
// params, the masks give mu_i, alpha_i no dependence on w_j, j >= i). With lam = the total
// dL/dw (the upstream gradient through the output guard plus what later steps pass back through
// the MADE), mode 0 writes g_w = the guard's share of gy, mode 1 dL/dparams [B][2d] of lam,
// mode 2 dL/dx. The caller iterates lam = g_w + MADE-input-VJP(mode 1) d times (nilpotent:
// the Jacobian is strictly triangular), which is autograd through the reference's d calls.
//   MAF forward  w_i = x_i exp(clamp(a_i,-5,5)) + mu_i, a = clamp(alpha,-3,3), ld = sum a
//   IAF inverse  w_i = (x_i - clamp(mu_i,-10,10)) exp(clamp(-a_i,-3,3)), a = clamp(alpha,-2,2), ld = -sum a
__global__ __launch_bounds__(256) void made_elem_seq_bwd_kernel(const float* __restrict__ x, const float* __restrict__ prm,
                                                                const float* __restrict__ w, const float* __restrict__ lam,
                                                                const float* __restrict__ gy, const float* __restrict__ gld,
                                                                float* __restrict__ out, int64_t B, int d, int variant,
                                                                int mode) {
#pragma clang fp contract(off)
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= B) return;
    const bool maf = variant == NFX_MAF_FORWARD;
    if (mode == 0) {
        for (int j = 0; j < d; ++j) out[s * d + j] = (gy && !nonfinite(w[s * d + j])) ? gy[s * d + j] : 0.f;
        return;
    }
    const float* mu = prm + s * 2 * d;
    const float* al = mu + d;
    const float lo = maf ? -3.f : -2.f, hi = maf ? 3.f : 2.f, lim = maf ? 100.f : 50.f;
    float gl = 0.f;
    if (mode == 1) {
        float ldr = 0.f;
        for (int j = 0; j < d; ++j) ldr = maf ? ldr + tclamp(al[j], lo, hi) : ldr - tclamp(al[j], lo, hi);
        const float g0 = gld ? gld[s] : 0.f;
        gl = (nonfinite(ldr) || !(ldr >= -lim && ldr <= lim)) ? 0.f : g0;
    }
    for (int j = 0; j < d; ++j) {
        const float alpha = al[j], m = mu[j], xv = x[s * d + j], l = lam[s * d + j];
        const float a = tclamp(alpha, lo, hi);
        const bool ain = alpha >= lo && alpha <= hi;
        const float e = maf ? exp_fast(tclamp(a, -5.f, 5.f)) : exp_fast(tclamp(-a, -3.f, 3.f));
        if (mode == 2) {
            const float gd = (!maf && gy && nonfinite(w[s * d + j])) ? gy[s * d + j] : 0.f;  // IAF guard: y = x
            out[s * d + j] = l * e + gd;
        } else if (maf) {
            out[s * 2 * d + j] = l;
            out[s * 2 * d + d + j] = ain ? l * xv * e + gl : 0.f;
        } else {
            const float xm = xv - tclamp(m, -10.f, 10.f);
            out[s * 2 * d + j] = (m >= -10.f && m <= 10.f) ? -(l * e) : 0.f;
            out[s * 2 * d + d + j] = ain ? -(l * xm * e) - gl : 0.f;
        }
    }
}

// Train-mode BatchNorm in a sequential direction (use_batch_norm=True, the MADE in train mode):
// every one of the reference's d calls normalises with the batch statistics of ITS partial vector,
// so step i's params are row i of call i's MADE output (no single-evaluation shortcut). The
// reverse sweep then differentiates call by call; one step's adjoint from lam (the total dL/dw,
// column i final once every later call has passed its input VJP back):
//   dL/dparams of call i = (dmu_i, dalpha_i) in row i, zeros elsewhere; dL/dx_i = lam_i e_i (+ the
//   IAF output guard's share). The log-det clamp decision uses the forward's running sum ldw.
__global__ __launch_bounds__(256) void made_elem_seq_step_bwd_kernel(
    const float* __restrict__ x, const float* __restrict__ prm, const float* __restrict__ w,
    const float* __restrict__ ldw, const float* __restrict__ lam, const float* __restrict__ gy,
    const float* __restrict__ gld, float* __restrict__ dprm, float* __restrict__ gx, int64_t B, int d, int i,
    int variant) {
#pragma clang fp contract(off)
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= B) return;
    const bool maf = variant == NFX_MAF_FORWARD;
    const float lo = maf ? -3.f : -2.f, hi = maf ? 3.f : 2.f, lim = maf ? 100.f : 50.f;
    const float ldr = ldw[s];
    const float gl = (nonfinite(ldr) || !(ldr >= -lim && ldr <= lim)) ? 0.f : (gld ? gld[s] : 0.f);
    const float m = prm[s * 2 * d + i], alpha = prm[s * 2 * d + d + i], xv = x[s * d + i], l = lam[s * d + i];
    const float a = tclamp(alpha, lo, hi);
    const bool ain = alpha >= lo && alpha <= hi;
    const float e = maf ? exp_fast(tclamp(a, -5.f, 5.f)) : exp_fast(tclamp(-a, -3.f, 3.f));
    for (int j = 0; j < 2 * d; ++j) dprm[s * 2 * d + j] = 0.f;
    if (maf) {
        dprm[s * 2 * d + i] = l;
        dprm[s * 2 * d + d + i] = ain ? l * xv * e + gl : 0.f;
    } else {
        const float xm = xv - tclamp(m, -10.f, 10.f);
        dprm[s * 2 * d + i] = (m >= -10.f && m <= 10.f) ? -(l * e) : 0.f;
        dprm[s * 2 * d + d + i] = ain ? -(l * xm * e) - gl : 0.f;
    }
    const float gd = (!maf && gy && nonfinite(w[s * d + i])) ? gy[s * d + i] : 0.f;  // IAF guard: y = x
    gx[s * d + i] = l * e + gd;
}

// out[:, j] = j < i ? w[:, j] : 0 — call i's conditioner input rebuilt from the finished vector
// (every column is written once, by its own step).
__global__ __launch_bounds__(256) void made_elem_prefix_kernel(const float* __restrict__ w, float* __restrict__ out,
                                                               int64_t B, int d, int i) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < B * d; e += (int64_t)gridDim.x * blockDim.x)
        out[e] = (int)(e % d) < i ? w[e] : 0.f;
}

// ---- affine coupling element math (coupling_layer.py:40-96) ---------------------------------
// s, b = clamp(raw, -10, 10); y = x m + (1 - m)(x exp(s) + b)  (forward) or
// x m + (1 - m)((x - b) exp(-s)) (inverse); ld = sum_j (1 - m) (+-s); guards: y, ld non-finite -> 0.
// A wave per sample, lanes over the dims (coalesced rows), log-det by a fixed-order wave
// reduction (as the MADE element kernels).
__global__ __launch_bounds__(256) void affine_elem_fwd_kernel(const float* __restrict__ x, const float* __restrict__ sr,
                                                              const float* __restrict__ br, const float* __restrict__ mask,
                                                              float* __restrict__ y, float* __restrict__ log_det,
                                                              int64_t B, int d, int dir, int accumulate) {
#pragma clang fp contract(off)
    const int lane = lane_id();
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t s = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); s < B; s += nw) {
        float part = 0.f;
        for (int j = lane; j < d; j += 64) {
            const float m = mask[j], om = 1.f - m, xv = x[s * d + j];
            const float sv = tclamp(sr[s * d + j], -10.f, 10.f), bv = tclamp(br[s * d + j], -10.f, 10.f);
            float t;
            if (dir > 0) {
                t = xv * exp_fast(sv) + bv;
                part = part + om * sv;
            } else {
                t = (xv - bv) * exp_fast(-sv);
                part = part + om * (-sv);
            }
            const float v = xv * m + om * t;
            y[s * d + j] = nonfinite(v) ? 0.f : v;
        }
        float ld = wave_sum_xor(part);
        if (lane == 0) {
            if (nonfinite(ld)) ld = 0.f;
            log_det[s] = accumulate ? log_det[s] + ld : ld;
        }
    }
}

// Its adjoint: gs, gb = dL/d(raw net outputs), gx = the direct dL/dx term.
__global__ __launch_bounds__(256) void affine_elem_bwd_kernel(const float* __restrict__ x, const float* __restrict__ sr,
                                                              const float* __restrict__ br, const float* __restrict__ mask,
                                                              const float* __restrict__ gy, const float* __restrict__ gld,
                                                              float* __restrict__ gs, float* __restrict__ gb,
                                                              float* __restrict__ gx, int64_t B, int d, int dir) {
#pragma clang fp contract(off)
    const int lane = lane_id();
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t s = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); s < B; s += nw) {
        float part = 0.f;
        for (int j = lane; j < d; j += 64) {
            const float om = 1.f - mask[j], sv = tclamp(sr[s * d + j], -10.f, 10.f);
            part = part + om * (dir > 0 ? sv : -sv);
        }
        const float ld = wave_sum_xor(part);
        const float gl = (gld && !nonfinite(ld)) ? gld[s] : 0.f;
        for (int j = lane; j < d; j += 64) {
            const float m = mask[j], om = 1.f - m, xv = x[s * d + j];
            const float s0 = sr[s * d + j], b0 = br[s * d + j];
            const float sv = tclamp(s0, -10.f, 10.f), bv = tclamp(b0, -10.f, 10.f);
            const bool sin = s0 >= -10.f && s0 <= 10.f, bin = b0 >= -10.f && b0 <= 10.f;
            const float g = gy ? gy[s * d + j] : 0.f;
            float v, e, dts, dtb;
            if (dir > 0) {
                e = exp_fast(sv);
                v = xv * m + om * (xv * e + bv);
                dts = xv * e;
                dtb = 1.f;
            } else {
                e = exp_fast(-sv);
                v = xv * m + om * ((xv - bv) * e);
                dts = -((xv - bv) * e);
                dtb = -e;
            }
            const float gv = nonfinite(v) ? 0.f : g;
            const float gvo = gv * om;
            gs[s * d + j] = sin ? gvo * dts + (dir > 0 ? gl * om : -(gl * om)) : 0.f;
            gb[s * d + j] = bin ? gvo * dtb : 0.f;
            gx[s * d + j] = gv * m + gvo * e;
        }
    }
}

// ---- BatchNorm1d of a conditioner (coupling_layer.py:18-35), any H --------------------------
// prepare: per-feature mean / invstd from the batch moments (train: float64 (n, mean, M2) triples
// from nfx_flowbn_moments, SyncBN-merged; the running statistics updated with the unbiased
// variance, as torch) or from the running statistics (eval); scale = gamma invstd,
// shift = beta - mean scale, so BN(z) = z scale + shift.
__global__ void bn_prepare_kernel(const double* __restrict__ stats, const float* __restrict__ gamma,
                                  const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar,
                                  double eps, double momentum, int update, int N, float* __restrict__ mean_o,
                                  float* __restrict__ invstd_o, float* __restrict__ scale_o, float* __restrict__ shift_o) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    double mean, var;
    if (stats) {
        const double cnt = stats[3 * n], m2 = stats[3 * n + 2];
        mean = stats[3 * n + 1];
        var = cnt > 0 ? m2 / cnt : 0.0;
        if (update) {
            const double unb = cnt > 1 ? m2 / (cnt - 1) : var;
            rmean[n] = (float)((1.0 - momentum) * (double)rmean[n] + momentum * mean);
            rvar[n] = (float)((1.0 - momentum) * (double)rvar[n] + momentum * unb);
        }
    } else {
        mean = (double)rmean[n];
        var = (double)rvar[n];
    }
    const float inv = (float)(1.0 / sqrt(var + eps));
    const float mf = (float)mean;
    const float sc = gamma[n] * inv;
    mean_o[n] = mf;
    invstd_o[n] = inv;
    scale_o[n] = sc;
    shift_o[n] = beta[n] - mf * sc;
}

// h = relu(z scale + shift) over [M][N]
__global__ void bn_apply_relu_kernel(const float* __restrict__ z, const float* __restrict__ scale,
                                     const float* __restrict__ shift, float* __restrict__ h, int64_t M, int N) {
    const int64_t total = M * N;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int n = (int)(i % N);
        h[i] = trelu(z[i] * scale[n] + shift[n]);
    }
}

// Backward sums over rows z: part[z][0][n] = sum g, part[z][1][n] = sum g (zv - mean) invstd (float64)
__global__ __launch_bounds__(256) void bn_bwd_sums_kernel(const float* __restrict__ g, const float* __restrict__ zv,
                                                          const float* __restrict__ mean, const float* __restrict__ invstd,
                                                          int64_t M, int N, int64_t rchunk, double* __restrict__ part) {
    __shared__ double red[2][8][33];
    const int cx = threadIdx.x & 31, rg = threadIdx.x >> 5;
    const int n = blockIdx.x * 32 + cx;
    const int64_t rb = (int64_t)blockIdx.y * rchunk, re = rb + rchunk < M ? rb + rchunk : M;
    double a = 0.0, b = 0.0;
    if (n < N) {
        const float mu = mean[n], is = invstd[n];
        for (int64_t m = rb + rg; m < re; m += 8) {
            const float gv = g[m * N + n];
            a += (double)gv;
            b += (double)(gv * ((zv[m * N + n] - mu) * is));
        }
    }
    red[0][rg][cx] = a;
    red[1][rg][cx] = b;
    __syncthreads();
    if (rg == 0 && n < N) {
        double sa = 0.0, sb = 0.0;
        for (int q = 0; q < 8; ++q) {
            sa += red[0][q][cx];
            sb += red[1][q][cx];
        }
        part[((int64_t)blockIdx.y * 2 + 0) * N + n] = sa;
        part[((int64_t)blockIdx.y * 2 + 1) * N + n] = sb;
    }
}

__global__ void reduce_f64_kernel(const double* __restrict__ part, int64_t nz, int64_t n, double* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        double v = 0.0;
        for (int64_t z = 0; z < nz; ++z) v += part[z * n + i];
        out[i] = v;
    }
}

// g_z = gamma invstd g (eval) or gamma invstd (g - sum g / cnt - xhat sum(g xhat) / cnt) (train)
__global__ void bn_bwd_apply_kernel(const float* __restrict__ g, const float* __restrict__ zv,
                                    const float* __restrict__ mean, const float* __restrict__ invstd,
                                    const float* __restrict__ gamma, const double* __restrict__ sums,
                                    const double* __restrict__ count, int train, float* __restrict__ gz, int64_t M, int N) {
    const int64_t total = M * N;
    const double cnt = train ? *count : 1.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int n = (int)(i % N);
        const float k = gamma[n] * invstd[n];
        float v = g[i];
        if (train) {
            const float xh = (zv[i] - mean[n]) * invstd[n];
            v = v - (float)(sums[n] / cnt) - xh * (float)(sums[N + n] / cnt);
        }
        gz[i] = v * k;
    }
}

// ---- ARQS (arqs.py:44-114), one sequential step at a time --------------------------------
// params [B][d * R] = MADE(state) viewed [B, d, R] (R = 3K-1); row i = (widths | heights |
// inner derivatives) of coordinate i. mode 0: forward step — state[:, i] = spline(xr[:, i]),
// ld += log-det (the reference's x_new[:, i] / log_det_jacobian +=); mode 1: reverse step —
// with lam = dL/d(state after step i): dL/d(row i) into gprm (row i + 1 of the previous reverse
// step zeroed), dL/dx[:, i] into gx, lam[:, i] = 0 (the column was overwritten; the MADE-input
// VJP is added by the caller); mode 2: state[:, i] = 0 (the state before step i).
struct RqsConsts {
    float min_w, cw, min_h, ch, min_d;
};

template <int K, bool INV>
__global__ __launch_bounds__(256) void arqs_step_kernel(const float* __restrict__ xr, const float* __restrict__ prm,
                                                        float* __restrict__ state, float* __restrict__ ld,
                                                        const float* __restrict__ gld, float* __restrict__ lam,
                                                        float* __restrict__ gprm, float* __restrict__ gx, int64_t B,
                                                        int d, int i, int mode, const RqsConsts C) {
    constexpr int R = 3 * K - 1;
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= B) return;
    if (mode == 2) {
        state[s * d + i] = 0.f;
        return;
    }
    const float* p = prm + (s * d + i) * R;
    float uw[K], uh[K], ud[K - 1];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uw[k] = p[k];
        uh[k] = p[K + k];
    }
#pragma unroll
    for (int k = 0; k < K - 1; ++k) ud[k] = p[2 * K + k];
    const float xv = xr[s * d + i];
    float o, l;
    if (mode == 0) {
        rqs_unit_eval<K, INV>(xv, uw, uh, ud, C.min_w, C.cw, C.min_h, C.ch, C.min_d, o, l);
        state[s * d + i] = o;
        ld[s] = ld[s] + l;
        return;
    }
    float g, guw[K], guh[K], gud[K - 1];
    rqs_unit_adjoint<K, INV>(xv, uw, uh, ud, C.min_w, C.cw, C.min_h, C.ch, C.min_d, lam[s * d + i],
                             gld ? gld[s] : 0.f, o, l, g, guw, guh, gud);
    float* gp = gprm + (s * d + i) * R;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        gp[k] = guw[k];
        gp[K + k] = guh[k];
    }
#pragma unroll
    for (int k = 0; k < K - 1; ++k) gp[2 * K + k] = gud[k];
    if (i + 1 < d) {
#pragma unroll
        for (int t = 0; t < R; ++t) gp[R + t] = 0.f;
    }
    gx[s * d + i] = g;
    lam[s * d + i] = 0.f;
}

static const void* arqs_step_pick(int K, bool inv) {
#define NFX_AS(k) \
    case k:       \
        return inv ? (const void*)arqs_step_kernel<k, true> : (const void*)arqs_step_kernel<k, false>;
    switch (K) {
        NFX_AS(2) NFX_AS(3) NFX_AS(4) NFX_AS(5) NFX_AS(6) NFX_AS(7) NFX_AS(8) NFX_AS(9) NFX_AS(10) NFX_AS(11)
    }
#undef NFX_AS
    return nullptr;
}

}  // namespace nfx

using namespace nfx;

extern "C" int nfx_linear_forward(const float* x, const float* w, const float* wmask, const float* b,
                                  const float* in_scale, const float* post_scale, const float* post_shift, float* y,
                                  int64_t M, int K, int N, int relu, void* stream) {
    if (M < 0 || K <= 0 || N <= 0) return set_error(NFX_EINVAL, "linear_forward: bad shape M=%lld K=%d N=%d", (long long)M, K, N);
    if (M == 0) return NFX_OK;
    if (!x || !w || !y) return set_error(NFX_EINVAL, "linear_forward: null pointer");
    GemmArgs g{};
    g.a = x; g.lda = K;
    g.b = w; g.ldb = K;
    g.c = y; g.ldc = N;
    g.M = M; g.N = N; g.K = K;
    g.kscale = in_scale;
    g.bmask = wmask;
    g.bias = b;
    if ((post_scale == nullptr) != (post_shift == nullptr))
        return set_error(NFX_EINVAL, "linear_forward: post_scale and post_shift go together");
    g.pscale = post_scale;
    g.pshift = post_shift;
    g.relu = relu;
    g.kchunk = K;
    return gemm_launch(g, 0, 1, 1, (hipStream_t)stream);
}

extern "C" int nfx_linear_backward_data(const float* gy, const float* w, const float* wmask, const float* act,
                                        const float* out_scale, float* gx, int64_t M, int N, int K, int accumulate,
                                        void* stream) {
    if (M < 0 || K <= 0 || N <= 0) return set_error(NFX_EINVAL, "linear_backward_data: bad shape M=%lld N=%d K=%d", (long long)M, N, K);
    if (M == 0) return NFX_OK;
    if (!gy || !w || !gx) return set_error(NFX_EINVAL, "linear_backward_data: null pointer");
    GemmArgs g{};
    g.a = gy; g.lda = N;
    g.b = w; g.ldb = K;
    g.bmask = wmask;
    g.c = gx; g.ldc = K;
    g.M = M; g.N = K; g.K = N;
    g.act = act; g.ldact = K;
    g.nscale = out_scale;
    g.accumulate = accumulate;
    g.kchunk = N;
    return gemm_launch(g, 0, 0, 1, (hipStream_t)stream);
}

static constexpr int kThin = 8;

// row splits of the thin weight gradient: about 8 blocks per CU, at least 256 rows each
static int64_t thin_splits(int64_t M, int N, int K) {
    const int64_t C = K <= kThin ? N : K;
    const int64_t gx = (C + 63) / 64;
    int64_t s = (8 * (int64_t)num_cus() + gx - 1) / gx;
    const int64_t maxs = (M + 255) / 256;
    if (s > maxs) s = maxs;
    if (s > 4096) s = 4096;
    return s < 1 ? 1 : s;
}

template <bool THIN_X>
static void thin_wgrad_go(int kt, dim3 grid, hipStream_t s, const float* gy, const float* x, const float* sc, int64_t M,
                          int N, int K, int64_t rchunk, float* pw, float* pb) {
    switch (kt) {
#define NFX_THIN(KT) case KT: thin_wgrad_kernel<KT, THIN_X><<<grid, 256, 0, s>>>(gy, x, sc, M, N, K, rchunk, pw, pb); break;
        NFX_THIN(1) NFX_THIN(2) NFX_THIN(3) NFX_THIN(4) NFX_THIN(5) NFX_THIN(6) NFX_THIN(7) NFX_THIN(8)
#undef NFX_THIN
    }
}

extern "C" size_t nfx_linear_workspace_bytes(int64_t M, int N, int K) {
    if (M <= 0 || N <= 0 || K <= 0) return 0;
    if (K <= kThin || N <= kThin) return (size_t)(thin_splits(M, N, K) * (int64_t)N * (K + 1) * sizeof(float));
    const int64_t s = wgrad_splits(N, K, M);
    const int64_t cs = colsum_chunks(M);
    // the large-tile GEMM also writes the bias partials [s][N] beside the weight partials
    const int64_t a = s * (int64_t)N * K + (gemm_tile_bn(N, K) ? s * (int64_t)N : 0), b = (cs < 1 ? 1 : cs) * (int64_t)N;
    return (size_t)((a > b ? a : b) * sizeof(float));
}

extern "C" int nfx_linear_backward_weight(const float* gy, const float* x, const float* in_scale, const float* wmask,
                                          float* gw, float* gb, int64_t M, int N, int K, void* workspace,
                                          void* stream) {
    if (M < 0 || K <= 0 || N <= 0) return set_error(NFX_EINVAL, "linear_backward_weight: bad shape M=%lld N=%d K=%d", (long long)M, N, K);
    if (!gw || (M > 0 && (!gy || !x || !workspace))) return set_error(NFX_EINVAL, "linear_backward_weight: null pointer");
    hipStream_t s = (hipStream_t)stream;
    float* ws = reinterpret_cast<float*>(workspace);
    if (M == 0) {
        (void)wmask;
        (void)hipMemsetAsync(gw, 0, (size_t)N * K * sizeof(float), s);
        if (gb) (void)hipMemsetAsync(gb, 0, (size_t)N * sizeof(float), s);
        return check_launch("linear_backward_weight(memset)");
    }
    const int64_t NK = (int64_t)N * K;
    if (K <= kThin || N <= kThin) {
        const bool thin_x = K <= kThin;
        const int64_t splits = thin_splits(M, N, K);
        const int64_t rchunk = (M + splits - 1) / splits;
        const int64_t nz = (M + rchunk - 1) / rchunk;
        const dim3 grid((unsigned)(((thin_x ? N : K) + 63) / 64), (unsigned)nz);
        float* pb = ws + nz * NK;
        if (thin_x) thin_wgrad_go<true>(K, grid, s, gy, x, in_scale, M, N, K, rchunk, ws, pb);
        else thin_wgrad_go<false>(N, grid, s, gy, x, in_scale, M, N, K, rchunk, ws, pb);
        int rc = check_launch("thin_wgrad_kernel");
        if (rc) return rc;
        split_reduce_kernel<<<(unsigned)((NK + 255) / 256 < 4096 ? (NK + 255) / 256 : 4096), 256, 0, s>>>(ws, nz, NK, gw, 0, wmask);
        rc = check_launch("split_reduce_kernel");
        if (rc || !gb) return rc;
        split_reduce_kernel<<<(unsigned)((N + 255) / 256), 256, 0, s>>>(pb, nz, N, gb, 0, nullptr);
        return check_launch("split_reduce_kernel");
    }
    // gw [N][K] = sum_m gy[m][n] x[m][k] s[k]: A(n, m) = gy[m * N + n] (TA = 1), B(m, k) = x[m * K + k]
    const int64_t splits = wgrad_splits(N, K, M);
    int64_t kchunk = (M + splits - 1) / splits;
    kchunk = (kchunk + kGBK - 1) / kGBK * kGBK;
    const int64_t nz = (M + kchunk - 1) / kchunk;
    GemmArgs g{};
    g.a = gy; g.lda = N;
    g.b = x; g.ldb = K;
    g.c = ws; g.ldc = K;
    g.M = N; g.N = K; g.K = M;
    g.kchunk = kchunk;
    // x * in_scale applies to B's n index here (the input features): scale after the sum
    g.nscale = in_scale;
    // the large-tile GEMM sums gy's columns (the bias gradient) from the tiles it stages anyway
    const bool fused_bias = gb && gemm_tile_bn(N, K);
    if (fused_bias) g.asum = ws + nz * NK;
    int rc = gemm_launch(g, 1, 0, nz, s);
    if (rc) return rc;
    split_reduce_kernel<<<(unsigned)((NK + 255) / 256 < 4096 ? (NK + 255) / 256 : 4096), 256, 0, s>>>(ws, nz, NK, gw, 0, wmask);
    rc = check_launch("split_reduce_kernel");
    if (rc || !gb) return rc;
    if (fused_bias) {
        split_reduce_kernel<<<(unsigned)((N + 255) / 256), 256, 0, s>>>(g.asum, nz, N, gb, 0, nullptr);
        return check_launch("split_reduce_kernel");
    }
    const int64_t cs = colsum_chunks(M);
    const int64_t rchunk = (M + cs - 1) / cs;
    const int64_t ncs = (M + rchunk - 1) / rchunk;
    if (N % 4 == 0 && aligned16(gy))
        colsum_kernel<true><<<dim3((unsigned)((N + 127) / 128), (unsigned)ncs), 256, 0, s>>>(gy, M, N, rchunk, ws);
    else
        colsum_kernel<false><<<dim3((unsigned)((N + 31) / 32), (unsigned)ncs), 256, 0, s>>>(gy, M, N, rchunk, ws);
    rc = check_launch("colsum_kernel");
    if (rc) return rc;
    split_reduce_kernel<<<(unsigned)((N + 255) / 256), 256, 0, s>>>(ws, ncs, N, gb, 0, nullptr);
    return check_launch("split_reduce_kernel");
}

// bounds (optional): device [3][d] = data_min | 2B/(data_max - data_min) | (data_max - data_min)/(2B)
// per dimension, rounded as the reference's expressions round them (the caller computes them).
static int spline_elem_fwd_launch(const float* x, const float* params, const float* mask, const float* bounds, float* y,
                                  float* log_det, int64_t B, int d, int K, float bound, float min_bin_width,
                                  float min_bin_height, float min_derivative, int direction, int accumulate,
                                  hipStream_t stream) {
    if (B < 0 || d <= 0) return set_error(NFX_EINVAL, "spline_elem_forward: bad shape B=%lld d=%d", (long long)B, d);
    if (K < 2 || K > 11) return set_error(NFX_EUNSUPPORTED, "spline_elem_forward: K=%d outside 2..11", K);
    if (direction != NFX_FORWARD && direction != NFX_INVERSE) return set_error(NFX_EINVAL, "spline_elem_forward: direction");
    if (B == 0) return NFX_OK;
    if (!x || !params || !mask || !y || !log_det) return set_error(NFX_EINVAL, "spline_elem_forward: null pointer");
    if (x == y) return set_error(NFX_EINVAL, "spline_elem_forward: x and y must not alias");
    typedef void (*fk)(const float*, const float*, const float*, float*, float*, int64_t, int, int, const SplineConsts,
                       const float*);
    fk k = (fk)spline_elem_pick<false>(K, direction < 0);
    const SplineConsts C = spline_consts(K, bound, min_bin_width, min_bin_height, min_derivative);
    const int64_t blocks = (B + 255) / 256;
    if (blocks > 0x7fffffff) return set_error(NFX_EUNSUPPORTED, "spline_elem_forward: B too large");
    k<<<(unsigned)blocks, 256, 0, stream>>>(x, params, mask, y, log_det, B, d, accumulate, C, bounds);
    return check_launch("spline_elem_fwd_kernel");
}

static int spline_elem_bwd_launch(const float* x, const float* params, const float* mask, const float* bounds,
                                  const float* gy, const float* gld, float* gparams, float* gx, int64_t B, int d, int K,
                                  float bound, float min_bin_width, float min_bin_height, float min_derivative,
                                  int direction, hipStream_t stream) {
    if (B < 0 || d <= 0) return set_error(NFX_EINVAL, "spline_elem_backward: bad shape B=%lld d=%d", (long long)B, d);
    if (K < 2 || K > 11) return set_error(NFX_EUNSUPPORTED, "spline_elem_backward: K=%d outside 2..11", K);
    if (direction != NFX_FORWARD && direction != NFX_INVERSE) return set_error(NFX_EINVAL, "spline_elem_backward: direction");
    if (B == 0) return NFX_OK;
    if (!x || !params || !mask || !gparams || !gx) return set_error(NFX_EINVAL, "spline_elem_backward: null pointer");
    typedef void (*bk)(const float*, const float*, const float*, const float*, const float*, float*, float*, int64_t,
                       int, const SplineConsts, const float*);
    bk k = (bk)spline_elem_pick<true>(K, direction < 0);
    const SplineConsts C = spline_consts(K, bound, min_bin_width, min_bin_height, min_derivative);
    const int64_t blocks = (B + 127) / 128;
    if (blocks > 0x7fffffff) return set_error(NFX_EUNSUPPORTED, "spline_elem_backward: B too large");
    k<<<(unsigned)blocks, 256, 0, stream>>>(x, params, mask, gy, gld, gparams, gx, B, d, C, bounds);
    return check_launch("spline_elem_bwd_kernel");
}

extern "C" int nfx_spline_elem_forward(const float* x, const float* params, const float* mask, float* y,
                                       float* log_det, int64_t B, int d, int K, float bound, float min_bin_width,
                                       float min_bin_height, float min_derivative, int direction, int accumulate,
                                       void* stream) {
    return spline_elem_fwd_launch(x, params, mask, nullptr, y, log_det, B, d, K, bound, min_bin_width, min_bin_height,
                                  min_derivative, direction, accumulate, (hipStream_t)stream);
}

extern "C" int nfx_spline_elem_forward_bounded(const float* x, const float* params, const float* mask,
                                               const float* bounds, float* y, float* log_det, int64_t B, int d, int K,
                                               float bound, float min_bin_width, float min_bin_height,
                                               float min_derivative, int direction, int accumulate, void* stream) {
    if (!bounds) return set_error(NFX_EINVAL, "spline_elem_forward_bounded: null bounds");
    return spline_elem_fwd_launch(x, params, mask, bounds, y, log_det, B, d, K, bound, min_bin_width, min_bin_height,
                                  min_derivative, direction, accumulate, (hipStream_t)stream);
}

extern "C" int nfx_spline_elem_backward(const float* x, const float* params, const float* mask, const float* gy,
                                        const float* gld, float* gparams, float* gx, int64_t B, int d, int K,
                                        float bound, float min_bin_width, float min_bin_height, float min_derivative,
                                        int direction, void* stream) {
    return spline_elem_bwd_launch(x, params, mask, nullptr, gy, gld, gparams, gx, B, d, K, bound, min_bin_width,
                                  min_bin_height, min_derivative, direction, (hipStream_t)stream);
}

extern "C" int nfx_spline_elem_backward_bounded(const float* x, const float* params, const float* mask,
                                                const float* bounds, const float* gy, const float* gld, float* gparams,
                                                float* gx, int64_t B, int d, int K, float bound, float min_bin_width,
                                                float min_bin_height, float min_derivative, int direction,
                                                void* stream) {
    if (!bounds) return set_error(NFX_EINVAL, "spline_elem_backward_bounded: null bounds");
    return spline_elem_bwd_launch(x, params, mask, bounds, gy, gld, gparams, gx, B, d, K, bound, min_bin_width,
                                  min_bin_height, min_derivative, direction, (hipStream_t)stream);
}

// ARQS data_min / data_max bounds (arqs.py:28-42) and their adjoints, per element, fp32 ops as
// the reference's tensor expressions: bounds = [lo | w][d] with w = data_max - data_min.
//   mode 0: (x - lo) / w      mode 1: x * w + lo      mode 2: g / w      mode 3: g * w
__global__ __launch_bounds__(256) void arqs_bounds_kernel(const float* __restrict__ in, const float* __restrict__ bnd,
                                                          float* __restrict__ out, int64_t B, int d, int mode) {
#pragma clang fp contract(off)
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < B * d; e += (int64_t)gridDim.x * blockDim.x) {
        const int j = (int)(e % d);
        const float v = in[e], lo = bnd[j], w = bnd[d + j];
        out[e] = mode == 0 ? (v - lo) / w : mode == 1 ? v * w + lo : mode == 2 ? v / w : v * w;
    }
}

extern "C" int nfx_arqs_bounds(const float* in, const float* bounds, float* out, int64_t B, int d, int mode,
                               void* stream) {
    if (B < 0 || d <= 0) return set_error(NFX_EINVAL, "arqs_bounds: bad shape B=%lld d=%d", (long long)B, d);
    if (mode < 0 || mode > 3) return set_error(NFX_EINVAL, "arqs_bounds: mode %d", mode);
    if (B == 0) return NFX_OK;
    if (!in || !bounds || !out) return set_error(NFX_EINVAL, "arqs_bounds: null pointer");
    const int64_t n = B * d;
    arqs_bounds_kernel<<<(unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096), 256, 0, (hipStream_t)stream>>>(
        in, bounds, out, B, d, mode);
    return check_launch("arqs_bounds_kernel");
}

// xr = to (x - lo) - bound per element (spline_coupling_layer.py:78-85, fp32 ops in order):
// the conditioner input of a layer with data_min / data_max bounds (times the mask in the GEMM).
__global__ __launch_bounds__(256) void spline_rescale_kernel(const float* __restrict__ x, const float* __restrict__ rs,
                                                             float* __restrict__ xr, int64_t B, int d, float bound) {
#pragma clang fp contract(off)
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < B * d; e += (int64_t)gridDim.x * blockDim.x) {
        const int j = (int)(e % d);
        xr[e] = rs[d + j] * (x[e] - rs[j]) - bound;
    }
}

extern "C" int nfx_spline_rescale(const float* x, const float* bounds, float* xr, int64_t B, int d, float bound,
                                  void* stream) {
    if (B < 0 || d <= 0) return set_error(NFX_EINVAL, "spline_rescale: bad shape B=%lld d=%d", (long long)B, d);
    if (B == 0) return NFX_OK;
    if (!x || !bounds || !xr) return set_error(NFX_EINVAL, "spline_rescale: null pointer");
    const int64_t n = B * d;
    spline_rescale_kernel<<<(unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096), 256, 0, (hipStream_t)stream>>>(
        x, bounds, xr, B, d, bound);
    return check_launch("spline_rescale_kernel");
}

// Blocks of 4 waves for the wave-per-sample element kernels (grid-stride beyond 16 Ki waves).
static unsigned wave_grid(int64_t B) {
    const int64_t b = (B + 3) / 4;
    return (unsigned)(b < 4096 ? (b < 1 ? 1 : b) : 4096);
}

static int made_elem_check(int64_t B, int d, const char* what) {
    if (B < 0 || d <= 0) return set_error(NFX_EINVAL, "%s: bad shape B=%lld d=%d", what, (long long)B, d);
    if ((B + 255) / 256 > 0x7fffffff) return set_error(NFX_EUNSUPPORTED, "%s: B too large", what);
    return NFX_OK;
}

extern "C" int nfx_made_elem_forward(const float* x, const float* params, float* y, float* log_det, int64_t B, int d,
                                     int variant, int accumulate, void* stream) {
    int rc = made_elem_check(B, d, "made_elem_forward");
    if (rc) return rc;
    if (variant != NFX_MAF_INVERSE && variant != NFX_IAF_FORWARD)
        return set_error(NFX_EINVAL, "made_elem_forward: parallel variants only (MAF inverse / IAF forward)");
    if (B == 0) return NFX_OK;
    if (!x || !params || !y || !log_det) return set_error(NFX_EINVAL, "made_elem_forward: null pointer");
    made_elem_fwd_kernel<<<wave_grid(B), 256, 0, (hipStream_t)stream>>>(x, params, y, log_det, B, d,
                                                                                      variant, accumulate);
    return check_launch("made_elem_fwd_kernel");
}

extern "C" int nfx_made_elem_seq_step_backward(const float* x, const float* params, const float* work,
                                               const float* work_ld, const float* lam, const float* grad_out,
                                               const float* grad_log_det, float* grad_params, float* grad_in,
                                               int64_t B, int d, int i, int variant, void* stream) {
    int rc = made_elem_check(B, d, "made_elem_seq_step_backward");
    if (rc) return rc;
    if (variant != NFX_MAF_FORWARD && variant != NFX_IAF_INVERSE)
        return set_error(NFX_EINVAL, "made_elem_seq_step_backward: sequential variants only (MAF forward / IAF inverse)");
    if (i < 0 || i >= d) return set_error(NFX_EINVAL, "made_elem_seq_step_backward: step %d outside 0..%d", i, d - 1);
    if (B == 0) return NFX_OK;
    if (!x || !params || !work || !work_ld || !lam || !grad_params || !grad_in)
        return set_error(NFX_EINVAL, "made_elem_seq_step_backward: null pointer");
    made_elem_seq_step_bwd_kernel<<<(unsigned)((B + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        x, params, work, work_ld, lam, grad_out, grad_log_det, grad_params, grad_in, B, d, i, variant);
    return check_launch("made_elem_seq_step_bwd_kernel");
}

extern "C" int nfx_made_elem_prefix(const float* work, float* out, int64_t B, int d, int i, void* stream) {
    int rc = made_elem_check(B, d, "made_elem_prefix");
    if (rc) return rc;
    if (i < 0 || i > d) return set_error(NFX_EINVAL, "made_elem_prefix: column count %d outside 0..%d", i, d);
    if (B == 0) return NFX_OK;
    if (!work || !out) return set_error(NFX_EINVAL, "made_elem_prefix: null pointer");
    const int64_t n = B * d;
    made_elem_prefix_kernel<<<(unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096), 256, 0,
                              (hipStream_t)stream>>>(work, out, B, d, i);
    return check_launch("made_elem_prefix_kernel");
}

extern "C" int nfx_made_elem_step(const float* x, const float* params, float* work, float* work_ld, int64_t B, int d,
                                  int i, int variant, void* stream) {
    int rc = made_elem_check(B, d, "made_elem_step");
    if (rc) return rc;
    if (variant != NFX_MAF_FORWARD && variant != NFX_IAF_INVERSE)
        return set_error(NFX_EINVAL, "made_elem_step: sequential variants only (MAF forward / IAF inverse)");
    if (i < 0 || i >= d) return set_error(NFX_EINVAL, "made_elem_step: step %d outside 0..%d", i, d - 1);
    if (B == 0) return NFX_OK;
    if (!x || !params || !work || !work_ld) return set_error(NFX_EINVAL, "made_elem_step: null pointer");
    made_elem_step_kernel<<<(unsigned)((B + 255) / 256), 256, 0, (hipStream_t)stream>>>(x, params, work, work_ld, B, d,
                                                                                       i, variant);
    return check_launch("made_elem_step_kernel");
}

extern "C" int nfx_made_elem_finish(const float* x, const float* work, const float* work_ld, float* y, float* log_det,
                                    int64_t B, int d, int variant, int accumulate, void* stream) {
    int rc = made_elem_check(B, d, "made_elem_finish");
    if (rc) return rc;
    if (variant != NFX_MAF_FORWARD && variant != NFX_IAF_INVERSE)
        return set_error(NFX_EINVAL, "made_elem_finish: sequential variants only");
    if (B == 0) return NFX_OK;
    if (!x || !work || !work_ld || !y || !log_det) return set_error(NFX_EINVAL, "made_elem_finish: null pointer");
    made_elem_finish_kernel<<<(unsigned)((B + 255) / 256), 256, 0, (hipStream_t)stream>>>(x, work, work_ld, y, log_det,
                                                                                         B, d, variant, accumulate);
    return check_launch("made_elem_finish_kernel");
}

extern "C" int nfx_made_elem_backward(const float* x, const float* params, const float* gy, const float* gld,
                                      float* gparams, float* gx, int64_t B, int d, int variant, void* stream) {
    int rc = made_elem_check(B, d, "made_elem_backward");
    if (rc) return rc;
    if (variant != NFX_MAF_INVERSE && variant != NFX_IAF_FORWARD)
        return set_error(NFX_EINVAL, "made_elem_backward: parallel variants only");
    if (B == 0) return NFX_OK;
    if (!x || !params || !gparams || !gx) return set_error(NFX_EINVAL, "made_elem_backward: null pointer");
    made_elem_bwd_kernel<<<wave_grid(B), 256, 0, (hipStream_t)stream>>>(x, params, gy, gld, gparams, gx,
                                                                                      B, d, variant);
    return check_launch("made_elem_bwd_kernel");
}

extern "C" int nfx_made_elem_seq_backward(const float* x, const float* params, const float* work, const float* lam,
                                          const float* gy, const float* gld, float* out, int64_t B, int d, int variant,
                                          int mode, void* stream) {
    int rc = made_elem_check(B, d, "made_elem_seq_backward");
    if (rc) return rc;
    if (variant != NFX_MAF_FORWARD && variant != NFX_IAF_INVERSE)
        return set_error(NFX_EINVAL, "made_elem_seq_backward: sequential variants only");
    if (mode < 0 || mode > 2) return set_error(NFX_EINVAL, "made_elem_seq_backward: mode %d", mode);
    if (B == 0) return NFX_OK;
    if (!x || !work || !out || (mode > 0 && (!params || !lam))) return set_error(NFX_EINVAL, "made_elem_seq_backward: null pointer");
    made_elem_seq_bwd_kernel<<<(unsigned)((B + 255) / 256), 256, 0, (hipStream_t)stream>>>(x, params, work, lam, gy, gld,
                                                                                          out, B, d, variant, mode);
    return check_launch("made_elem_seq_bwd_kernel");
}

static unsigned elem_grid(int64_t n) {
    const int64_t b = (n + 255) / 256;
    return (unsigned)(b < 65536 ? (b < 1 ? 1 : b) : 65536);
}

extern "C" int nfx_affine_elem_forward(const float* x, const float* s_raw, const float* b_raw, const float* mask,
                                       float* y, float* log_det, int64_t B, int d, int direction, int accumulate,
                                       void* stream) {
    int rc = made_elem_check(B, d, "affine_elem_forward");
    if (rc) return rc;
    if (direction != NFX_FORWARD && direction != NFX_INVERSE) return set_error(NFX_EINVAL, "affine_elem_forward: direction");
    if (B == 0) return NFX_OK;
    if (!x || !s_raw || !b_raw || !mask || !y || !log_det) return set_error(NFX_EINVAL, "affine_elem_forward: null pointer");
    affine_elem_fwd_kernel<<<wave_grid(B), 256, 0, (hipStream_t)stream>>>(x, s_raw, b_raw, mask, y, log_det,
                                                                                        B, d, direction, accumulate);
    return check_launch("affine_elem_fwd_kernel");
}

extern "C" int nfx_affine_elem_backward(const float* x, const float* s_raw, const float* b_raw, const float* mask,
                                        const float* gy, const float* gld, float* gs, float* gb, float* gx, int64_t B,
                                        int d, int direction, void* stream) {
    int rc = made_elem_check(B, d, "affine_elem_backward");
    if (rc) return rc;
    if (direction != NFX_FORWARD && direction != NFX_INVERSE) return set_error(NFX_EINVAL, "affine_elem_backward: direction");
    if (B == 0) return NFX_OK;
    if (!x || !s_raw || !b_raw || !mask || !gs || !gb || !gx) return set_error(NFX_EINVAL, "affine_elem_backward: null pointer");
    affine_elem_bwd_kernel<<<wave_grid(B), 256, 0, (hipStream_t)stream>>>(x, s_raw, b_raw, mask, gy, gld, gs,
                                                                                        gb, gx, B, d, direction);
    return check_launch("affine_elem_bwd_kernel");
}

extern "C" int nfx_bn_prepare(const double* stats, const float* gamma, const float* beta, float* running_mean,
                              float* running_var, double eps, double momentum, int update_running, int N, float* mean,
                              float* invstd, float* scale, float* shift, void* stream) {
    if (N <= 0) return set_error(NFX_EINVAL, "bn_prepare: N=%d", N);
    if (!gamma || !beta || !running_mean || !running_var || !mean || !invstd || !scale || !shift)
        return set_error(NFX_EINVAL, "bn_prepare: null pointer");
    bn_prepare_kernel<<<(N + 255) / 256, 256, 0, (hipStream_t)stream>>>(stats, gamma, beta, running_mean, running_var, eps,
                                                                         momentum, stats ? update_running : 0, N, mean,
                                                                         invstd, scale, shift);
    return check_launch("bn_prepare_kernel");
}

extern "C" int nfx_bn_apply_relu(const float* z, const float* scale, const float* shift, float* h, int64_t M, int N,
                                 void* stream) {
    if (M < 0 || N <= 0) return set_error(NFX_EINVAL, "bn_apply_relu: bad shape");
    if (M == 0) return NFX_OK;
    if (!z || !scale || !shift || !h) return set_error(NFX_EINVAL, "bn_apply_relu: null pointer");
    bn_apply_relu_kernel<<<elem_grid(M * N), 256, 0, (hipStream_t)stream>>>(z, scale, shift, h, M, N);
    return check_launch("bn_apply_relu_kernel");
}

extern "C" size_t nfx_bn_workspace_bytes(int64_t M, int N) {
    if (M <= 0 || N <= 0) return 0;
    int64_t cs = (M + 4095) / 4096;
    if (cs > 1024) cs = 1024;
    return (size_t)(cs * 2 * (int64_t)N * sizeof(double));
}

extern "C" int nfx_bn_backward_sums(const float* g, const float* z, const float* mean, const float* invstd, double* sums,
                                    int64_t M, int N, void* workspace, void* stream) {
    if (M < 0 || N <= 0) return set_error(NFX_EINVAL, "bn_backward_sums: bad shape");
    if (!sums) return set_error(NFX_EINVAL, "bn_backward_sums: null sums");
    hipStream_t s = (hipStream_t)stream;
    if (M == 0) {
        (void)hipMemsetAsync(sums, 0, 2 * (size_t)N * sizeof(double), s);
        return check_launch("bn_backward_sums(memset)");
    }
    if (!g || !z || !mean || !invstd || !workspace) return set_error(NFX_EINVAL, "bn_backward_sums: null pointer");
    int64_t cs = (M + 4095) / 4096;
    if (cs > 1024) cs = 1024;
    const int64_t rchunk = (M + cs - 1) / cs, nz = (M + rchunk - 1) / rchunk;
    double* part = reinterpret_cast<double*>(workspace);
    bn_bwd_sums_kernel<<<dim3((unsigned)((N + 31) / 32), (unsigned)nz), 256, 0, s>>>(g, z, mean, invstd, M, N, rchunk, part);
    int rc = check_launch("bn_bwd_sums_kernel");
    if (rc) return rc;
    reduce_f64_kernel<<<(unsigned)((2 * N + 255) / 256), 256, 0, s>>>(part, nz, 2 * (int64_t)N, sums);
    return check_launch("reduce_f64_kernel");
}

extern "C" int nfx_bn_backward_apply(const float* g, const float* z, const float* mean, const float* invstd,
                                     const float* gamma, const double* sums, const double* count, int train, float* gz,
                                     int64_t M, int N, void* stream) {
    if (M < 0 || N <= 0) return set_error(NFX_EINVAL, "bn_backward_apply: bad shape");
    if (M == 0) return NFX_OK;
    if (!g || !gamma || !invstd || !gz || (train && (!z || !mean || !sums || !count)))
        return set_error(NFX_EINVAL, "bn_backward_apply: null pointer");
    bn_bwd_apply_kernel<<<elem_grid(M * N), 256, 0, (hipStream_t)stream>>>(g, z, mean, invstd, gamma, sums, count, train,
                                                                          gz, M, N);
    return check_launch("bn_bwd_apply_kernel");
}

extern "C" int nfx_arqs_step(const float* xr, const float* params, float* state, float* log_det, const float* gld,
                             float* lam, float* gparams, float* gx, int64_t B, int d, int K, int i, int direction,
                             int mode, float min_bin_width, float min_bin_height, float min_derivative, void* stream) {
    int rc = made_elem_check(B, d, "arqs_step");
    if (rc) return rc;
    if (K < 2 || K > 11) return set_error(NFX_EUNSUPPORTED, "arqs_step: K=%d outside 2..11", K);
    if (i < 0 || i >= d) return set_error(NFX_EINVAL, "arqs_step: step %d outside 0..%d", i, d - 1);
    if (direction != NFX_FORWARD && direction != NFX_INVERSE) return set_error(NFX_EINVAL, "arqs_step: direction");
    if (mode < 0 || mode > 2) return set_error(NFX_EINVAL, "arqs_step: mode %d", mode);
    if (B == 0) return NFX_OK;
    if (!state || (mode != 2 && (!xr || !params)) || (mode == 0 && !log_det) || (mode == 1 && (!lam || !gparams || !gx)))
        return set_error(NFX_EINVAL, "arqs_step: null pointer");
    RqsConsts C;
    C.min_w = min_bin_width;
    C.cw = (float)(1.0 - (double)min_bin_width * K);
    C.min_h = min_bin_height;
    C.ch = (float)(1.0 - (double)min_bin_height * K);
    C.min_d = min_derivative;
    typedef void (*ak)(const float*, const float*, float*, float*, const float*, float*, float*, float*, int64_t, int, int,
                       int, const RqsConsts);
    ak k = (ak)arqs_step_pick(K, direction < 0);
    k<<<(unsigned)((B + 255) / 256), 256, 0, (hipStream_t)stream>>>(xr, params, state, log_det, gld, lam, gparams, gx, B,
                                                                     d, i, mode, C);
    return check_launch("arqs_step_kernel");
}
