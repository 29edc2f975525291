// MADE affine flows with wide hidden layers: 128 < H <= 256 (HT = 5..8 hidden tiles of 32).
//
// Same math and packed image as the H <= 128 kernels (nfx_made_kernel.h); what changes is where
// the activations live.
// * Parallel directions (MAF.inverse, IAF.forward; masked_autoregressive_flow.py:18-44,
//   inverse_autoregressive_flow.py:30-63): one wave per 32-sample tile; a layer's HT output
//   tiles are MFMA accumulators (<= 128 registers) and its input is the previous layer's tiles
//   parked in a wave-private LDS buffer in accumulator-register order (= the B operands, 16-byte
//   reads, 32 KB per wave at H = 256), weights read from L2 in A-operand order, x streamed
//   through a [32][33] LDS stage per 32-dimension chunk (coalesced rows in, conflict-free column
//   reads), output layer in (mu, alpha) tile pairs with the affine epilogue on the staged chunk.
// * Sequential directions (MAF.forward, IAF.inverse; masked_autoregressive_flow.py:46-78,
//   inverse_autoregressive_flow.py:65-103): one lane per sample as made_seq_kernel — each hidden
//   unit computed once when the input of its degree is known, each output once (one MADE
//   evaluation instead of d) — with the layer-1 pre-activations in registers (a unit's register
//   turns into its h1 value when it completes: later rank-1 updates add W1m[a][i] * x_i = exact
//   zeros to it, the mask being zero past the unit's degree) and h2 / h3 in per-lane LDS rows.
//   Weights are wave-uniform (scalar loads).
#include "nfx_made_kernel.h"

namespace nfx {

constexpr int kBigWaves = 4;
constexpr int kBigStage = 32 * kStageStride;  // [32 samples][33]

// Per-wave LDS: the stage, then the activation tiles of one layer in accumulator-register
// order [tile][r / 4][lane][r % 4] — exactly the next layer's B operands, 16-byte reads.
__host__ __device__ constexpr int big_wave_floats(int HT) { return kBigStage + HT * 1024; }

// x[32 samples][32 dims] of a tile (dims dim0..dim0+31) into the wave's stage, zero-padded.
__device__ __forceinline__ void big_stage_in(const float* __restrict__ in, int64_t base, int d, int64_t B,
                                             int dim0, float* st) {
    const int lane = lane_id();
#pragma unroll 8
    for (int i = 0; i < 16; ++i) {
        const int idx = i * 64 + lane;
        const int s = idx >> 5, dd = idx & 31;
        const int64_t row = base + s;
        const int dim = dim0 + dd;
        st[s * kStageStride + dd] = (row < B && dim < d) ? in[row * d + dim] : 0.f;
    }
}

__device__ __forceinline__ void big_stage_out(float* __restrict__ out, int64_t base, int d, int64_t B,
                                              int dim0, const float* st) {
    const int lane = lane_id();
#pragma unroll 8
    for (int i = 0; i < 16; ++i) {
        const int idx = i * 64 + lane;
        const int s = idx >> 5, dd = idx & 31;
        const int64_t row = base + s;
        const int dim = dim0 + dd;
        if (row < B && dim < d) out[row * d + dim] = st[s * kStageStride + dd];
    }
}

// relu'd accumulator tiles -> the wave's activation buffer
template <int HT>
__device__ __forceinline__ void big_put(float* act, f32x16 (&a)[HT]) {
    const int lane = lane_id();
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int rq = 0; rq < 4; ++rq)
            *reinterpret_cast<f32x4*>(act + ((t * 4 + rq) * 64 + lane) * 4) =
                f32x4{trelu(a[t][4 * rq]), trelu(a[t][4 * rq + 1]), trelu(a[t][4 * rq + 2]), trelu(a[t][4 * rq + 3])};
}

// a[hto] = b + W[hto][kt] . act[kt] over all tiles (weights from L2, B operands from LDS)
template <int HT>
__device__ __forceinline__ void big_layer(const float* __restrict__ W, int woff, int boff, const float* act,
                                          f32x16 (&a)[HT]) {
    const int lane = lane_id(), h = lane >> 5;
#pragma unroll
    for (int t = 0; t < HT; ++t) a[t] = load_bias16(W + boff + t * 32, h);
#pragma unroll 1
    for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {
            const f32x4 bv = *reinterpret_cast<const f32x4*>(act + ((kt * 4 + rq) * 64 + lane) * 4);
#pragma unroll
            for (int t = 0; t < HT; ++t) {
                const f32x4 w = *reinterpret_cast<const f32x4*>(W + woff + (((t * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) a[t] = mfma32(w[rr], bv[rr], a[t]);
            }
        }
    }
}

template <int HT, int VAR>
__global__ __launch_bounds__(kBigWaves * 64) void made_big_par_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d, int accumulate, int64_t ntiles) {
    const MadeLayout L = made_layout(d, HT);
    extern __shared__ f32x4 lds4[];
    const int wave = threadIdx.x >> 6;
    float* stg = reinterpret_cast<float*>(lds4) + wave * big_wave_floats(HT);
    float* act = stg + kBigStage;
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    const float* W = packed;

    for (int64_t t = (int64_t)blockIdx.x * kBigWaves + wave; t < ntiles; t += (int64_t)gridDim.x * kBigWaves) {
        const int64_t base = t * 32;
        // ---- layer 1: K streamed in 32-dim chunks through the stage ----
        f32x16 a[HT];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) a[ht] = load_bias16(W + L.b1 + ht * 32, h);
        for (int kc = 0; kc < L.NKC; ++kc) {
            big_stage_in(in, base, d, B, 32 * kc, stg);
            wave_lds_sync();
#pragma unroll
            for (int g = 0; g < 4; ++g) {
#pragma unroll
                for (int ht = 0; ht < HT; ++ht) {
                    const f32x4 w = *reinterpret_cast<const f32x4*>(W + L.w1 + ((ht * 4 * L.NKC + kc * 4 + g) * 64 + lane) * 4);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr)
                        a[ht] = mfma32(w[rr], stg[col * kStageStride + 8 * g + 2 * rr + h], a[ht]);
                }
            }
            wave_lds_sync();
        }
        big_put<HT>(act, a);
        wave_lds_sync();
        // ---- layers 2, 3: B operands from LDS, the new layer overwrites the old one ----
        big_layer<HT>(W, L.w2, L.b2, act, a);
        wave_lds_sync();
        big_put<HT>(act, a);
        wave_lds_sync();
        big_layer<HT>(W, L.w3, L.b3, act, a);
        wave_lds_sync();
        big_put<HT>(act, a);
        wave_lds_sync();
        // ---- layer 4 in (mu, alpha) tile pairs + affine epilogue on the staged x chunk ----
        float acc = 0.f;
        for (int j = 0; j < L.NJ; ++j) {
            f32x16 mu = load_bias16(W + L.b4 + (j * 2 + 0) * 32, h);
            f32x16 al = load_bias16(W + L.b4 + (j * 2 + 1) * 32, h);
#pragma unroll 1
            for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) {
                    const f32x4 bv = *reinterpret_cast<const f32x4*>(act + ((kt * 4 + rq) * 64 + lane) * 4);
                    const f32x4 wm = *reinterpret_cast<const f32x4*>(
                        W + L.w4 + ((((j * 2 + 0) * HT + kt) * 4 + rq) * 64 + lane) * 4);
                    const f32x4 wa = *reinterpret_cast<const f32x4*>(
                        W + L.w4 + ((((j * 2 + 1) * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        mu = mfma32(wm[rr], bv[rr], mu);
                        al = mfma32(wa[rr], bv[rr], al);
                    }
                }
            }
            big_stage_in(in, base, d, B, 32 * j, stg);
            wave_lds_sync();
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = crow(r, h);
                if (32 * j + row < d) {
                    float* p = stg + col * kStageStride + row;
                    *p = made_affine<VAR>(*p, mu[r], al[r], acc);
                }
            }
            wave_lds_sync();
            big_stage_out(out, base, d, B, 32 * j, stg);
            wave_lds_sync();
        }
        // lanes col and col + 32 hold the two row halves of sample base + col
        const float s = acc + __shfl_xor(acc, 32, 64);
        const int64_t so = base + col;
        if (h == 0 && so < B) {
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
        wave_lds_sync();
    }
}

template <int HT, int VAR>
__global__ __launch_bounds__(64) void made_big_seq_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d, int H, int accumulate) {
    constexpr int Hp = 32 * HT;
    constexpr int RS = Hp + 4;  // per-lane LDS row stride (conflict-free ds_read_b128 across lanes)
    const MadeLayout L = made_layout(d, HT);
    extern __shared__ f32x4 lds4[];
    const int lane = threadIdx.x;
    float* h2s = reinterpret_cast<float*>(lds4) + lane * RS;
    float* h3s = h2s + 64 * RS;
    const int64_t s = (int64_t)blockIdx.x * 64 + lane;
    const bool valid = s < B;
    const float* P = packed;

    float p1[Hp];  // layer-1 pre-activation of an incomplete unit, h1 of a completed one
#pragma unroll
    for (int a = 0; a < Hp; ++a) p1[a] = P[L.s_b1 + a];
#pragma unroll
    for (int a = 0; a < Hp; a += 4) {
        *reinterpret_cast<f32x4*>(h2s + a) = f32x4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f32x4*>(h3s + a) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    float ld = 0.f;
    bool poison = false;
    int p = 0;  // next unit (in completion order) to complete
    const float* ord = P + L.s_deg;

    for (int i = 0; i < d; ++i) {
        // output i from the units of degree < i (incomplete units: h3 = 0 and masked weights)
        float mu = 0.f, al = 0.f;
        const float* w_mu = P + L.s_w4 + (size_t)i * Hp;
        const float* w_al = P + L.s_w4 + (size_t)(d + i) * Hp;
#pragma unroll 8
        for (int a = 0; a < Hp; a += 4) {
            const f32x4 hv = *reinterpret_cast<const f32x4*>(h3s + a);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                mu = fmaf(w_mu[a + c], hv[c], mu);
                al = fmaf(w_al[a + c], hv[c], al);
            }
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
        // rank-1 update with the new input x_i (zero weights for the completed units)
        const float* w1c = P + L.s_w1t + (size_t)i * Hp;
#pragma unroll
        for (int a = 0; a < Hp; ++a) p1[a] = fmaf(w1c[a], xi, p1[a]);
        // the units of degree i complete: layer 1 for all of them, then 2, then 3
        int q = p;
        while (q < H && (int)ord[Hp + q] == i) ++q;
        if (q > p) {
            for (int k = p; k < q; ++k) {
                const int a = (int)ord[2 * Hp + k];
#pragma unroll
                for (int b = 0; b < Hp; ++b) p1[b] = (b == a) ? trelu(p1[b]) : p1[b];
            }
            for (int k = p; k < q; ++k) {
                const int a = (int)ord[2 * Hp + k];
                const float* w = P + L.s_w2 + (size_t)a * Hp;
                float v = 0.f;
#pragma unroll
                for (int b = 0; b < Hp; ++b) v = fmaf(w[b], p1[b], v);
                h2s[a] = trelu(v + P[L.s_b2 + a]);
            }
            for (int k = p; k < q; ++k) {
                const int a = (int)ord[2 * Hp + k];
                const float* w = P + L.s_w3 + (size_t)a * Hp;
                float v = 0.f;
#pragma unroll 8
                for (int b = 0; b < Hp; b += 4) {
                    const f32x4 hv = *reinterpret_cast<const f32x4*>(h2s + b);
                    v = fmaf(w[b], hv[0], v);
                    v = fmaf(w[b + 1], hv[1], v);
                    v = fmaf(w[b + 2], hv[2], v);
                    v = fmaf(w[b + 3], hv[3], v);
                }
                h3s[a] = trelu(v + P[L.s_b3 + a]);
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

template <int HT>
static int big_launch_ht(const float* packed, const float* in, float* out, float* log_det, int64_t B, int d,
                         int H, int variant, int accumulate, hipStream_t s) {
    if (variant == NFX_MAF_INVERSE || variant == NFX_IAF_FORWARD) {
        auto k = variant == NFX_MAF_INVERSE ? made_big_par_kernel<HT, NFX_MAF_INVERSE>
                                            : made_big_par_kernel<HT, NFX_IAF_FORWARD>;
        const size_t lds = (size_t)kBigWaves * big_wave_floats(HT) * sizeof(float);
        int rc = prepare_lds((const void*)k, lds);
        if (rc) return rc;
        const int64_t ntiles = (B + 31) / 32;
        const int grid = resident_grid((const void*)k, kBigWaves * 64, lds, (ntiles + kBigWaves - 1) / kBigWaves);
        k<<<grid, kBigWaves * 64, lds, s>>>(packed, in, out, log_det, B, d, accumulate, ntiles);
        return check_launch("made_big_par_kernel");
    }
    auto k = variant == NFX_MAF_FORWARD ? made_big_seq_kernel<HT, NFX_MAF_FORWARD>
                                        : made_big_seq_kernel<HT, NFX_IAF_INVERSE>;
    const size_t lds = 2 * 64 * (size_t)(32 * HT + 4) * sizeof(float);
    int rc = prepare_lds((const void*)k, lds);
    if (rc) return rc;
    const int64_t grid = (B + 63) / 64;
    k<<<(unsigned)grid, 64, lds, s>>>(packed, in, out, log_det, B, d, H, accumulate);
    return check_launch("made_big_seq_kernel");
}

int made_big_launch(const float* packed, const float* in, float* out, float* log_det, int64_t B, int d, int H,
                    int variant, int accumulate, hipStream_t s) {
    switch ((H + 31) / 32) {
        case 5: return big_launch_ht<5>(packed, in, out, log_det, B, d, H, variant, accumulate, s);
        case 6: return big_launch_ht<6>(packed, in, out, log_det, B, d, H, variant, accumulate, s);
        case 7: return big_launch_ht<7>(packed, in, out, log_det, B, d, H, variant, accumulate, s);
        case 8: return big_launch_ht<8>(packed, in, out, log_det, B, d, H, variant, accumulate, s);
        default: return set_error(NFX_EUNSUPPORTED, "made_affine: no wide-hidden kernel for H=%d", H);
    }
}

}  // namespace nfx
