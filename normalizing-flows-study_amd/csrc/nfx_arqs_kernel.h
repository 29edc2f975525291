// ARQS (autoregressive rational-quadratic spline flow) kernel template; design notes in
// nfx_arqs.hip.
#pragma once
#include "nfx_rqs_unit.h"

namespace nfx {

// Packed weight image (floats), MADE(d, H, output_dim_multiplier = R = 3K-1), masks and eval
// BatchNorm folded in:
//   w2 [HT][HT][4][64][4]  A operand of hidden layer 2: [out tile][k tile][r/4][lane][r%4]
//   w3 [HT][HT][4][64][4]  hidden layer 3
//   b1, b2, b3 [HT][2][16] biases at accumulator register r of half h (row crow(r, h))
//   w1t [d][HT][2][16]     input column j of layer 1, accumulator layout (rank-1 updates)
//   w4 [d][HT][4][64][4]   output rows i*R .. i*R+R-1 (the reference's view(b, d, R)[:, i]),
//                          A operand of one 32-row tile per step i, rows >= R zero
//   b4 [d][2][16]
struct ArqsLayout {
    int d, HT, R;
    int w2, w3, b1, b2, b3, w1t, w4, b4, total;
};

__host__ __device__ constexpr ArqsLayout arqs_layout(int d, int HT, int R) {
    ArqsLayout L{};
    L.d = d;
    L.HT = HT;
    L.R = R;
    int o = 0;
    L.w2 = o; o += HT * HT * 1024;
    L.w3 = o; o += HT * HT * 1024;
    L.b1 = o; o += HT * 32;
    L.b2 = o; o += HT * 32;
    L.b3 = o; o += HT * 32;
    L.w1t = o; o += d * HT * 32;
    L.w4 = o; o += d * HT * 1024;
    L.b4 = o; o += d * 32;
    L.total = o;
    return L;
}

struct ArqsArgs {
    const float* packed;
    const float* in;
    float* out;
    float* logdet;
    int64_t B;
    int64_t ntiles;
    int d;
    int accumulate;
    int rescale;       // data_min/data_max given (arqs.py:28-42)
    float lo, span;    // fp32(data_min), fp32(data_max - data_min)
    float min_w, cw, min_h, ch, min_d;
};

// Workgroup = HT waves, one 32-sample tile at a time (grid-stride); wave w owns hidden output
// tile w of layers 2 and 3. Per step i (arqs.py:53-80 / :86-112):
//   layer 1   pre1 += W1[:, i-1] x_{i-1} (rank-1, every wave keeps all HT tiles)
//   layer 2   own tile from relu(pre1) — no exchange
//   layer 3   own tile from every wave's layer-2 tile (exchanged through LDS)
//   output    own tile's partial of the step's R rows; partials meet in LDS
//   spline    32 threads: one sample each, unit RQS on column i (rqs_unit_eval)
template <int HT, int K, bool INV>
__global__ __launch_bounds__(64 * HT) void arqs_kernel(ArqsArgs A) {
    constexpr int R = 3 * K - 1;
    static_assert(R <= 32, "one 32-row output tile per step");
    const ArqsLayout L = arqs_layout(A.d, HT, R);
    __shared__ float xbuf[HT][16][64];
    __shared__ float obuf[32];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    const float* P = A.packed;
    // the wave's layer-2/3 row tiles stay in registers for the whole kernel
    f32x4 w2r[HT][4], w3r[HT][4];
    {
        const f32x4* g2 = reinterpret_cast<const f32x4*>(P + L.w2) + lane;
        const f32x4* g3 = reinterpret_cast<const f32x4*>(P + L.w3) + lane;
#pragma unroll
        for (int kt = 0; kt < HT; ++kt)
#pragma unroll
            for (int rq = 0; rq < 4; ++rq) {
                w2r[kt][rq] = g2[((w * HT + kt) * 4 + rq) * 64];
                w3r[kt][rq] = g3[((w * HT + kt) * 4 + rq) * 64];
            }
    }
    const f32x16 b2v = load_bias16(P + L.b2 + w * 32, h);
    const f32x16 b3v = load_bias16(P + L.b3 + w * 32, h);

    for (int64_t t = blockIdx.x; t < A.ntiles; t += gridDim.x) {
        const int64_t s = t * 32 + col;
        const bool own = threadIdx.x < 32 && s < A.B;  // spline thread of sample s
        f32x16 pre1[HT];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) pre1[ht] = load_bias16(P + L.b1 + ht * 32, h);
        float ld = 0.f;
        for (int i = 0; i < A.d; ++i) {
            // this step's output-layer A operand (k tile w) and bias, issued early
            f32x4 w4r[4];
            {
                const f32x4* g4 = reinterpret_cast<const f32x4*>(P + L.w4) + lane;
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) w4r[rq] = g4[((i * HT + w) * 4 + rq) * 64];
            }
            const float xin = own ? A.in[s * A.d + i] : 0.f;
            // layer 2 (own tile)
            f32x16 a = b2v;
#pragma unroll
            for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                for (int rq = 0; rq < 4; ++rq)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) a = mfma32(w2r[kt][rq][rr], trelu(pre1[kt][4 * rq + rr]), a);
#pragma unroll
            for (int r = 0; r < 16; ++r) xbuf[w][r][lane] = trelu(a[r]);
            __syncthreads();
            // layer 3 (own tile) from every layer-2 tile
            f32x16 c = b3v;
#pragma unroll
            for (int kt = 0; kt < HT; ++kt) {
                float hv[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) hv[r] = xbuf[kt][r][lane];
#pragma unroll
                for (int rq = 0; rq < 4; ++rq)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) c = mfma32(w3r[kt][rq][rr], hv[4 * rq + rr], c);
            }
            __syncthreads();  // every wave has read xbuf
            // output rows i*R.., partial over this wave's hidden tile (bias carried by wave 0)
            f32x16 o4 = w == 0 ? load_bias16(P + L.b4 + i * 32, h) : f32x16{};
#pragma unroll
            for (int rq = 0; rq < 4; ++rq)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) o4 = mfma32(w4r[rq][rr], trelu(c[4 * rq + rr]), o4);
#pragma unroll
            for (int r = 0; r < 16; ++r) xbuf[w][r][lane] = o4[r];
            __syncthreads();
            if (threadIdx.x < 32) {
#pragma clang fp contract(off)
                // parameter j of sample col sits at register r, half hj of every wave's partial,
                // with j = crow(r, hj)
                float prm[R];
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    const int hj = (j >> 2) & 1, r = (j & 3) + 4 * (j >> 3);
                    float v = xbuf[0][r][hj * 32 + col];
#pragma unroll
                    for (int ww = 1; ww < HT; ++ww) v = v + xbuf[ww][r][hj * 32 + col];
                    prm[j] = v;
                }
                float uw[K], uh[K], ud[K - 1];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    uw[k] = prm[k];
                    uh[k] = prm[K + k];
                }
#pragma unroll
                for (int k = 0; k < K - 1; ++k) ud[k] = prm[2 * K + k];
                const float v = A.rescale ? (xin - A.lo) / A.span : xin;
                float o, l;
                rqs_unit_eval<K, INV>(v, uw, uh, ud, A.min_w, A.cw, A.min_h, A.ch, A.min_d, o, l);
                obuf[col] = o;
                if (own) {
                    A.out[s * A.d + i] = A.rescale ? o * A.span + A.lo : o;
                    ld = ld + l;
                }
            }
            __syncthreads();
            // layer-1 rank-1 update with the new coordinate
            const float xo = obuf[col];
#pragma unroll
            for (int ht = 0; ht < HT; ++ht) {
                const f32x16 w1 = load_bias16(P + L.w1t + (i * HT + ht) * 32, h);
#pragma unroll
                for (int r = 0; r < 16; ++r) pre1[ht][r] = fmaf(w1[r], xo, pre1[ht][r]);
            }
        }
        if (own) A.logdet[s] = A.accumulate ? A.logdet[s] + ld : ld;
    }
}

typedef void (*arqs_kernel_t)(ArqsArgs);

template <int HT>
arqs_kernel_t arqs_pick_ht(int K, int inverse);

}  // namespace nfx
