// Wide-input MADE-affine kernel (d > 64, H <= 64; e.g. the d=784 IAF of BASELINE cfg5) for the
// parallel directions (MAF.inverse = density, IAF.forward = sampling).
//
// Reference: made.py:81-140, masked_autoregressive_flow.py:18-44,
// inverse_autoregressive_flow.py:30-63 (see nfx_made_kernel.h for the shared conventions).
//
// The packed weights (W1 [H x d], W4 [2d x H]) are far larger than LDS, and one wave's 64-sample
// chunk would re-read all of them from L2 with the A-operand loads sitting in front of the MFMAs.
// Here the 8 waves of a workgroup (2 per SIMD) walk the same weight stream in lockstep: layer 1
// in 32-input slices, layer 4 in 32-output (mu, alpha) block pairs, each slice staged ONCE into
// an LDS double buffer by all 512 threads (one 16-byte load each, issued a step ahead) and read
// by eight 64-sample chunks; W2/W3 and the biases stay LDS-resident. Every wave prefetches its
// next x slice into registers while the current slice's MFMAs run, so HBM latency hides
// behind matrix work, and x moves through a wave-private stride-33 LDS tile (coalesced rows in,
// conflict-free sample columns out, as in the small-d kernels).
//
// Structural zeros (made_live_kernel, nfx_made.hip): under the MADE masks, hidden tile ht only
// sees inputs up to its top degree, hidden layers are block-lower-triangular and output block j
// only sees hidden tiles of lower degree. Layer 1 runs in segments — inputs [0, E_0) feed every
// tile, [E_0, E_1) tiles >= 1, ... (E = prefix max of the per-tile extents, so always a superset
// of the nonzero blocks) — and layers 2-4 stop each output tile at its extent. This is exact
// (bit-identical to the dense product) when every input of the chunk is finite and within the
// overflow-safe bound; a chunk failing that test recomputes the skipped layer-1 blocks and runs
// layers 2-4 dense, reproducing the reference's 0*inf = NaN contamination.
#pragma once
#include <type_traits>

#include "nfx_made_kernel.h"

namespace nfx {

constexpr int kWideWaves = 8;

// Layout of the dynamic LDS (floats) for HT hidden tiles.
struct WideLds {
    int r23, nr23, rb1, rb4, nrb4, wb, wbuf, xt, total;
};

__host__ __device__ inline WideLds wide_lds(const MadeLayout& L, int HT, int nw = kWideWaves) {
    WideLds W{};
    int o = 0;
    W.r23 = o; W.nr23 = L.w4 - L.w2; o += W.nr23;    // w2 b2 w3 b3 (resident)
    W.rb1 = o; o += HT * 32;                          // b1
    W.rb4 = o; W.nrb4 = L.par_total - L.b4; o += W.nrb4;  // b4
    o = (o + 3) & ~3;
    W.wb = o; W.wbuf = 2 * HT * 1024; o += 2 * W.wbuf;    // two staging buffers (W1 slice / W4 block)
    W.xt = o; o += nw * kStageFloats;                     // wave-private x tiles [64][33]
    W.total = o;
    return W;
}

// 2-tile (64-sample) hidden output tile over its first NK input tiles.
template <int HT, int NK>
__device__ __forceinline__ void hidden_tile2(const float* __restrict__ W, int woff, int boff, int hto,
                                             const f32x16 (&hin)[HT][2], f32x16& o0, f32x16& o1) {
    const int lane = lane_id(), h = lane >> 5;
    f32x16 a0, a1;
    load_bias16_x2(W + boff + hto * 32, h, a0, a1);
#pragma unroll
    for (int kt = 0; kt < NK; ++kt) {
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
    o0 = a0;
    o1 = a1;
}

template <int HT, int N>
__device__ __forceinline__ void hidden_tile2_n(int n, const float* __restrict__ W, int woff, int boff, int hto,
                                               const f32x16 (&hin)[HT][2], f32x16& o0, f32x16& o1) {
    if constexpr (N == 0) {
        hidden_tile2<HT, 0>(W, woff, boff, hto, hin, o0, o1);
    } else {
        if (n >= N) {
            hidden_tile2<HT, N>(W, woff, boff, hto, hin, o0, o1);
            return;
        }
        hidden_tile2_n<HT, N - 1>(n, W, woff, boff, hto, hin, o0, o1);
    }
}

// Layer-4 block pair j for both sample tiles over its first NK hidden tiles. wb = the staged
// block [which][kt][rq][lane][4]; bias from the LDS copy of b4.
template <int HT, int NK>
__device__ __forceinline__ void out_pair2(const float* __restrict__ wb, const float* __restrict__ b4, int j,
                                          const f32x16 (&hin)[HT][2], f32x16& mu0, f32x16& mu1,
                                          f32x16& al0, f32x16& al1) {
    const int lane = lane_id(), h = lane >> 5;
    load_bias16_x2(b4 + (j * 2 + 0) * 32, h, mu0, mu1);
    load_bias16_x2(b4 + (j * 2 + 1) * 32, h, al0, al1);
#pragma unroll
    for (int kt = 0; kt < NK; ++kt) {
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {
            const f32x4 wm = *reinterpret_cast<const f32x4*>(wb + ((0 * HT + kt) * 4 + rq) * 256 + lane * 4);
            const f32x4 wa = *reinterpret_cast<const f32x4*>(wb + ((1 * HT + kt) * 4 + rq) * 256 + lane * 4);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const float b0 = hin[kt][0][4 * rq + rr], b1 = hin[kt][1][4 * rq + rr];
                mu0 = mfma32(wm[rr], b0, mu0);
                mu1 = mfma32(wm[rr], b1, mu1);
                al0 = mfma32(wa[rr], b0, al0);
                al1 = mfma32(wa[rr], b1, al1);
            }
        }
    }
}

template <int HT, int N>
__device__ __forceinline__ void out_pair2_n(int n, const float* __restrict__ wb, const float* __restrict__ b4, int j,
                                            const f32x16 (&hin)[HT][2], f32x16& mu0, f32x16& mu1,
                                            f32x16& al0, f32x16& al1) {
    if constexpr (N == 0) {
        out_pair2<HT, 0>(wb, b4, j, hin, mu0, mu1, al0, al1);
    } else {
        if (n >= N) {
            out_pair2<HT, N>(wb, b4, j, hin, mu0, mu1, al0, al1);
            return;
        }
        out_pair2_n<HT, N - 1>(n, wb, b4, j, hin, mu0, mu1, al0, al1);
    }
}

// Stage one weight slice (n4 <= 1024 float4s, contiguous in the packed image) into an LDS
// buffer: each of the NT threads moves at most 1024 / NT float4s; `reg` carries them across the
// compute step.
template <int NT>
struct WideStage {
    f32x4 v[1024 / NT];
};

template <int NT>
__device__ __forceinline__ void wide_fetch(const float* __restrict__ src, int n4, WideStage<NT>& s) {
    const f32x4* p = reinterpret_cast<const f32x4*>(src);
#pragma unroll
    for (int q = 0; q < 1024 / NT; ++q) {
        const int e = threadIdx.x + q * NT;
        s.v[q] = e < n4 ? p[e] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
}

template <int NT>
__device__ __forceinline__ void wide_store(float* __restrict__ dst, int n4, const WideStage<NT>& s) {
    f32x4* p = reinterpret_cast<f32x4*>(dst);
#pragma unroll
    for (int q = 0; q < 1024 / NT; ++q) {
        const int e = threadIdx.x + q * NT;
        if (e < n4) p[e] = s.v[q];
    }
}

// NW waves per workgroup (8, or 4 when 8-wave workgroups would not cover every CU, e.g. the
// 64Ki per-GPU shard of cfg5f): each wave owns one 64-sample chunk per round.
template <int HT, int VAR, bool LOGP, int NW>
__global__ __launch_bounds__(64 * NW) void made_wide_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d, int accumulate, int64_t nchunks,
    float* __restrict__ logp, double* __restrict__ partials, double* __restrict__ sums, float cgauss) {
    const MadeLayout L = made_layout(d, HT);
    constexpr int NT = 64 * NW;
    const WideLds S = wide_lds(L, HT, NW);
    extern __shared__ f32x4 lds4[];
    float* lds = reinterpret_cast<float*>(lds4);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;

    // resident: w2 b2 w3 b3, b1, b4
    for (int i = threadIdx.x; i < S.nr23; i += NT) lds[S.r23 + i] = packed[L.w2 + i];
    for (int i = threadIdx.x; i < HT * 32; i += NT) lds[S.rb1 + i] = packed[L.b1 + i];
    for (int i = threadIdx.x; i < S.nrb4; i += NT) lds[S.rb4 + i] = packed[L.b4 + i];
    const float* W23 = lds + S.r23 - L.w2;  // indexable with the packed-image offsets
    const float* B1 = lds + S.rb1;
    const float* B4 = lds + S.rb4;
    float* xt = lds + S.xt + wave * kStageFloats;

    // structural-zero extents (wave-uniform scalar loads)
    const int* nkp = reinterpret_cast<const int*>(packed);
    const int NKC = L.NKC, NJ = L.NJ;
    int E[HT], nk2[HT], nk3[HT];
    bool full2 = true, full3 = true;
    {
        int run = 0;
#pragma unroll
        for (int i = 0; i < HT; ++i) {
            const int e = nkp[L.nk1 + i];
            run = e > run ? e : run;
            E[i] = (i == HT - 1) ? NKC : (run < NKC ? run : NKC);
            nk2[i] = nkp[L.nk2 + i];
            nk3[i] = nkp[L.nk3 + i];
            full2 = full2 && nk2[i] >= HT;
            full3 = full3 && nk3[i] >= HT;
        }
    }
    const float tsafe = packed[L.tsafe];
    const int n4w1 = HT * 256, n4w4 = 2 * HT * 256;
    double lpacc = 0.0;

    for (int64_t cb = (int64_t)blockIdx.x * NW; cb < nchunks; cb += (int64_t)gridDim.x * NW) {
        const int64_t c = cb + wave;
        const int64_t base = c * 64;
        const int rows = c < nchunks ? (int)(B - base < 64 ? B - base : 64) : 0;
        // x rows through range-checked buffer ops: lanes past d and rows past B read 0 / drop stores
        const auto rs_in = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in) + (rows > 0 ? base * d : 0), 0,
                                                             rows * d * 4, 0x00020000);
        const auto rs_out = __builtin_amdgcn_make_buffer_rsrc(out + (rows > 0 ? base * d : 0), 0, rows * d * 4,
                                                              0x00020000);
        const int rowstep = 2 * d * 4;
        auto voff = [&](int kc) {
            const int dim = 32 * kc + col;
            return dim < d ? (h * d + dim) * 4 : (1 << 30);
        };
        float pf[32];
        auto load_x = [&](int kc) {
            const int vo = voff(kc);
#pragma unroll
            for (int i = 0; i < 32; ++i)
                pf[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_in, vo, i * rowstep, 0));
        };
        float xmax = 0.f;
        auto put_x = [&](bool track) {
#pragma unroll
            for (int i = 0; i < 32; ++i) {
                xt[(2 * i + h) * kStageStride + col] = pf[i];
                if (track) xmax = tmax(xmax, fabsf(pf[i]));
            }
        };

        // ---- layer 1: 32-input slices, W1 slice kc staged in buffer kc & 1 ----
        __syncthreads();  // previous iteration's readers of the staging buffers are done
        load_x(0);
        {
            // stage slice 0: the HT tiles' 1024-float slices are strided by 4*NKC*256 floats
            f32x4* dst = reinterpret_cast<f32x4*>(lds + S.wb);
            for (int e = threadIdx.x; e < n4w1; e += NT) {
                const int ht = e >> 8, q = e & 255;
                dst[e] = reinterpret_cast<const f32x4*>(packed + L.w1 + (ht * 4 * NKC) * 256)[q];
            }
        }
        __syncthreads();

        f32x16 h1[HT][2];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) load_bias16_x2(B1 + ht * 32, h, h1[ht][0], h1[ht][1]);

        int kc = 0;
        auto l1_step = [&](auto seg) {
            constexpr int SEG = decltype(seg)::value;
            const float* wbk = lds + S.wb + (kc & 1) * S.wbuf;
            put_x(true);
            wave_lds_sync();
            // prefetch the next slice: x rows (registers) and the W1 slice (registers -> LDS)
            constexpr int NQ1 = (2 * 256 + NT - 1) / NT;  // float4s per thread of a W1 slice (HT <= 2)
            f32x4 wn[NQ1];
#pragma unroll
            for (int qq = 0; qq < NQ1; ++qq) wn[qq] = f32x4{0.f, 0.f, 0.f, 0.f};
            const bool more = kc + 1 < NKC;
            if (more) {
                load_x(kc + 1);
#pragma unroll
                for (int qq = 0; qq < NQ1; ++qq) {
                    const int e = threadIdx.x + qq * NT;
                    if (e < n4w1) {
                        const int ht = e >> 8, q = e & 255;
                        wn[qq] = reinterpret_cast<const f32x4*>(packed + L.w1 + (ht * 4 * NKC + (kc + 1) * 4) * 256)[q];
                    }
                }
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                f32x4 w[HT];
#pragma unroll
                for (int ht = SEG; ht < HT; ++ht)
                    w[ht] = *reinterpret_cast<const f32x4*>(wbk + (ht * 4 + g) * 256 + lane * 4);
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int k = 8 * g + 2 * rr + h;
                    const float b0 = xt[col * kStageStride + k];
                    const float b1 = xt[(32 + col) * kStageStride + k];
#pragma unroll
                    for (int ht = SEG; ht < HT; ++ht) {
                        h1[ht][0] = mfma32(w[ht][rr], b0, h1[ht][0]);
                        h1[ht][1] = mfma32(w[ht][rr], b1, h1[ht][1]);
                    }
                }
            }
            wave_lds_sync();
            if (more) {
#pragma unroll
                for (int qq = 0; qq < NQ1; ++qq) {
                    const int e = threadIdx.x + qq * NT;
                    if (e < n4w1) reinterpret_cast<f32x4*>(lds + S.wb + ((kc + 1) & 1) * S.wbuf)[e] = wn[qq];
                }
            }
            __syncthreads();
            ++kc;
        };
        for (; kc < E[0];) l1_step(std::integral_constant<int, 0>{});
        if constexpr (HT > 1) {
            for (; kc < E[1];) l1_step(std::integral_constant<int, 1>{});
        }
        const bool dense = __builtin_amdgcn_ballot_w64(!(xmax <= tsafe)) != 0;
        if constexpr (HT > 1) {
            if (dense && E[0] < NKC) {
                // rare: non-finite or huge inputs -> add the skipped (all-zero) blocks of tile 0 so
                // 0*inf contaminates exactly as the reference's dense product does
                for (int k2 = E[0]; k2 < NKC; ++k2) {
                    load_x(k2);
                    put_x(false);
                    wave_lds_sync();
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const f32x4 w = *reinterpret_cast<const f32x4*>(packed + L.w1 + ((k2 * 4 + g) * 64 + lane) * 4);
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) {
                            const int k = 8 * g + 2 * rr + h;
                            h1[0][0] = mfma32(w[rr], xt[col * kStageStride + k], h1[0][0]);
                            h1[0][1] = mfma32(w[rr], xt[(32 + col) * kStageStride + k], h1[0][1]);
                        }
                    }
                    wave_lds_sync();
                }
            }
        }
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                h1[ht][0][r] = trelu(h1[ht][0][r]);
                h1[ht][1][r] = trelu(h1[ht][1][r]);
            }
        }

        // ---- layers 2, 3 (LDS-resident weights) ----
        f32x16 h2[HT][2];
        if (dense || full2) {
            made_hidden<HT>(W23, L.w2, L.b2, h1, h2);
        } else {
#pragma unroll
            for (int hto = 0; hto < HT; ++hto) hidden_tile2_n<HT, HT>(nk2[hto], W23, L.w2, L.b2, hto, h1, h2[hto][0], h2[hto][1]);
        }
        if (dense || full3) {
            made_hidden<HT>(W23, L.w3, L.b3, h2, h1);
        } else {
#pragma unroll
            for (int hto = 0; hto < HT; ++hto) hidden_tile2_n<HT, HT>(nk3[hto], W23, L.w3, L.b3, hto, h2, h1[hto][0], h1[hto][1]);
        }

        // ---- layer 4 in (mu, alpha) block pairs + affine epilogue ----
        {
            f32x4* dst = reinterpret_cast<f32x4*>(lds + S.wb);
            const f32x4* src = reinterpret_cast<const f32x4*>(packed + L.w4);
            for (int e = threadIdx.x; e < n4w4; e += NT) dst[e] = src[e];
        }
        __syncthreads();
        float acc0 = 0.f, acc1 = 0.f, zsq = 0.f;
        for (int j = 0; j < NJ; ++j) {
            const float* wbj = lds + S.wb + (j & 1) * S.wbuf;
            load_x(j);  // x slice j for the epilogue, in flight during the MFMAs
            WideStage<NT> nx;
            const bool more = j + 1 < NJ;
            if (more) wide_fetch(packed + L.w4 + (j + 1) * 2 * HT * 1024, n4w4, nx);
            f32x16 mu0, mu1, al0, al1;
            out_pair2_n<HT, HT>(dense ? HT : nkp[L.nk4 + j], wbj, B4, j, h1, mu0, mu1, al0, al1);
            put_x(false);
            wave_lds_sync();
            // rows past d: zero weights and bias (alpha = 0 adds nothing to the log-det) and a
            // zero x column; their z lands in the tile padding and is never stored
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = crow(r, h);
                float* p0 = xt + col * kStageStride + row;
                float* p1 = xt + (32 + col) * kStageStride + row;
                *p0 = made_affine<VAR>(*p0, mu0[r], al0[r], acc0);
                *p1 = made_affine<VAR>(*p1, mu1[r], al1[r], acc1);
            }
            wave_lds_sync();
            {
                const int vo = voff(j);
#pragma unroll
                for (int i = 0; i < 32; ++i)
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xt[(2 * i + h) * kStageStride + col]), rs_out,
                                                          vo, i * rowstep, 0);
            }
            if constexpr (LOGP) {
                // sum z^2 of sample `lane` in dimension order (as nfx_gauss_logprob does)
                const int n = d - 32 * j < 32 ? d - 32 * j : 32;
                for (int dd = 0; dd < n; ++dd) {
                    const float v = xt[lane * kStageStride + dd];
                    zsq = (j == 0 && dd == 0) ? gauss_sq0(v) : gauss_sq(zsq, v);
                }
            }
            wave_lds_sync();
            if (more) wide_store(lds + S.wb + ((j + 1) & 1) * S.wbuf, n4w4, nx);
            __syncthreads();
        }
        // per-sample alpha sum: lane l <-> sample base + l
        const float s = halves_sum(acc0, acc1);
        const int64_t so = base + lane;
        if (lane < rows) {
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
            const float ldt = accumulate ? logdet[so] + ld : ld;
            logdet[so] = ldt;
            if constexpr (LOGP) {
                const float lp = gauss_lp(zsq, cgauss, ldt);
                logp[so] = lp;
                lpacc += (double)lp;
            }
        }
    }
    if constexpr (LOGP) {
        logp_commit<NT>(lpacc, partials, sums, B);
    }
}

template <int HT>
made_par_kernel_t made_wide_pick_ht(int variant, bool logp, int nw);

}  // namespace nfx
