// A whole chain of RQ-spline coupling layers (d = 2) in ONE launch: the cfg3 log_prob (8x
// SplineCouplingLayer(2, 64, K=8), normalizing_flow_model.py:48-65 over
// spline_coupling_layer.py:139-180) and RealNVPSpline, at large batches and strong-scaled shards.
//
// The affine streaming chain's structure (nfx_affine_schain.hip) around spline_coupling_kernel's
// arithmetic (spline_unit_apply: the same operations in the same order, so the chain equals the
// per-layer launches bit for bit): one workgroup per CU carries a slice of rows and their running
// log-det in LDS through every layer; the next layer's packed image is DMA'd into the other half
// of an LDS double buffer while the current layer runs; one barrier per layer.
#pragma once
#include "nfx_chain.h"
#include "nfx_spline_kernel.h"

namespace nfx {

template <int HT>
__host__ __device__ constexpr int spline_schain_wpad() {
    return (spline_layout(HT, 2).total + 255) & ~255;  // floats; a multiple of one 1-KiB DMA piece
}

template <int HT, int K, int DIR, bool LOGP, int NW>
__global__ __launch_bounds__(64 * NW) void spline_schain_kernel(
    NfxChainPacks packs, int nl, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, SplineConsts C, int accumulate, int64_t nchunks, int slice_chunks,
    float* __restrict__ logp, double* __restrict__ partials, double* __restrict__ sums, float cgauss,
    uint64_t seed, uint64_t* rng, float* __restrict__ zout) {
#pragma clang fp contract(off)
    constexpr int D = 2;
    constexpr SplineLayout L = spline_layout(HT, D);
    constexpr int WPAD = spline_schain_wpad<HT>();
    constexpr int NTH = 64 * NW;
    extern __shared__ f32x4 lds4[];
    float* wbuf = reinterpret_cast<float*>(lds4);     // [2][WPAD] weight images
    float* sx = wbuf + 2 * WPAD;                       // [slice_chunks * 64][2] rows
    float* sld = sx + (size_t)slice_chunks * 64 * D;   // [slice_chunks * 64] running log-det

    const uint32_t wbuf_lds = lds_addr_of(lds4);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = lane_id(), h = lane >> 5;
    const int64_t c0 = nchunks * blockIdx.x / gridDim.x, c1 = nchunks * (blockIdx.x + 1) / gridDim.x;

    auto stage = [&](int li, int buf) {
        const float* src = packs.p[DIR > 0 ? li : nl - 1 - li];
        for (int c = wave; c < WPAD / 256; c += NW) {
            int idx = c * 256 + lane * 4;
            if (idx > L.total - 4) idx = L.total - 4;  // tail lanes re-read the last float4 into padding
            lds_dma_x4(src + idx, wbuf_lds + (uint32_t)(buf * WPAD + c * 256) * 4u);
        }
    };

#ifdef NFX_SCHAIN_TIMING
    // timing build only (tools/schain_timing.py): workgroup 0's waves 0 and 4 accumulate clock64
    // ticks per stage
    long long tacc[6] = {0, 0, 0, 0, 0, 0};
    long long tmark = clock64();
#define NFX_CMARK(k) do { const long long t_ = clock64(); tacc[k] += t_ - tmark; tmark = t_; } while (0)
#else
#define NFX_CMARK(k) do { } while (0)
#endif
    double lpacc = 0.0;
    int g = 0;  // layers run so far by this workgroup: weight buffer g & 1
    if (c0 < c1) stage(0, 0);
    for (int64_t s0 = c0; s0 < c1; s0 += slice_chunks) {
        const int64_t s1 = s0 + slice_chunks < c1 ? s0 + slice_chunks : c1;
        const int64_t r0 = s0 * 64;
        const int rows = (int)((B < s1 * 64 ? B : s1 * 64) - r0);
        if (rng) {  // the fused sampling pass: z ~ N(0, I) drawn here (base_draw, nfx_chain.h)
            const uint64_t off = __hip_atomic_load(rng, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (int e = threadIdx.x; e < rows; e += NTH) {
                float z[D];
                base_draw<D>(r0 + e, seed, off, z);
                sx[e * D] = z[0];
                sx[e * D + 1] = z[1];
                if (zout) {
                    zout[(r0 + e) * D] = z[0];
                    zout[(r0 + e) * D + 1] = z[1];
                }
            }
        } else {
            for (int e = threadIdx.x; e < rows * D; e += NTH) sx[e] = in[r0 * D + e];
        }
        for (int e = threadIdx.x; e < rows; e += NTH) sld[e] = accumulate ? logdet[r0 + e] : 0.f;
        const int nch = (int)(s1 - s0);
        const int F = nch / NW, R = nch - F * NW;
        const bool split = 2 * R <= NW;
        const int nfull = split ? F : F + (wave < R ? 1 : 0);
        const bool half = split && wave < 2 * R;
        const int half_base = F * NW * 64 + wave * 32;

        NFX_CMARK(4);  // slice prologue
        for (int li = 0; li < nl; ++li) {
            NFX_CMARK(3);  // layer start + row io
            lds_dma_wait();
            __syncthreads();
            NFX_CMARK(0);  // barrier
            if (li + 1 < nl)
                stage(li + 1, (g + 1) & 1);
            else if (s0 + slice_chunks < c1)
                stage(0, (g + 1) & 1);
            const float* W = wbuf + (g & 1) * WPAD;
            const bool first = li == 0 && !accumulate;
            const int NT = (int)W[L.meta];
            const float mkb = h < D ? W[L.mask + h] : 0.f;

            auto unit = [&](auto tiles_c, int ub) {
                constexpr int TILES = decltype(tiles_c)::value;
                const int so = ub + lane;
                const bool act = lane < 32 * TILES && so < rows;
                float xr[D];
                if (act) {
                    const f32x2 v = *reinterpret_cast<const f32x2*>(sx + so * D);
                    xr[0] = v.x;
                    xr[1] = v.y;
                } else {
                    xr[0] = xr[1] = 0.f;
                }
                // layer-1 operands as spline_coupling_kernel<DS = 2>: one half-wave row swap
                float xb[2][4];
                {
                    const float other = halves_other(xr[0], xr[1]);
                    float xraw[2] = {h ? other : xr[0], h ? xr[1] : other};
#pragma unroll
                    for (int st = 0; st < 2; ++st) {
                        float xv = xraw[st];
                        if (C.rescale) xv = C.rs_to_scale * (xv - C.rs_lo) - C.bound;
                        xb[st][0] = xv * mkb;
                        xb[st][1] = xb[st][2] = xb[st][3] = 0.f;  // k-steps >= KS1 = 1 are not issued
                    }
                }
                float y[D];
                float ld;
#ifdef NFX_SCHAIN_TIMING
                {
                    const float* Wz = W + opaque_zero();
                    f32x16 h2[HT][2];
                    spline_unit_hidden<HT, TILES>(Wz, L, 1, xb, h2);
                    float prm[32];
                    spline_unit_params<HT, TILES>(Wz, L, h2, 0, prm);
                    NFX_CMARK(1);  // MFMA part (one transformed dim)
#pragma unroll
                    for (int j = 0; j < D; ++j) y[j] = xr[j];
                    ld = 0.f;
                    spline_unit_dim<K, DIR, D>(C, (int)Wz[L.tdim], 0, prm, xr, y, ld);
                    NFX_CMARK(2);  // spline
                }
#else
                if constexpr (NW > 8 && HT > 1)  // (the 168-VGPR budget: one tile's activations at a time)
                    spline_unit_apply_tseq<HT, K, DIR, D, TILES>(W + opaque_zero(), L, C, 1, NT, xb, xr, y, ld);
                else
                    spline_unit_apply<HT, K, DIR, D, TILES>(W + opaque_zero(), L, C, 1, NT, xb, xr, y, ld);
#endif
                if (act) {
                    float yo[D];
#pragma unroll
                    for (int j = 0; j < D; ++j) yo[j] = nonfinite(y[j]) ? 0.f : y[j];
                    *reinterpret_cast<f32x2*>(sx + so * D) = f32x2{yo[0], yo[1]};
                    if (nonfinite(ld)) ld = 0.f;
                    sld[so] = first ? ld : sld[so] + ld;
                }
            };
            for (int u = 0; u < nfull; ++u) unit(std::integral_constant<int, 2>{}, (wave + u * NW) * 64);
            if (half) unit(std::integral_constant<int, 1>{}, half_base);
            ++g;
        }
        NFX_CMARK(3);
        __syncthreads();
        for (int e = threadIdx.x; e < rows * D; e += NTH) out[r0 * D + e] = sx[e];
        for (int e = threadIdx.x; e < rows; e += NTH) {
            const float ldt = sld[e];
            logdet[r0 + e] = ldt;
            if constexpr (LOGP) {
                const float* rw = sx + (size_t)e * D;
                const float m = gauss_sq(gauss_sq0(rw[0]), rw[1]);
                const float lp = gauss_lp(m, cgauss, ldt);
                logp[r0 + e] = lp;
                lpacc += (double)lp;
            }
        }
        __syncthreads();
    }
    NFX_CMARK(5);  // slice epilogue
#ifdef NFX_SCHAIN_TIMING
    if (blockIdx.x == 0 && lane == 0 && (wave == 0 || wave == 4))
        for (int k = 0; k < 6; ++k) out[(wave ? 6 : 0) + k] = (float)tacc[k];
#endif
    if constexpr (LOGP) {
        logp_commit<NTH>(lpacc, partials, sums, B);
    }
    if (rng) {  // every workgroup read rng[0] in its slices; the last one to get here moves it on
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            uint64_t* cnt = rng + 1;
            const uint64_t prev = __hip_atomic_fetch_add(cnt, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (prev == (uint64_t)gridDim.x - 1) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                __hip_atomic_store(rng, __hip_atomic_load(rng, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(cnt, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

typedef void (*spline_schain_t)(NfxChainPacks, int, const float*, float*, float*, int64_t, SplineConsts, int, int64_t,
                                int, float*, double*, double*, float, uint64_t, uint64_t*, float*);

constexpr int kSplineSchainWaves = 12;
// Strong-scaled shards (at most one 64-row unit per wave and layer): 8 waves, two per SIMD, which
// leaves the unit body 256 VGPRs instead of 168 (no scratch spills); the twelve-wave kernel would
// leave a third of its waves idle there anyway.
constexpr int kSplineSchainWavesSmall = 8;

template <int HT>
spline_schain_t spline_schain_pick_ht(int K, int dir, bool logp, bool small);

}  // namespace nfx
