// A whole chain of affine coupling layers in ONE launch at LARGE batches (the streaming layout):
// the cfg2 log_prob (RealNVP(2, 8, 64), normalizing_flow_model.py:48-65 over
// coupling_layer.py:70-96) at the full 1M batch and at its strong-scaled per-GPU shards.
//
// Per layer the arithmetic is affine_coupling_kernel's (nfx_affine_kernel.h: a wave owns
// 64-sample chunks, both conditioner nets on fp32 MFMA, the output layer on VALU with the
// half-wave combine, the same epilogue roundings), so the chain equals the per-layer streaming
// launches bit for bit. What changes is what happens BETWEEN layers. A per-layer launch pays,
// every layer: the dispatch ramp of its workgroups, the copy of the layer's weight image into
// each workgroup's LDS, the HBM latency of its first rows and the tail of its last wave — about
// 5 us per layer at a 125k-sample shard (22.3 us per layer vs 17.4 us of MFMA + VALU work). Here
// one workgroup per CU carries a slice of rows and their running log-det in LDS through ALL
// layers; the next layer's weight image is copied into the second half of a double buffer by
// LDS-DMA while the current layer computes, and one barrier per layer hands it over. HBM
// traffic is the rows in and out once per chain (8d + 8 bytes per sample for the whole chain).
//
// Work split: workgroup b owns chunks [b*C/G, (b+1)*C/G) of the C 64-sample chunks, processed in
// slices that fit its LDS; within a slice wave w takes chunks w, w+NW, ... and leftover chunks
// go out as 32-sample half chunks when that balances the SIMDs better (as the per-layer kernel).
// A sample is always processed by the same lane of the same wave, so layer l+1 reads only what
// that lane wrote in layer l: the per-layer barrier is needed for the weight buffer alone.
#include "nfx_chain.h"

namespace nfx {

// Staged image per layer: the split tail (affine_split; H <= 64 always has one here), padded to
// a multiple of one 1-KiB DMA piece.
template <int HT, int D>
__host__ __device__ constexpr int schain_wpad() {
    return (affine_split(D, HT).total + 255) & ~255;  // floats
}

template <int HT, int D, int DIR, bool LOGP, int NW>
__global__ __launch_bounds__(64 * NW) void affine_schain_kernel(
    NfxChainPacks packs, int nl, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int accumulate, int64_t nchunks, int slice_chunks,
    float* __restrict__ logp, double* __restrict__ partials, double* __restrict__ sums, float cgauss) {
    constexpr AffineLayout L = affine_layout(D, HT);
    constexpr AffineSplit SL = affine_split(D, HT);
    static_assert(affine_has_split(D, HT), "the streaming chain runs the split nets");
    constexpr int KS1 = L.KS1;
    constexpr int WPAD = schain_wpad<HT, D>();
    constexpr int NT = 64 * NW;
    extern __shared__ f32x4 lds4[];
    float* wbuf = reinterpret_cast<float*>(lds4);  // [2][WPAD] weight images
    float* sx = wbuf + 2 * WPAD;                    // [slice_chunks * 64][D] rows
    float* sld = sx + (size_t)slice_chunks * 64 * D;  // [slice_chunks * 64] running log-det

    const uint32_t wbuf_lds = lds_addr_of(lds4);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    const int64_t c0 = nchunks * blockIdx.x / gridDim.x, c1 = nchunks * (blockIdx.x + 1) / gridDim.x;

    // DMA layer li's packed image (module order reversed for an inverse chain) into buffer buf.
    auto stage = [&](int li, int buf) {
        const float* src = packs.p[DIR > 0 ? li : nl - 1 - li] + L.s;
        for (int c = wave; c < WPAD / 256; c += NW) {
            int idx = c * 256 + lane * 4;
            if (idx > SL.total - 4) idx = SL.total - 4;  // tail lanes re-read the last float4 into padding
            lds_dma_x4(src + idx, wbuf_lds + (uint32_t)(buf * WPAD + c * 256) * 4u);
        }
    };

    double lpacc = 0.0;
    int g = 0;  // layers run so far by this workgroup: weight buffer g & 1
    if (c0 < c1) stage(0, 0);
    for (int64_t s0 = c0; s0 < c1; s0 += slice_chunks) {
        const int64_t s1 = s0 + slice_chunks < c1 ? s0 + slice_chunks : c1;
        const int64_t r0 = s0 * 64;
        const int rows = (int)((B < s1 * 64 ? B : s1 * 64) - r0);
        for (int e = threadIdx.x; e < rows * D; e += NT) sx[e] = in[r0 * D + e];
        for (int e = threadIdx.x; e < rows; e += NT) sld[e] = accumulate ? logdet[r0 + e] : 0.f;
        const int nch = (int)(s1 - s0);
        const int F = nch / NW, R = nch - F * NW;
        const bool split = 2 * R <= NW;
        const int nfull = split ? F : F + (wave < R ? 1 : 0);
        const bool half = split && wave < 2 * R;
        const int half_base = F * NW * 64 + wave * 32;

        for (int li = 0; li < nl; ++li) {
            lds_dma_wait();   // this wave's DMA pieces (and the slice loads) have landed
            __syncthreads();  // every wave's pieces landed; every wave is done with the other buffer
            if (li + 1 < nl)
                stage(li + 1, (g + 1) & 1);
            else if (s0 + slice_chunks < c1)
                stage(0, (g + 1) & 1);
            const float* W = wbuf + (g & 1) * WPAD;
            const float* Pg = packs.p[DIR > 0 ? li : nl - 1 - li];  // fp32 image: fallback tiles
            const bool first = li == 0 && !accumulate;
            float mk[D], mkb[KS1];
#pragma unroll
            for (int j = 0; j < D; ++j) mk[j] = W[SL.mask + j];
#pragma unroll
            for (int ks = 0; ks < KS1; ++ks) mkb[ks] = (2 * ks + h < D) ? W[SL.mask + 2 * ks + h] : 0.f;

            auto unit = [&](auto tiles_c, int ub) {
                constexpr int TILES = decltype(tiles_c)::value;
                const int so = ub + lane;  // slice-local sample of this lane
                const bool act = lane < 32 * TILES && so < rows;
                float xr[D];
                if (act) {
                    load_row<D>(sx + so * D, xr);
                } else {
#pragma unroll
                    for (int j = 0; j < D; ++j) xr[j] = 0.f;
                }
                float xb[2][KS1];
                if constexpr (D == 2) {
                    // lanes 0..31 hold samples ub+col, lanes 32..63 ub+32+col; operand (st, k = h)
                    // of lane (col, h) is x[ub+32st+col][h]: one half-wave swap of the row
                    const float other = halves_other(xr[0], xr[1]);
                    xb[0][0] = (h ? other : xr[0]) * mkb[0];
                    xb[1][0] = (h ? xr[1] : other) * mkb[0];
                } else {
#pragma unroll
                    for (int st = 0; st < 2; ++st) {
                        const int s = ub + 32 * st + col;
#pragma unroll
                        for (int ks = 0; ks < KS1; ++ks) {
                            const int k = 2 * ks + h;
                            xb[st][ks] = (32 * st + col < 32 * TILES && s < rows && k < D) ? sx[s * D + k] * mkb[ks] : 0.f;
                        }
                    }
                }
                const float* Wi = W + opaque_zero();
                float sv[D], bv[D];
                affine_nets_split<HT, D, TILES>(Wi, SL, Pg, L, xb, sv, bv);
                if (act) {
#pragma clang fp contract(off)  // separate mul/add roundings, as affine_coupling_kernel / the reference
                    float y[D];
                    float ld = 0.f;
#pragma unroll
                    for (int j = 0; j < D; ++j) {
                        const float m = mk[j], om = 1.f - m;
                        const float xa = xr[j] * m;
                        float t;
                        if constexpr (DIR < 0) {
                            t = (xr[j] - bv[j]) * exp_fast(-sv[j]);
                            ld = ld + om * (-sv[j]);
                        } else {
                            t = xr[j] * exp_fast(sv[j]) + bv[j];
                            ld = ld + om * sv[j];
                        }
                        const float v = xa + om * t;
                        y[j] = nonfinite(v) ? 0.f : v;
                    }
                    if (nonfinite(ld)) ld = 0.f;
                    store_row<D>(sx + so * D, y);
                    sld[so] = first ? ld : sld[so] + ld;
                }
            };
            for (int u = 0; u < nfull; ++u) unit(std::integral_constant<int, 2>{}, (wave + u * NW) * 64);
            if (half) unit(std::integral_constant<int, 1>{}, half_base);
            ++g;
        }
        __syncthreads();  // rows of every wave final
        for (int e = threadIdx.x; e < rows * D; e += NT) out[r0 * D + e] = sx[e];
        for (int e = threadIdx.x; e < rows; e += NT) {
            const float ldt = sld[e];
            logdet[r0 + e] = ldt;
            if constexpr (LOGP) {
                const float* rw = sx + (size_t)e * D;
                float m = gauss_sq0(rw[0]);
#pragma unroll
                for (int j = 1; j < D; ++j) m = gauss_sq(m, rw[j]);
                const float lp = gauss_lp(m, cgauss, ldt);
                logp[r0 + e] = lp;
                lpacc += (double)lp;
            }
        }
        __syncthreads();  // the next slice overwrites the rows
    }
    if constexpr (LOGP) {
        logp_commit<NT>(lpacc, partials, sums, B);
    }
}

typedef void (*schain_t)(NfxChainPacks, int, const float*, float*, float*, int64_t, int, int64_t, int, float*,
                         double*, double*, float);

// Waves per workgroup: one workgroup per CU (its LDS holds two weight images + the row slice),
// 3 waves per SIMD as the per-layer kernel runs (<= 168 VGPRs).
constexpr int kSchainWaves = 12;

template <int HT, int D>
static schain_t schain_pick_d(int dir, bool logp) {
    if (dir > 0) return affine_schain_kernel<HT, D, 1, false, kSchainWaves>;
    return logp ? affine_schain_kernel<HT, D, -1, true, kSchainWaves> : affine_schain_kernel<HT, D, -1, false, kSchainWaves>;
}

static schain_t schain_pick(int HT, int D, int dir, bool logp) {
    if (HT == 1) return D == 2 ? schain_pick_d<1, 2>(dir, logp) : D == 4 ? schain_pick_d<1, 4>(dir, logp) : schain_pick_d<1, 8>(dir, logp);
    if (HT == 2) return D == 2 ? schain_pick_d<2, 2>(dir, logp) : D == 4 ? schain_pick_d<2, 4>(dir, logp) : schain_pick_d<2, 8>(dir, logp);
    return nullptr;
}

static int schain_wpad_rt(int HT, int D) {
    return (affine_split(D, HT).total + 255) & ~255;
}

constexpr size_t kSchainLds = 160 * 1024;   // gfx950 LDS per CU
constexpr size_t kSchainStatic = 1024;      // block_sum_f64's static LDS, rounded up

// Chunks of rows one workgroup can hold next to the two weight images (0: does not fit).
static int64_t schain_slice_cap(int HT, int D) {
    const size_t w = 2 * (size_t)schain_wpad_rt(HT, D) * sizeof(float);
    if (w + kSchainStatic >= kSchainLds) return 0;
    return (int64_t)((kSchainLds - kSchainStatic - w) / (64 * (D + 1) * sizeof(float)));
}

bool schain_supported(int64_t B, int d, int H) {
    (void)B;
    const int HT = (H + 31) / 32;
    return (d == 2 || d == 4 || d == 8) && HT >= 1 && HT <= 2 && schain_slice_cap(HT, d) >= 1;
}

int schain_launch(const NfxChainPacks& P, int nl, const float* in, float* out, float* log_det, int64_t B, int d,
                  int H, int direction, int accumulate, float* logp, double* sums, void* workspace, hipStream_t s) {
    const bool fused = sums != nullptr;
    const int HT = (H + 31) / 32;
    if (!schain_supported(B, d, H))
        return set_error(NFX_EUNSUPPORTED, "affine_chain (streaming): d=%d H=%d outside d in {2,4,8}, H <= 64", d, H);
    schain_t k = schain_pick(HT, d, direction, fused);
    const int64_t nchunks = (B + 63) / 64;
    int64_t grid = num_cus();
    if (grid > nchunks) grid = nchunks;
    if (grid > kMaxPartials) grid = kMaxPartials;
    const int64_t per_wg = (nchunks + grid - 1) / grid;
    const int64_t cap = schain_slice_cap(HT, d);
    const int64_t nslices = (per_wg + cap - 1) / cap;
    const int64_t slice = (per_wg + nslices - 1) / nslices;  // equal slices
    const size_t lds = (2 * (size_t)schain_wpad_rt(HT, d) + (size_t)slice * 64 * (d + 1)) * sizeof(float);
    int rc = prepare_lds((const void*)k, lds);
    if (rc) return rc;
    k<<<(unsigned)grid, 64 * kSchainWaves, lds, s>>>(P, nl, in, out, log_det, B, accumulate, nchunks, (int)slice,
                                                      logp, reinterpret_cast<double*>(workspace), sums,
                                                      gauss_const(d));
    return check_launch("affine_schain_kernel");
}

}  // namespace nfx
