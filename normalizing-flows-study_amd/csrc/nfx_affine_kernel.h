// Affine-coupling kernel template (see nfx_affine.hip for the design notes).
#pragma once
#include <type_traits>

#include "nfx_common.h"

namespace nfx {

__host__ __device__ constexpr int up4(int v) { return (v + 3) & ~3; }

// Packed weight image (floats). Per net (s_net = 0, b_net = 1):
//   w1 [HT][KS1][64]        A operand of layer 1 (BN folded)
//   b1 [HT][2][16]          bias of layer 1 at accumulator register r of half h (BN folded)
//   w2 [HT][HT][4][64][4]   A operand of layer 2: [out tile][k tile][r/4][lane][r%4]
//   b2 [HT][2][16]
//   w3 [d][HT][2][16]       output layer, by (j, k tile, half, r) for the VALU dot    (d <= 8)
//   b3 [up4(d)]
//   w3 [NJ][HT][4][64][4]   output layer as MFMA A-operand tiles, NJ = ceil(d/32)     (d > 8)
//   b3 [NJ][2][16]          its bias in accumulator order
// then mask [up4(d)].
struct AffineLayout {
    int d, HT, KS1;
    int w1, b1, w2, b2, w3, b3, net, mask, total;
    int s;  // base of the split tail (affine_split), == the fp32 image's end
};

// Split tail (d <= 8, H <= 64), appended to the image and derived from it on device
// (nfx_affine_split_pack): what affine_net_split reads, contiguous so that a kernel stages only
// this region into LDS. Per net: w1 b1 b2 w3 b3 (copies, the fp32 formats above) and W2 as three
// bf16 pieces W2 ~ W2_0 + W2_1 + W2_2 (round-to-nearest split, split_block) in v_mfma_f32_32x32x16_bf16
// A-operand order [out tile][k block][piece][lane][4 dwords]; then the mask and two safety words:
// ok[0] = 1 when every W2 entry is finite with |w| <= 1e6, ok[1] = xsafe, the largest |x * m|
// for which every layer-1 activation stays <= 1e30 (so no bf16 piece product or layer-2 partial
// sum can overflow).
struct AffineSplit {
    int w1, b1, b2, w3, b3, w2s, net, mask, ok, total;
};

__host__ __device__ constexpr AffineSplit affine_split(int d, int HT) {
    AffineSplit S{};
    int o = 0;
    S.w1 = o; o += HT * ((d + 1) / 2) * 64;
    S.b1 = o; o += HT * 32;
    S.b2 = o; o += HT * 32;
    S.w3 = o; o += d * HT * 32;
    S.b3 = o; o += up4(d);
    S.w2s = o; o += HT * 2 * HT * 768;
    S.net = o;
    S.mask = 2 * o;
    S.ok = S.mask + up4(d);
    S.total = S.ok + 4;
    return S;
}

__host__ __device__ constexpr bool affine_has_split(int d, int HT) { return d <= 8 && HT <= 2; }

__host__ __device__ constexpr AffineLayout affine_layout(int d, int HT) {
    AffineLayout L{};
    L.d = d;
    L.HT = HT;
    L.KS1 = (d + 1) / 2;
    int o = 0;
    L.w1 = o; o += HT * L.KS1 * 64;
    L.b1 = o; o += HT * 32;
    L.w2 = o; o += HT * HT * 16 * 64;
    L.b2 = o; o += HT * 32;
    if (d <= 8) {  // VALU output layer (affine_coupling_kernel)
        L.w3 = o; o += d * HT * 32;
        L.b3 = o; o += up4(d);
    } else {       // MFMA output layer (affine_wide_kernel): A-operand tiles + accumulator-order bias
        const int NJ = (d + 31) / 32;
        L.w3 = o; o += NJ * HT * 1024;
        L.b3 = o; o += NJ * 32;
    }
    L.net = o;
    L.mask = 2 * o;
    L.total = 2 * o + up4(d);
    L.s = L.total;
    if (affine_has_split(d, HT)) L.total += affine_split(d, HT).total;
    return L;
}

template <int D>
__device__ __forceinline__ void load_row(const float* __restrict__ p, float (&v)[D]) {
    if constexpr (D == 2) {
        float2 t = *reinterpret_cast<const float2*>(p);
        v[0] = t.x; v[1] = t.y;
    } else if constexpr (D == 4) {
        float4 t = *reinterpret_cast<const float4*>(p);
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else {
#pragma unroll
        for (int j = 0; j < D; ++j) v[j] = p[j];
    }
}

template <int D>
__device__ __forceinline__ void store_row(float* __restrict__ p, const float (&v)[D]) {
    if constexpr (D == 2) {
        *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
    } else if constexpr (D == 4) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
        for (int j = 0; j < D; ++j) p[j] = v[j];
    }
}

// Conditioner MLP of one net for a 64-sample chunk; returns clamp(net(x*m), -10, 10)[j] for the
// lane's own sample (lane l <-> sample chunk*64 + l). TILES = 1: a 32-sample half chunk (sample
// tile 1 is skipped; lanes 32..63 return unused values).
template <int HT, int D, int TILES = 2>
__device__ __forceinline__ void affine_net(const float* __restrict__ P, const AffineLayout& L,
                                           const float (&xb)[2][(D + 1) / 2], float (&res)[D]) {
    constexpr int KS1 = (D + 1) / 2;
    const int lane = lane_id(), h = lane >> 5;

    // Layer 1: [H x d] * [d x 32] per sample tile, bias-initialised accumulators, ReLU.
    f32x16 h1[HT][2];
#pragma unroll
    for (int ht = 0; ht < HT; ++ht) {
        f32x16 a0, a1;
        load_bias16_x2(P + L.b1 + ht * 32, h, a0, a1);
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks) {
            const float w = P[L.w1 + (ht * KS1 + ks) * 64 + lane];
            a0 = mfma32(w, xb[0][ks], a0);
            if constexpr (TILES == 2) a1 = mfma32(w, xb[1][ks], a1);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            a0[r] = trelu(a0[r]);
            if constexpr (TILES == 2) a1[r] = trelu(a1[r]);
        }
        h1[ht][0] = a0;
        h1[ht][1] = a1;
    }

    // Layer 2 (H x H) tile by tile; each finished tile is ReLU'd and folded into the
    // output-layer partial dot products right away (keeps one tile of h2 live).
    float part[D][2];
#pragma unroll
    for (int j = 0; j < D; ++j) part[j][0] = part[j][1] = 0.f;
    const f32x4* wg = reinterpret_cast<const f32x4*>(P + L.w2) + lane;
#pragma unroll
    for (int hto = 0; hto < HT; ++hto) {
        f32x16 a0, a1;
        load_bias16_x2(P + L.b2 + hto * 32, h, a0, a1);
#pragma unroll
        for (int kt = 0; kt < HT; ++kt) {
#pragma unroll
            for (int rq = 0; rq < 4; ++rq) {
                // (a one-group-ahead weight prefetch here measured 5% slower: the compiler
                // then interleaves both nets at 217 VGPRs = 2 waves/SIMD instead of 3)
                const f32x4 w = wg[((hto * HT + kt) * 4 + rq) * 64];
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    a0 = mfma32(w[rr], h1[kt][0][4 * rq + rr], a0);
                    if constexpr (TILES == 2) a1 = mfma32(w[rr], h1[kt][1][4 * rq + rr], a1);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const f32x16 w3 = load_bias16(P + L.w3 + (j * HT + hto) * 32, h);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                part[j][0] = fmaf(w3[r], trelu(a0[r]), part[j][0]);
                if constexpr (TILES == 2) part[j][1] = fmaf(w3[r], trelu(a1[r]), part[j][1]);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < D; ++j)
        res[j] = tclamp(halves_sum(part[j][0], part[j][1]) + P[L.b3 + j], -10.f, 10.f);
}

// ---- layer 2 as bf16x3-split MFMAs (H <= 64, d <= 8; round 6) ----------------------------------
// fp32 has no fast matrix path on gfx950 (v_mfma_f32_32x32x2_f32 runs at 1/16 of the bf16 rate).
// Layer 2 (H x H, 97 % of the conditioner's flops) instead splits both operands into three bf16
// pieces and sums the six products a_i * w_j with i + j <= 2 on v_mfma_f32_32x32x16_bf16 (fp32
// accumulate; every piece product is exact in fp32). Activations split exactly by truncation
// (a0 = top 8 significant bits, a1 the next 8, a2 the rest: |a1| <= 2^-8 |a|, |a2| <= 2^-16 |a|),
// weights by round-to-nearest at pack time (|w1| <= 2^-9 |w|, |w2| <= 2^-18 |w|, random signs),
// so the dropped a1w2, a2w1, a2w2 are unbiased and below 2^-25 of the term: the layer keeps fp32
// accuracy (not the fp32 chain's bits; all-truncation pieces measured a systematic NLL shift of
// 4e-8, this split 1e-9, profiles/r06_split/). Six 32-cycle
// MFMAs replace the eight 64-cycle fp32 MFMAs of a 16-deep k block, and the splitting VALU issues
// in their shadow. A 32-row sample tile whose masked input fails |x * m| <= xsafe (non-finite or
// huge), or a layer whose W2 is not finite / exceeds 1e6, runs the fp32 chain instead, so
// non-finite rows keep the reference's inf / NaN propagation; the decision is per 32-row tile
// (32-aligned in every kernel), so a row's bits depend only on its own tile.
#ifndef NFX_SPLIT_TERMS
#define NFX_SPLIT_TERMS 6  // piece products per k block (8: + w1 x2, w2 x1)
#endif
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 mfma_bf16(u32x4 a, u32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                    0, 0, 0);
}

// The three pieces (fp32 bit patterns, zero low halves) of a finite activation x, by truncation:
// x0 keeps x's top 8 significant bits, x1 the next 8 of the exact remainder, x2 the rest (exact).
__device__ __forceinline__ void split3(float x, uint32_t& u0, uint32_t& u1, uint32_t& u2) {
    u0 = __float_as_uint(x) & 0xffff0000u;
    const float r1 = x - __uint_as_float(u0);
    u1 = __float_as_uint(r1) & 0xffff0000u;
    u2 = __float_as_uint(r1 - __uint_as_float(u1));
}

// bf16x2 word: element lo in bits 0..15, hi in 16..31 (the high halves of the two patterns).
__device__ __forceinline__ uint32_t pack_bf16(uint32_t lo, uint32_t hi) {
    return __builtin_amdgcn_perm(hi, lo, 0x07060302u);
}

// B-operand pieces of k block kb of an activation tile: the lane's registers 8 (kb & 1) + j,
// j = 0..7 (hidden units 32 (kb >> 1) + crow(8 (kb & 1) + j, h); the pack orders W2's k to match).
__device__ __forceinline__ void split_block(const f32x16& a, int half, u32x4 (&xp)[3]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint32_t l0, l1, l2, h0, h1, h2;
        split3(a[8 * half + 2 * q], l0, l1, l2);
        split3(a[8 * half + 2 * q + 1], h0, h1, h2);
        xp[0][q] = pack_bf16(l0, h0);
        xp[1][q] = pack_bf16(l1, h1);
        xp[2][q] = pack_bf16(l2, h2);
    }
}

// Conditioner MLP of one net on the split tail S (LDS) for a 64-sample chunk (TILES = 2) or a
// 32-sample half chunk. Returns clamp(net(x*m), -10, 10)[j] for the lane's sample, as affine_net.
template <int HT, int D, int TILES = 2>
__device__ __forceinline__ void affine_net_split(const float* __restrict__ S, const AffineSplit& SL,
                                                 const float (&xb)[2][(D + 1) / 2], float (&res)[D]) {
    constexpr int KS1 = (D + 1) / 2;
    const int lane = lane_id(), h = lane >> 5;

    f32x16 h1[HT][2];
#pragma unroll
    for (int ht = 0; ht < HT; ++ht) {
        f32x16 a0, a1;
        load_bias16_x2(S + SL.b1 + ht * 32, h, a0, a1);
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks) {
            const float w = S[SL.w1 + (ht * KS1 + ks) * 64 + lane];
            a0 = mfma32(w, xb[0][ks], a0);
            if constexpr (TILES == 2) a1 = mfma32(w, xb[1][ks], a1);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            a0[r] = trelu(a0[r]);
            if constexpr (TILES == 2) a1[r] = trelu(a1[r]);
        }
        h1[ht][0] = a0;
        h1[ht][1] = a1;
    }

    float part[D][2];
#pragma unroll
    for (int j = 0; j < D; ++j) part[j][0] = part[j][1] = 0.f;
    auto fold = [&](int hto, const f32x16& a, int st) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const f32x16 w3 = load_bias16(S + SL.w3 + (j * HT + hto) * 32, h);
#pragma unroll
            for (int r = 0; r < 16; ++r) part[j][st] = fmaf(w3[r], trelu(a[r]), part[j][st]);
        }
    };
    const u32x4* w2s = reinterpret_cast<const u32x4*>(S + SL.w2s) + lane;
    // sample tile outer: the tile's activations are split once (h1 of the tile dies), then per
    // output tile the k blocks accumulate the big product w0 x0 into hi (bias-initialised) and
    // the small ones into lo, added once at the end: the running sum takes only 2 HT MFMA
    // roundings instead of 6 per k block
#pragma unroll
    for (int st = 0; st < TILES; ++st) {
        u32x4 xp[2 * HT][3];
#pragma unroll
        for (int kb = 0; kb < 2 * HT; ++kb) split_block(h1[kb >> 1][st], kb & 1, xp[kb]);
        const u32x4* w2 = w2s + opaque_zero();  // re-read per tile: no 96-VGPR cache of W2
#pragma unroll
        for (int hto = 0; hto < HT; ++hto) {
            f32x16 hi = load_bias16(S + SL.b2 + hto * 32 + opaque_zero(), h), lo = {};
#pragma unroll
            for (int kb = 0; kb < 2 * HT; ++kb) {
                const int g = (hto * 2 * HT + kb) * 3;
                const u32x4 w[3] = {w2[g * 64], w2[(g + 1) * 64], w2[(g + 2) * 64]};
#if NFX_SPLIT_TERMS == 8
                lo = mfma_bf16(w[2], xp[kb][1], lo);
                lo = mfma_bf16(w[1], xp[kb][2], lo);
#endif
                lo = mfma_bf16(w[2], xp[kb][0], lo);
                lo = mfma_bf16(w[1], xp[kb][1], lo);
                lo = mfma_bf16(w[0], xp[kb][2], lo);
                lo = mfma_bf16(w[1], xp[kb][0], lo);
                lo = mfma_bf16(w[0], xp[kb][1], lo);
                hi = mfma_bf16(w[0], xp[kb][0], hi);
            }
            fold(hto, hi + lo, st);
        }
    }
#pragma unroll
    for (int j = 0; j < D; ++j)
        res[j] = tclamp(halves_sum(part[j][0], part[j][1]) + S[SL.b3 + j], -10.f, 10.f);
}

// Both conditioner nets of a unit: the split nets from the staged tail S, and — only when a
// 32-row sample tile has a masked input beyond xsafe (non-finite or huge; NaN fails the test) or
// the layer's W2 is unsafe — the fp32 nets (affine_net) from the layer's fp32 image Pg in global
// memory, whose results replace the split ones on that tile's lanes (lane l holds sample
// ub + l: tile l >> 5). The choice is per 32-aligned tile, so a row's bits never depend on
// rows outside its tile.
template <int HT, int D, int TILES>
__device__ __forceinline__ void affine_nets_split(const float* __restrict__ S, const AffineSplit& SL,
                                                  const float* __restrict__ Pg, const AffineLayout& L,
                                                  const float (&xb)[2][(D + 1) / 2], float (&sv)[D], float (&bv)[D]) {
    constexpr int KS1 = (D + 1) / 2;
    const bool wok = S[SL.ok] != 0.f;
    const float xs = S[SL.ok + 1];
    bool fast[2];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
        bool bad = false;
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks) bad = bad || !(fabsf(xb[st][ks]) <= xs);
        fast[st] = wok && __builtin_amdgcn_ballot_w64(bad) == 0;
    }
    affine_net_split<HT, D, TILES>(S, SL, xb, sv);
    __builtin_amdgcn_sched_barrier(0);  // one net's activations live at a time
    affine_net_split<HT, D, TILES>(S + SL.net, SL, xb, bv);
    if (!(fast[0] && (TILES == 1 || fast[1]))) {
        __builtin_amdgcn_sched_barrier(0);
        const float* P = Pg + opaque_zero();  // (no hoisted global addresses for this rare path)
        float s2[D], b2[D];
        affine_net<HT, D, TILES>(P, L, xb, s2);
        __builtin_amdgcn_sched_barrier(0);
        affine_net<HT, D, TILES>(P + L.net, L, xb, b2);
        if (!fast[lane_id() >> 5]) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                sv[j] = s2[j];
                bv[j] = b2[j];
            }
        }
    }
}

// LOGP: fused log_prob epilogue for the last layer of an inverse chain — logp = -0.5*(c +
// sum_j z_j^2) + total log-det per sample, and one float64 partial sum per workgroup.
template <int HT, int D, int DIR, bool LOGP>
__global__ __launch_bounds__(256) void affine_coupling_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int accumulate, int64_t nchunks,
    float* __restrict__ logp, double* __restrict__ partials, double* __restrict__ sums, float cgauss) {
    constexpr AffineLayout L = affine_layout(D, HT);
    constexpr int KS1 = L.KS1;
    // H <= 64: only the split tail is staged (layer 2 on the split bf16 MFMAs, affine_net_split)
    constexpr bool SPLIT = affine_has_split(D, HT);
    constexpr AffineSplit SL = affine_split(D, HT);
    constexpr int MASK = SPLIT ? SL.mask : L.mask;
    extern __shared__ f32x4 lds4[];
    {
        const f32x4* src = reinterpret_cast<const f32x4*>(packed + (SPLIT ? L.s : 0));
        for (int i = threadIdx.x; i < (SPLIT ? SL.total : L.total) / 4; i += 256) lds4[i] = src[i];
    }
    __syncthreads();
    const float* sm = reinterpret_cast<const float*>(lds4);

    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    float mk[D], mkb[KS1];
#pragma unroll
    for (int j = 0; j < D; ++j) mk[j] = sm[MASK + j];
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks) mkb[ks] = (2 * ks + h < D) ? sm[MASK + 2 * ks + h] : 0.f;

    // Work split: every wave takes F = nchunks / nwaves whole 64-sample chunks (grid-stride); the
    // R leftover chunks go out as 2R 32-sample half chunks, one to each of the first 2R waves
    // (when 2R <= nwaves), so a SIMD's last round is half a chunk instead of a whole one: at
    // B = 1M, 15.26 chunks per SIMD ran as 16, now as 15.5. (Otherwise the first R waves take
    // one more whole chunk.)
    const int64_t wv = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t F = nchunks / nwaves, R = nchunks - F * nwaves;
    const bool split = 2 * R <= nwaves;
    const int64_t nfull = split ? F : F + (wv < R ? 1 : 0);
    const bool half = split && wv < 2 * R;
    const int64_t half_base = F * nwaves * 64 + wv * 32;

    // Software pipeline: the x rows (both layouts) and the incoming log-det of the next unit are
    // loaded while the current one computes, so HBM latency never sits in front of the MFMAs.
    struct Fetch {
        float xb[2][KS1];  // layer-1 B operands x[base+32st+col][2ks+h] (unmasked)
        float xr[D];       // the lane's own sample row
        float ldin;        // log-det accumulated so far (accumulate = 1)
    };
    // unit u < nfull: chunk wv + u nwaves (64 samples); u == nfull: the half chunk, if any
    auto fetch = [&](int64_t u, Fetch& f) {
        const int64_t base = u < nfull ? (wv + u * nwaves) * 64 : half_base;
        const int nsamp = u < nfull ? 64 : (u == nfull && half ? 32 : 0);
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            const int64_t s = base + 32 * st + col;
#pragma unroll
            for (int ks = 0; ks < KS1; ++ks) {
                const int k = 2 * ks + h;
                f.xb[st][ks] = (32 * st + col < nsamp && k < D && s < B) ? in[s * D + k] : 0.f;
            }
        }
        const int64_t so = base + lane;
        if (lane < nsamp && so < B) {
            load_row<D>(in + so * D, f.xr);
            f.ldin = accumulate ? logdet[so] : 0.f;
        } else {
#pragma unroll
            for (int j = 0; j < D; ++j) f.xr[j] = 0.f;
            f.ldin = 0.f;
        }
    };

    double lpacc = 0.0;
    // one unit: 2 sample tiles (TILES = 2) or the half chunk (TILES = 1, lanes 0..31)
    auto unit = [&](auto tiles_c, int64_t base, const Fetch& cur) {
        constexpr int TILES = decltype(tiles_c)::value;
        const float* smi = sm + opaque_zero();
        float xb[2][KS1];
#pragma unroll
        for (int st = 0; st < 2; ++st) {
#pragma unroll
            for (int ks = 0; ks < KS1; ++ks) xb[st][ks] = cur.xb[st][ks] * mkb[ks];
        }

        float sv[D], bv[D];
        if constexpr (SPLIT) {
            affine_nets_split<HT, D, TILES>(smi, SL, packed, L, xb, sv, bv);
        } else {
            affine_net<HT, D, TILES>(smi, L, xb, sv);
            affine_net<HT, D, TILES>(smi + L.net, L, xb, bv);
        }

        const int64_t so = base + lane;
        if (lane < 32 * TILES && so < B) {
#pragma clang fp contract(off)  // separate mul/add roundings, as the reference's torch ops
            float y[D];
            float ld = 0.f;
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const float m = mk[j], om = 1.f - m;
                const float xa = cur.xr[j] * m;
                float t;
                if constexpr (DIR < 0) {
                    t = (cur.xr[j] - bv[j]) * exp_fast(-sv[j]);
                    ld = ld + om * (-sv[j]);
                } else {
                    t = cur.xr[j] * exp_fast(sv[j]) + bv[j];
                    ld = ld + om * sv[j];
                }
                const float v = xa + om * t;
                y[j] = nonfinite(v) ? 0.f : v;
            }
            if (nonfinite(ld)) ld = 0.f;
            store_row<D>(out + so * D, y);
            const float ldt = accumulate ? cur.ldin + ld : ld;
            logdet[so] = ldt;
            if constexpr (LOGP) {
                float m = gauss_sq0(y[0]);
#pragma unroll
                for (int j = 1; j < D; ++j) m = gauss_sq(m, y[j]);
                const float lp = gauss_lp(m, cgauss, ldt);
                logp[so] = lp;
                lpacc += (double)lp;
            }
        }
    };

    Fetch cur;
    fetch(0, cur);
    for (int64_t u = 0; u < nfull; ++u) {
        Fetch nxt;
        fetch(u + 1, nxt);
        unit(std::integral_constant<int, 2>{}, (wv + u * nwaves) * 64, cur);
        cur = nxt;
    }
    if (half) unit(std::integral_constant<int, 1>{}, half_base, cur);
    if constexpr (LOGP) {
        logp_commit<256>(lpacc, partials, sums, B);
    }
}


// ---- wide coupling layers (8 < d <= 64, e.g. UCI-shaped RealNVP d = 43 / 63) -------------------
// A wave owns a 32-sample tile whose [32 x d] x block sits in a wave-private LDS tile (odd row
// stride, conflict-free column reads), loaded and stored row by row with coalesced accesses.
// Layer 1 (K = d) reads its B operands (x * mask) from the tile, layers 2 and 3 (H -> d, one
// 32-row MFMA tile per 32 output dims) keep activations in accumulator registers, and the
// affine epilogue runs in accumulator layout on the tile in place. Weights (both nets) are
// read from L2 (up to ~260 KB at H = 128, beyond LDS).
constexpr int kWideWaves = 4;

template <int HT>
__device__ __forceinline__ void wide_net(const float* __restrict__ P, const AffineLayout& L, const float* xt, int S,
                                         const float* __restrict__ mask, int d, f32x16 (&res)[2]) {
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    f32x16 h1[HT];
#pragma unroll
    for (int ht = 0; ht < HT; ++ht) h1[ht] = load_bias16(P + L.b1 + ht * 32, h);
    for (int ks = 0; ks < L.KS1; ++ks) {
        const int k = 2 * ks + h;
        const float xb = k < d ? xt[col * S + k] * mask[k] : 0.f;
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) h1[ht] = mfma32(P[L.w1 + (ht * L.KS1 + ks) * 64 + lane], xb, h1[ht]);
    }
#pragma unroll
    for (int ht = 0; ht < HT; ++ht)
#pragma unroll
        for (int r = 0; r < 16; ++r) h1[ht][r] = trelu(h1[ht][r]);
    f32x16 h2[HT];
#pragma unroll
    for (int hto = 0; hto < HT; ++hto) {
        f32x16 a = load_bias16(P + L.b2 + hto * 32, h);
#pragma unroll
        for (int kt = 0; kt < HT; ++kt)
#pragma unroll
            for (int rq = 0; rq < 4; ++rq) {
                const f32x4 w = *reinterpret_cast<const f32x4*>(P + L.w2 + (((hto * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) a = mfma32(w[rr], h1[kt][4 * rq + rr], a);
            }
#pragma unroll
        for (int r = 0; r < 16; ++r) a[r] = trelu(a[r]);
        h2[hto] = a;
    }
    const int NJ = (d + 31) / 32;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (j < NJ) {
            f32x16 a = load_bias16(P + L.b3 + j * 32, h);
#pragma unroll
            for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) {
                    const f32x4 w = *reinterpret_cast<const f32x4*>(P + L.w3 + (((j * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) a = mfma32(w[rr], h2[kt][4 * rq + rr], a);
                }
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = tclamp(a[r], -10.f, 10.f);
            res[j] = a;
        } else {
            res[j] = f32x16{};
        }
    }
}

template <int HT, int DIR, bool LOGP>
__global__ __launch_bounds__(64 * kWideWaves) void affine_wide_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d, int accumulate, int64_t ntiles,
    float* __restrict__ logp, double* __restrict__ partials, double* __restrict__ sums, float cgauss) {
    const AffineLayout L = affine_layout(d, HT);
    const int S = d | 1;
    extern __shared__ f32x4 lds4[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float* xt = reinterpret_cast<float*>(lds4) + wave * 32 * S;
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    const float* mask = packed + L.mask;
    double lpacc = 0.0;
    for (int64_t t = (int64_t)blockIdx.x * kWideWaves + wave; t < ntiles; t += (int64_t)gridDim.x * kWideWaves) {
        const int64_t base = t * 32;
        const int rows = (int)(B - base < 32 ? B - base : 32);
        const float* src = in + base * d;
        for (int i = lane; i < 32 * d; i += 64) {
            const int r = i / d, c = i - r * d;
            xt[r * S + c] = r < rows ? src[i] : 0.f;
        }
        const float ldin = (accumulate && lane < rows) ? logdet[base + lane] : 0.f;
        wave_lds_sync();
        const float* Pw = packed + opaque_zero();
        f32x16 sv[2], bv[2];
        wide_net<HT>(Pw, L, xt, S, mask, d, sv);
        wide_net<HT>(Pw + L.net, L, xt, S, mask, d, bv);
        float ldp = 0.f;
        {
#pragma clang fp contract(off)  // separate mul/add roundings, as the reference's torch ops
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int dim = 32 * j + crow(r, h);
                    if (dim < d) {
                        float* px = xt + col * S + dim;
                        const float xv = *px, m = mask[dim], om = 1.f - m;
                        float tv;
                        if constexpr (DIR < 0) {
                            tv = (xv - bv[j][r]) * exp_fast(-sv[j][r]);
                            ldp = ldp + om * (-sv[j][r]);
                        } else {
                            tv = xv * exp_fast(sv[j][r]) + bv[j][r];
                            ldp = ldp + om * sv[j][r];
                        }
                        const float v = xv * m + om * tv;
                        *px = nonfinite(v) ? 0.f : v;
                    }
                }
        }
        float ld = halves_sum(ldp, ldp);  // lanes 0..31: sample col
        if (nonfinite(ld)) ld = 0.f;
        wave_lds_sync();
        float* dst = out + base * d;
        for (int i = lane; i < rows * d; i += 64) {
            const int r = i / d, c = i - r * d;
            dst[i] = xt[r * S + c];
        }
        if (lane < rows) {
            const float ldt = accumulate ? ldin + ld : ld;
            logdet[base + lane] = ldt;
            if constexpr (LOGP) {
                float m = gauss_sq0(xt[lane * S]);
                for (int c = 1; c < d; ++c) m = gauss_sq(m, xt[lane * S + c]);
                const float lp = gauss_lp(m, cgauss, ldt);
                logp[base + lane] = lp;
                lpacc += (double)lp;
            }
        }
        wave_lds_sync();
    }
    if constexpr (LOGP) {
        logp_commit<64 * kWideWaves>(lpacc, partials, sums, B);
    }
}

typedef void (*affine_kernel_t)(const float*, const float*, float*, float*, int64_t, int, int64_t,
                                float*, double*, double*, float);

template <int HT>
affine_kernel_t affine_pick_ht(int d, int dir, bool logp);

// Writes the split tail of an eval image after its fp32 part (no-op without one); same stream.
int affine_split_pack(float* packed, int d, int H, hipStream_t s);

}  // namespace nfx
