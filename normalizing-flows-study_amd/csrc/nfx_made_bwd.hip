// Backward (training) pass of the PARALLEL MADE directions — MaskedAutoregressiveFlow.inverse
// (MAF density, masked_autoregressive_flow.py:18-44) and InverseAutoregressiveFlow.forward (IAF
// sampling, inverse_autoregressive_flow.py:30-63) under autograd, no BatchNorm.
// SURVEY.md §8(f) item 1. Two kernels:
//   made_bwd_kernel<HT, VAR>   d <= 64, H <= 64: weights (forward image + padded transposed
//                              copy) LDS-resident, x tiles by LDS-DMA;
//   made_bwdw_kernel<HT, VAR>  d <= 4096, H <= 128 (e.g. IAF(784, 64) sampling): x streamed
//                              through a 32 x 32 LDS stage per input chunk, the output layer per
//                              (mu, alpha) block pair in two passes, weights read from L2.
// Both serve both parallel directions (VAR = NFX_MAF_INVERSE | NFX_IAF_FORWARD epilogue).
// Batch limit: the feature-major factor rows are addressed with 32-bit buffer offsets, so
// nfx_made_affine_backward accepts B <= nfx_made_backward_max_batch(d, H) (the host chunks the
// batch above it).
//
// One fused kernel per layer recomputes the forward on fp32 MFMA (same tile kernel structure
// as made_tile_kernel: a wave owns 32 samples, hidden activations stay in accumulator registers)
// and runs the data-gradient chain back through the net on MFMA with the TRANSPOSED weights:
// the (mu, alpha) gradients δ4 come out of the affine epilogue's backward in accumulator layout,
// which is exactly the B operand of gh3 = W4mᵀ δ4; each ReLU backward masks with the kept
// activations; gx = the epilogue's direct term + W1mᵀ δ1. The weight gradients are reductions
// over the SAMPLE dimension (K = B), which the per-sample tile layout cannot contract without a
// transpose per tile, so the kernel writes the per-sample factors feature-major (δ4ᵀ, δ3ᵀ, δ2ᵀ,
// δ1ᵀ, h3ᵀ, h2ᵀ, h1ᵀ: coalesced 128-byte rows, one half-wave per feature row, row pitch B)
// and the weight gradients are MFMA sample contractions over them
// (nfx_made_wgrad.hip: gW4 = δ4·h3ᵀ, …, gW1 = δ1·xᵀ), masked like the reference's weight*mask.
//
// Epilogue backward (MAF density), per element (torch semantics of the reference ops):
//   a = clamp(alpha, -3, 3); e = exp(-a); zr = (x - mu) * e; z = finite(zr) ? zr : 0
//   ld_raw = -sum a; ld1 = finite(ld_raw) ? ld_raw : 0; ld = clamp(ld1, -100, 100)
//   gzr = finite(zr) ? gz : 0;  gld1 = gld * [-100 <= ld1 <= 100] * finite(ld_raw)
//   gx += gzr * e;  gmu = -gzr * e;  galpha = [-3 <= alpha <= 3] * (-(gzr * (x - mu) * e) - gld1)
#include "nfx_made_kernel.h"
#include "nfx_pack.h"

namespace nfx {

__global__ void made_bwd_pack_kernel(NfxMlpRaw net, int d, int H, float* packed) {
    const int HT = (H + 31) / 32;
    const MadeLayout L = made_layout(d, HT);
    for (int i = L.t4 + blockIdx.x * blockDim.x + threadIdx.x; i < L.rimg; i += gridDim.x * blockDim.x) {
        float v = 0.f;
        int base, nk;
        if (i < L.t3) { base = L.t4; nk = 2 * L.NJ; }
        else if (i < L.t2) { base = L.t3; nk = HT; }
        else if (i < L.t1) { base = L.t2; nk = HT; }
        else { base = L.t1; nk = HT; }
        const int t = i - base, rr = t & 3, lane = (t >> 2) & 63, rq = (t >> 8) & 3;
        const int kt = (t >> 10) % nk, ot = (t >> 10) / nk;
        const int row = 32 * ot + (lane & 31);                     // out index (rows of the transposed)
        const int kk = crow(4 * rq + rr, lane >> 5);               // k index inside the k tile
        if (i < L.t3) {
            const int j = kt >> 1, which = kt & 1, o = 32 * j + kk;  // output block (mu | alpha)
            v = (row < H && o < d) ? mlp_weight(net, 3, H, which * d + o, row) : 0.f;
        } else if (i < L.t1) {
            const int layer = i < L.t2 ? 2 : 1, k = 32 * kt + kk;
            v = (row < H && k < H) ? mlp_weight(net, layer, H, k, row) : 0.f;
        } else {
            const int k = 32 * kt + kk;                              // hidden unit
            v = (row < d && k < H) ? mlp_weight(net, 0, d, k, row) : 0.f;
        }
        packed[i] = v;
    }
}

// Feature-major store of one accumulator tile: rows `row0 + crow(r, h)` (< nrows) of a
// [nrows x B] matrix, columns = the tile's 32 samples (base + col < B). Raw buffer stores: the
// lane offset carries the sample and the lane half's +4 rows, the row of each register rides in
// the scalar offset, and the descriptor's range check drops rows >= nrows; lanes past B get an
// offset outside every range. No per-element branches or 64-bit address math.
__device__ __forceinline__ void store_fm(float* __restrict__ dst, const f32x16& t, int row0, int nrows, int64_t B,
                                         int64_t P, int64_t base) {
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, (int)(((int64_t)nrows * P - base) * 4),
                                                      0x00020000);
    const int vo = base + col < B ? (int)((col + 4 * h * P) * 4) : (int)0xFFFFFFF0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int rowu = row0 + (r & 3) + 8 * (r >> 2);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(t[r]), rs, vo, (int)(rowu * P * 4), 0);
    }
}

// ReLU-backward masks of HT accumulator tiles as bits (tile ot, register r -> bit ot*16 + r):
// the backward needs only (h > 0), so the activations can be written out and die early.
template <int HT>
__device__ __forceinline__ uint32_t relu_bits(const f32x16 (&t)[HT]) {
    uint32_t m = 0;
#pragma unroll
    for (int ot = 0; ot < HT; ++ot)
#pragma unroll
        for (int r = 0; r < 16; ++r) m |= (t[ot][r] > 0.f ? 1u : 0u) << (ot * 16 + r);
    return m;
}

// A-operand (weights) x B-operand (accumulator-layout tiles) chain over NK k tiles, A from
// global/L2 in [out tile][k tile][r/4][lane][r%4] order.
template <int NK>
__device__ __forceinline__ f32x16 chain_gmem(const float* __restrict__ A, int ot, int nk_total,
                                             const f32x16* bt, f32x16 acc) {
    const int lane = lane_id();
#pragma unroll
    for (int kt = 0; kt < NK; ++kt) {
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {
            const f32x4 w = *reinterpret_cast<const f32x4*>(A + (((ot * nk_total + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) acc = mfma32(w[rr], bt[kt][4 * rq + rr], acc);
        }
    }
    return acc;
}

// chain_gmem over k tiles [K0, NK) only: the leading k tiles of a transposed MADE weight tile
// row are structurally zero (sorted degrees), so they are skipped whole; k0 is wave-uniform and
// selects a straight-line variant (no branches around individual MFMAs).
template <int NK, int K0>
__device__ __forceinline__ f32x16 chain_gmem_k(const float* __restrict__ A, int ot, int nk_total, const f32x16* bt,
                                               f32x16 acc) {
    const int lane = lane_id();
#pragma unroll
    for (int kt = K0; kt < NK; ++kt) {
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {
            const f32x4 w = *reinterpret_cast<const f32x4*>(A + (((ot * nk_total + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) acc = mfma32(w[rr], bt[kt][4 * rq + rr], acc);
        }
    }
    return acc;
}
template <int NK, int K0 = 0>
__device__ __forceinline__ f32x16 chain_gmem_from(int k0, const float* __restrict__ A, int ot, int nk_total,
                                                  const f32x16* bt, f32x16 acc) {
    if constexpr (K0 >= NK) {
        return acc;
    } else {
        if (k0 <= K0) return chain_gmem_k<NK, K0>(A, ot, nk_total, bt, acc);
        return chain_gmem_from<NK, K0 + 1>(k0, A, ot, nk_total, bt, acc);
    }
}

// All 16 x HT values of a tile set finite (wave-wide): skipping structurally-zero weight blocks
// is then exact (a zero weight times a finite operand adds an exact zero).
template <int HT>
__device__ __forceinline__ bool tiles_finite(const f32x16* t) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < HT; ++k)
#pragma unroll
        for (int r = 0; r < 16; ++r) ok = ok && !nonfinite(t[k][r]);
    return __builtin_amdgcn_ballot_w64(!ok) == 0;
}

__host__ __device__ constexpr int NKC_(int d) { return (d + 31) / 32; }
__host__ __device__ constexpr int NJ_(int d) { return (d + 31) / 32; }

// ---- made_bwd_kernel's LDS weight image ----
// The forward A-operand tiles ([rq][lane][4], 1024 floats) are copied into LDS with padding —
// rq blocks 264 floats apart, the upper lane half shifted by 4 — so that they serve BOTH chains:
// the forward recompute reads them as before (16-byte reads, contiguous per half wave), and the
// data-gradient chain reads the TRANSPOSED tile from the same copy, one dword per MFMA k-step:
// lane (i, kh) at step s needs W[row crow(s, kh)][col i] of the forward tile, which lives at
//   (i >> 3) * 264 + ((i >> 2) & 1) * 132 + (i & 3) + 4 crow(s, kh)      (hidden / output layers,
//   whose k index is the accumulator row crow(., .))
//   (i >> 3) * 264 + (i & 1) * 132 + ((i >> 1) & 3) + 4 crow(s, kh)      (layer 1, k = 2 s + kh);
// modulo 32 banks the lane-dependent part is 8a + 4c + b over the 32 lanes of a half: no
// conflicts. No transposed image is read from L2 any more.
constexpr int kPadRQ = 264, kPadH = 4, kPadTile = 4 * kPadRQ;
struct BwdLds {
    int w1, w2, w3, w4, b1, b2, b3, b4, x, total;
};
__host__ __device__ constexpr BwdLds bwd_lds(int d, int HT) {
    const int NKC = (d + 31) / 32, NJ = NKC;
    BwdLds b{};
    int o = 0;
    b.w1 = o; o += HT * NKC * kPadTile;
    b.w2 = o; o += HT * HT * kPadTile;
    b.w3 = o; o += HT * HT * kPadTile;
    b.w4 = o; o += NJ * 2 * HT * kPadTile;
    b.b1 = o; o += HT * 32;
    b.b2 = o; o += HT * 32;
    b.b3 = o; o += HT * 32;
    b.b4 = o; o += NJ * 64;
    b.x = (o + 3) & ~3;  // per-wave x tiles follow
    b.total = b.x;
    return b;
}

// hidden / output tile `tile` of a padded layer over its first NK k tiles (bias, MFMA chain)
template <int HT, int NK>
__device__ __forceinline__ f32x16 pad_tile(const float* wl, const float* bl, int hto, const f32x16 (&hin)[HT],
                                           int lo, int h) {
    f32x16 a = load_bias16(bl + hto * 32, h);
#pragma unroll
    for (int kt = 0; kt < NK; ++kt) {
        const float* tp = wl + (hto * HT + kt) * kPadTile + lo;
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {
            const f32x4 w = *reinterpret_cast<const f32x4*>(tp + rq * kPadRQ);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) a = mfma32(w[rr], hin[kt][4 * rq + rr], a);
        }
    }
    return a;
}
template <int HT, int N>
__device__ __forceinline__ f32x16 pad_tile_n(int n, const float* wl, const float* bl, int hto, const f32x16 (&hin)[HT],
                                             int lo, int h) {
    if constexpr (N == 0) {
        return pad_tile<HT, 0>(wl, bl, hto, hin, lo, h);
    } else {
        if (n >= N) return pad_tile<HT, N>(wl, bl, hto, hin, lo, h);
        return pad_tile_n<HT, N - 1>(n, wl, bl, hto, hin, lo, h);
    }
}
template <int HT>
__device__ __forceinline__ void pad_hidden(const float* wl, const float* bl, const f32x16 (&hin)[HT], f32x16 (&hout)[HT],
                                           const int (&nk)[HT], bool dense, int lo, int h) {
#pragma unroll
    for (int hto = 0; hto < HT; ++hto) {
        f32x16 a = pad_tile_n<HT, HT>(dense ? HT : nk[hto], wl, bl, hto, hin, lo, h);
#pragma unroll
        for (int r = 0; r < 16; ++r) a[r] = trelu(a[r]);
        hout[hto] = a;
    }
}

// transposed chain: acc += sum over k tiles kt in [K0, NK) of (forward tile kt * stride + ot)^T
// . bt[kt]; `tb` = this lane's transposed-read base inside a tile (see above)
template <int NK, int K0>
__device__ __forceinline__ f32x16 tchain_k(const float* wl, int stride, int ot, int tb, const f32x16* bt, f32x16 acc) {
#pragma unroll
    for (int kt = K0; kt < NK; ++kt) {
        const float* tp = wl + (kt * stride + ot) * kPadTile + tb;
        // the tile's 16 dwords in flight together (counted waits), then the 16 MFMAs
        float a[16];
#pragma unroll
        for (int st = 0; st < 16; ++st) a[st] = tp[4 * ((st & 3) + 8 * (st >> 2))];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int st = 0; st < 16; ++st) acc = mfma32(a[st], bt[kt][st], acc);
    }
    return acc;
}
template <int NK, int K0 = 0>
__device__ __forceinline__ f32x16 tchain_from(int k0, const float* wl, int stride, int ot, int tb, const f32x16* bt,
                                              f32x16 acc) {
    if constexpr (K0 >= NK) {
        return acc;
    } else {
        if (k0 <= K0) return tchain_k<NK, K0>(wl, stride, ot, tb, bt, acc);
        return tchain_from<NK, K0 + 1>(k0, wl, stride, ot, tb, bt, acc);
    }
}

// Waves per workgroup (LDS: the padded forward weight image + one x tile per wave, one workgroup per
// CU): 8 (2 per SIMD) for large batches; 4 (1 per SIMD, 512 registers: no scratch spills) when
// the batch has at most one 32-sample tile per wave of 4-wave workgroups on every CU — the figure
// models' 2,000 points then run on 16 CUs instead of 8 (0.88 vs 1.04 ms per trainfig_maf step),
// while cfg4t's 15.6k tiles run faster at 2 waves per SIMD (89.9 vs 85.9 M samples/s).
constexpr int kBwdWaves = 8;
constexpr int kBwdWavesSmall = 4;

template <int HT, int VAR, int NW>
__global__ __launch_bounds__(64 * NW) void made_bwd_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, const float* __restrict__ gout,
    const float* __restrict__ gld_in, float* __restrict__ gin, float* __restrict__ acts, int64_t B, int d,
    int H, int64_t ntiles) {
    const MadeLayout L = made_layout(d, HT);
    constexpr int S = kTileStride;
    extern __shared__ f32x4 lds4[];
    float* lds = reinterpret_cast<float*>(lds4);
    // the padded forward weight image (both the recompute and the transposed chains read it)
    const BwdLds BL = bwd_lds(d, HT);
    {
        const f32x4* src = reinterpret_cast<const f32x4*>(packed);
        const int nt1 = HT * NKC_(d), nt23 = HT * HT, nt4 = NJ_(d) * 2 * HT;
        const int ntiles_w = nt1 + 2 * nt23 + nt4;
        for (int i = threadIdx.x; i < ntiles_w * 256; i += 64 * NW) {
            const int tl = i >> 8, q = i & 255, rq = q >> 6, ln = q & 63;
            int srco, dsto;
            if (tl < nt1) { srco = L.w1 + tl * 1024; dsto = BL.w1 + tl * kPadTile; }
            else if (tl < nt1 + nt23) { srco = L.w2 + (tl - nt1) * 1024; dsto = BL.w2 + (tl - nt1) * kPadTile; }
            else if (tl < nt1 + 2 * nt23) { srco = L.w3 + (tl - nt1 - nt23) * 1024; dsto = BL.w3 + (tl - nt1 - nt23) * kPadTile; }
            else { srco = L.w4 + (tl - nt1 - 2 * nt23) * 1024; dsto = BL.w4 + (tl - nt1 - 2 * nt23) * kPadTile; }
            *reinterpret_cast<f32x4*>(lds + dsto + rq * kPadRQ + ln * 4 + (ln >> 5) * kPadH) = src[(srco >> 2) + q];
        }
        for (int i = threadIdx.x; i < HT * 32; i += 64 * NW) {
            lds[BL.b1 + i] = packed[L.b1 + i];
            lds[BL.b2 + i] = packed[L.b2 + i];
            lds[BL.b3 + i] = packed[L.b3 + i];
        }
        for (int i = threadIdx.x; i < NJ_(d) * 64; i += 64 * NW) lds[BL.b4 + i] = packed[L.b4 + i];
    }
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float* xt = lds + BL.x + wave * 32 * S;  // x tile; later the direct dL/dx term
    const int rowb = d * 4;
    const int NJ = L.NJ, NKC = L.NKC;
    // feature-major factors: [d4 (2d) | d3 | d2 | d1 (H each) | h3, 1 | h2, 1 | h1, 1 (H+1 each) |
    // x, 1 (d+1)] rows x B — the trailing ones rows turn each weight-gradient GEMM into the
    // bias gradient as well (its last column)
    const int64_t P = B;  // factor row pitch (nfx_made_factor_pitch)
    float* D4 = acts;
    float* D3 = D4 + (int64_t)2 * d * P;
    float* D2 = D3 + (int64_t)H * P;
    float* D1 = D2 + (int64_t)H * P;
    float* H3 = D1 + (int64_t)H * P;
    float* H2 = H3 + (int64_t)(H + 1) * P;
    float* H1 = H2 + (int64_t)(H + 1) * P;
    float* X1 = H1 + (int64_t)(H + 1) * P;

    // Structural-zero extents of the forward image (made_live_kernel) and their transposed
    // starts: W^T tile (ot, kt) of a layer is nonzero iff W block (kt, ot) is, i.e. iff
    // ot < nk[kt]; nk is non-decreasing in kt (sorted degrees), so the nonzero kt form a suffix.
    const int* nkp = reinterpret_cast<const int*>(packed);
    int nk1[HT], nk2[HT], nk3[HT], nk4[2];
    bool full2 = true, full3 = true;
#pragma unroll
    for (int i = 0; i < HT; ++i) {
        nk1[i] = nkp[L.nk1 + i];
        nk2[i] = nkp[L.nk2 + i];
        nk3[i] = nkp[L.nk3 + i];
        full2 = full2 && nk2[i] >= HT;
        full3 = full3 && nk3[i] >= HT;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) nk4[j] = j < NJ ? nkp[L.nk4 + j] : HT;
    auto kstart = [&](const int* nk, int n, int ot) {
        int k0 = n;
        for (int k = n - 1; k >= 0; --k)
            if (nk[k] > ot) k0 = k;
        return k0;
    };
    const float tsafe = packed[L.tsafe];

    for (int64_t t = (int64_t)blockIdx.x * NW + wave; t < ntiles; t += (int64_t)gridDim.x * NW) {
        // the per-lane constants are recomputed per tile from threadIdx.x (a few VALU ops) rather
        // than kept live across the loop: at the 256-VGPR budget they would be spilled, and each
        // reload waits behind the tile's factor stores (one in-order vmcnt for loads and stores)
        const int lane = (int)(threadIdx.x & 63) + opaque_zero(), h = lane >> 5, col = lane & 31;
        const int voff = lane < d ? lane * 4 : (1 << 30);
        const int64_t base = t * 32;
        const int rows = (int)(B - base < 32 ? B - base : 32);
        float xmax = 0.f;
        {
            // the tile's 32 rows go straight into LDS (buffer_load ... lds: all 32 in flight, no
            // registers held), then the overflow-safe bound check reads them back. Out-of-range
            // lanes of an LDS-DMA write nothing, so the padding dims >= d are zeroed explicitly
            // (layer 1 multiplies them by zero weights: stale NaN there would poison the sample);
            // rows >= B stay stale, which only touches the tile's unused sample columns.
            const auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in) + base * d, 0, rows * rowb, 0x00020000);
            if (lane >= d) {
#pragma unroll
                for (int r = 0; r < 32; ++r) xt[r * S + lane] = 0.f;
            }
#pragma unroll
            for (int r = 0; r < 32; ++r)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(xt + r * S), 4, voff,
                                                     r * rowb, 0, 0);
            // the DMA completes under vmcnt; wait explicitly before any LDS read of the tile
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int r = 0; r < 32; ++r) xmax = tmax(xmax, fabsf(xt[r * S + lane]));  // NaN-propagating
        }
        // Skip structurally-zero blocks only when the tile's inputs are finite and within the
        // overflow-safe bound (every forward activation finite: bit-identical to dense, as in
        // made_tile_kernel); the backward chains additionally check their operand tiles.
        const bool dense = __builtin_amdgcn_ballot_w64(!(xmax <= tsafe)) != 0;
        wave_lds_sync();
        // opaque offsets keep the compiler from hoisting every (loop-invariant) weight read out
        // of the tile loop into registers
        const float* Wl = lds + opaque_zero();
        const int lo = lane * 4 + h * kPadH;                                              // forward reads
        const int tbh = ((col >> 3) * kPadRQ + ((col >> 2) & 1) * (128 + kPadH) + (col & 3) + 16 * h);  // W2..W4^T
        const int tb1 = ((col >> 3) * kPadRQ + (col & 1) * (128 + kPadH) + ((col >> 1) & 3) + 16 * h);  // W1^T
        {
            // x and the ones rows, feature-major: half-wave h writes dim row 2i+h of 32 samples
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(X1 + base, 0, (int)(((int64_t)(d + 1) * P - base) * 4),
                                                              0x00020000);
            const int vo = base + col < B ? (int)((col + h * P) * 4) : (int)0xFFFFFFF0;
#pragma unroll
            for (int i = 0; i < 32; ++i)
                if (2 * i < d)
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(2 * i + h < d ? xt[col * S + 2 * i + h] : 1.f), rs,
                                                          vo, (int)(2 * i * P * 4), 0);
            if (h == 0 && base + col < B) {
                if ((d & 1) == 0) X1[(int64_t)d * P + base + col] = 1.f;  // odd d: written above (row 2i+1 = d)
                H3[(int64_t)H * P + base + col] = 1.f;
                H2[(int64_t)H * P + base + col] = 1.f;
                H1[(int64_t)H * P + base + col] = 1.f;
            }
        }

        // ---- forward recompute (structurally-zero blocks skipped unless dense) ----
        f32x16 h1[HT], h2[HT], h3[HT];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
            f32x16 a = load_bias16(Wl + BL.b1 + ht * 32, h);
            const int nkc = dense ? NKC : nk1[ht];
            for (int kc = 0; kc < nkc; ++kc) {
                const float* tp = Wl + BL.w1 + (ht * NKC + kc) * kPadTile + lo;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x4 w = *reinterpret_cast<const f32x4*>(tp + g * kPadRQ);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) a = mfma32(w[rr], xt[col * S + 32 * kc + 8 * g + 2 * rr + h], a);
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = trelu(a[r]);
            h1[ht] = a;
        }
        pad_hidden<HT>(Wl + BL.w2, Wl + BL.b2, h1, h2, nk2, dense || full2, lo, h);
        const uint32_t m1 = relu_bits<HT>(h1);
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) store_fm(H1, h1[ht], 32 * ht, H, B, P, base);
        pad_hidden<HT>(Wl + BL.w3, Wl + BL.b3, h2, h3, nk3, dense || full3, lo, h);
        const uint32_t m2 = relu_bits<HT>(h2);
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) store_fm(H2, h2[ht], 32 * ht, H, B, P, base);

        // layer 4 for every output block (kept for the log-det sum), then the epilogue backward.
        // d4[j*2 + 0] = mu / δmu rows of block j, d4[j*2 + 1] = alpha / δalpha rows (t4 k order).
        f32x16 d4[4];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (j < NJ) {
                // output tiles (j, mu) = tile index 2j, (j, alpha) = 2j + 1 of the padded w4
                d4[2 * j] = pad_tile_n<HT, HT>(dense ? HT : nk4[j], Wl + BL.w4, Wl + BL.b4, 2 * j, h3, lo, h);
                d4[2 * j + 1] = pad_tile_n<HT, HT>(dense ? HT : nk4[j], Wl + BL.w4, Wl + BL.b4, 2 * j + 1, h3, lo, h);
            } else {
                d4[2 * j] = d4[2 * j + 1] = f32x16{};
            }
        }
        const uint32_t m3 = relu_bits<HT>(h3);
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) store_fm(H3, h3[ht], 32 * ht, H, B, P, base);

        // ld_raw = -sum_i clamp(alpha_i, -3, 3) (MAF inverse) / +sum_i clamp(alpha_i, -2, 2) (IAF
        // forward) of the lane's sample, summed in the forward kernel's order (rows past d: 0)
        constexpr bool IAF = VAR == NFX_IAF_FORWARD;
        constexpr float ALO = IAF ? -2.f : -3.f, AHI = IAF ? 2.f : 3.f, LDLIM = IAF ? 50.f : 100.f;
        float asum0 = 0.f;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) asum0 = asum0 + tclamp(d4[2 * j + 1][r], ALO, AHI);
        const float ldraw = IAF ? halves_sum(asum0, asum0) : -halves_sum(asum0, asum0);
        const float gld = (lane < 32 && col < rows) ? gld_in[base + col] : 0.f;
        float gld1 = nonfinite(ldraw) ? 0.f : gld;
        const float ld1 = nonfinite(ldraw) ? 0.f : ldraw;
        if (!(ld1 >= -LDLIM && ld1 <= LDLIM)) gld1 = 0.f;
        const float gld1s = __shfl(gld1, col, 64);  // both lane halves of sample col

        // epilogue backward; the direct dz/dx term replaces x in the tile (same lane, same slot).
        // dL/dz in accumulator layout straight from global: lane (col, h), block j holds dims
        // 32j + 8q + 4h + 0..3 of sample col -> four 16-byte loads (range check: rows >= B read 0;
        // dims >= d belong to the next row and are zeroed)
        const auto rgz = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(gout) + base * d, 0, rows * rowb,
                                                           0x00020000);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            float gzr[16];
            if (j < NJ) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int dim0 = 32 * j + 8 * q + 4 * h;
                    const auto u = __builtin_amdgcn_raw_buffer_load_b128(rgz, col * rowb + dim0 * 4, 0, 0);
#pragma unroll
                    for (int e = 0; e < 4; ++e) gzr[4 * q + e] = dim0 + e < d ? __uint_as_float(u[e]) : 0.f;
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int dim = 32 * j + crow(r, h);
                float* px = xt + col * S + dim;
                const float xv = *px;
                const float gz = j < NJ ? gzr[r] : 0.f;
                const float alpha = d4[2 * j + 1][r];
                if constexpr (IAF) {
                    // inverse_autoregressive_flow.py:39-54: y = x exp(clamp(a,-2,2)) + clamp(mu,-10,10),
                    // y = finite ? y : x
                    const float mu = d4[2 * j][r];
                    const float a = tclamp(alpha, -2.f, 2.f);
                    const float e = exp_fast(a);
                    const float yr = xv * e + tclamp(mu, -10.f, 10.f);  // same expression as the forward kernel
                    const bool bad = nonfinite(yr);
                    const float gyr = bad ? 0.f : gz;
                    *px = bad ? gz : gyr * e;
                    d4[2 * j][r] = (mu >= -10.f && mu <= 10.f) ? gyr : 0.f;                    // δmu
                    d4[2 * j + 1][r] = (alpha >= -2.f && alpha <= 2.f) ? gyr * xv * e + gld1s : 0.f;  // δalpha
                } else {
                    const float a = tclamp(alpha, -3.f, 3.f);
                    const float e = exp_fast(-a);
                    const float xm = xv - d4[2 * j][r];
                    const float zr = xm * e;
                    const float gzr = nonfinite(zr) ? 0.f : gz;
                    const float ge = gzr * e;
                    *px = ge;
                    d4[2 * j][r] = -ge;                                          // δmu
                    const float ga = -(gzr * xm * e) - gld1s;
                    d4[2 * j + 1][r] = (alpha >= -3.f && alpha <= 3.f) ? ga : 0.f;  // δalpha
                }
            }
        }

        // ---- data-gradient chain on MFMA with the transposed weights (L2); every factor is
        // written feature-major as soon as it is final so it can die ----
        // the structurally-zero leading k tiles of each transposed row are skipped when the
        // chain's operand tiles are finite (0 * finite = exact 0), else the dense chain runs
        const bool d4ok = !dense && tiles_finite<4>(d4);
        f32x16 g[HT];
#pragma unroll
        for (int ot = 0; ot < HT; ++ot) {
            const int k4 = d4ok ? 2 * kstart(nk4, NJ, ot) : 0;
            f32x16 acc = NJ == 2 ? tchain_from<4>(k4, Wl + BL.w4, HT, ot, tbh, d4, f32x16{})
                                 : tchain_from<2>(k4, Wl + BL.w4, HT, ot, tbh, d4, f32x16{});
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = ((m3 >> (ot * 16 + r)) & 1u) ? acc[r] : 0.f;
            g[ot] = acc;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (j < NJ) {
                store_fm(D4, d4[2 * j], 32 * j, d, B, P, base);                        // mu rows
                store_fm(D4 + (int64_t)d * P, d4[2 * j + 1], 32 * j, d, B, P, base);   // alpha rows
            }
        }
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
            store_fm(D3, g[ht], 32 * ht, H, B, P, base);
        }
        const bool g3ok = !dense && tiles_finite<HT>(g);
        f32x16 g2[HT];
#pragma unroll
        for (int ot = 0; ot < HT; ++ot) {
            f32x16 acc = tchain_from<HT>(g3ok ? kstart(nk3, HT, ot) : 0, Wl + BL.w3, HT, ot, tbh, g, f32x16{});
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = ((m2 >> (ot * 16 + r)) & 1u) ? acc[r] : 0.f;
            g2[ot] = acc;
        }
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
            store_fm(D2, g2[ht], 32 * ht, H, B, P, base);
        }
        const bool g2ok = !dense && tiles_finite<HT>(g2);
#pragma unroll
        for (int ot = 0; ot < HT; ++ot) {
            f32x16 acc = tchain_from<HT>(g2ok ? kstart(nk2, HT, ot) : 0, Wl + BL.w2, HT, ot, tbh, g2, f32x16{});
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = ((m1 >> (ot * 16 + r)) & 1u) ? acc[r] : 0.f;
            g[ot] = acc;
        }
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
            store_fm(D1, g[ht], 32 * ht, H, B, P, base);
        }
        // gx = direct term (in the tile) + W1mᵀ δ1, accumulator layout rows = dims
        wave_lds_sync();
        const bool g1ok = !dense && tiles_finite<HT>(g);
#pragma unroll
        for (int ot = 0; ot < 2; ++ot) {
            if (ot < NKC) {
                const f32x16 gx = tchain_from<HT>(g1ok ? kstart(nk1, HT, ot) : 0, Wl + BL.w1, NKC, ot, tb1, g, f32x16{});
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    float* px = xt + col * S + 32 * ot + crow(r, h);
                    *px = *px + gx[r];
                }
            }
        }

        // ---- gx rows out of the tile, coalesced ----
        wave_lds_sync();
        {
            const auto ro = __builtin_amdgcn_make_buffer_rsrc(gin + base * d, 0, rows * rowb, 0x00020000);
#pragma unroll
            for (int r = 0; r < 32; ++r)
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(xt[r * S + lane]), ro, voff, r * rowb, 0);
        }
        wave_lds_sync();
    }
}


// ---- general shapes: any d (<= 4096), H <= 128 (made_bwdw_kernel) ---------------------------
// Same math as made_bwd_kernel, for the shapes whose [32 x d] x tile does not fit a wave's LDS
// (e.g. the IAF(784, 64) sampling direction under autograd): the input layer streams x through a
// [32 x 32] LDS stage per 32-dimension chunk; the output layer runs per (mu, alpha) block pair j
// in two passes — pass A only sums clamp(alpha) (the log-det clamp decides every block's
// gradient), pass B recomputes the block, runs the epilogue backward on the staged x / gz chunk,
// writes the direct dL/dx term of the chunk, the block's δ rows, and folds δ into the layer-3
// adjoint at once (gh3 += W4mᵀ δ_j, MFMA); after the hidden chain, gx += W1mᵀ δ1 is added per
// input chunk (read-modify-write of the wave's own gx rows).
constexpr int kBwdwWaves = 4;
constexpr int kS32 = 33;  // [32 samples][33] stage stride (conflict-free column reads)

__device__ __forceinline__ void stage32_in(const float* __restrict__ src, int64_t base, int d, int64_t B, int dim0,
                                           float* st) {
    const int lane = lane_id();
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
        const int idx = i * 64 + lane, sm = idx >> 5, dd = idx & 31;
        const int64_t row = base + sm;
        const int dim = dim0 + dd;
        st[sm * kS32 + dd] = (row < B && dim < d) ? src[row * d + dim] : 0.f;
    }
}

__device__ __forceinline__ void stage32_out(float* __restrict__ dst, int64_t base, int d, int64_t B, int dim0,
                                            const float* st) {
    const int lane = lane_id();
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
        const int idx = i * 64 + lane, sm = idx >> 5, dd = idx & 31;
        const int64_t row = base + sm;
        const int dim = dim0 + dd;
        if (row < B && dim < d) dst[row * d + dim] = st[sm * kS32 + dd];
    }
}

template <int HT, int VAR>
__global__ __launch_bounds__(64 * kBwdwWaves) void made_bwdw_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, const float* __restrict__ gout,
    const float* __restrict__ gld_in, float* __restrict__ gin, float* __restrict__ acts, int64_t B, int d,
    int H, int64_t ntiles) {
    const MadeLayout L = made_layout(d, HT);
    constexpr bool IAF = VAR == NFX_IAF_FORWARD;
    constexpr float ALO = IAF ? -2.f : -3.f, AHI = IAF ? 2.f : 3.f, LDLIM = IAF ? 50.f : 100.f;
    extern __shared__ f32x4 lds4[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float* xt = reinterpret_cast<float*>(lds4) + wave * 2 * 32 * kS32;
    float* gt = xt + 32 * kS32;
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    const int NKC = L.NKC, NJ = L.NJ;
    const int64_t P = B;  // factor row pitch (nfx_made_factor_pitch)
    float* D4 = acts;
    float* D3 = D4 + (int64_t)2 * d * P;
    float* D2 = D3 + (int64_t)H * P;
    float* D1 = D2 + (int64_t)H * P;
    float* H3 = D1 + (int64_t)H * P;
    float* H2 = H3 + (int64_t)(H + 1) * P;
    float* H1 = H2 + (int64_t)(H + 1) * P;
    float* X1 = H1 + (int64_t)(H + 1) * P;

    for (int64_t t = (int64_t)blockIdx.x * kBwdwWaves + wave; t < ntiles; t += (int64_t)gridDim.x * kBwdwWaves) {
        const int64_t base = t * 32;
        const float* Wf = packed + opaque_zero();
        const bool live = base + col < B;
        // ---- layer 1 over 32-dimension chunks of x (x rows also written feature-major) ----
        f32x16 h1[HT];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) h1[ht] = load_bias16(Wf + L.b1 + ht * 32, h);
        for (int kc = 0; kc < NKC; ++kc) {
            wave_lds_sync();
            stage32_in(in, base, d, B, 32 * kc, xt);
            wave_lds_sync();
#pragma unroll
            for (int g = 0; g < 4; ++g) {
#pragma unroll
                for (int ht = 0; ht < HT; ++ht) {
                    const f32x4 w = *reinterpret_cast<const f32x4*>(Wf + L.w1 + ((ht * 4 * NKC + kc * 4 + g) * 64 + lane) * 4);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) h1[ht] = mfma32(w[rr], xt[col * kS32 + 8 * g + 2 * rr + h], h1[ht]);
                }
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int dim = 32 * kc + 2 * i + h;
                if (live && dim < d) X1[(int64_t)dim * P + base + col] = xt[col * kS32 + 2 * i + h];
            }
        }
#pragma unroll
        for (int ht = 0; ht < HT; ++ht)
#pragma unroll
            for (int r = 0; r < 16; ++r) h1[ht][r] = trelu(h1[ht][r]);
        f32x16 h2[HT], h3[HT];
        made_hidden1<HT>(Wf, L.w2, L.b2, h1, h2);
        uint32_t m1[HT], m2[HT], m3[HT];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
            m1[ht] = 0u;
#pragma unroll
            for (int r = 0; r < 16; ++r) m1[ht] |= (h1[ht][r] > 0.f ? 1u : 0u) << r;
            store_fm(H1, h1[ht], 32 * ht, H, B, P, base);
        }
        made_hidden1<HT>(Wf, L.w3, L.b3, h2, h3);
#pragma unroll
        for (int ht = 0; ht < HT; ++ht) {
            m2[ht] = m3[ht] = 0u;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                m2[ht] |= (h2[ht][r] > 0.f ? 1u : 0u) << r;
                m3[ht] |= (h3[ht][r] > 0.f ? 1u : 0u) << r;
            }
            store_fm(H2, h2[ht], 32 * ht, H, B, P, base);
            store_fm(H3, h3[ht], 32 * ht, H, B, P, base);
        }

        // ---- pass A: the log-det sum (alpha rows only) ----
        float asum0 = 0.f;
        for (int j = 0; j < NJ; ++j) {
            f32x16 al = load_bias16(Wf + L.b4 + (j * 2 + 1) * 32, h);
#pragma unroll
            for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) {
                    const f32x4 wa = *reinterpret_cast<const f32x4*>(Wf + L.w4 + ((((j * 2 + 1) * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) al = mfma32(wa[rr], h3[kt][4 * rq + rr], al);
                }
#pragma unroll
            for (int r = 0; r < 16; ++r) asum0 = asum0 + tclamp(al[r], ALO, AHI);
        }
        const float ssum = halves_sum(asum0, asum0);
        const float ldraw = IAF ? ssum : -ssum;
        const float gld = (lane < 32 && live) ? gld_in[base + col] : 0.f;
        float gld1 = nonfinite(ldraw) ? 0.f : gld;
        const float ld1 = nonfinite(ldraw) ? 0.f : ldraw;
        if (!(ld1 >= -LDLIM && ld1 <= LDLIM)) gld1 = 0.f;
        const float gld1s = __shfl(gld1, col, 64);

        // ---- pass B: per output block, epilogue backward + gh3 accumulation ----
        f32x16 g3[HT];
#pragma unroll
        for (int ot = 0; ot < HT; ++ot) g3[ot] = f32x16{};
        for (int j = 0; j < NJ; ++j) {
            f32x16 mu = load_bias16(Wf + L.b4 + (j * 2 + 0) * 32, h);
            f32x16 al = load_bias16(Wf + L.b4 + (j * 2 + 1) * 32, h);
#pragma unroll
            for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) {
                    const f32x4 wm = *reinterpret_cast<const f32x4*>(Wf + L.w4 + ((((j * 2 + 0) * HT + kt) * 4 + rq) * 64 + lane) * 4);
                    const f32x4 wa = *reinterpret_cast<const f32x4*>(Wf + L.w4 + ((((j * 2 + 1) * HT + kt) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        mu = mfma32(wm[rr], h3[kt][4 * rq + rr], mu);
                        al = mfma32(wa[rr], h3[kt][4 * rq + rr], al);
                    }
                }
            wave_lds_sync();
            stage32_in(in, base, d, B, 32 * j, xt);
            stage32_in(gout, base, d, B, 32 * j, gt);
            wave_lds_sync();
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int dd = crow(r, h);
                float* px = xt + col * kS32 + dd;
                const float xv = *px;
                const float gz = gt[col * kS32 + dd];
                const float alpha = al[r];
                if constexpr (IAF) {
                    const float m = mu[r];
                    const float a = tclamp(alpha, -2.f, 2.f);
                    const float e = exp_fast(a);
                    const float yr = xv * e + tclamp(m, -10.f, 10.f);
                    const bool bad = nonfinite(yr);
                    const float gyr = bad ? 0.f : gz;
                    *px = bad ? gz : gyr * e;
                    mu[r] = (m >= -10.f && m <= 10.f) ? gyr : 0.f;
                    al[r] = (alpha >= -2.f && alpha <= 2.f) ? gyr * xv * e + gld1s : 0.f;
                } else {
                    const float a = tclamp(alpha, -3.f, 3.f);
                    const float e = exp_fast(-a);
                    const float xm = xv - mu[r];
                    const float zr = xm * e;
                    const float gzr = nonfinite(zr) ? 0.f : gz;
                    const float ge = gzr * e;
                    *px = ge;
                    mu[r] = -ge;
                    al[r] = (alpha >= -3.f && alpha <= 3.f) ? -(gzr * xm * e) - gld1s : 0.f;
                }
            }
            wave_lds_sync();
            stage32_out(gin, base, d, B, 32 * j, xt);  // direct dL/dx term of the chunk
            store_fm(D4, mu, 32 * j, d, B, P, base);
            store_fm(D4 + (int64_t)d * P, al, 32 * j, d, B, P, base);
#pragma unroll
            for (int ot = 0; ot < HT; ++ot) {
#pragma unroll
                for (int which = 0; which < 2; ++which) {
                    const f32x16& dl = which ? al : mu;
#pragma unroll
                    for (int rq = 0; rq < 4; ++rq) {
                        const f32x4 w = *reinterpret_cast<const f32x4*>(
                            Wf + L.t4 + (((ot * 2 * NJ + 2 * j + which) * 4 + rq) * 64 + lane) * 4);
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr) g3[ot] = mfma32(w[rr], dl[4 * rq + rr], g3[ot]);
                    }
                }
            }
        }
        // ---- hidden chain ----
#pragma unroll
        for (int ot = 0; ot < HT; ++ot) {
#pragma unroll
            for (int r = 0; r < 16; ++r) g3[ot][r] = ((m3[ot] >> r) & 1u) ? g3[ot][r] : 0.f;
            store_fm(D3, g3[ot], 32 * ot, H, B, P, base);
        }
        f32x16 g2[HT];
#pragma unroll
        for (int ot = 0; ot < HT; ++ot) {
            f32x16 acc = chain_gmem<HT>(Wf + L.t3, ot, HT, g3, f32x16{});
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = ((m2[ot] >> r) & 1u) ? acc[r] : 0.f;
            g2[ot] = acc;
            store_fm(D2, acc, 32 * ot, H, B, P, base);
        }
#pragma unroll
        for (int ot = 0; ot < HT; ++ot) {
            f32x16 acc = chain_gmem<HT>(Wf + L.t2, ot, HT, g2, f32x16{});
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = ((m1[ot] >> r) & 1u) ? acc[r] : 0.f;
            g3[ot] = acc;  // δ1
            store_fm(D1, acc, 32 * ot, H, B, P, base);
        }
        // ---- gx += W1mᵀ δ1 per input chunk ----
        for (int kc = 0; kc < NKC; ++kc) {
            const f32x16 gx = chain_gmem<HT>(Wf + L.t1, kc, HT, g3, f32x16{});
            wave_lds_sync();
            stage32_in(gin, base, d, B, 32 * kc, xt);
            wave_lds_sync();
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float* px = xt + col * kS32 + crow(r, h);
                *px = *px + gx[r];
            }
            wave_lds_sync();
            stage32_out(gin, base, d, B, 32 * kc, xt);
        }
        wave_lds_sync();
    }
}

}  // namespace nfx

using namespace nfx;

extern "C" int nfx_made_pack_backward(const NfxMlpRaw* net, int d, int H, float* packed, void* stream) {
    if (!net || !packed) return set_error(NFX_EINVAL, "made_pack_backward: null pointer");
    if (d <= 0 || d > 4096 || H <= 0 || H > 256)
        return set_error(NFX_EUNSUPPORTED, "made_pack_backward: d=%d H=%d outside d<=4096, H<=256", d, H);
    const MadeLayout L = made_layout(d, (H + 31) / 32);
    int blocks = (L.rimg - L.t4 + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    made_bwd_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(*net, d, H, packed);
    return check_launch("made_bwd_pack_kernel");
}

// Largest batch one backward call accepts: every feature-major factor region (at most
// max(2d, d + 1, 32 HT + 1) rows of pitch B) must stay within a 32-bit buffer range, and the
// weight-gradient contraction reads 32-row tiles with 32-bit offsets (32 B 4 < 2^31).
extern "C" int64_t nfx_made_backward_max_batch(int d, int H) {
    if (d <= 0 || H <= 0) return 0;
    const int64_t HT = (H + 31) / 32;
    int64_t rows = 2 * (int64_t)d;
    if (d + 1 > rows) rows = d + 1;
    if (32 * HT + 1 > rows) rows = 32 * HT + 1;
    const int64_t lim = ((int64_t)1 << 31) - 1;
    const int64_t b1 = lim / (4 * rows), b2 = lim / (4 * 32);
    return b1 < b2 ? b1 : b2;
}

extern "C" size_t nfx_made_backward_factor_floats(int64_t B, int d, int H) {
    if (B < 0 || d <= 0 || H <= 0) return 0;
    return (size_t)B * (size_t)(3 * d + 6 * H + 4);
}

extern "C" int nfx_made_affine_backward(const float* packed, const float* in, const float* grad_out,
                                        const float* grad_log_det, float* grad_in, float* factors,
                                        int64_t B, int d, int H, int variant, void* stream) {
    if (variant != NFX_MAF_INVERSE && variant != NFX_IAF_FORWARD)
        return set_error(NFX_EUNSUPPORTED, "made_affine_backward: parallel directions only (NFX_MAF_INVERSE, "
                                           "NFX_IAF_FORWARD); the sequential ones are nfx_made_seq_backward");
    if (B < 0 || d <= 0 || H <= 0) return set_error(NFX_EINVAL, "made_affine_backward: bad shape");
    if (d > 4096 || H > 128)
        return set_error(NFX_EUNSUPPORTED, "made_affine_backward: d=%d H=%d outside d<=4096, H<=128", d, H);
    if (B > nfx_made_backward_max_batch(d, H))
        return set_error(NFX_EUNSUPPORTED, "made_affine_backward: B=%lld above nfx_made_backward_max_batch(%d, %d) = "
                                           "%lld (32-bit factor offsets); split the batch", (long long)B, d, H,
                         (long long)nfx_made_backward_max_batch(d, H));
    if (B == 0) return NFX_OK;
    if (!packed || !in || !grad_out || !grad_log_det || !grad_in || !factors)
        return set_error(NFX_EINVAL, "made_affine_backward: null pointer");
    const int HT = (H + 31) / 32;
    if (d > 64 || H > 64) {  // general shapes: x streamed in 32-dimension chunks
        typedef void (*bwdw_t)(const float*, const float*, const float*, const float*, float*, float*, int64_t, int,
                               int, int64_t);
        const bool iaf = variant == NFX_IAF_FORWARD;
        bwdw_t kw = nullptr;
        switch (HT) {
            case 1: kw = iaf ? made_bwdw_kernel<1, NFX_IAF_FORWARD> : made_bwdw_kernel<1, NFX_MAF_INVERSE>; break;
            case 2: kw = iaf ? made_bwdw_kernel<2, NFX_IAF_FORWARD> : made_bwdw_kernel<2, NFX_MAF_INVERSE>; break;
            case 3: kw = iaf ? made_bwdw_kernel<3, NFX_IAF_FORWARD> : made_bwdw_kernel<3, NFX_MAF_INVERSE>; break;
            default: kw = iaf ? made_bwdw_kernel<4, NFX_IAF_FORWARD> : made_bwdw_kernel<4, NFX_MAF_INVERSE>; break;
        }
        const size_t ldsw = (size_t)kBwdwWaves * 2 * 32 * kS32 * sizeof(float);
        const int64_t nt = (B + 31) / 32;
        const int gw = resident_grid((const void*)kw, 64 * kBwdwWaves, ldsw, (nt + kBwdwWaves - 1) / kBwdwWaves);
        kw<<<gw, 64 * kBwdwWaves, ldsw, (hipStream_t)stream>>>(packed, in, grad_out, grad_log_det, grad_in, factors, B,
                                                                d, H, nt);
        return check_launch("made_bwdw_kernel");
    }
    const MadeLayout L = made_layout(d, HT);
    (void)L;
    const bool iaf = variant == NFX_IAF_FORWARD;
    const int64_t ntiles = (B + 31) / 32;
    const bool small = ntiles <= (int64_t)kBwdWavesSmall * num_cus();
    const int nw = small ? kBwdWavesSmall : kBwdWaves;
    const size_t lds = ((size_t)bwd_lds(d, HT).total + (size_t)nw * 32 * kTileStride) * sizeof(float);
    const void* k;
    if (small)
        k = HT == 1 ? (iaf ? (const void*)made_bwd_kernel<1, NFX_IAF_FORWARD, kBwdWavesSmall>
                           : (const void*)made_bwd_kernel<1, NFX_MAF_INVERSE, kBwdWavesSmall>)
                    : (iaf ? (const void*)made_bwd_kernel<2, NFX_IAF_FORWARD, kBwdWavesSmall>
                           : (const void*)made_bwd_kernel<2, NFX_MAF_INVERSE, kBwdWavesSmall>);
    else
        k = HT == 1 ? (iaf ? (const void*)made_bwd_kernel<1, NFX_IAF_FORWARD, kBwdWaves>
                           : (const void*)made_bwd_kernel<1, NFX_MAF_INVERSE, kBwdWaves>)
                    : (iaf ? (const void*)made_bwd_kernel<2, NFX_IAF_FORWARD, kBwdWaves>
                           : (const void*)made_bwd_kernel<2, NFX_MAF_INVERSE, kBwdWaves>);
    int rc = prepare_lds(k, lds);
    if (rc) return rc;
    const int threads = 64 * nw;
    const int grid = resident_grid(k, threads, lds, (ntiles + nw - 1) / nw);
    hipStream_t s = (hipStream_t)stream;
    typedef void (*bwd_t)(const float*, const float*, const float*, const float*, float*, float*, int64_t, int, int,
                          int64_t);
    reinterpret_cast<bwd_t>(const_cast<void*>(k))<<<grid, threads, lds, s>>>(packed, in, grad_out, grad_log_det, grad_in,
                                                                          factors, B, d, H, ntiles);
    return check_launch("made_bwd_kernel");
}
