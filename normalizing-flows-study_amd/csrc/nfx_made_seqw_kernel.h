// Sequential MADE-affine directions with ONE WAVE PER SAMPLE (MAF.forward = sampling,
// IAF.inverse = density; H <= 64) — the strong-scaling layout of made_seqs_kernel.
//
// Reference: masked_autoregressive_flow.py:46-78, inverse_autoregressive_flow.py:65-103 (d full
// MADE calls on the partially filled vector). Same math and same one-MADE-evaluation schedule as
// made_seqs_kernel (nfx_made_seqs_kernel.h: units complete when the input of their degree is
// known; the steps of a segment between two completions share h3 and are evaluated as one
// chunk of up to 16 steps), but a sample gets all 64 lanes instead of 16, so the chain of ~d/12
// dependent chunks a sample must run is ~4x shorter per chunk — the batch no longer has to be
// large for the GPU to be fast (8,192 samples at 4 per wave are only 2 waves per SIMD; 1,024
// samples, the 8-way shard of cfg5i, would run on 32 CUs):
//   1. lane (rq, j) = (lane >> 4, lane & 15) forms step j's mu/alpha partial dot products over
//      the completed ranks of quads 16 m + 4 rq .. + 3 (h3 by rank in LDS, zero until complete;
//      W4 (mu, alpha) pair rows by rank, packed FMAs), then the 4 rank quarters meet with two
//      lane swaps (v_permlane16_swap, v_permlane32_swap): every row holds the full mu/alpha;
//   2. every row evaluates the chunk's affine maps (row 0 stores them);
//   3. lane u owns the unit of completion rank u: its layer-1 pre-activation takes the chunk's
//      new inputs (DPP row broadcasts) as rank-1 updates, in step order (one FMA per step);
//   4. the units of degree D_{g+1} complete: h1 on the owning lane, then layer 2 and layer 3 of
//      each as a 64-lane product + wave all-reduce (4 DPP row stages + 2 lane swaps, every lane
//      gets the bit-identical sum), h3 written to the wave's LDS row.
// Steps are staged exactly as in made_seqs_kernel (64-step blocks of the block-ready image,
// 16-byte LDS-DMA into a double buffer, the next block in flight; blocks end at segment ends);
// a workgroup of NWV waves = NWV samples shares them. Log-det and the fused Gaussian term are
// summed in step order; non-finite steps poison the later ones exactly as made_seqs_kernel does.
#pragma once
#include "nfx_made_seqs_kernel.h"

namespace nfx {

// per wave: x, z, alpha block tiles; the h3 row; 64 floats where masked stores land
constexpr int kSeqwTile = 3 * kSeqsStep + kSeqsH3 + 64;

__host__ __device__ inline int seqw_blkf(int Hp) { return kSeqsStep * Hp + kSeqsStep * seqs_w4_stride(Hp) + 2 * kSeqsStep; }
// LDS: tables (5 Hp) | W2, W3 rank-ordered images (2 Hp^2) | two staged blocks | per-wave tiles
__host__ __device__ inline int seqw_lds_floats(int Hp, int nwv) {
    return 5 * Hp + 2 * Hp * Hp + 2 * seqw_blkf(Hp) + nwv * kSeqwTile;
}

// Sum over all 64 lanes; every lane gets the same (bit-identical) value.
__device__ __forceinline__ float wave_allsum(float v) {
    v = row16_allsum(v);
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(t[0]) + __uint_as_float(t[1]);
}
// Sum over the 4 rows (lanes j, 16 + j, 32 + j, 48 + j), every row gets it.
__device__ __forceinline__ float rows4_sum(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(t[0]) + __uint_as_float(t[1]);
}

template <int HT, int VAR, bool LOGP, int NWV>
__global__ __launch_bounds__(NWV * 64) void made_seqw_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d, int H, int accumulate, float* __restrict__ logp,
    double* __restrict__ partials, float cgauss) {
    constexpr int Hp = 32 * HT;
    constexpr int UPL = Hp / 16;
    constexpr int RS4 = seqs_w4_stride(Hp);
    constexpr int W4F = kSeqsStep * Hp;
    constexpr int B4F = W4F + kSeqsStep * RS4;
    const int BLKF = seqw_blkf(Hp);
    const MadeLayout L = made_layout(d, HT);
    const SeqsLds S = seqs_lds(Hp);  // image offsets (w2, w3, tab) and the table layout
    extern __shared__ f32x4 lds4[];
    float* lds = reinterpret_cast<float*>(lds4);
    const float* P = packed;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = lane_id(), rq = lane >> 4, jl = lane & 15;
    const bool own = lane < Hp;                                   // lane owns the unit of rank `lane`
    const int posu = own ? (lane % 16) * UPL + lane / 16 : 0;    // its position (w1t / W2 / W3 column)

    const float* img = P + L.rimg;
    {
        const f32x4* src = reinterpret_cast<const f32x4*>(img + S.tab);
        for (int i = threadIdx.x; i < 5 * Hp / 4; i += NWV * 64) lds4[i] = src[i];
        // W2 / W3 rows by completion rank (columns by position): the completion chain reads them
        // from LDS, not L2 — an L2 round trip per completing unit would sit on every chunk's chain
        const f32x4* sw = reinterpret_cast<const f32x4*>(img + S.w2);
        for (int i = threadIdx.x; i < 2 * Hp * Hp / 4; i += NWV * 64) lds4[5 * Hp / 4 + i] = sw[i];
    }
    __syncthreads();
    const float* w23 = lds + 5 * Hp;  // [W2 rank rows | W3 rank rows], S.w3 - S.w2 = Hp * Hp
    const int tl = lane & (Hp - 1);
    const int degv = (int)lds[S.deg + tl];
    const int gendv = (int)lds[S.gend + tl];
    const int b2v = __float_as_int(lds[S.b2 + tl]);
    const int b3v = __float_as_int(lds[S.b3 + tl]);
    const float b1u = own ? lds[S.b1 + posu] : 0.f;
    float* blk0 = lds + 5 * Hp + 2 * Hp * Hp;
    float* xin_t = blk0 + 2 * BLKF + wave * kSeqwTile;
    float* zout_t = xin_t + kSeqsStep;
    float* at_t = zout_t + kSeqsStep;
    float* h3_t = at_t + kSeqsStep;   // [kSeqsH3] h3 by rank (0 until complete)
    float* dump = h3_t + kSeqsH3;     // [64]

    auto blk_end = [&](int i0) -> int {
        const int lim = i0 + kSeqsStep;
        if (lim >= d) return d;
        const int e = degv + 1;
        const uint64_t m = __ballot(lane < H && e > i0 && e <= lim);
        if (m == 0) return lim;
        return __builtin_amdgcn_readlane(e, 63 - __builtin_clzll(m));
    };
    constexpr int N1 = kSeqsStep * Hp / 256, N4 = kSeqsStep * RS4 / 256;
    static_assert(N1 * 256 == kSeqsStep * Hp && N4 * 256 == kSeqsStep * RS4, "whole 1 KiB pieces");
    auto blk_stage = [&](int i0, int buf) {
        float* dst = blk0 + buf * BLKF;
        const float* sw1 = P + L.sw1 + (size_t)i0 * Hp;
        const float* sw4 = P + L.sw4 + (size_t)i0 * RS4;
        for (int j = wave; j < N1 + N4 + 2; j += NWV) {
            if (j < N1) {
                seqs_dma_x4(sw1 + 256 * j + 4 * lane, dst + 256 * j);
            } else if (j < N1 + N4) {
                seqs_dma_x4(sw4 + 256 * (j - N1) + 4 * lane, dst + W4F + 256 * (j - N1));
            } else {
                const int jb = j - N1 - N4;
                seqs_dma_dword(P + L.sb4 + (size_t)jb * (d + kSeqsPadRows) + i0 + lane, dst + B4F + 64 * jb);
            }
        }
    };
    // the wave's sample row of the block: one coalesced range-checked load (lane l: step i0 + l)
    auto x_load = [&](int64_t s, int i0, int n) -> float {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in) + (s < B ? s : 0) * d, 0,
                                                          s < B ? d * 4 : 0, 0x00020000);
        const int voff = lane < n ? (i0 + lane) * 4 : (int)0x7FFFFFF0;
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, 0, 0));
    };

#ifdef NFX_SEQW_TIMING
    long long tacc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    long long tmark = clock64();
#define NFX_WMARK(k) do { const long long t_ = clock64(); tacc[k] += t_ - tmark; tmark = t_; } while (0)
#else
#define NFX_WMARK(k) do { } while (0)
#endif
    double lpacc = 0.0;
    for (int64_t gb = (int64_t)blockIdx.x * NWV; gb < B; gb += (int64_t)gridDim.x * NWV) {
        const int64_t s = gb + wave;
        const bool valid = s < B;
        float pre1 = b1u, h1 = 0.f, h2 = 0.f;
        for (int e = lane; e < kSeqsH3; e += 64) h3_t[e] = 0.f;
        float ld = 0.f, zsq = 0.f;
        bool poisoned = false;
        int gi = 0;
        int nextdeg = H > 0 ? __builtin_amdgcn_readlane(degv, 0) : d;

        int i0 = 0, n = blk_end(0), buf = 0;
        float xr = x_load(s, 0, n);
        __syncthreads();  // previous group's readers of the staging buffers are done
        blk_stage(0, 0);
        seqs_dma_wait();
        __syncthreads();

        while (i0 < d) {
            const float* blk = blk0 + buf * BLKF;
            const float* w1b = blk;
            const float* w4b = blk + W4F;
            const float* bmb = blk + B4F;
            const float* bab = bmb + kSeqsStep;
            xin_t[lane] = xr;
            if (lane >= n) zout_t[lane] = at_t[lane] = 0.f;
            const int i0n = i0 + n;
            NFX_WMARK(7);  // tiles
            const int nn = i0n < d ? blk_end(i0n) - i0n : 0;
            NFX_WMARK(8);  // next block end (ballot)
            if (nn > 0) {
                blk_stage(i0n, buf ^ 1);
                xr = x_load(s, i0n, nn);
            }
            seqs_lds_order();
            NFX_WMARK(6);  // block start: tiles, next block's DMA and x loads
            for (int ii = 0; ii < n;) {
                const int i = i0 + ii;
                int nc = n - ii < 16 ? n - ii : 16;
                if (nextdeg - i + 1 < nc) nc = nextdeg - i + 1;
                const int rj = ii + jl;
                // step inputs and biases first: nothing below waits on their LDS round trip
                const float xin = xin_t[rj];
                const float bmu = bmb[rj], bal = bab[rj];
                // 1. step rj's mu/alpha over all ranks of this lane's quads: a fixed, fully unrolled
                // trip (h3 is exactly 0 for the ranks that have not completed, so they add zeros) —
                // every LDS read issues at once instead of one dependent round trip per quad
                f32x2 acc0 = {0.f, 0.f}, acc1 = {0.f, 0.f};
                {
                    const float* wr = w4b + rj * RS4 + 8 * rq;
                    const float* hr = h3_t + 4 * rq;
#pragma unroll
                    for (int m = 0; m < Hp / 16; ++m) {
                        const f32x4 hv = *reinterpret_cast<const f32x4*>(hr + 16 * m);
                        const f32x4 w0 = *reinterpret_cast<const f32x4*>(wr + 32 * m);
                        const f32x4 w1 = *reinterpret_cast<const f32x4*>(wr + 32 * m + 4);
                        acc0 = pk_fma(f32x2{w0[0], w0[1]}, hv[0], acc0);
                        acc1 = pk_fma(f32x2{w0[2], w0[3]}, hv[1], acc1);
                        acc0 = pk_fma(f32x2{w1[0], w1[1]}, hv[2], acc0);
                        acc1 = pk_fma(f32x2{w1[2], w1[3]}, hv[3], acc1);
                    }
                }
                // step-3 rows and the next completing unit's W2/W3 entries (latency overlaps 1-2)
                float w1v[16];
#pragma unroll
                for (int j = 0; j < 16; ++j) w1v[j] = own ? w1b[(ii + j) * Hp + posu] : 0.f;
                const float w2n = own && gi < Hp ? w23[gi * Hp + posu] : 0.f;
                const float w3n = own && gi < Hp ? w23[Hp * Hp + gi * Hp + posu] : 0.f;
                const float b2n = lds[S.b2 + (gi < Hp ? gi : 0)], b3n = lds[S.b3 + (gi < Hp ? gi : 0)];
                float mu = rows4_sum(acc0[0] + acc1[0]) + bmu;
                float al = rows4_sum(acc0[1] + acc1[1]) + bal;
                NFX_WMARK(0);  // dot products + row reduction
                // 2. step rj's affine map (every row; row 0 stores)
                const bool vj = jl < nc;
                mu = poisoned ? __builtin_nanf("") : mu;
                al = poisoned ? __builtin_nanf("") : al;
                float vi, vo, a;
                if constexpr (VAR == NFX_MAF_FORWARD) {
                    a = tclamp(al, -3.f, 3.f);
                    vi = xin * exp_fast(a) + mu;
                } else {
                    a = tclamp(al, -2.f, 2.f);
                    const float m = tclamp(mu, -10.f, 10.f);
                    vi = (xin - m) * exp_fast(-a);
                }
                const uint64_t bad = __ballot(vj && nonfinite(vi));
                const unsigned rowbad = (unsigned)bad & 0xFFFFu;  // every row holds the same steps
                const bool kill = rowbad != 0u && jl > __builtin_ctz(rowbad | 0x10000u);
                vi = kill ? __builtin_nanf("") : vi;
                a = kill ? __builtin_nanf("") : a;
                poisoned = poisoned || rowbad != 0u;
                if constexpr (VAR == NFX_MAF_FORWARD) vo = nonfinite(vi) ? 0.f : vi;
                else vo = nonfinite(vi) ? xin : vi;
                {
                    const bool st = vj && rq == 0;
                    *(st ? zout_t + rj : dump + lane) = vo;
                    *(st ? at_t + rj : dump + lane) = a;
                }
                NFX_WMARK(1);  // affine map, poison ballot, stores
                // 3. rank-1 updates of the owned unit's layer-1 pre-activation, step order
                float cv[16];
                seqs_row_bcast16(vj ? vi : 0.f, cv);
#pragma unroll
                for (int j = 0; j < 16; ++j) pre1 = fmaf(w1v[j], cv[j], pre1);
                seqs_lds_order();
                NFX_WMARK(2);  // broadcasts + rank-1 updates
                // 4. the units of degree nextdeg (ranks gi .. q-1) complete
                if (i + nc - 1 == nextdeg) {
                    const int q = __builtin_amdgcn_readlane(gendv, gi);
                    if (lane >= gi && lane < q) h1 = trelu(pre1);
                    {
                        const float v = wave_allsum(w2n * h1);
                        const float h2p = trelu(v + b2n);
                        if (lane == gi) h2 = h2p;
                    }
                    for (int p = gi + 1; p < q; ++p) {
                        const float w = own ? w23[p * Hp + posu] : 0.f;
                        const float v = wave_allsum(w * h1);
                        const float h2p = trelu(v + __int_as_float(__builtin_amdgcn_readlane(b2v, p)));
                        if (lane == p) h2 = h2p;
                    }
                    {
                        const float v = wave_allsum(w3n * h2);
                        const float h3p = trelu(v + b3n);
                        if (lane == 0) h3_t[gi] = h3p;
                    }
                    for (int p = gi + 1; p < q; ++p) {
                        const float w = own ? w23[Hp * Hp + p * Hp + posu] : 0.f;
                        const float v = wave_allsum(w * h2);
                        const float h3p = trelu(v + __int_as_float(__builtin_amdgcn_readlane(b3v, p)));
                        if (lane == 0) h3_t[p] = h3p;
                    }
                    seqs_lds_order();
                    gi = q;
                    nextdeg = gi < H ? __builtin_amdgcn_readlane(degv, gi) : d;
                }
                NFX_WMARK(3);  // completion
                ii += nc;
            }
            seqs_lds_order();
            // log-det and z^2 of the block in step order (steps past the block hold zeros)
#pragma unroll 4
            for (int j = 0; j < kSeqsStep; j += 4) {
                const f32x4 ta = *reinterpret_cast<const f32x4*>(at_t + j);
                const f32x4 tz = *reinterpret_cast<const f32x4*>(zout_t + j);
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    if constexpr (VAR == NFX_MAF_FORWARD) ld = ld + ta[c];
                    else ld = ld - ta[c];
                    if constexpr (LOGP) zsq = gauss_sq(zsq, tz[c]);
                }
            }
            if (valid && lane < n) out[s * d + i0 + lane] = zout_t[lane];
            NFX_WMARK(4);  // block sums + output row
            seqs_dma_wait();
            __syncthreads();
            NFX_WMARK(5);  // vmcnt(0) + barrier
            i0 = i0n;
            n = nn;
            buf ^= 1;
        }
        if (valid && lane == 0) {
            if (nonfinite(ld)) ld = 0.f;
            ld = (VAR == NFX_MAF_FORWARD) ? tclamp(ld, -100.f, 100.f) : tclamp(ld, -50.f, 50.f);
            const float ldt = accumulate ? logdet[s] + ld : ld;
            logdet[s] = ldt;
            if constexpr (LOGP) {
                const float lp = gauss_lp(zsq, cgauss, ldt);
                logp[s] = lp;
                lpacc += (double)lp;
            }
        }
    }
#ifdef NFX_SEQW_TIMING
    // timing build only: workgroup 0's first lane overwrites sample 0's first outputs
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (int k = 0; k < 9; ++k) out[k] = (float)tacc[k];
#endif
    if constexpr (LOGP) {
        const double t = block_sum_f64<NWV * 64>(lpacc);
        if (threadIdx.x == 0) partials[blockIdx.x] = t;
    }
}

typedef void (*made_seqw_kernel_t)(const float*, const float*, float*, float*, int64_t, int, int, int, float*,
                                   double*, float);

}  // namespace nfx
