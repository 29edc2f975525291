// Sequential MADE-affine directions with ONE WAVE PER SAMPLE (MAF.forward = sampling,
// IAF.inverse = density; H <= 64) — the strong-scaling layout of made_seqs_kernel.
//
// Reference: masked_autoregressive_flow.py:46-78, inverse_autoregressive_flow.py:65-103 (d full
// MADE calls on the partially filled vector). Same math and same one-MADE-evaluation schedule as
// made_seqs_kernel (nfx_made_seqs_kernel.h: units complete when the input of their degree is
// known; the steps of a segment between two completions share h3 and are evaluated as one
// chunk of up to 16 steps), but a sample gets all 64 lanes instead of 16. A sample's time is its
// chain of ~d/12 dependent chunks, each a string of dependent instructions (wave64 issues in
// order), so the kernel is built to keep that string short:
//   1. lane (rq, j) = (lane >> 4, lane & 15) forms step j's mu/alpha partial dot products over
//      ranks 16 m + 4 rq .. + 3 (h3 by rank in REGISTERS — no LDS round trip on the chain; W4
//      (mu, alpha) pair rows prefetched into registers during the previous chunk), then the 4
//      row partials meet with two lane swaps (v_permlane16_swap, v_permlane32_swap);
//   2. every row evaluates the chunk's affine maps; row 0 stores the outputs to global memory
//      directly and the lanes keep per-lane log-det partials;
//   3. lane u owns the unit of completion rank u: its layer-1 pre-activation takes the chunk's
//      new inputs (DPP row broadcasts) as rank-1 updates;
//   4. the unit of degree D_{g+1} completes: its layer-2 and layer-3 sums over the units that
//      completed BEFORE it (final h1 / h2) are all-reduced off the chain while steps 1-3 run, so
//      on the chain only the diagonal terms remain: h1 = relu(pre1), h2 = relu(P2 + W2_gg h1 +
//      b2), h3 = relu(P3 + W3_gg h2 + b3). (Several units of one degree take the general path:
//      64-lane products + wave all-reduces, every lane gets the bit-identical sum.)
// Steps are staged as in made_seqs_kernel (64-step blocks of the block-ready image, 16-byte
// LDS-DMA into a double buffer, the next block in flight) by a separate staging wave, which also
// sums the fused Gaussian term's z^2 in step order (as nfx_gauss_logprob does) one block behind;
// the NWV compute waves (= NWV samples) of a workgroup share the staged blocks. Non-finite steps
// poison the later ones exactly as made_seqs_kernel does.
#pragma once
#include "nfx_made_seqs_kernel.h"

namespace nfx {

// per compute wave: the x block tile and two z block tiles (alternate blocks); then one z^2 sum
// per sample slot
constexpr int kSeqwTile = 3 * kSeqsStep;

__host__ __device__ inline int seqw_blkf(int Hp) { return kSeqsStep * Hp + kSeqsStep * seqs_w4_stride(Hp) + 2 * kSeqsStep; }
// LDS: tables (5 Hp) | W2, W3 rank-ordered images (2 Hp^2) | two staged blocks | per-wave tiles | z^2 sums
__host__ __device__ inline int seqw_lds_floats(int Hp, int nwv) {
    return 5 * Hp + 2 * Hp * Hp + 2 * seqw_blkf(Hp) + nwv * kSeqwTile + 16;
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
// Workgroup barrier over LDS only: unlike __syncthreads() it does not wait for the wave's global
// stores (vmcnt), which the compute waves leave in flight.
__device__ __forceinline__ void seqw_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// The next chunk's W4 rows, biases and inputs, read one chunk ahead.
template <int NM>
struct SeqwOps {
    f32x4 w4[2 * NM];  // step rj's (mu, alpha) pairs for ranks 16 m + 4 rq + c
    float xin, bmu, bal;
};

// Workgroup = NWV compute waves (one sample each) + one staging wave. The staging wave issues the
// LDS-DMA of every block and sums z^2 of the finished blocks in step order (LOGP), so the compute
// waves' instruction streams hold only the sample's dependent chain.
template <int HT, int VAR, bool LOGP, int NWV>
__global__ __launch_bounds__((NWV + 1) * 64) void made_seqw_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d, int H, int accumulate, float* __restrict__ logp,
    double* __restrict__ partials, float cgauss) {
    constexpr int Hp = 32 * HT;
    constexpr int UPL = Hp / 16;
    constexpr int NM = Hp / 16;  // rank groups of 16: h3r[4 m + c] = h3 of rank 16 m + 4 rq + c
    constexpr int RS4 = seqs_w4_stride(Hp);
    constexpr int W4F = kSeqsStep * Hp;
    constexpr int B4F = W4F + kSeqsStep * RS4;
    constexpr int N1 = kSeqsStep * Hp / 256, N4 = kSeqsStep * RS4 / 256;
    static_assert(N1 * 256 == kSeqsStep * Hp && N4 * 256 == kSeqsStep * RS4, "whole 1 KiB pieces");
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
        for (int i = threadIdx.x; i < 5 * Hp / 4; i += (NWV + 1) * 64) lds4[i] = src[i];
        // W2 / W3 rows by completion rank (columns by position)
        const f32x4* sw = reinterpret_cast<const f32x4*>(img + S.w2);
        for (int i = threadIdx.x; i < 2 * Hp * Hp / 4; i += (NWV + 1) * 64) lds4[5 * Hp / 4 + i] = sw[i];
    }
    __syncthreads();
    const float* w23 = lds + 5 * Hp;  // [W2 rank rows | W3 rank rows]
    const int tl = lane & (Hp - 1);
    const int degv = (int)lds[S.deg + tl];
    const int gendv = (int)lds[S.gend + tl];
    const int b2v = __float_as_int(lds[S.b2 + tl]);
    const int b3v = __float_as_int(lds[S.b3 + tl]);
    float* blk0 = lds + 5 * Hp + 2 * Hp * Hp;
    float* tiles = blk0 + 2 * BLKF;
    float* zsum_t = tiles + NWV * kSeqwTile;  // [16] z^2 per sample slot

    auto blk_end = [&](int i0) -> int {
        const int lim = i0 + kSeqsStep;
        if (lim >= d) return d;
        const int e = degv + 1;
        const uint64_t m = __ballot(lane < H && e > i0 && e <= lim);
        if (m == 0) return lim;
        return __builtin_amdgcn_readlane(e, 63 - __builtin_clzll(m));
    };
    double lpacc = 0.0;

    if (wave == NWV) {
        // ---------------- staging wave ----------------
        auto stage = [&](int i0, int buf) {
            float* dst = blk0 + buf * BLKF;
            const float* sw1 = P + L.sw1 + (size_t)i0 * Hp;
            const float* sw4 = P + L.sw4 + (size_t)i0 * RS4;
#pragma unroll 4
            for (int j = 0; j < N1; ++j) seqs_dma_x4(sw1 + 256 * j + 4 * lane, dst + 256 * j);
#pragma unroll 4
            for (int j = 0; j < N4; ++j) seqs_dma_x4(sw4 + 256 * j + 4 * lane, dst + W4F + 256 * j);
            seqs_dma_dword(P + L.sb4 + i0 + lane, dst + B4F);
            seqs_dma_dword(P + L.sb4 + (size_t)(d + kSeqsPadRows) + i0 + lane, dst + B4F + 64);
        };
        // step-order z^2 of sample slot `lane` over the block in tile `par`
        auto zsq_block = [&](int par, float z) -> float {
            if (lane < NWV) {
                const float* zt = tiles + lane * kSeqwTile + kSeqsStep * (1 + par);
#pragma unroll 4
                for (int j = 0; j < kSeqsStep; j += 4) {
                    const f32x4 tz = *reinterpret_cast<const f32x4*>(zt + j);
#pragma unroll
                    for (int c = 0; c < 4; ++c) z = gauss_sq(z, tz[c]);
                }
            }
            return z;
        };
        for (int64_t gb = (int64_t)blockIdx.x * NWV; gb < B; gb += (int64_t)gridDim.x * NWV) {
            float z = 0.f;
            int i0 = 0, n = blk_end(0), buf = 0, par = 0;
            seqw_lds_barrier();  // A: the previous group is done with the staging buffers
            stage(0, 0);
            seqs_dma_wait();
            seqw_lds_barrier();  // B: block 0 is in LDS
            bool prev = false;
            while (i0 < d) {
                const int i0n = i0 + n;
                const int nn = i0n < d ? blk_end(i0n) - i0n : 0;
                if (nn > 0) stage(i0n, buf ^ 1);
                if (LOGP && prev) z = zsq_block(par ^ 1, z);  // the block before this one
                seqs_dma_wait();
                seqw_lds_barrier();  // C: block done by every compute wave; the next one is in LDS
                prev = true;
                i0 = i0n;
                n = nn;
                buf ^= 1;
                par ^= 1;
            }
            if constexpr (LOGP) {
                z = zsq_block(par ^ 1, z);
                if (lane < NWV) zsum_t[lane] = z;
                seqw_lds_barrier();  // D: the sums are in LDS
            }
        }
    } else {
        // ---------------- compute waves: one sample each ----------------
        const float b1u = own ? lds[S.b1 + posu] : 0.f;
        float* xin_t = tiles + wave * kSeqwTile;
        auto x_load = [&](int64_t s, int i0, int n) -> float {
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in) + (s < B ? s : 0) * d, 0,
                                                              s < B ? d * 4 : 0, 0x00020000);
            const int voff = lane < n ? (i0 + lane) * 4 : (int)0x7FFFFFF0;
            return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, 0, 0));
        };
        // operands of the chunk at block position ii (rows past the block clamp to its last row:
        // their steps are masked out)
        auto load_ops = [&](const float* blk, int ii, SeqwOps<NM>& o) {
            const int rj = ii + jl < kSeqsStep ? ii + jl : kSeqsStep - 1;
            const float* wr = blk + W4F + rj * RS4 + 8 * rq;
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                o.w4[2 * m] = *reinterpret_cast<const f32x4*>(wr + 32 * m);
                o.w4[2 * m + 1] = *reinterpret_cast<const f32x4*>(wr + 32 * m + 4);
            }
            o.bmu = blk[B4F + rj];
            o.bal = blk[B4F + kSeqsStep + rj];
            o.xin = xin_t[rj];
        };
#ifdef NFX_SEQW_TIMING
        long long tacc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        long long tmark = clock64();
#define NFX_WMARK(k) do { const long long t_ = clock64(); tacc[k] += t_ - tmark; tmark = t_; } while (0)
#else
#define NFX_WMARK(k) do { } while (0)
#endif
        for (int64_t gb = (int64_t)blockIdx.x * NWV; gb < B; gb += (int64_t)gridDim.x * NWV) {
            const int64_t s = gb + wave;
            const bool valid = s < B;
            float* orow = out + (valid ? s : 0) * d;
            float pre1 = b1u, h1 = 0.f, h2 = 0.f;
            float h3r[4 * NM];
#pragma unroll
            for (int k = 0; k < 4 * NM; ++k) h3r[k] = 0.f;
            float ldl = 0.f;  // per-lane log-det partial (steps ii + jl of every chunk)
            bool poisoned = false;
            int gi = 0;
            int nextdeg = H > 0 ? __builtin_amdgcn_readlane(degv, 0) : d;

            int i0 = 0, n = blk_end(0), buf = 0, par = 0;
            float xr = x_load(s, 0, n);
            seqw_lds_barrier();  // A
            seqw_lds_barrier();  // B
            while (i0 < d) {
                const float* blk = blk0 + buf * BLKF;
                float* zt = xin_t + kSeqsStep * (1 + par);
                xin_t[lane] = xr;
                if (LOGP && lane >= n) zt[lane] = 0.f;
                const int i0n = i0 + n;
                const int nn = i0n < d ? blk_end(i0n) - i0n : 0;
                if (nn > 0) xr = x_load(s, i0n, nn);
                seqs_lds_order();
                SeqwOps<NM> opa, opb;
                load_ops(blk, 0, opa);
                NFX_WMARK(6);  // block start
                int ii = 0;
                auto chunk = [&](SeqwOps<NM>& c, SeqwOps<NM>& nx) {
                    const int i = i0 + ii;
                    int nc = n - ii < 16 ? n - ii : 16;
                    if (nextdeg - i + 1 < nc) nc = nextdeg - i + 1;
                    const bool completes = i + nc - 1 == nextdeg;
                    const int ii2 = ii + nc;
                    const int rj = ii + jl;
                    // this chunk's LDS reads: unit gi's W2 / W3 rows and diagonal, the W1t rows
                    const int gc = gi < Hp ? gi : Hp - 1;
                    const int pg = (gc % 16) * UPL + gc / 16;
                    const float w2n = own ? w23[gc * Hp + posu] : 0.f;
                    const float w3n = own ? w23[Hp * Hp + gc * Hp + posu] : 0.f;
                    const float wd2 = w23[gc * Hp + pg], wd3 = w23[Hp * Hp + gc * Hp + pg];
                    float w1v[16];
#pragma unroll
                    for (int j = 0; j < 16; ++j) w1v[j] = own ? blk[(ii + j) * Hp + posu] : 0.f;  // rows past
                    // the block (ii + j < 80) read the finite W4 part of the same buffer; their steps are masked
                    // 1. step rj's mu/alpha over the lane's ranks, then the 4 rows meet
                    f32x2 a0 = {0.f, 0.f}, a1 = {0.f, 0.f}, a2 = {0.f, 0.f}, a3 = {0.f, 0.f};
#pragma unroll
                    for (int m = 0; m < NM; ++m) {
                        const f32x4 w0 = c.w4[2 * m], w1 = c.w4[2 * m + 1];
                        a0 = pk_fma(f32x2{w0[0], w0[1]}, h3r[4 * m], a0);
                        a1 = pk_fma(f32x2{w0[2], w0[3]}, h3r[4 * m + 1], a1);
                        a2 = pk_fma(f32x2{w1[0], w1[1]}, h3r[4 * m + 2], a2);
                        a3 = pk_fma(f32x2{w1[2], w1[3]}, h3r[4 * m + 3], a3);
                    }
                    const f32x2 at = (a0 + a1) + (a2 + a3);
                    float mu = rows4_sum(at[0]) + c.bmu;
                    float al = rows4_sum(at[1]) + c.bal;
                    // unit gi's layer-2 / layer-3 sums over the units completed before it
                    const float P2 = wave_allsum(w2n * h1);
                    const float P3 = wave_allsum(w3n * h2);
                    NFX_WMARK(0);  // loads, dot products + row reduction, partial sums
                    // 2. step rj's affine map (every row)
                    const bool vj = jl < nc;
                    mu = poisoned ? __builtin_nanf("") : mu;
                    al = poisoned ? __builtin_nanf("") : al;
                    float vi, vo, a;
                    if constexpr (VAR == NFX_MAF_FORWARD) {
                        a = tclamp(al, -3.f, 3.f);
                        vi = c.xin * exp_fast(a) + mu;
                    } else {
                        a = tclamp(al, -2.f, 2.f);
                        const float m = tclamp(mu, -10.f, 10.f);
                        vi = (c.xin - m) * exp_fast(-a);
                    }
                    const uint64_t bad = __ballot(vj && nonfinite(vi));
                    const unsigned rowbad = (unsigned)bad & 0xFFFFu;  // every row holds the same steps
                    const bool kill = rowbad != 0u && jl > __builtin_ctz(rowbad | 0x10000u);
                    vi = kill ? __builtin_nanf("") : vi;
                    a = kill ? __builtin_nanf("") : a;
                    poisoned = poisoned || rowbad != 0u;
                    if constexpr (VAR == NFX_MAF_FORWARD) vo = nonfinite(vi) ? 0.f : vi;
                    else vo = nonfinite(vi) ? c.xin : vi;
                    if constexpr (VAR == NFX_MAF_FORWARD) ldl = vj ? ldl + a : ldl;
                    else ldl = vj ? ldl - a : ldl;
                    if (vj && rq == 0) {
                        if (valid) orow[i + jl] = vo;
                        if constexpr (LOGP) zt[rj] = vo;
                    }
                    NFX_WMARK(1);  // affine map, poison ballot, stores
                    // 3. rank-1 updates of the owned unit's layer-1 pre-activation
                    float cv[16];
                    seqs_row_bcast16(vj ? vi : 0.f, cv);
                    {
                        float t0 = 0.f, t1 = 0.f, t2 = 0.f, t3 = 0.f;
#pragma unroll
                        for (int j = 0; j < 16; j += 4) {
                            t0 = fmaf(w1v[j], cv[j], t0);
                            t1 = fmaf(w1v[j + 1], cv[j + 1], t1);
                            t2 = fmaf(w1v[j + 2], cv[j + 2], t2);
                            t3 = fmaf(w1v[j + 3], cv[j + 3], t3);
                        }
                        pre1 = pre1 + ((t0 + t1) + (t2 + t3));
                    }
                    // the next chunk's W4 rows, biases and inputs (the completion reads no LDS)
                    load_ops(blk, ii2 < n ? ii2 : ii, nx);
                    NFX_WMARK(2);  // broadcasts + rank-1 updates
                    // 4. the units of degree nextdeg (ranks gi .. q-1) complete
                    const int q = __builtin_amdgcn_readlane(gendv, gc);
                    const bool one = completes && q == gi + 1;
                    {
                        // one unit completes (branch-free): only the diagonal terms are left on the chain
                        const float h1g = trelu(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(pre1), gc)));
                        const float h2g = trelu(fmaf(wd2, h1g, P2) + __int_as_float(__builtin_amdgcn_readlane(b2v, gc)));
                        const float h3g = trelu(fmaf(wd3, h2g, P3) + __int_as_float(__builtin_amdgcn_readlane(b3v, gc)));
                        const bool mine = one && lane == gi;
                        h1 = mine ? h1g : h1;
                        h2 = mine ? h2g : h2;
                        // h3r slot 4 (gc >> 4) + (gc & 3) of the lanes of row (gc >> 2) & 3: a uniform
                        // register index
                        const int slot = __builtin_amdgcn_readfirstlane(4 * (gc >> 4) + (gc & 3));
                        const bool row = one && rq == ((gc >> 2) & 3);
                        h3r[slot] = row ? h3g : h3r[slot];
                    }
                    if (completes && !one) {
                        // several units of one degree: 64-lane products + wave all-reduces
                        if (lane >= gi && lane < q) h1 = trelu(pre1);
                        for (int p = gi; p < q; ++p) {
                            const float w = own ? w23[p * Hp + posu] : 0.f;
                            const float h2p = trelu(wave_allsum(w * h1) + __int_as_float(__builtin_amdgcn_readlane(b2v, p)));
                            if (lane == p) h2 = h2p;
                        }
                        for (int p = gi; p < q; ++p) {
                            const float w = own ? w23[Hp * Hp + p * Hp + posu] : 0.f;
                            const float h3p = trelu(wave_allsum(w * h2) + __int_as_float(__builtin_amdgcn_readlane(b3v, p)));
                            const int slot = __builtin_amdgcn_readfirstlane(4 * (p >> 4) + (p & 3));
                            const bool row = rq == ((p >> 2) & 3);
                            h3r[slot] = row ? h3p : h3r[slot];
                        }
                    }
                    if (completes) {
                        gi = q;
                        nextdeg = gi < H ? __builtin_amdgcn_readlane(degv, gi) : d;
                    }
                    NFX_WMARK(3);  // completion
                    ii = ii2;
                };
                for (;;) {  // two operand sets alternate: no register copies of loads in flight
                    chunk(opa, opb);
                    if (ii >= n) break;
                    chunk(opb, opa);
                    if (ii >= n) break;
                }
                seqw_lds_barrier();  // C
                NFX_WMARK(5);  // barrier
                i0 = i0n;
                n = nn;
                buf ^= 1;
                par ^= 1;
            }
            float ld = row16_allsum(ldl);
            float zsq = 0.f;
            if constexpr (LOGP) {
                seqw_lds_barrier();  // D
                zsq = zsum_t[wave];
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
    }
    if constexpr (LOGP) {
        const double t = block_sum_f64<(NWV + 1) * 64>(lpacc);
        if (threadIdx.x == 0) partials[blockIdx.x] = t;
    }
}

typedef void (*made_seqw_kernel_t)(const float*, const float*, float*, float*, int64_t, int, int, int, float*,
                                   double*, float);

}  // namespace nfx
