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
//   4. the unit of degree D_{g+1} completes. Lane p also keeps unit p's layer-2 and layer-3 sums
//      over the units completed so far (acc2, acc3: one FMA each per completion, with the
//      completing unit's outgoing weights — W2 / W3 held transposed in LDS), so on the chain
//      only the diagonal terms remain: h1 = relu(pre1), h2 = relu(acc2_g + W2_gg h1 + b2),
//      h3 = relu(acc3_g + W3_gg h2 + b3) — no all-reduce. (Several units of one degree: the
//      group's sums take every member first, MADE connecting equal degrees.)
// Steps are staged as in made_seqs_kernel (64-step blocks of the block-ready image, 16-byte
// LDS-DMA into a double buffer, the next block in flight) by a separate staging wave, which also
// sums the fused Gaussian term's z^2 in step order (as nfx_gauss_logprob does) one block behind;
// the NWV compute waves (= NWV samples) of a workgroup share the staged blocks. Non-finite steps
// poison the later ones exactly as made_seqs_kernel does.
#pragma once
#include "nfx_made_seqs_kernel.h"

namespace nfx {

// per compute wave: two x block tiles and two z block tiles (alternate blocks) and 64 floats where
// masked lanes' stores land; then one z^2 sum per sample slot
constexpr int kSeqwTile = 5 * kSeqsStep;

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
// Row sums of two values at once (rows hold partials m_r, a_r): three lane swaps instead of four
// (V_PERMLANE16_SWAP: odd rows of the first operand <-> even rows of the second; V_PERMLANE32_SWAP:
// upper half of the first <-> lower half of the second); every lane ends with both sums.
__device__ __forceinline__ void rows4_sum2(float m, float a, float& ms, float& as) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(a), false, false);
    const float c = __uint_as_float(r[0]) + __uint_as_float(r[1]);  // rows: m0+m1, a0+a1, m2+m3, a2+a3
    const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(c), __float_as_uint(c), false, false);
    const float e = __uint_as_float(t[0]) + __uint_as_float(t[1]);  // rows: m, a, m, a
    const auto u = __builtin_amdgcn_permlane16_swap(__float_as_uint(e), __float_as_uint(e), false, false);
    ms = __uint_as_float(u[0]);
    as = __uint_as_float(u[1]);
}
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
    double* __restrict__ partials, double* __restrict__ sums, float cgauss) {
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
        // W2 / W3 TRANSPOSED by completion rank: wt[l][u][p] = W_l[rank p][rank u] (the image holds
        // rows by rank p, columns by position), so lane p reads unit u's outgoing weights as one row
        const float* sw = img + S.w2;
        for (int e = threadIdx.x; e < 2 * Hp * Hp; e += (NWV + 1) * 64) {
            const int l = e / (Hp * Hp), r = e % (Hp * Hp), u = r / Hp, pr = r % Hp;
            lds[5 * Hp + e] = sw[l * Hp * Hp + pr * Hp + (u % 16) * UPL + u / 16];
        }
    }
    __syncthreads();
    const float* w2t = lds + 5 * Hp;  // [u][p]: W2[p][u]
    const float* w3t = w2t + Hp * Hp;  // [u][p]: W3[p][u]
    const int tl = lane & (Hp - 1);
    const int degv = (int)lds[S.deg + tl];
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
        // a block's weight rows, and every compute wave's inputs for it (the x tile of the block's
        // parity: no global loads in the compute waves, whose vmcnt waits would also wait for
        // their output stores' acknowledgements). Lanes past the block read later inputs of the
        // row (finite; their steps are masked), rows past B read row 0.
        auto stage = [&](int64_t gb, int i0, int buf) {
            float* dst = blk0 + buf * BLKF;
            const float* sw1 = P + L.sw1 + (size_t)i0 * Hp;
            const float* sw4 = P + L.sw4 + (size_t)i0 * RS4;
#pragma unroll 4
            for (int j = 0; j < N1; ++j) seqs_dma_x4(sw1 + 256 * j + 4 * lane, dst + 256 * j);
#pragma unroll 4
            for (int j = 0; j < N4; ++j) seqs_dma_x4(sw4 + 256 * j + 4 * lane, dst + W4F + 256 * j);
            seqs_dma_dword(P + L.sb4 + i0 + lane, dst + B4F);
            seqs_dma_dword(P + L.sb4 + (size_t)(d + kSeqsPadRows) + i0 + lane, dst + B4F + 64);
            const int col = i0 + lane < d ? i0 + lane : d - 1;
#pragma unroll
            for (int w = 0; w < NWV; ++w) {
                const int64_t sw = gb + w < B ? gb + w : 0;
                seqs_dma_dword(in + sw * d + col, tiles + w * kSeqwTile + kSeqsStep * buf);
            }
        };
        // step-order z^2 of sample slot `lane` over the block in tile `par`
        auto zsq_block = [&](int par, float z) -> float {
            if (lane < NWV) {
                const float* zt = tiles + lane * kSeqwTile + kSeqsStep * (2 + par);
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
            seqs_lds_barrier();  // A: the previous group is done with the staging buffers
            stage(gb, 0, 0);
            seqs_dma_wait();
            seqs_lds_barrier();  // B: block 0 is in LDS
            bool prev = false;
            while (i0 < d) {
                const int i0n = i0 + n;
                const int nn = i0n < d ? blk_end(i0n) - i0n : 0;
                if (nn > 0) stage(gb, i0n, buf ^ 1);
                if (LOGP && prev) z = zsq_block(par ^ 1, z);  // the block before this one
                seqs_dma_wait();
                seqs_lds_barrier();  // C: block done by every compute wave; the next one is in LDS
                prev = true;
                i0 = i0n;
                n = nn;
                buf ^= 1;
                par ^= 1;
            }
            if constexpr (LOGP) {
                z = zsq_block(par ^ 1, z);
                if (lane < NWV) zsum_t[lane] = z;
                seqs_lds_barrier();  // D: the sums are in LDS
            }
        }
    } else {
        // ---------------- compute waves: one sample each ----------------
        const float b1u = own ? lds[S.b1 + posu] : 0.f;
        float* xin_t = tiles + wave * kSeqwTile;
        const float* xt = xin_t;  // the block's x tile (parity par)
        // operands of the chunk at block position ii (rows past the block clamp to its last row:
        // their steps are masked out)
        const uint32_t* ctab = reinterpret_cast<const uint32_t*>(P + L.ctab);
        auto load_desc = [&](int kb, SeqsDesc& o) { seqs_desc_load_at(ctab, kb, o); };
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
            o.xin = xt[rj];
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
            const auto orsrc = __builtin_amdgcn_make_buffer_rsrc(out + (valid ? s : 0) * d, 0, valid ? d * 4 : 0,
                                                                  0x00020000);
            // pre1: the owned unit's layer-1 pre-activation; acc2 / acc3: its layer-2 / layer-3 sums
            // over the units completed so far (in completion order)
            float pre1 = b1u, acc2 = 0.f, acc3 = 0.f;
            float h3r[4 * NM];
#pragma unroll
            for (int k = 0; k < 4 * NM; ++k) h3r[k] = 0.f;
            float ldl = 0.f;  // per-lane log-det partial (steps ii + jl of every chunk)
            bool poisoned = false;
            int kc = 0;  // byte offset of the chunk's entry in the schedule

            int i0 = 0, n = blk_end(0), buf = 0, par = 0;
            seqs_lds_barrier();  // A
            seqs_lds_barrier();  // B
            while (i0 < d) {
                const float* blk = blk0 + buf * BLKF;
                const int zoff = kSeqsStep * (2 + par);
                float* zt = xin_t + zoff;
                xt = xin_t + kSeqsStep * par;
                if (LOGP && lane >= n) zt[lane] = 0.f;
                const int i0n = i0 + n;
                const int nn = i0n < d ? blk_end(i0n) - i0n : 0;
                seqs_lds_order();
                SeqwOps<NM> opa, opb;
                SeqsDesc da, db;
                load_desc(kc, da);
                load_ops(blk, 0, opa);
                NFX_WMARK(6);  // block start
                bool done = false;
                auto chunk = [&](SeqwOps<NM>& c, SeqwOps<NM>& nx, SeqsDesc& dc, SeqsDesc& dn) {
                    seqs_desc_wait(dc);
                    load_desc(kc + 32, dn);
                    // the chunk's schedule (made_seqs_chunk_kernel): no per-chunk bookkeeping
                    const int ii = dc[0] & 0xff, nc = (dc[0] >> 8) & 0xff;
                    const bool completes = (dc[0] >> 16) & 1u, one = (dc[0] >> 17) & 1u;
                    done = (dc[0] >> 18) & 1u;
                    const int gc = dc[1] & 0xff, q = (dc[1] >> 8) & 0xff, slot = (dc[1] >> 16) & 0xff;
                    const int pg = (int)(dc[2] & 0xffffu);
                    const float b2g = __uint_as_float(dc[3]), b3g = __uint_as_float(dc[4]);
                    const float wd2 = __uint_as_float(dc[5]), wd3 = __uint_as_float(dc[6]);
                    const int i = i0 + ii, ii2 = ii + nc, rj = ii + jl;
                    const unsigned rowm = one && rq == (int)(dc[1] >> 24) ? ~0u : 0u;  // lanes holding h3 of gc
                    // this chunk's LDS reads: unit gc's outgoing W2 / W3 weights, the W1t rows (all
                    // units' for the rank-1 updates; unit gc's for its own pre-activation)
                    const float w2o = w2t[gc * Hp + tl], w3o = w3t[gc * Hp + tl];
                    const float w1g = blk[rj * Hp + pg];
                    float w1v[16];
#pragma unroll
                    for (int j = 0; j < 16; ++j) w1v[j] = own ? blk[(ii + j) * Hp + posu] : 0.f;  // rows past
                    // the block (ii + j < 80) read the finite W4 part of the same buffer; their steps are masked
                    // keep these reads at the chunk start (the scheduler would sink them next to their
                    // uses, exposing their latency in the rank-1 updates and the running sums)
                    __builtin_amdgcn_sched_barrier(0);
                    // unit gc's layer-1 pre-activation before this chunk, its layer-2 / layer-3 sums over
                    // the units completed before it, its own (diagonal) weights
                    const float p1g = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pre1), gc));
                    const float P2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(acc2), gc));
                    const float P3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(acc3), gc));
                    // a poisoned sample's biases are NaN: every later step is NaN
                    const float bmu = poisoned ? __builtin_nanf("") : c.bmu;
                    const float bal = poisoned ? __builtin_nanf("") : c.bal;
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
                    float mu, al;
                    rows4_sum2(at[0], at[1], mu, al);
                    mu = mu + bmu;
                    al = al + bal;
                    NFX_WMARK(0);  // loads, dot products + row reduction
                    // 2. step rj's affine map (every row)
                    const bool vj = jl < nc;
                    float vi, a;
                    if constexpr (VAR == NFX_MAF_FORWARD) {
                        a = tclamp(al, -3.f, 3.f);
                        vi = c.xin * exp_fast(a) + mu;
                    } else {
                        a = tclamp(al, -2.f, 2.f);
                        const float m = tclamp(mu, -10.f, 10.f);
                        vi = (c.xin - m) * exp_fast(-a);
                    }
                    const float vz = vj ? vi : 0.f;
                    // 3. the chain: unit gc completes. Its pre-activation takes the chunk's inputs as one
                    // row sum; then only the diagonal terms of layers 2 and 3 are left. (A non-finite
                    // step poisons the sample below; what it leaves in the sums reaches only steps that
                    // the poison turns to NaN anyway.)
                    {
                        const float h1g = trelu(p1g + row16_allsum(vz * w1g));
                        const float h2g = trelu(fmaf(wd2, h1g, P2) + b2g);
                        const float h3g = trelu(fmaf(wd3, h2g, P3) + b3g);
                        // select by bit mask (v_bfi_b32): one instruction, no exec-mask branch
                        h3r[slot] = __uint_as_float((__float_as_uint(h3g) & rowm) | (__float_as_uint(h3r[slot]) & ~rowm));
                        // every unit's running sums take unit gc's outputs
                        acc2 = one ? fmaf(w2o, h1g, acc2) : acc2;
                        acc3 = one ? fmaf(w3o, h2g, acc3) : acc3;
                    }
                    NFX_WMARK(1);  // affine map + completion
                    // 4. off the chain: the poison rule, outputs, log-det
                    const uint64_t bad = __builtin_amdgcn_ballot_w64(vj && nonfinite(vi));
                    const unsigned rowbad = (unsigned)bad & 0xFFFFu;  // every row holds the same steps
                    const bool kill = rowbad != 0u && jl > __builtin_ctz(rowbad | 0x10000u);
                    const float vk = kill ? __builtin_nanf("") : vi;
                    a = kill ? __builtin_nanf("") : a;
                    poisoned = poisoned || rowbad != 0u;
                    float vo;
                    if constexpr (VAR == NFX_MAF_FORWARD) vo = nonfinite(vk) ? 0.f : vk;
                    else vo = nonfinite(vk) ? c.xin : vk;
                    if constexpr (VAR == NFX_MAF_FORWARD) ldl = vj ? ldl + a : ldl;
                    else ldl = vj ? ldl - a : ldl;
                    {
                        // branch-free stores (a branch here would split the chunk's scheduling region):
                        // out of range for the other lanes, which the buffer store drops
                        const bool st = vj && rq == 0;
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(vo), orsrc, st ? (i + jl) * 4 : (int)0x7FFFFFF0,
                                                              0, 0);
                        if constexpr (LOGP) xin_t[st ? zoff + rj : 4 * kSeqsStep + lane] = vo;
                    }
                    // 5. rank-1 updates of every owned unit's layer-1 pre-activation
                    float cv[16];
                    seqs_row_bcast16(vz, cv);
                    {
                        // step pairs as packed FMAs: lanes (2j, 2j + 1) of the pair accumulators
                        f32x2 t0 = {0.f, 0.f}, t1 = {0.f, 0.f};
#pragma unroll
                        for (int j = 0; j < 16; j += 4) {
                            t0 = __builtin_elementwise_fma(f32x2{w1v[j], w1v[j + 1]}, f32x2{cv[j], cv[j + 1]}, t0);
                            t1 = __builtin_elementwise_fma(f32x2{w1v[j + 2], w1v[j + 3]}, f32x2{cv[j + 2], cv[j + 3]}, t1);
                        }
                        const f32x2 tt = t0 + t1;
                        pre1 = pre1 + (tt[0] + tt[1]);
                    }
                    // the next chunk's W4 rows, biases and inputs
                    load_ops(blk, done ? ii : ii2, nx);
                    NFX_WMARK(2);  // poison, stores, broadcasts + rank-1 updates
                    if (completes && !one) {
                        // several units of one degree (MADE connects equal degrees): h1 of the group,
                        // then its layer-2 sums, then layer 3
                        const float h1v = trelu(pre1);
                        for (int p = gc; p < q; ++p)
                            acc2 = fmaf(w2t[p * Hp + tl], __int_as_float(__builtin_amdgcn_readlane(__float_as_int(h1v), p)), acc2);
                        const float h2v = trelu(acc2 + __int_as_float(b2v));
                        for (int p = gc; p < q; ++p)
                            acc3 = fmaf(w3t[p * Hp + tl], __int_as_float(__builtin_amdgcn_readlane(__float_as_int(h2v), p)), acc3);
                        const float h3v = trelu(acc3 + __int_as_float(b3v));
                        for (int p = gc; p < q; ++p) {
                            const float h3p = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(h3v), p));
                            const int slot = __builtin_amdgcn_readfirstlane(4 * (p >> 4) + (p & 3));
                            const bool row = rq == ((p >> 2) & 3);
                            h3r[slot] = row ? h3p : h3r[slot];
                        }
                    }
                    NFX_WMARK(3);  // completion
                    kc += 32;
                };
                for (;;) {  // two operand / schedule sets alternate: no register copies of loads in flight
                    chunk(opa, opb, da, db);
                    if (done) break;
                    chunk(opb, opa, db, da);
                    if (done) break;
                }
                seqs_lds_barrier();  // C
                NFX_WMARK(5);  // barrier
                i0 = i0n;
                n = nn;
                buf ^= 1;
                par ^= 1;
            }
            float ld = row16_allsum(ldl);
            float zsq = 0.f;
            if constexpr (LOGP) {
                seqs_lds_barrier();  // D
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
        logp_commit<(NWV + 1) * 64>(lpacc, partials, sums, B);
    }
}

typedef void (*made_seqw_kernel_t)(const float*, const float*, float*, float*, int64_t, int, int, int, float*,
                                   double*, double*, float);

}  // namespace nfx
