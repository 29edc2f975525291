// Sequential MADE-affine directions with a sample's hidden units spread over 16 lanes
// (MAF.forward = sampling, IAF.inverse = density; H <= 64).
//
// Reference: masked_autoregressive_flow.py:46-78, inverse_autoregressive_flow.py:65-103 (d full
// MADE calls on the partially filled vector). Same algorithm as made_seq_kernel (nfx_made_kernel.h):
// every hidden unit is computed once, when the input of its degree is known, and every output
// once — one MADE evaluation per sample instead of d. What changes is the mapping: one lane per
// sample leaves a small batch (cfg5i: 8,192 samples = 128 waves) with most of the GPU idle and
// every step's dependency chain exposed. Here a 16-lane DPP row owns one sample (4 samples per
// wave) and each lane owns Hp/16 hidden units: an output's dot product is Hp/16 FMAs per lane
// plus a 4-step DPP butterfly, the rank-1 update of the layer-1 pre-activations is Hp/16 FMAs
// per lane, and a completing unit's layer-2/3 dot products are split the same way.
// Weights: W2/W3, biases and the completion-order tables are LDS-resident; the per-step rows
// (W1ᵀ column, W4 mu/alpha rows) are staged in 32-step blocks into an LDS double buffer by the
// whole 512-thread workgroup, a block ahead; x (resp. z) rows move through per-wave LDS tiles.
#pragma once
#include "nfx_made_kernel.h"

namespace nfx {

constexpr int kSeqgWaves = 8;   // 512-thread workgroups
constexpr int kSeqgStep = 32;   // steps per staged block

struct SeqgLds {
    int w2, w3, b1, b2, b3, ord, blk, blkf, wv, total;
};

__host__ __device__ inline SeqgLds seqg_lds(int Hp) {
    SeqgLds S{};
    int o = 0;
    S.w2 = o; o += Hp * Hp;
    S.w3 = o; o += Hp * Hp;
    S.b1 = o; o += Hp;
    S.b2 = o; o += Hp;
    S.b3 = o; o += Hp;
    S.ord = o; o += 3 * Hp;
    S.blk = o; S.blkf = 3 * kSeqgStep * Hp + 2 * kSeqgStep; o += 2 * S.blkf;  // w1t | w4mu | w4al | b4mu | b4al
    S.wv = o; o += kSeqgWaves * 2 * 4 * kSeqgStep;  // per wave: in tile [4][32], out tile [4][32]
    S.total = o;
    return S;
}

// Sum over the 16 lanes of a DPP row (one sample): xor-1, xor-2 quad swaps, then the 8- and
// 16-lane mirrors. Every lane of the row ends with the total.
__device__ __forceinline__ float row16_sum(float v) {
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
    return v;
}

template <int UPL>
__device__ __forceinline__ void lds_row(const float* p, float (&w)[UPL]) {
    if constexpr (UPL == 4) {
        const f32x4 t = *reinterpret_cast<const f32x4*>(p);
        w[0] = t[0]; w[1] = t[1]; w[2] = t[2]; w[3] = t[3];
    } else {
#pragma unroll
        for (int u = 0; u < UPL; ++u) w[u] = p[u];
    }
}

template <int HT, int VAR>
__global__ __launch_bounds__(512) void made_seqg_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d, int H, int accumulate) {
    constexpr int Hp = 32 * HT;
    constexpr int UPL = Hp / 16;  // hidden units per lane
    const MadeLayout L = made_layout(d, HT);
    const SeqgLds S = seqg_lds(Hp);
    extern __shared__ f32x4 lds4[];
    float* lds = reinterpret_cast<float*>(lds4);
    const float* P = packed;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = lane_id(), slot = lane >> 4, sub = lane & 15;

    for (int i = threadIdx.x; i < Hp * Hp; i += 512) {
        lds[S.w2 + i] = P[L.s_w2 + i];
        lds[S.w3 + i] = P[L.s_w3 + i];
    }
    for (int i = threadIdx.x; i < Hp; i += 512) {
        lds[S.b1 + i] = P[L.s_b1 + i];
        lds[S.b2 + i] = P[L.s_b2 + i];
        lds[S.b3 + i] = P[L.s_b3 + i];
    }
    for (int i = threadIdx.x; i < 3 * Hp; i += 512) lds[S.ord + i] = P[L.s_deg + i];
    __syncthreads();  // the per-group state below reads b1 before the group's first barrier
    const float* ordD = lds + S.ord + Hp;      // degree of the k-th unit in completion order
    const float* ordU = lds + S.ord + 2 * Hp;  // its unit index
    float* xin_t = lds + S.wv + wave * 2 * 4 * kSeqgStep;
    float* vout_t = xin_t + 4 * kSeqgStep;

    const int nblk = (d + kSeqgStep - 1) / kSeqgStep;

    for (int64_t gb = (int64_t)blockIdx.x * kSeqgWaves * 4; gb < B; gb += (int64_t)gridDim.x * kSeqgWaves * 4) {
        const int64_t s = gb + wave * 4 + slot;  // this row's sample
        const bool valid = s < B;
        // per-lane state: owned units sub*UPL + u
        float pre1[UPL], h1v[UPL], h2v[UPL], h3v[UPL];
#pragma unroll
        for (int u = 0; u < UPL; ++u) {
            pre1[u] = lds[S.b1 + sub * UPL + u];
            h1v[u] = h2v[u] = h3v[u] = 0.f;
        }
        float ld = 0.f;
        bool poison = false;
        int p = 0;

        // stage block 0 (weights: whole workgroup; x rows: per wave)
        auto stage_blk = [&](int kb, int buf) {
            float* dst = lds + S.blk + buf * S.blkf;
            const int i0 = kb * kSeqgStep;
            const int n = d - i0 < kSeqgStep ? d - i0 : kSeqgStep;
            for (int e = threadIdx.x; e < n * Hp; e += 512) {
                dst[e] = P[L.s_w1t + (size_t)i0 * Hp + e];
                dst[kSeqgStep * Hp + e] = P[L.s_w4 + (size_t)i0 * Hp + e];
                dst[2 * kSeqgStep * Hp + e] = P[L.s_w4 + (size_t)(d + i0) * Hp + e];
            }
            for (int e = threadIdx.x; e < n; e += 512) {
                dst[3 * kSeqgStep * Hp + e] = P[L.s_b4 + i0 + e];
                dst[3 * kSeqgStep * Hp + kSeqgStep + e] = P[L.s_b4 + d + i0 + e];
            }
        };
        __syncthreads();  // previous group's readers of the staging buffers are done
        stage_blk(0, 0);
        __syncthreads();

        for (int kb = 0; kb < nblk; ++kb) {
            const int i0 = kb * kSeqgStep;
            const int n = d - i0 < kSeqgStep ? d - i0 : kSeqgStep;
            const float* blk = lds + S.blk + (kb & 1) * S.blkf;
            // this wave's 4 input rows for the block: 2 values per lane, coalesced 128-byte rows
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int e = lane + 64 * q, r = e >> 5, c = e & 31;
                const int64_t sr = gb + wave * 4 + r;
                xin_t[e] = (sr < B && c < n) ? in[sr * d + i0 + c] : 0.f;
            }
            // stage the next block into the other buffer (its readers finished last block)
            if (kb + 1 < nblk) stage_blk(kb + 1, (kb + 1) & 1);
            wave_lds_sync();

            for (int ii = 0; ii < n; ++ii) {
                const int i = i0 + ii;
                float wm[UPL], wa[UPL];
                lds_row<UPL>(blk + kSeqgStep * Hp + ii * Hp + sub * UPL, wm);
                lds_row<UPL>(blk + 2 * kSeqgStep * Hp + ii * Hp + sub * UPL, wa);
                float pm = 0.f, pa = 0.f;
#pragma unroll
                for (int u = 0; u < UPL; ++u) {
                    pm = fmaf(wm[u], h3v[u], pm);
                    pa = fmaf(wa[u], h3v[u], pa);
                }
                float mu = row16_sum(pm) + blk[3 * kSeqgStep * Hp + ii];
                float al = row16_sum(pa) + blk[3 * kSeqgStep * Hp + kSeqgStep + ii];
                if (poison) {
                    mu = __builtin_nanf("");
                    al = mu;
                }
                const float xin = xin_t[slot * kSeqgStep + ii];
                float vi, vo;
                if constexpr (VAR == NFX_MAF_FORWARD) {
                    // masked_autoregressive_flow.py:57-65
                    const float a = tclamp(al, -3.f, 3.f);
                    vi = xin * exp_fast(a) + mu;
                    ld = ld + a;
                    vo = nonfinite(vi) ? 0.f : vi;
                } else {
                    // inverse_autoregressive_flow.py:79-88
                    const float a = tclamp(al, -2.f, 2.f);
                    const float m = tclamp(mu, -10.f, 10.f);
                    vi = (xin - m) * exp_fast(-a);
                    ld = ld - a;
                    vo = nonfinite(vi) ? xin : vi;
                }
                if (sub == 0) vout_t[slot * kSeqgStep + ii] = vo;
                if (nonfinite(vi)) poison = true;
                // rank-1 update of the owned layer-1 pre-activations with the new input
                float w1[UPL];
                lds_row<UPL>(blk + ii * Hp + sub * UPL, w1);
#pragma unroll
                for (int u = 0; u < UPL; ++u) pre1[u] = fmaf(w1[u], vi, pre1[u]);
                // hidden units of degree i complete: layer 1, then 2, then 3 of the level
                int q = p;
                while (q < H && (int)ordD[q] == i) ++q;
                if (q > p) {
                    for (int k = p; k < q; ++k) {
                        const int a = (int)ordU[k];
#pragma unroll
                        for (int u = 0; u < UPL; ++u)
                            if (a == sub * UPL + u) h1v[u] = trelu(pre1[u]);
                    }
                    for (int k = p; k < q; ++k) {
                        const int a = (int)ordU[k];
                        float w[UPL];
                        lds_row<UPL>(lds + S.w2 + a * Hp + sub * UPL, w);
                        float v = 0.f;
#pragma unroll
                        for (int u = 0; u < UPL; ++u) v = fmaf(w[u], h1v[u], v);
                        v = trelu(row16_sum(v) + lds[S.b2 + a]);
#pragma unroll
                        for (int u = 0; u < UPL; ++u)
                            if (a == sub * UPL + u) h2v[u] = v;
                    }
                    for (int k = p; k < q; ++k) {
                        const int a = (int)ordU[k];
                        float w[UPL];
                        lds_row<UPL>(lds + S.w3 + a * Hp + sub * UPL, w);
                        float v = 0.f;
#pragma unroll
                        for (int u = 0; u < UPL; ++u) v = fmaf(w[u], h2v[u], v);
                        v = trelu(row16_sum(v) + lds[S.b3 + a]);
#pragma unroll
                        for (int u = 0; u < UPL; ++u)
                            if (a == sub * UPL + u) h3v[u] = v;
                    }
                    p = q;
                }
            }
            wave_lds_sync();
            // this wave's 4 output rows for the block
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                const int e = lane + 64 * qq, r = e >> 5, c = e & 31;
                const int64_t sr = gb + wave * 4 + r;
                if (sr < B && c < n) out[sr * d + i0 + c] = vout_t[e];
            }
            __syncthreads();  // every wave is done with this block's buffer
        }
        if (valid && sub == 0) {
            if (nonfinite(ld)) ld = 0.f;
            ld = (VAR == NFX_MAF_FORWARD) ? tclamp(ld, -100.f, 100.f) : tclamp(ld, -50.f, 50.f);
            logdet[s] = accumulate ? logdet[s] + ld : ld;
        }
    }
}

template <int HT>
made_seq_kernel_t made_seqg_pick_ht(int variant);

}  // namespace nfx
