// Sequential MADE-affine directions, segment-parallel (MAF.forward = sampling, IAF.inverse =
// density; H <= 64).
//
// Reference: masked_autoregressive_flow.py:46-78, inverse_autoregressive_flow.py:65-103 (d full
// MADE calls on the partially filled vector). As in made_seq_kernel (nfx_made_kernel.h) every
// hidden unit is computed once, when the input of its degree is known (made.py:56,63: unit a of
// every hidden layer sees only inputs <= deg(a)), so a sample costs ONE MADE evaluation. What
// this kernel adds is the observation that between two completion events the last hidden layer
// does not change: output i reads only units with deg < i (made.py:72-78), so all steps in
// (D_g, D_{g+1}] -- a "segment", ~d/H steps -- take their mu/alpha from the same h3 and are
// mutually independent. They are evaluated together, in chunks of up to 16 steps:
//   1. a 16-lane DPP row owns one sample (4 samples per wave); lane j forms step j's mu/alpha
//      dot products over the COMPLETED units (ranks < gi) in full: the step's staged W4 row
//      holds (mu, alpha) weight pairs by completion rank, the sample's h3 row sits in LDS by
//      rank (0 until the unit completes; one broadcast read serves the 16 lanes), so no
//      cross-lane reduction is needed and the work grows with the completed units;
//   2. lane j evaluates step j's affine map;
//   3. the rank-1 updates of the layer-1 pre-activations with the chunk's new inputs (DPP row
//      broadcasts), in step order, over the lane's INCOMPLETE units only (W1[a][i] is masked to
//      zero for i > deg(a)); lane `sub` owns the hidden units of completion rank sub + 16k;
//   4. the units of degree D_{g+1} complete (layer 1, then 2, then 3, row all-reduces; the
//      layer-3 value is written to the sample's h3 row).
// Owning ranks sub + 16k (interleaved) keeps the completed/incomplete split within one unit per
// lane at every segment, so the skipping in 3 is lane-uniform (template-specialised on
// floor(c/16) completed slots).
// The log-det and the fused Gaussian term are summed in step order (the reference's sequential
// fp32 `ld -= alpha_i` and nfx_gauss_logprob's in-order z^2 sum), so results equal the
// per-step formulation's up to the reduction order inside each mu/alpha dot product.
// A non-finite step poisons every later step (the reference feeds NaN/Inf through the dense
// masked matmul: 0*NaN = NaN), found per chunk with a wave ballot.
// Weights (permuted to rank order at pack time): biases and the degree tables LDS-resident, W2/W3
// rows read from the L2-resident image at the chunk start; per-step rows (W1^T column, W4
// mu/alpha rows, b4) staged in 64-step blocks into an LDS double buffer by LDS-DMA, the next
// block in flight while the current one is processed; mu/alpha weights interleaved per rank so
// the pair of dot products is one packed FMA (v_pk_fma_f32).
#pragma once
#include "nfx_made_kernel.h"

namespace nfx {

constexpr int kSeqsWaves = 8;  // compute waves per workgroup (4 samples each)
// + one staging wave that issues the blocks' LDS-DMA (else the compute waves share it)
constexpr bool kSeqsStager = true;  // required: the staging wave also owns the block sums
constexpr int kSeqsThreads = 64 * (kSeqsWaves + (kSeqsStager ? 1 : 0));
constexpr int kSeqsStep = 64;  // steps per staged block
constexpr int kSeqsH3 = 68;  // per-sample h3 row (by rank, Hp <= 64) + 4 pad floats
// per wave: the x block tile; z and alpha block tiles, double-buffered (the staging wave sums and
// stores block k while the wave computes block k + 1); h3 rows; 64 floats where the lanes past a
// chunk store
constexpr int kSeqsTile = 4 * kSeqsStep + 2 * 2 * 4 * kSeqsStep + 4 * kSeqsH3 + 64;

// seqs_w4_stride (nfx_made_kernel.h): row stride of the interleaved (mu, alpha) W4 block rows,
// 2 Hp + 4, so that the 16 lanes of a row group, reading the same 16-byte column of 16
// consecutive rows, hit 16 different bank granules ((ii + j)(Hp / 2 + 1) + 2 q = ii + j + 2 q mod 16).
static_assert(kSeqsPadRows == kSeqsStep, "a staged block is copied whole from the padded rows");

struct SeqsLds {
    int w2, w3, tab;                                         // rank-ordered image in global memory
    int b1, b2, b3, deg, gend, tabn, wv, blk, blkf, total;  // LDS
};

// Rank-ordered image in global memory (P + L.rimg, built at pack time by made_seqs_image_kernel):
// W2 / W3 rows by completion rank, columns by position (unit of rank p sits at position
// pos(p) = (p % 16) * UPL + p / 16: lane sub's slots k = 0..UPL-1 are contiguous), then the
// tables (b1 by position; b2, b3, degree, group end by rank). The completion chain reads its W2 /
// W3 rows from there (L2-resident, issued at the chunk start).
// LDS (floats): the tables | per-wave tiles (low addresses, so every tile access is a base VGPR +
// immediate offset) | two staged blocks: w1t [64][Hp] by position | w4 [64][Hp][mu, alpha] by RANK
// (+4 pad floats per row) | b4 [mu 64 | alpha 64].
__host__ __device__ inline SeqsLds seqs_lds(int Hp) {
    SeqsLds S{};
    S.w2 = 0;
    S.w3 = Hp * Hp;
    S.tab = 2 * Hp * Hp;
    int o = 0;
    S.b1 = o; o += Hp;    // by position
    S.b2 = o; o += Hp;    // by rank
    S.b3 = o; o += Hp;    // by rank
    S.deg = o; o += Hp;   // degree by rank (padded units 1e9)
    S.gend = o; o += Hp;  // first rank after rank p's degree group
    S.tabn = o;
    S.wv = o; o += kSeqsWaves * kSeqsTile;
    S.blk = o; S.blkf = kSeqsStep * Hp + kSeqsStep * seqs_w4_stride(Hp) + 2 * kSeqsStep; o += 2 * S.blkf;
    S.total = o;
    return S;
}

// One global_load_lds_dword: lane l's dword from `src` (per lane) to LDS lds_dst + 4l. Issued as
// inline asm so the compiler does not know an LDS write is in flight: the builtin makes it wait
// vmcnt(0) before every later ds_read (it cannot tell the DMA targets the other buffer), which
// would expose the load latency once per block. Completion is waited for explicitly
// (seqs_dma_wait) before the barrier that publishes the buffer.
__device__ __forceinline__ void seqs_dma_dword(const float* src, float* lds_dst) {
    const uint32_t m = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) float*)lds_dst);
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dword %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(__builtin_amdgcn_readfirstlane(m))
        : "memory");
}
__device__ __forceinline__ void seqs_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// One global_load_lds_dwordx4: lane l's 16 bytes from `src` (per lane) to LDS lds_dst + 16 l.
__device__ __forceinline__ void seqs_dma_x4(const float* src, float* lds_dst) {
    const uint32_t m = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) float*)lds_dst);
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(__builtin_amdgcn_readfirstlane(m))
        : "memory");
}

// Workgroup barrier over LDS only: unlike __syncthreads() it does not wait for the wave's global
// stores (vmcnt), which the compute waves leave in flight.
__device__ __forceinline__ void seqs_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// A chunk's schedule entry (made_seqs_chunk_kernel), scalar-loaded (s_load_dwordx8) one chunk
// ahead. Inline asm: the compiler would not use a scalar load here (the kernel's stores and asm
// memory clobbers make every global read "clobberable" for it) and would read the entry with
// vector loads + 8 v_readfirstlane instead. seqs_desc_wait is the matching wait; taking the entry
// as an operand, it orders every use after it.
typedef uint32_t SeqsDesc __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void seqs_desc_load(const uint32_t* p, SeqsDesc& o) {
    asm volatile("s_load_dwordx8 %0, %1, 0x0" : "=s"(o) : "s"(p) : "memory");
}
// Entry at byte offset `off` from the table base (an SGPR offset: one s_add per chunk for the
// address instead of the 64-bit index arithmetic).
__device__ __forceinline__ void seqs_desc_load_at(const uint32_t* base, int off, SeqsDesc& o) {
    asm volatile("s_load_dwordx8 %0, %1, %2" : "=s"(o) : "s"(base), "s"(off) : "memory");
}
__device__ __forceinline__ void seqs_desc_wait(SeqsDesc& o) { asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(o)); }

// Keeps the compiler from moving LDS accesses across this point. A wave's DS operations execute
// in order, so wave-private tiles need nothing more -- and, unlike a fence, this emits no
// s_waitcnt vmcnt that would drain the next block's LDS-DMA in flight.
__device__ __forceinline__ void seqs_lds_order() { asm volatile("" ::: "memory"); }

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    // every control used here reads a valid lane for every lane, so no `old` value is needed
    // (mov_dpp leaves it undefined: no zeroing v_mov before each DPP op, and the DPP combiner can
    // fold the move into the consuming add)
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

// out[c] = v of lane c of this lane's 16-lane DPP row (row_newbcast:c, GFX90A+ encoding 0x150 + c).
template <int C = 0>
__device__ __forceinline__ void seqs_row_bcast16(float v, float (&out)[16]) {
    if constexpr (C < 16) {
        out[C] = dpp<0x150 + C>(v);
        seqs_row_bcast16<C + 1>(v, out);
    }
}

// Sum over the 16 lanes of a DPP row; every lane of the row ends with the total.
__device__ __forceinline__ float row16_allsum(float v) {
    v = v + dpp<0xB1>(v);   // quad xor 1
    v = v + dpp<0x4E>(v);   // quad xor 2
    v = v + dpp<0x141>(v);  // row_half_mirror
    v = v + dpp<0x140>(v);  // row_mirror
    return v;
}

// N consecutive floats of a lane's slots starting at slot K0 (16-byte aligned row base).
template <int K0, int N, int UPL>
__device__ __forceinline__ void seqs_slots(const float* row, float (&w)[UPL]) {
    if constexpr (N == 0) {
        return;
    } else if constexpr (K0 == 0 && N >= 3 && UPL == 4) {
        const f32x4 t = *reinterpret_cast<const f32x4*>(row);
        w[0] = t[0]; w[1] = t[1]; w[2] = t[2]; w[3] = t[3];
    } else if constexpr (K0 % 2 == 0 && N >= 2) {
        const float2 t = *reinterpret_cast<const float2*>(row + K0);
        w[K0] = t.x; w[K0 + 1] = t.y;
        if constexpr (N > 2) seqs_slots<K0 + 2, N - 2, UPL>(row, w);
    } else {
        w[K0] = row[K0];
        if constexpr (N > 1) seqs_slots<K0 + 1, N - 1, UPL>(row, w);
    }
}

__device__ __forceinline__ f32x2 pk_fma(f32x2 a, float b, f32x2 c) {
    return __builtin_elementwise_fma(a, f32x2{b, b}, c);
}

// Step 3 for slots k >= K0 (the others are completed in every lane): pre1 += W1t[i] * v_i in
// step order, pairs of slots as packed FMAs. w = this lane's slots of the chunk's 16 W1t rows,
// read before steps 1-2 finish (they depend only on the chunk position), so their LDS latency
// hides behind the reduce-scatter and the affine map.
template <int K0, int UPL>
__device__ __forceinline__ void seqs_rank1(const float (&w)[16][UPL], const float (&cv)[16],
                                           f32x2 (&pre1)[UPL / 2]) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        if constexpr (K0 % 2 == 1) pre1[K0 / 2][1] = fmaf(w[j][K0], cv[j], pre1[K0 / 2][1]);
#pragma unroll
        for (int k = (K0 + 1) / 2; k < UPL / 2; ++k)
            pre1[k] = pk_fma(f32x2{w[j][2 * k], w[j][2 * k + 1]}, cv[j], pre1[k]);
    }
}

// Unit p (rank, uniform) of a hidden layer: relu(row sum of w . hin + bias[p]), stored into the
// owning lane's slot (every lane of the row gets the value from the all-reduce).
template <int UPL>
__device__ __forceinline__ float seqs_unit_value(int p, const float (&w)[UPL], const float (&hin)[UPL], int bv) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < UPL; ++k) v = fmaf(w[k], hin[k], v);
    return trelu(row16_allsum(v) + __int_as_float(__builtin_amdgcn_readlane(bv, p)));
}
template <int UPL>
__device__ __forceinline__ void seqs_unit(int p, int sub, const float (&w)[UPL], const float (&hin)[UPL], int bv,
                                          float (&hout)[UPL]) {
    const float v = seqs_unit_value<UPL>(p, w, hin, bv);
#pragma unroll
    for (int k = 0; k < UPL; ++k)
        if (p == sub + 16 * k) hout[k] = v;
}

template <int HT, int VAR, bool LOGP>
__global__ __launch_bounds__(kSeqsThreads) void made_seqs_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d, int H, int accumulate, float* __restrict__ logp,
    double* __restrict__ partials, double* __restrict__ sums, float cgauss) {
    constexpr int Hp = 32 * HT;
    constexpr int UPL = Hp / 16;  // hidden-unit slots per lane
    constexpr int RS4 = seqs_w4_stride(Hp);
    constexpr int W4F = kSeqsStep * Hp;  // block image offsets
    constexpr int B4F = W4F + kSeqsStep * RS4;
    const MadeLayout L = made_layout(d, HT);
    const SeqsLds S = seqs_lds(Hp);
    extern __shared__ f32x4 lds4[];
    float* lds = reinterpret_cast<float*>(lds4);
    const float* P = packed;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = lane_id(), slot = lane >> 4, sub = lane & 15;

    // the tables of the rank-ordered image (prepared once at pack time, made_seqs_image_kernel):
    // one coalesced copy
    const float* img = P + L.rimg;
    {
        const f32x4* src = reinterpret_cast<const f32x4*>(img + S.tab);
        for (int i = threadIdx.x; i < S.tabn / 4; i += kSeqsThreads) lds4[i] = src[i];
    }
    __syncthreads();
    // Per-rank tables held one entry per lane (Hp <= 64) and read with v_readlane at a uniform
    // rank: the completion chain (next degree, group end, layer-2/3 biases) has no LDS round trip.
    const int tl = lane & (Hp - 1);
    const int degv = (int)lds[S.deg + tl];
    const int b2v = __float_as_int(lds[S.b2 + tl]);
    const int b3v = __float_as_int(lds[S.b3 + tl]);
    // compute wave w's tiles; the staging wave reads every wave's z / alpha tiles
    auto wtile = [&](int w) { return lds + S.wv + w * kSeqsTile; };
    float* xin_t = wtile(wave);                     // [4][64] inputs of the block
    float* zt2 = xin_t + 4 * kSeqsStep;             // [2][4][64] guarded outputs of the block (by parity)
    float* at2 = zt2 + 2 * 4 * kSeqsStep;           // [2][4][64] clamped alphas of the block (by parity)
    float* h3_t = at2 + 2 * 4 * kSeqsStep;          // [4][kSeqsH3] h3 by rank (0 until complete)
    // Staged blocks end where a segment ends (after the step of a completion degree) whenever a
    // segment boundary falls within kSeqsStep steps, so that no chunk is cut by a block boundary
    // (at cfg5i: 65 chunks per sample instead of 77). Block [i0, blk_end(i0)), uniform.
    auto blk_end = [&](int i0) -> int {
        const int lim = i0 + kSeqsStep;
        if (lim >= d) return d;
        // lane g < H holds rank g's degree; degrees ascend with the rank, so the highest lane
        // whose segment end falls in (i0, lim] has the largest one
        const int e = degv + 1;
        const uint64_t m = __ballot(lane < H && e > i0 && e <= lim);
        if (m == 0) return lim;  // no segment ends inside: a full block
        return __builtin_amdgcn_readlane(e, 63 - __builtin_clzll(m));
    };
    // Block staging by LDS-DMA: a block is kSeqsStep consecutive rows of the block-ready image
    // (made_seqs_image_kernel: w1t rows by position, W4 pair rows by rank + pads, b4), copied
    // whole with 16-byte LDS-DMA pieces (1 KiB per wave instruction) — rows past the block (the
    // next block's, or zero rows past d) are finite, which the lanes past a chunk rely on.
    // Issued a block ahead into the other buffer.
    constexpr int N1 = kSeqsStep * Hp / 256, N4 = kSeqsStep * RS4 / 256;
    static_assert(N1 * 256 == kSeqsStep * Hp && N4 * 256 == kSeqsStep * RS4, "whole 1 KiB pieces");
    auto blk_stage = [&](int i0, int buf) {
        float* dst = lds + S.blk + buf * S.blkf;
        const float* sw1 = P + L.sw1 + (size_t)i0 * Hp;
        const float* sw4 = P + L.sw4 + (size_t)i0 * RS4;
        for (int j = kSeqsStager ? 0 : wave; j < N1 + N4 + 2; j += kSeqsStager ? 1 : kSeqsWaves) {
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
    // the wave's 4 rows of the block's inputs: range-checked buffer loads (rows >= B and dims
    // past the block read 0), no branches
    auto x_load = [&](int64_t gb, int i0, int n, float (&xr)[4]) {
        const int64_t r0 = gb + wave * 4;
        const int64_t nrows = B - r0 < 4 ? (B - r0 > 0 ? B - r0 : 0) : 4;
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in) + (r0 < B ? r0 : 0) * d, 0,
                                                          (int)(nrows * d * 4), 0x00020000);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int voff = lane < n ? (q * d + i0 + lane) * 4 : (int)0x7FFFFFF0;
            xr[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, 0, 0));
        }
    };

#ifdef NFX_SEQS_TIMING
    long long tacc[7] = {0, 0, 0, 0, 0, 0, 0};
    long long tmark = clock64();
#define NFX_TMARK(k) do { const long long t_ = clock64(); tacc[k] += t_ - tmark; tmark = t_; } while (0)
#else
#define NFX_TMARK(k) do { } while (0)
#endif
    static_assert(kSeqsStager, "the staging wave sums the blocks and writes the results");
    double lpacc = 0.0;
    if (wave == kSeqsWaves) {
        // staging wave: the LDS-DMA of every block, and — one block behind the compute waves — the
        // block's log-det / z^2 terms in step order for all 32 samples (serial chains the compute
        // waves would otherwise run on all 64 lanes for 4 samples). Lane l < 32 owns sample l
        // (compute wave l / 4, row l % 4). No global stores here but the per-sample results: the
        // DMA waits (vmcnt) would otherwise also wait for the stores' write acknowledgements.
        const int lane = lane_id();
        const int sw = (lane & 31) >> 2, sq = lane & 3;
        auto sums = [&](int i0b, int nb, int pb, float& ld, float& zsq) {
            const float* zt = wtile(sw) + 4 * kSeqsStep + pb * 4 * kSeqsStep + sq * kSeqsStep;
            const float* at = zt + 2 * 4 * kSeqsStep;
            auto step = [&](float a, float z) {
                if constexpr (VAR == NFX_MAF_FORWARD) ld = ld + a;
                else ld = ld - a;
                if constexpr (LOGP) zsq = gauss_sq(zsq, z);
            };
            int j = 0;
            for (; j + 4 <= nb; j += 4) {
                const f32x4 a4 = *reinterpret_cast<const f32x4*>(at + j);
                const f32x4 z4 = *reinterpret_cast<const f32x4*>(zt + j);
#pragma unroll
                for (int c = 0; c < 4; ++c) step(a4[c], z4[c]);
            }
            for (; j < nb; ++j) step(at[j], zt[j]);
            (void)i0b;
        };
        for (int64_t gb = (int64_t)blockIdx.x * kSeqsWaves * 4; gb < B; gb += (int64_t)gridDim.x * kSeqsWaves * 4) {
            float ld = 0.f, zsq = 0.f;
            int i0 = 0, n = blk_end(0), buf = 0;
            int i0p = 0, np = 0;  // the previous block (its tiles have parity buf ^ 1)
            seqs_lds_barrier();  // A: the previous group is done with the staging buffers
            blk_stage(0, 0);
            seqs_dma_wait();
            seqs_lds_barrier();  // B: block 0 is in LDS
            while (i0 < d) {
                const int i0n = i0 + n;
                const int nn = i0n < d ? blk_end(i0n) - i0n : 0;
                if (nn > 0) blk_stage(i0n, buf ^ 1);
                if (np > 0) sums(i0p, np, buf ^ 1, ld, zsq);
                seqs_dma_wait();
                seqs_lds_barrier();  // C: every compute wave is done with the block; the next is in
                i0p = i0;
                np = n;
                i0 = i0n;
                n = nn;
                buf ^= 1;
            }
            // the group's last block (parity buf ^ 1), then the per-sample results
            sums(i0p, np, buf ^ 1, ld, zsq);
            const int64_t s = gb + (lane & 31);
            if (lane < 32 && s < B) {
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
    } else {
    const uint32_t* ctab = reinterpret_cast<const uint32_t*>(P + L.ctab);
    for (int64_t gb = (int64_t)blockIdx.x * kSeqsWaves * 4; gb < B; gb += (int64_t)gridDim.x * kSeqsWaves * 4) {
        const int64_t s = gb + wave * 4 + slot;  // this row's sample
        const bool valid = s < B;
        f32x2 pre1[UPL / 2];
        float h1v[UPL], h2v[UPL];
#pragma unroll
        for (int k = 0; k < UPL; ++k) {
            pre1[k / 2][k % 2] = lds[S.b1 + sub * UPL + k];
            h1v[k] = h2v[k] = 0.f;
        }
        for (int e = lane; e < 4 * kSeqsH3; e += 64) h3_t[e] = 0.f;
        bool poisoned = false;
        int kc = 0;  // byte offset of the chunk's entry in the schedule (made_seqs_chunk_kernel)

        float xr[4];
        int i0 = 0, n = blk_end(0), buf = 0;
        x_load(gb, i0, n, xr);
        seqs_lds_barrier();  // A
        seqs_lds_barrier();  // B

        while (i0 < d) {
            // The block's LDS offset is laundered through an empty asm: the staged blocks sit above
            // 64 KiB, past the reach of a ds_read's immediate offset, and with the constant visible
            // the compiler re-adds it to every read (8 v_add per 16 ranks of the dot products)
            // instead of keeping the whole base in the address VGPR.
            int blk_off = S.blk + buf * S.blkf;
            asm volatile("" : "+v"(blk_off));
            const float* blk = lds + blk_off;
            const float* w1b = blk;
            const float* w4b = blk + W4F;
            const float* bmb = blk + B4F;
            const float* bab = bmb + kSeqsStep;
            float* zout_t = zt2 + buf * 4 * kSeqsStep;  // this block's z / alpha tiles (the staging
            float* at_t = at2 + buf * 4 * kSeqsStep;    // wave reads them during the next block)
#pragma unroll
            for (int q = 0; q < 4; ++q) xin_t[q * kSeqsStep + lane] = xr[q];
            const int i0n = i0 + n;
            const int nn = i0n < d ? blk_end(i0n) - i0n : 0;
            if (nn > 0) x_load(gb, i0n, nn, xr);
            seqs_lds_order();
            SeqsDesc da, db;
            seqs_desc_load_at(ctab, kc, da);

            NFX_TMARK(6);  // block start: input tile, block end, LDS-DMA and x issue
            auto chunk = [&](SeqsDesc& dc, SeqsDesc& dn) -> bool {
                seqs_desc_wait(dc);
                seqs_desc_load_at(ctab, kc + 32, dn);
                // the chunk's schedule: first step, size, completion, completed units before it
                const int ii = dc[0] & 0xff, nc = (dc[0] >> 8) & 0xff;
                const bool completes = (dc[0] >> 16) & 1u, last = (dc[0] >> 18) & 1u;
                const int q = (dc[1] >> 8) & 0xff, gi = (int)(dc[2] >> 16);
                const int i = i0 + ii;
                // 1. lane sub forms step ii + sub's mu/alpha dot products over the completed ranks
                // (< gi; ranks past it hold h3 = 0): the step's W4 row pair (mu, alpha) by rank
                // against the sample's h3 row (one broadcast read per 4 ranks), two chains
                f32x2 acc0 = {0.f, 0.f}, acc1 = {0.f, 0.f};
                {
                    const float* wr = w4b + (ii + sub) * RS4;
                    const float* hr = h3_t + slot * kSeqsH3;
                    const int nq = (gi + 3) >> 2;
#pragma unroll 4
                    for (int qd = 0; qd < nq; ++qd) {
                        const f32x4 hv = *reinterpret_cast<const f32x4*>(hr + 4 * qd);
                        const f32x4 w0 = *reinterpret_cast<const f32x4*>(wr + 8 * qd);
                        const f32x4 w1 = *reinterpret_cast<const f32x4*>(wr + 8 * qd + 4);
                        acc0 = pk_fma(f32x2{w0[0], w0[1]}, hv[0], acc0);
                        acc1 = pk_fma(f32x2{w0[2], w0[3]}, hv[1], acc1);
                        acc0 = pk_fma(f32x2{w1[0], w1[1]}, hv[2], acc0);
                        acc1 = pk_fma(f32x2{w1[2], w1[3]}, hv[3], acc1);
                    }
                }
                // step-3 rows now: their LDS latency overlaps the reductions and step 2; likewise
                // the W2/W3 rows of the next unit to complete (rank gi)
                float w1v[16][UPL], w2n[UPL], w3n[UPL];
                seqs_slots<0, UPL, UPL>(img + S.w2 + gi * Hp + sub * UPL, w2n);
                seqs_slots<0, UPL, UPL>(img + S.w3 + gi * Hp + sub * UPL, w3n);
                {
                    const float* w1r = w1b + ii * Hp + sub * UPL;
#pragma unroll
                    for (int j = 0; j < 16; ++j) seqs_slots<0, UPL, UPL>(w1r + j * Hp, w1v[j]);
                }
                NFX_TMARK(0);  // chunk start + dot products
                // 2. lane sub evaluates step ii + sub (lanes past the chunk compute garbage, unused)
                const bool vj = sub < nc;
                const int rj = ii + sub;
                float mu = (acc0[0] + acc1[0]) + bmb[rj];
                float al = (acc0[1] + acc1[1]) + bab[rj];
                mu = poisoned ? __builtin_nanf("") : mu;
                al = poisoned ? __builtin_nanf("") : al;
                const float xin = xin_t[slot * kSeqsStep + rj];
                float vi, vo, a;
                if constexpr (VAR == NFX_MAF_FORWARD) {
                    // masked_autoregressive_flow.py:57-65
                    a = tclamp(al, -3.f, 3.f);
                    vi = xin * exp_fast(a) + mu;
                } else {
                    // inverse_autoregressive_flow.py:79-88
                    a = tclamp(al, -2.f, 2.f);
                    const float m = tclamp(mu, -10.f, 10.f);
                    vi = (xin - m) * exp_fast(-a);
                }
                // the first non-finite step of the chunk poisons the later ones (and the rest)
                const uint64_t bad = __ballot(vj && nonfinite(vi));
                const unsigned rowbad = (unsigned)(bad >> (slot * 16)) & 0xFFFFu;
                const bool kill = rowbad != 0u && sub > __builtin_ctz(rowbad | 0x10000u);
                vi = kill ? __builtin_nanf("") : vi;
                a = kill ? __builtin_nanf("") : a;
                poisoned = poisoned || rowbad != 0u;
                if constexpr (VAR == NFX_MAF_FORWARD) vo = nonfinite(vi) ? 0.f : vi;
                else vo = nonfinite(vi) ? xin : vi;
                {
                    // branch-free: lanes past the chunk store into the tile's spare 64 floats
                    float* dump = h3_t + 4 * kSeqsH3 + lane;
                    *(vj ? zout_t + slot * kSeqsStep + rj : dump) = vo;
                    *(vj ? at_t + slot * kSeqsStep + rj : dump) = a;
                }
                NFX_TMARK(1);  // rank-1 / W2 / W3 row reads, affine map, poison ballot, step stores
                // every lane of the row needs the chunk's 16 values: DPP row broadcasts
                // (row_newbcast:c), no LDS round trip on the chunk's critical path
                const float cvl = vj ? vi : 0.f;
                float cv[16];
                seqs_row_bcast16(cvl, cv);
                // 3. rank-1 updates of the incomplete slots' layer-1 pre-activations, step order
                const int kc3 = gi >> 4;
                switch (kc3 < UPL ? kc3 : UPL) {
                    case 0: seqs_rank1<0, UPL>(w1v, cv, pre1); break;
                    case 1: seqs_rank1<1, UPL>(w1v, cv, pre1); break;
                    case 2: if constexpr (UPL > 2) seqs_rank1<2, UPL>(w1v, cv, pre1); break;
                    case 3: if constexpr (UPL > 3) seqs_rank1<3, UPL>(w1v, cv, pre1); break;
                    default: break;
                }
                seqs_lds_order();  // the chunk tile is rewritten by the next chunk
                NFX_TMARK(2);  // broadcasts + rank-1 updates
                // 4. the units of degree nextdeg (ranks gi .. q-1) complete: layer 1, 2, 3
                if (completes) {
#pragma unroll
                    for (int k = 0; k < UPL; ++k) {
                        const int p = sub + 16 * k;
                        if (p >= gi && p < q) h1v[k] = trelu(pre1[k / 2][k % 2]);
                    }
                    // layer 2 of every unit of the group, then layer 3 (a unit's h3 reads the h2
                    // of its own group); rank gi with the rows read at the chunk start
                    seqs_unit<UPL>(gi, sub, w2n, h1v, b2v, h2v);
                    for (int p = gi + 1; p < q; ++p) {
                        float w[UPL];
                        seqs_slots<0, UPL, UPL>(img + S.w2 + p * Hp + sub * UPL, w);
                        seqs_unit<UPL>(p, sub, w, h1v, b2v, h2v);
                    }
                    // layer 3 into the sample's LDS h3 row (step 1 reads it by rank)
                    float* h3r = h3_t + slot * kSeqsH3;
                    {
                        const float v = seqs_unit_value<UPL>(gi, w3n, h2v, b3v);
                        if (sub == 0) h3r[gi] = v;
                    }
                    for (int p = gi + 1; p < q; ++p) {
                        float w[UPL];
                        seqs_slots<0, UPL, UPL>(img + S.w3 + p * Hp + sub * UPL, w);
                        const float v = seqs_unit_value<UPL>(p, w, h2v, b3v);
                        if (sub == 0) h3r[p] = v;
                    }
                }
                NFX_TMARK(3);  // completion
                (void)i;
                kc += 32;
                return last;
            };
            for (;;) {  // two schedule entries alternate: no copy of a scalar load in flight
                if (chunk(da, db)) break;
                if (chunk(db, da)) break;
            }
            seqs_lds_order();
            // this wave's 4 output rows for the block (coalesced; the sums: the staging wave)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t so = gb + wave * 4 + q;
                if (so < B && lane < n) out[so * d + i0 + lane] = zout_t[q * kSeqsStep + lane];
            }
            NFX_TMARK(4);  // output rows
            seqs_lds_barrier();  // C: the next block is in LDS, every wave is done with this one
            NFX_TMARK(5);  // barrier
            i0 = i0n;
            n = nn;
            buf ^= 1;
        }
        (void)valid;
    }
    }
#ifdef NFX_SEQS_TIMING
    // timing build only: workgroup 0's first lane overwrites sample 0's first outputs
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (int k = 0; k < 7; ++k) out[k] = (float)tacc[k];
#endif
    if constexpr (LOGP) {
        logp_commit<kSeqsThreads>(lpacc, partials, sums, B);
    }
}

// Pack-time: the rank-ordered LDS prologue image of made_seqs_kernel (W2/W3 rows by completion
// rank, columns by position, biases, degree tables), from the unit-order copies and the degree
// tables made_live_kernel wrote. One launch per pack.
template <int HT>
__global__ __launch_bounds__(256) void made_seqs_image_kernel(float* __restrict__ packed, int d, int H) {
    constexpr int Hp = 32 * HT;
    constexpr int UPL = Hp / 16;
    const MadeLayout L = made_layout(d, HT);
    const SeqsLds S = seqs_lds(Hp);
    const float* P = packed;
    const float* ordD = P + L.s_deg + Hp;
    const float* ordU = P + L.s_deg + 2 * Hp;
    float* img = packed + L.rimg;
    auto rank_at = [](int pos) { return (pos % UPL) * 16 + pos / UPL; };
    for (int e = blockIdx.x * 256 + threadIdx.x; e < Hp * Hp; e += gridDim.x * 256) {
        const int p = e / Hp, q = rank_at(e % Hp);
        const int a = (int)ordU[p], b = (int)ordU[q];
        img[S.w2 + e] = P[L.s_w2 + a * Hp + b];
        img[S.w3 + e] = P[L.s_w3 + a * Hp + b];
    }
    float* tab = img + S.tab;
    // block-ready step rows (made_seqs_kernel's LDS-DMA staging source), zero rows past d
    const int rows = d + kSeqsPadRows;
    constexpr int RS4 = seqs_w4_stride(Hp);
    for (int e = blockIdx.x * 256 + threadIdx.x; e < rows * Hp; e += gridDim.x * 256) {
        const int i = e / Hp, pos = e % Hp;
        packed[L.sw1 + e] = i < d ? P[L.s_w1t + (size_t)i * Hp + (int)ordU[rank_at(pos)]] : 0.f;
    }
    for (int e = blockIdx.x * 256 + threadIdx.x; e < rows * RS4; e += gridDim.x * 256) {
        const int i = e / RS4, c = e % RS4;
        float v = 0.f;
        if (i < d && c < 2 * Hp) v = P[L.s_w4 + (size_t)((c & 1) * d + i) * Hp + (int)ordU[c >> 1]];
        packed[L.sw4 + e] = v;
    }
    for (int e = blockIdx.x * 256 + threadIdx.x; e < 2 * rows; e += gridDim.x * 256) {
        const int jb = e / rows, i = e % rows;
        packed[L.sb4 + e] = i < d ? P[L.s_b4 + jb * d + i] : 0.f;
    }
    for (int p = blockIdx.x * 256 + threadIdx.x; p < Hp; p += gridDim.x * 256) {
        tab[S.b1 + p] = P[L.s_b1 + (int)ordU[rank_at(p)]];
        tab[S.b2 + p] = P[L.s_b2 + (int)ordU[p]];
        tab[S.b3 + p] = P[L.s_b3 + (int)ordU[p]];
        tab[S.deg + p] = ordD[p];
        int q = p + 1;
        while (q < H && ordD[q] == ordD[p]) ++q;
        tab[S.gend + p] = (float)q;
    }
}

// The chunk schedule of the sequential directions, built once at pack time (one lane, serially,
// over LDS copies of the rank tables). It depends only on the degrees, so the sequential kernels
// read it instead of recomputing the bookkeeping per chunk. Entry k (8 words at P + L.ctab):
//   [0] ii (block-relative first step) | nc << 8 | completes << 16 | one << 17 | last-in-block << 18
//   [1] gc (= min(gi, Hp - 1)) | q (group end of gc) << 8 | h3 register slot << 16 | row << 24
//   [2] pos(gc) (its W1t / W2 / W3 column) | gi (completed units before the chunk) << 16   [3] b2[gc]   [4] b3[gc]   [5] W2[gc][gc]   [6] W3[gc][gc]
//   [7] i0 of the chunk's block
// Blocks are made_seqs_kernel's (64 steps, or ending at the last segment end inside them).
template <int HT>
__global__ __launch_bounds__(64) void made_seqs_chunk_kernel(float* __restrict__ packed, int d, int H) {
    constexpr int Hp = 32 * HT;
    constexpr int UPL = Hp / 16;
    const MadeLayout L = made_layout(d, HT);
    const SeqsLds S = seqs_lds(Hp);
    const float* img = packed + L.rimg;
    __shared__ int deg[Hp], gend[Hp];
    __shared__ float b2[Hp], b3[Hp], wd2[Hp], wd3[Hp];
    for (int p = threadIdx.x; p < Hp; p += 64) {
        deg[p] = p < H ? (int)img[S.tab + S.deg + p] : d;
        gend[p] = (int)img[S.tab + S.gend + p];
        b2[p] = img[S.tab + S.b2 + p];
        b3[p] = img[S.tab + S.b3 + p];
        const int pos = (p % 16) * UPL + p / 16;
        wd2[p] = img[S.w2 + p * Hp + pos];
        wd3[p] = img[S.w3 + p * Hp + pos];
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    uint32_t* tab = reinterpret_cast<uint32_t*>(packed + L.ctab);
    const int cap = seqs_max_chunks(d, Hp) - 1;
    int gi = 0, nextdeg = H > 0 ? deg[0] : d, k = 0;
    for (int i0 = 0; i0 < d && k < cap;) {
        int n = kSeqsStep;
        if (i0 + kSeqsStep >= d) {
            n = d - i0;
        } else {
            // the largest segment end (degree + 1) inside (i0, i0 + 64]
            for (int g = 0; g < H; ++g) {
                const int e = deg[g] + 1;
                if (e > i0 && e <= i0 + kSeqsStep) n = e - i0;
            }
        }
        for (int ii = 0; ii < n && k < cap;) {
            const int i = i0 + ii;
            int nc = n - ii < 16 ? n - ii : 16;
            if (nextdeg - i + 1 < nc) nc = nextdeg - i + 1;
            const bool completes = i + nc - 1 == nextdeg;
            const int gc = gi < Hp ? gi : Hp - 1;
            const int q = gend[gc];
            const bool one = completes && q == gi + 1;
            const bool last = ii + nc >= n;
            uint32_t* e = tab + 8 * k;
            e[0] = (uint32_t)ii | (uint32_t)nc << 8 | (uint32_t)completes << 16 | (uint32_t)one << 17 | (uint32_t)last << 18;
            e[1] = (uint32_t)gc | (uint32_t)q << 8 | (uint32_t)(4 * (gc >> 4) + (gc & 3)) << 16 | (uint32_t)((gc >> 2) & 3) << 24;
            e[2] = (uint32_t)((gc % 16) * UPL + gc / 16) | (uint32_t)gi << 16;
            e[3] = __float_as_uint(b2[gc]);
            e[4] = __float_as_uint(b3[gc]);
            e[5] = __float_as_uint(wd2[gc]);
            e[6] = __float_as_uint(wd3[gc]);
            e[7] = (uint32_t)i0;
            if (completes) {
                gi = q;
                nextdeg = gi < H ? deg[gi] : d;
            }
            ii += nc;
            ++k;
        }
        i0 += n;
    }
    uint32_t* e = tab + 8 * k;  // sentinel: a valid, never-consumed prefetch target
    for (int j = 0; j < 8; ++j) e[j] = 0u;
}

typedef void (*made_seqs_kernel_t)(const float*, const float*, float*, float*, int64_t, int, int, int, float*,
                                   double*, double*, float);

template <int HT>
made_seqs_kernel_t made_seqs_pick_ht(int variant, bool logp);

}  // namespace nfx
