// Sequential MADE-affine directions, PUSH formulation, one wave per sample (MAF.forward =
// sampling, IAF.inverse = density; H <= 64, d <= 1024) — the strong-scaling shard kernel.
//
// Reference: masked_autoregressive_flow.py:46-78, inverse_autoregressive_flow.py:65-103 (d full
// MADE calls on the partially filled vector). As in made_seqs_kernel / made_seqw_kernel every
// hidden unit is computed once, when the input of its degree is known, so a sample costs one
// MADE evaluation; what differs is where the work sits relative to the sample's dependent chain
// (unit g completes -> the steps up to the next completion -> unit g + 1 completes -> ...).
// Those kernels PULL each step's (mu, alpha) as a dot product over the completed units' h3 when
// the step is reached, and keep every unit's layer-1 pre-activation current with per-chunk rank-1
// updates; both sit on the chain's instruction stream (~212 instructions per chunk in
// made_seqw_kernel, one wave per SIMD issuing one instruction per 4 cycles). Here:
//   * every step's (mu, alpha) accumulator lives in a register of the lane that owns the step
//     (lane l of slot s = step 64 s + l; 13 slots at d = 784), initialised with the biases; when
//     unit g completes, its h3 is PUSHED into every later step at once: one packed FMA per slot
//     with unit g's (mu, alpha) output column, streamed from the L2-resident pw4 image one stage
//     ahead. A step's (mu, alpha) is complete when it is reached; the chunk of steps between two
//     completions is evaluated where it lies (its lanes, under the chunk's lane mask);
//   * the layer-1 pre-activation of the unit that completes is formed only then, as one wave sum
//     of W1[g][step] * z[step] over the slots so far (pw1 row, prefetched one stage ahead);
//     layers 2 and 3 keep made_seqw_kernel's running per-unit sums (acc2, acc3; lane p = unit of
//     completion rank p), so only the diagonal terms are on the chain;
//   * the log-det and the fused Gaussian z^2 are summed in step order (the reference's
//     sequential fp32 `ld -= alpha_i`, nfx_gauss_logprob's z^2 order) by a fifth, summing wave
//     from per-slot LDS tiles the compute waves publish (an LDS counter per slot), so the compute
//     waves carry no serial reductions;
//   * the outputs stay in registers until the sample is done (no global stores in flight to
//     stall the prefetch's vmcnt waits).
// The slots are unrolled at compile time (S = ceil(d / 64)), so every register index is static.
// Non-finite steps poison every later step exactly as in made_seqw_kernel (kill the chunk's later
// lanes, NaN into every accumulator), on a branch that finite inputs never take; several units of
// one degree (MADE connects equal degrees) complete on a separate path.
#pragma once
#include "nfx_made_seqw_kernel.h"

namespace nfx {

constexpr int kSeqpWaves = 4;                        // compute waves per workgroup, one sample each
constexpr int kSeqpThreads = 64 * (kSeqpWaves + 1);  // + the summing wave

// Schedule entry (16 words at P + L.ptab, made_seqp_chunk_kernel):
//   [0], [1] lane mask of the chunk's steps in slot K; [4] flags | g << 8 | n2 << 16 (g = the unit
//   the chunk completes, or the next one to complete; n2 = the steps of slot K + 1 a crossing chunk
//   also covers); [5] byte offset of unit g's pw4 column; [6], [7] byte offsets of unit u's pw1 row
//   and pw23 row (u = the unit the next chunk completes); [8], [9], [14] b1[g], W2[g][g], W3[g][g];
//   [2, 3] / [10, 11] / [12, 13] lane masks (all ones or 0) switching on unit g's layer-1 / -2 / -3
//   results: all three when g alone completes; several units of one degree (MADE connects equal
//   degrees) complete as one chunk with layer 1 of the first unit, then empty chunks with layer 1
//   of each other unit, layer 2 of each (W2[g][g] = 0: the running sums already hold the whole
//   group) and layer 3 of each.
constexpr uint32_t kSpSlotEnd = 1u;  // the slot's last chunk (crossing chunks included)
constexpr uint32_t kSpCross = 2u;    // the chunk also covers the start of slot K + 1

typedef uint32_t SeqpDesc __attribute__((ext_vector_type(16)));
__device__ __forceinline__ void seqp_desc_load(const uint32_t* base, int off, SeqpDesc& o) {
    asm volatile("s_load_dwordx16 %0, %1, %2" : "=s"(o) : "s"(base), "s"(off) : "memory");
}
__device__ __forceinline__ void seqp_desc_wait(SeqpDesc& o) { asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(o)); }

// LDS: per compute wave a z tile and an alpha tile of S slots, then S slot counters
__host__ __device__ inline int seqp_lds_floats(int S) { return kSeqpWaves * 2 * 64 * S + 64; }

// Per-lane state of one sample. Slot s: step 64 s + lane. The prefetched images come in 16-byte
// pieces: W4q[j] = unit g's (mu, alpha) weights of slots 2j, 2j + 1; W1q[j] = unit u's W1 weights
// of slots 4j .. 4j + 3. acc23 = (layer-2, layer-3) running sums of unit `lane` (biases included).
template <int S>
struct SeqpState {
    float X[S], Z[S], Al[S];
    f32x2 A[S];
    f32x4 W4q[(S + 1) / 2], W1q[(S + 3) / 4];
    f32x2 w23, acc23;
    float h3g;
#ifdef NFX_SEQP_TIMING
    long long tacc[8], tmark;
#endif
};
// Stage clocks (timing build only, -DNFX_SEQP_TIMING; tools/seqp_timing.py): ticks since the last
// mark added to stage k.
#ifdef NFX_SEQP_TIMING
#define NFX_PMARK(st, k) do { const long long t_ = clock64(); (st).tacc[k] += t_ - (st).tmark; (st).tmark = t_; } while (0)
#else
#define NFX_PMARK(st, k) do { } while (0)
#endif

struct SeqpCtx {
    __amdgpu_buffer_rsrc_t pr;  // the packed image (byte offsets)
    int lane;
    float* zt;  // this wave's z tile
    float* at;  // this wave's alpha tile
    int* cnt;   // slot counters
};

__device__ __forceinline__ f32x2 seqp_ld2(const SeqpCtx& c, int voff, int soff) {
    return __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(c.pr, voff, soff, 0));
}
__device__ __forceinline__ f32x4 seqp_ld4(const SeqpCtx& c, int voff, int soff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(c.pr, voff, soff, 0));
}
// lane in mask ? t : f (one v_cndmask with the SGPR-pair mask)
__device__ __forceinline__ float seqp_sel(uint64_t m, float t, float f) {
    float r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
    return r;
}
__device__ __forceinline__ uint64_t seqp_mask(uint32_t lo, uint32_t hi) { return (uint64_t)hi << 32 | lo; }
// Keeps a value materialised here: the compiler may not sink its computation past this point
// (a sunk push would keep the prefetch registers live across their reload, i.e. copies that wait).
template <typename T>
__device__ __forceinline__ void seqp_pin(T& v) { asm volatile("" : "+v"(v)); }
// A use of every element here: a prefetched 16-byte piece whose elements are not all read (slots
// before the current one or past the last) would otherwise free those registers for temporaries
// while the load is in flight (a write-after-write hazard the hardware resolves by waiting).
template <typename T>
__device__ __forceinline__ void seqp_use(const T& v) { asm volatile("" ::"v"(v)); }

// Sum over the wave: row sums, then rows 0 + 1 and 2 + 3 (row_bcast:15), then all four
// (row_bcast:31; lanes of disabled rows keep their value); the total is lane 63's, returned
// uniform. (The s_nop covers the DPP read-after-VALU-write hazard the asm hides from the compiler.)
__device__ __forceinline__ float seqp_wave_sum(float v) {
#ifdef NFX_SEQP_ABL_SUM  // timing ablation only (wrong results): no cross-lane reduction
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
#endif
    v = row16_allsum(v);
    asm volatile(
        "s_nop 1\n\t"
        "v_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
        : "+v"(v));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// The affine map of slot K under mask M: z and the clamped alpha kept for the mask's lanes
// (separate roundings, as the reference's torch ops). Returns the raw value.
template <int VAR>
__device__ __forceinline__ float seqp_affine(const f32x2 p, float x, uint64_t M, float& z, float& al) {
#pragma clang fp contract(off)
    float v, a;
#ifdef NFX_SEQP_ABL_AFF  // timing ablation only (wrong results): the affine map without clamp / exp
    a = p[1];
    v = x - p[0];
    z = seqp_sel(M, v, z);
    al = seqp_sel(M, a, al);
    return v;
#endif
    if constexpr (VAR == NFX_MAF_FORWARD) {
        a = tclamp(p[1], -3.f, 3.f);
        v = x * exp_fast(a) + p[0];
    } else {
        a = tclamp(p[1], -2.f, 2.f);
        const float m = tclamp(p[0], -10.f, 10.f);
        v = (x - m) * exp_fast(-a);
    }
    z = seqp_sel(M, v, z);
    al = seqp_sel(M, a, al);
    return v;
}

// One chunk of slot K. Branch-free on the hot path, and ordered so that each prefetched register
// is dead before its next load is issued (no copies that would wait for loads in flight): the
// last completion's h3 is pushed, unit g's column re-issued, the chunk's steps evaluated, unit g
// completed (its results selected away where the flags say so), unit u's rows issued.
// Returns true at the slot's last chunk.
template <int K, int S, int VAR>
__device__ __forceinline__ bool seqp_chunk(SeqpState<S>& st, const SeqpCtx& c, SeqpDesc& e) {
    constexpr int KE = K + 1 < S ? K + 1 : S - 1;  // the completion sum's last slot
    constexpr int KL = K + 2 < S ? K + 2 : S - 1;  // the prefetched W1 row's last slot
#ifdef NFX_SEQP_NEAR
    // timing ablation only (wrong results): the chain wave's share of a two-wave split — pushes
    // into slots K .. K + 2, the layer-1 sum over slots K - 1 .. K + 1
    constexpr int SP = K + 3 < S ? K + 3 : S;
    constexpr int S0 = K > 0 ? K - 1 : 0;
#else
    constexpr int SP = S;
    constexpr int S0 = 0;
#endif
    // 1. the last completion's h3 into every later step (needs nothing from the entry)
#pragma unroll
    for (int j = (K > 0 ? K - 1 : 0) / 2; j < (SP + 1) / 2; ++j) seqp_use(st.W4q[j]);
#pragma unroll
    for (int s = K; s < SP; ++s) {
        const f32x4 w = st.W4q[s / 2];
        st.A[s] = pk_fma((s & 1) ? f32x2{w[2], w[3]} : f32x2{w[0], w[1]}, st.h3g, st.A[s]);
        seqp_pin(st.A[s]);
    }
    seqp_desc_wait(e);
    NFX_PMARK(st, 0);  // push + entry
    const uint32_t fl = e[4];
    const int g = (fl >> 8) & 0xff;
    const uint64_t M = seqp_mask(e[0], e[1]);
    const uint64_t M2 = ((1ull << ((fl >> 16) & 63)) - 1ull);
    // 2. unit g's column in flight until the next chunk pushes it
#pragma unroll
    for (int j = K / 2; j < (SP + 1) / 2; ++j) st.W4q[j] = seqp_ld4(c, 16 * c.lane + 1024 * j, (int)e[5]);
    // 3. the chunk's steps
    const float v = seqp_affine<VAR>(st.A[K], st.X[K], M, st.Z[K], st.Al[K]);
    float v2 = 0.f;
    if constexpr (K + 1 < S) {
        if (fl & kSpCross) v2 = seqp_affine<VAR>(st.A[K + 1], st.X[K + 1], M2, st.Z[K + 1], st.Al[K + 1]);
    }
    NFX_PMARK(st, 1);  // column issue + affine
    // 4. unit g's layer-1 sum over every step so far (b1 in lane 0), the diagonal terms of layers 2, 3
    {
        float t = seqp_sel(1ull, __uint_as_float(e[8]), 0.f);
#pragma unroll
        for (int j = S0 / 4; j <= KL / 4; ++j) seqp_use(st.W1q[j]);
#pragma unroll
        for (int s = S0; s <= KE; ++s) t = fmaf(st.W1q[s / 4][s % 4], st.Z[s], t);
        const float wd2 = __uint_as_float(e[9]), wd3 = __uint_as_float(e[14]);
        const float P2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(st.acc23[0]), g));
        const float P3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(st.acc23[1]), g));
        const float tsum = seqp_wave_sum(t);
        NFX_PMARK(st, 2);  // W1 wait + layer-1 sum
#ifdef NFX_SEQP_ABL_CHAIN  // timing ablation only (wrong results): layers 1-3 of the completing unit skipped
        const float h1 = tsum, h2 = tsum + wd2 * 0.f * P2, h3 = tsum + wd3 * 0.f * P3;
#else
        const float h1 = trelu(tsum);
        const float h2 = trelu(fmaf(wd2, h1, P2));
        const float h3 = trelu(fmaf(wd3, h2, P3));
#endif
        const uint64_t c1 = seqp_mask(e[2], e[3]), c2 = seqp_mask(e[10], e[11]), c3 = seqp_mask(e[12], e[13]);
        st.acc23 = __builtin_elementwise_fma(st.w23, f32x2{seqp_sel(c1, h1, 0.f), seqp_sel(c2, h2, 0.f)}, st.acc23);
        seqp_pin(st.acc23);
        st.h3g = seqp_sel(c3, h3, 0.f);
        NFX_PMARK(st, 3);  // layers 1-3 chain
    }
    // 5. the rows of unit u, in flight until the next chunk completes it
#pragma unroll
    for (int j = S0 / 4; j <= KL / 4; ++j) st.W1q[j] = seqp_ld4(c, 16 * c.lane + 1024 * j, (int)e[6]);
    st.w23 = seqp_ld2(c, 8 * c.lane, (int)e[7]);
    // 6. a non-finite step kills the chunk's later steps; NaN through the next push poisons every
    // later one (cold)
    const uint64_t bad = __ballot(nonfinite(v)) & M;
    const uint64_t bad2 = (K + 1 < S && (fl & kSpCross)) ? __ballot(nonfinite(v2)) & M2 : 0ull;
    if (bad | bad2) {
        uint64_t k1 = 0, k2 = 0;
        if (bad) {
            k1 = M & ~((2ull << __builtin_ctzll(bad)) - 1ull);
            k2 = (fl & kSpCross) ? M2 : 0ull;
        } else {
            k2 = M2 & ~((2ull << __builtin_ctzll(bad2)) - 1ull);
        }
        st.Z[K] = seqp_sel(k1, __builtin_nanf(""), st.Z[K]);
        st.Al[K] = seqp_sel(k1, __builtin_nanf(""), st.Al[K]);
        if constexpr (K + 1 < S) {
            st.Z[K + 1] = seqp_sel(k2, __builtin_nanf(""), st.Z[K + 1]);
            st.Al[K + 1] = seqp_sel(k2, __builtin_nanf(""), st.Al[K + 1]);
        }
        st.h3g = __builtin_nanf("");
    }
    NFX_PMARK(st, 4);  // rows issue + poison check
    return (fl & kSpSlotEnd) != 0;
}

template <int VAR>
__device__ __forceinline__ float seqp_guard(float z, float x) {
    if constexpr (VAR == NFX_MAF_FORWARD) return nonfinite(z) ? 0.f : z;
    else return nonfinite(z) ? x : z;
}

// Slot K: its chunks (each chunk's entry is scalar-loaded as it starts; the push before its
// first use covers the latency), then the slot's guarded outputs and alphas go to the LDS tiles
// for the summing wave.
template <int K, int S, int VAR>
__device__ __forceinline__ void seqp_slots(SeqpState<S>& st, const SeqpCtx& c, const uint32_t* ctab, int& kc,
                                           int kcap) {
    for (;;) {
        SeqpDesc e;
        seqp_desc_load(ctab, kc, e);
        kc = kc + 64 < kcap ? kc + 64 : kcap;  // the last entry is a slot-ending sentinel
        if (seqp_chunk<K, S, VAR>(st, c, e)) break;
    }
    c.zt[64 * K + c.lane] = seqp_guard<VAR>(st.Z[K], st.X[K]);
    c.at[64 * K + c.lane] = st.Al[K];
    if (c.lane == 0) __hip_atomic_fetch_add(&c.cnt[K], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    NFX_PMARK(st, 5);  // slot end
    if constexpr (K + 1 < S) seqp_slots<K + 1, S, VAR>(st, c, ctab, kc, kcap);
}

template <int HT, int VAR, bool LOGP, int S>
__global__ __launch_bounds__(kSeqpThreads) void made_seqp_kernel(
    const float* __restrict__ packed, const float* __restrict__ in, float* __restrict__ out,
    float* __restrict__ logdet, int64_t B, int d, int H, int accumulate, float* __restrict__ logp,
    double* __restrict__ partials, double* __restrict__ sums, float cgauss) {
    constexpr int Hp = 32 * HT;
    const MadeLayout L = made_layout(d, HT);
    extern __shared__ f32x4 lds4[];
    float* lds = reinterpret_cast<float*>(lds4);
    int* cnt = reinterpret_cast<int*>(lds + kSeqpWaves * 2 * 64 * S);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = lane_id();
    if (threadIdx.x < S) cnt[threadIdx.x] = 0;
    __syncthreads();
    double lpacc = 0.0;

    if (wave == kSeqpWaves) {
        // ---------------- summing wave: lane w < 4 sums compute wave w's sample in step order
        const float* zt = lds + (lane & 3) * 2 * 64 * S;
        const float* at = zt + 64 * S;
        for (int64_t gb = (int64_t)blockIdx.x * kSeqpWaves; gb < B; gb += (int64_t)gridDim.x * kSeqpWaves) {
            float ld = 0.f, zsq = 0.f;
            for (int k = 0; k < S; ++k) {
                // (bounded: a schedule fault cannot hang the device, only garble this group)
                for (int spin = 0; spin < (1 << 24) &&
                                   __hip_atomic_load(&cnt[k], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < kSeqpWaves;
                     ++spin)
                    __builtin_amdgcn_s_sleep(1);
                const int n = d - 64 * k < 64 ? d - 64 * k : 64;
                const float* zr = zt + 64 * k;
                const float* ar = at + 64 * k;
                auto step = [&](float av, float zv) {
                    if constexpr (VAR == NFX_MAF_FORWARD) ld = ld + av;
                    else ld = ld - av;
                    if constexpr (LOGP) zsq = gauss_sq(zsq, zv);
                };
                int j = 0;
                for (; j + 4 <= n; j += 4) {
                    const f32x4 a4 = *reinterpret_cast<const f32x4*>(ar + j);
                    const f32x4 z4 = *reinterpret_cast<const f32x4*>(zr + j);
#pragma unroll
                    for (int u = 0; u < 4; ++u) step(a4[u], z4[u]);
                }
                for (; j < n; ++j) step(ar[j], zr[j]);
            }
            if (lane < S) cnt[lane] = 0;
            const int64_t s = gb + lane;
            if (lane < kSeqpWaves && s < B) {
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
            __syncthreads();  // the tiles and counters are free for the next group
        }
    } else {
        // ---------------- compute waves: one sample each
        SeqpCtx c;
        c.pr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(packed), 0, 0x7FFFFFFF, 0x00020000);
        c.lane = lane;
        c.zt = lds + wave * 2 * 64 * S;
        c.at = c.zt + 64 * S;
        c.cnt = cnt;
        const uint32_t* ctab = reinterpret_cast<const uint32_t*>(packed + L.ptab);
        constexpr int S2 = (S + 1) / 2, S4 = (S + 3) / 4;
        for (int64_t gb = (int64_t)blockIdx.x * kSeqpWaves; gb < B; gb += (int64_t)gridDim.x * kSeqpWaves) {
            const int64_t s = gb + wave;
            const bool valid = s < B;
            const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in) + (valid ? s : 0) * d, 0, d * 4,
                                                              0x00020000);
            SeqpState<S> st;
#pragma unroll
            for (int k = 0; k < S; ++k) {
                st.X[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, 4 * (64 * k + lane), 0, 0));
                st.A[k] = seqp_ld2(c, 8 * lane + 512 * k, 4 * L.pb4);
                st.Z[k] = 0.f;
                st.Al[k] = 0.f;
            }
            // nothing pushed before the first chunk; unit 0's rows; the running sums start at b2, b3
#pragma unroll
            for (int j = 0; j < S2; ++j) st.W4q[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < S4; ++j) st.W1q[j] = seqp_ld4(c, 16 * lane + 1024 * j, 4 * L.pw1);
            st.w23 = seqp_ld2(c, 8 * lane, 4 * L.pw23);
            st.acc23 = f32x2{lane < Hp ? packed[L.ptb + Hp + (lane & (Hp - 1))] : 0.f,
                             lane < Hp ? packed[L.ptb + 2 * Hp + (lane & (Hp - 1))] : 0.f};
            st.h3g = 0.f;
#ifdef NFX_SEQP_TIMING
            for (int k = 0; k < 8; ++k) st.tacc[k] = 0;
            st.tmark = clock64();
#endif
            int kc = 0;
            seqp_slots<0, S, VAR>(st, c, ctab, kc, 64 * (seqp_max_chunks(d, Hp) - 1));
            const auto orr = __builtin_amdgcn_make_buffer_rsrc(out + (valid ? s : 0) * d, 0, valid ? d * 4 : 0,
                                                               0x00020000);
#pragma unroll
            for (int k = 0; k < S; ++k)
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(seqp_guard<VAR>(st.Z[k], st.X[k])), orr,
                                                      4 * (64 * k + lane), 0, 0);
            NFX_PMARK(st, 6);  // stores
#ifdef NFX_SEQP_TIMING
            // timing build only: workgroup 0's first lane overwrites sample 0's first outputs
            if (blockIdx.x == 0 && threadIdx.x == 0 && gb == 0)
                for (int k = 0; k < 8; ++k) out[k] = (float)st.tacc[k];
#endif
            __syncthreads();  // the summing wave is done with this group's tiles
        }
    }
    if constexpr (LOGP) {
        logp_commit<kSeqpThreads>(lpacc, partials, sums, B);
    }
}

typedef void (*made_seqp_kernel_t)(const float*, const float*, float*, float*, int64_t, int, int, int, float*,
                                   double*, double*, float);

}  // namespace nfx
