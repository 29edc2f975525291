// Shared device helpers for the gfx950 flow kernels.
//
// MFMA tile convention used by every conditioner MLP in this library
// (v_mfma_f32_32x32x2_f32, exact fp32, 64 FLOP/clk/SIMD):
//   D[32 x 32] += A[32 x 2] * B[2 x 32]
//   A: lane l holds A[i = l & 31][k = l >> 5]       (weights, packed on device by *_pack)
//   B: lane l holds B[k = l >> 5][j = l & 31]       (activations, column j = one sample)
//   C/D: lane l, register r holds D[crow(r, l >> 5)][l & 31]
// Activations therefore live "hidden-unit rows x sample columns": a layer's accumulator tile
// is directly the B operand of the next layer (k-step (kt, r) reads register r of tile kt),
// with the weight operand permuted on the host side of the pack to match. No LDS round trip
// and no lane shuffles between layers.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nfx.h"

namespace nfx {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Row of register r in lane-half h of a 32x32 fp32 MFMA accumulator.
__host__ __device__ constexpr int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// torch.clamp semantics: NaN propagates (fminf/fmaxf = IEEE minNum/maxNum would drop it).
// gfx950 has the IEEE-754-2019 NaN-propagating v_maximum3_f32 / v_minimum3_f32, reached
// through the elementwise maximum/minimum builtins: one instruction per bound.
__device__ __forceinline__ float tmax(float a, float b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ float tmin(float a, float b) { return __builtin_elementwise_minimum(a, b); }
__device__ __forceinline__ float tclamp(float v, float lo, float hi) { return tmin(tmax(v, lo), hi); }
__device__ __forceinline__ float tclamp_min(float v, float lo) { return tmax(v, lo); }
// torch.relu == clamp_min(0): NaN propagates.
__device__ __forceinline__ float trelu(float v) { return tmax(v, 0.f); }
// torch.isnan(v) | torch.isinf(v)
__device__ __forceinline__ bool nonfinite(float v) { return !__builtin_isfinite(v); }

// Sum of lane-halves with the lane<->sample convention of the small-d epilogues:
// lanes 0..31 return p0[l] + p0[l+32], lanes 32..63 return p1[l-32] + p1[l].
// v_permlane32_swap: vdst[32..63] <-> vsrc[0..31]; afterwards vdst + vsrc is exactly that.
__device__ __forceinline__ float halves_sum(float p0, float p1) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(p0), __float_as_uint(p1), false,
                                              false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// Same exchange without the add: lanes 0..31 get p0[l+32] (the other half of tile 0),
// lanes 32..63 get p1[l-32] (the other half of tile 1).
__device__ __forceinline__ float halves_other(float p0, float p1) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(p0), __float_as_uint(p1), false,
                                              false);
    return (threadIdx.x & 32) ? __uint_as_float(r[0]) : __uint_as_float(r[1]);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// 16 bias values of one accumulator tile for lane-half h: 4 x 16-byte reads, same address for
// every lane of the half (broadcast), straight into the accumulator registers.
__device__ __forceinline__ f32x16 load_bias16(const float* __restrict__ tile, int h) {
    const f32x4* p = reinterpret_cast<const f32x4*>(tile + 16 * h);
    const f32x4 a = p[0], b = p[1], c = p[2], e = p[3];
    return f32x16{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3], c[0], c[1], c[2], c[3], e[0], e[1], e[2], e[3]};
}

// The same bias tile into two accumulators (the two sample tiles of a 64-sample chunk) with two
// LDS reads instead of one read + 16 v_mov: LDS bandwidth is idle here, while the fp32 vector
// pipe is the bound (the copies cost as much as 16 VALU ops per tile). The opaque zero keeps the
// compiler from merging the two reads.
__device__ __forceinline__ int opaque_zero();
__device__ __forceinline__ void load_bias16_x2(const float* __restrict__ tile, int h, f32x16& a0, f32x16& a1) {
    a0 = load_bias16(tile, h);
    a1 = load_bias16(tile + opaque_zero(), h);
}

// A zero the compiler cannot see through. Offsetting the LDS weight pointer by it inside a
// grid-stride loop stops LICM from hoisting every (loop-invariant) weight read out of the
// loop into registers, which would otherwise blow the VGPR budget and spill.
__device__ __forceinline__ int opaque_zero() {
    int z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    return z;
}

__device__ __forceinline__ void wave_lds_sync() {
    // A wave's DS operations execute in order; this only stops the compiler from moving LDS
    // accesses across the point (the tile is wave-private, no workgroup barrier needed).
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup sum of a float64 (NT threads, wave64 shuffles then one LDS hop). Result valid in
// thread 0. Deterministic order.
template <int NT>
__device__ __forceinline__ double block_sum_f64(double v) {
    __shared__ double red[NT / 64];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < NT / 64; ++w) t += red[w];
    return t;
}

// exp(x) for finite x <= 87 (the affine/MADE callers clamp the scale exponent to +-10 first):
// x*log2(e) is carried as a compensated pair (t, e), the hardware exp2 takes the rounded t and
// the product's rounding error is folded back as exp2(t) * (1 + e*ln2). A few ulp like expf, in
// 6 instructions instead of OCML's 13 (range reduction and overflow paths are not needed here;
// results below 2^-126 flush to 0 where expf returns a subnormal). NaN propagates. An infinite
// argument gives NaN (inf - inf in the correction): use exp_safe where x may be -inf.
__device__ __forceinline__ float exp_fast(float x) {
    const float t = x * 1.44269502f;
    const float e = __builtin_fmaf(x, 1.44269502f, -t) + x * 1.9259629e-8f;
    const float r = __builtin_amdgcn_exp2f(t);
    return __builtin_fmaf(r, e * 0.693147182f, r);
}
// exp_fast for arguments that may be -inf or hugely negative (spline softmax numerators
// p_k - max p, softplus inputs): one NaN-propagating max first, so exp(-inf) = 0 like expf.
// Below -103.3 expf is already 0; between -103.3 and -87.3 it is subnormal and this flushes
// (the spline consumers add min_bin_width / min_derivative = 1e-3 to it, so no output changes).
__device__ __forceinline__ float exp_safe(float x) { return exp_fast(tmax(x, -128.f)); }

// fp32(d * log(2*pi)) exactly as torch's MultivariateNormal.log_prob rounds it.
inline float gauss_const(int d) { return (float)((double)d * 1.8378770664093453); }

// Gaussian log-density pieces with every rounding explicit (no FMA contraction), so the fused
// epilogues and nfx_gauss_logprob produce bit-identical logp: m = sum_j z_j^2 in order, then
// logp = -0.5 * (m + c) + log_det (separate mul/add, as torch's CPU kernels round).
// (__fadd_rn/__fmul_rn alone do not stop the backend from fusing; the pragma does.)
__device__ __forceinline__ float gauss_sq0(float v) { return v * v; }
__device__ __forceinline__ float gauss_sq(float m, float v) {
#pragma clang fp contract(off)
    return m + v * v;
}
__device__ __forceinline__ float gauss_lp(float m, float c, float ld) {
#pragma clang fp contract(off)
    return -0.5f * (m + c) + ld;
}

// Capacity (doubles) of the partial-sum workspace shared by nfx_gauss_logprob and the fused
// *_logprob layer epilogues; every launch that writes partials uses at most this many blocks.
// The workspace holds kMaxPartials doubles of partials, then the 64-bit arrival word of
// logp_commit (any content on entry, below).
constexpr int kMaxPartials = 4096;  // < 2^16: the arrival word's count field

// End of a fused log_prob epilogue: each workgroup's float64 sum of its log-densities goes to
// partials[blockIdx.x]; the LAST workgroup to arrive (agent-scope counter after the workspace's
// partials) reduces them into sums = [sum, (double)B] and resets the counter — no separate finish
// launch. The reduction replays gauss_finish_kernel's order exactly (256 strided accumulators, a
// shuffle-down tree per 64, the four wave sums in order), so fused and unfused results agree bit
// for bit whatever the workgroup size NT (a multiple of 64).
//
// The arrival word is 64-bit: [63:16] a tag, [15:0] the count (round 6; ABI version 3). A clean
// word holds the fixed tag kLogpClean with count 0, and every launch's last workgroup stores that
// back. A workgroup adds 1 to the word (one atomic, as the ABI-2 counter did) and, when the value
// it got back carries the clean tag, its count IS the arrival index. Anything else in the word — a
// workspace that was never initialised (torch.empty, 0xFF fills, a reused allocation holding
// other data, or all zeros) — is overwritten by ONE compare-and-swap to "clean tag, count 1" by
// the first workgroup to find it; workgroups that met the foreign value meanwhile retry on the
// clean word, so the count stays exact. Only that first launch on a fresh workspace pays the
// swaps (nfx_gauss_workspace_init writes the clean word instead). A foreign word matches the tag
// with probability 2^-48. (A count left mid-launch cannot be met: a launch that does not finish
// faults the device and ends the process.)
constexpr uint64_t kLogpClean = 0x4E46584C5047ull << 16;  // "NFXLPG", count 0

template <int NT>
__device__ __forceinline__ void logp_commit(double v, double* partials, double* sums, int64_t B) {
    static_assert(NT % 64 == 0, "whole waves");
    const double t = block_sum_f64<NT>(v);
    __shared__ int last;
    __shared__ double red4[4];
    uint64_t* cnt = reinterpret_cast<uint64_t*>(partials + kMaxPartials);
    if (threadIdx.x == 0) {
        partials[blockIdx.x] = t;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        uint64_t prev = __hip_atomic_fetch_add(cnt, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while ((prev & ~0xFFFFull) != kLogpClean) {
            // foreign word (rare): my add did not count. Claim the word, or add to the clean one
            uint64_t cur = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((cur & ~0xFFFFull) == kLogpClean) {
                prev = __hip_atomic_fetch_add(cnt, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (__hip_atomic_compare_exchange_strong(cnt, &cur, kLogpClean | 1u, __ATOMIC_RELAXED,
                                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                prev = kLogpClean;
            }
        }
        last = (unsigned)(prev & 0xFFFFu) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int n = (int)gridDim.x, lane = threadIdx.x & 63;
    for (int vw = threadIdx.x >> 6; vw < 4; vw += NT / 64) {
        double acc = 0.0;
        for (int i = vw * 64 + lane; i < n; i += 256) acc += partials[i];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
        if (lane == 0) red4[vw] = acc;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int w = 0; w < 4; ++w) s += red4[w];
        sums[0] = s;
        sums[1] = (double)B;
        __hip_atomic_store(cnt, kLogpClean, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace nfx

// Error reporting shared by the C-ABI translation units (nfx_abi.hip).
namespace nfx {
int set_error(int code, const char* fmt, ...);
int check_launch(const char* what);
int num_cus();
// Workgroups that fill every CU at the kernel's occupancy, capped by the available work.
int resident_grid(const void* kernel, int threads, size_t lds_bytes, int64_t work_groups);
// Raise the dynamic-LDS limit of `kernel` when it needs more than 64 KiB.
int prepare_lds(const void* kernel, size_t bytes);
// out[i] = sum_w part[w * len + i] (float partials of nw workgroups, float64 result, fixed order).
int train_sum_finish(const float* part, int nw, int len, double* out, hipStream_t s);
// Reduce n float64 partials into sums[0] = total, sums[1] = (double)B (one 256-thread block).
int gauss_finish(const double* partials, int n, double* sums, int64_t B, hipStream_t s);
}  // namespace nfx
