// Shared pieces of the one-launch coupling chains (nfx_affine_chain.hip: small-batch layout,
// nfx_affine_schain.hip: streaming layout for large batches).
#pragma once
#include "nfx_affine_kernel.h"

namespace nfx {

constexpr int kChainMax = 64;
struct NfxChainPacks {
    const float* p[kChainMax];
};

// LDS-DMA of 16 bytes per lane: lane l's float4 at `src` (per-lane address) lands at LDS
// lds_dst + 16 l. Issued as inline asm so the compiler does not see an LDS write in flight (the
// builtin would make it wait vmcnt(0) before every later ds_read, which cannot alias the other
// buffer the DMA targets); completion is waited for explicitly (lds_dma_wait) before the
// barrier that publishes the buffer.
// lds_addr: the LDS byte address (lds_addr_of of the shared array + offset).
__device__ __forceinline__ void lds_dma_x4(const float* src, uint32_t lds_addr) {
    const uint32_t m = lds_addr;
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
template <typename T>
__device__ __forceinline__ uint32_t lds_addr_of(T* shared_array) {
    return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) T*)shared_array);
}
__device__ __forceinline__ void lds_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---- the on-device base draw of the fused sampling chain (nfx_affine_chain_sample) ----------
// Philox4x32-10 (Salmon et al., SC'11 — the counter-based generator torch's CUDA/HIP normal_
// uses; not its stream: a separate generator state), counter = (sample row, word block, offset),
// key = seed; Box-Muller turns each pair of words into two N(0, 1) values.
__device__ __forceinline__ void philox4x32_10(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = 0xD2511F53u * c[0], hi0 = __umulhi(0xD2511F53u, c[0]);
        const uint32_t lo1 = 0xCD9E8D57u * c[2], hi1 = __umulhi(0xCD9E8D57u, c[2]);
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = lo1;
        c[2] = n2;
        c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}
// Two standard normals from two uniform words (u1 in (0, 1], so log never sees 0).
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
    const float u1 = ((float)(a >> 8) + 1.f) * 5.9604645e-8f;  // (0, 1], 2^-24 steps
    const float u2 = (float)(b >> 8) * 5.9604645e-8f;          // [0, 1)
    const float r = sqrtf(-2.f * logf(u1));
    float sn, cs;
    sincospif(2.f * u2, &sn, &cs);
    z0 = r * cs;
    z1 = r * sn;
}
// The D base values of sample `row` (D <= 8: one Philox block per four values).
template <int D>
__device__ __forceinline__ void base_draw(int64_t row, uint64_t seed, uint64_t offset, float (&z)[D]) {
#pragma unroll
    for (int blk = 0; blk < (D + 3) / 4; ++blk) {
        uint32_t c[4] = {(uint32_t)row, (uint32_t)((uint64_t)row >> 32) ^ ((uint32_t)blk << 24), (uint32_t)offset,
                         (uint32_t)(offset >> 32)};
        philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
        float g[4];
        box_muller(c[0], c[1], g[0], g[1]);
        box_muller(c[2], c[3], g[2], g[3]);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (4 * blk + q < D) z[4 * blk + q] = g[q];
    }
}

// Streaming chain (nfx_affine_schain.hip): which (B, d, H) it takes and its launch.
int schain_launch(const NfxChainPacks& P, int nl, const float* in, float* out, float* log_det, int64_t B, int d,
                  int H, int direction, int accumulate, float* logp, double* sums, void* workspace, hipStream_t s);
bool schain_supported(int64_t B, int d, int H);
// The affine kernel policy (nfx_affine_kernel_policy; nfx_affine.hip).
int affine_policy_get();
// AUTO: the small-batch chain up to this batch, the streaming chain above it.
constexpr int64_t kSmallChainMaxB = 1 << 16;

}  // namespace nfx
