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

// Streaming chain (nfx_affine_schain.hip): which (B, d, H) it takes and its launch.
int schain_launch(const NfxChainPacks& P, int nl, const float* in, float* out, float* log_det, int64_t B, int d,
                  int H, int direction, int accumulate, float* logp, double* sums, void* workspace, hipStream_t s);
bool schain_supported(int64_t B, int d, int H);
// The affine kernel policy (nfx_affine_kernel_policy; nfx_affine.hip).
int affine_policy_get();
// AUTO: the small-batch chain up to this batch, the streaming chain above it.
constexpr int64_t kSmallChainMaxB = 1 << 16;

}  // namespace nfx
