// Micro-benchmark: dependent back-to-back v_mfma_f32_32x32x2_f32 on ONE accumulator vs 2 / 4
// independent accumulators (one wave per SIMD and two waves per SIMD).
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_chain.hip -o build/ubench_chain
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ void chain(float* out, int n, float seed) {
    f32x16 c[NACC];
#pragma unroll
    for (int k = 0; k < NACC; ++k) c[k] = f32x16{seed + k};
    const float a = seed + threadIdx.x, b = seed - threadIdx.x;
    for (int i = 0; i < n; i += NACC) {
#pragma unroll
        for (int k = 0; k < NACC; ++k) c[k] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c[k], 0, 0, 0);
    }
    float r = 0.f;
#pragma unroll
    for (int k = 0; k < NACC; ++k) r += c[k][k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int NACC>
static float run(float* d, int cus, int threads, int n) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    chain<NACC><<<cus, threads>>>(d, n, 1.f);
    (void)hipEventRecord(e0);
    for (int it = 0; it < 5; ++it) chain<NACC><<<cus, threads>>>(d, n, 1.f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5 * 1e3f;
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* d;
    (void)hipMalloc(&d, (size_t)cus * 1024 * sizeof(float));
    const int n = 8192;
    for (int threads = 256; threads <= 512; threads += 256) {
        const float ideal = (float)n * (threads / 256) * 64 / 2.4e3f;
        printf("waves/SIMD=%d ideal %.1f us: 1 acc %.1f  2 acc %.1f  4 acc %.1f\n", threads / 256, ideal,
               run<1>(d, cus, threads, n), run<2>(d, cus, threads, n), run<4>(d, cus, threads, n));
    }
    (void)hipFree(d);
    return 0;
}
