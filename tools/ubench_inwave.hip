// Micro-benchmark: VALU fillers between one wave's OWN fp32 MFMAs (v_mfma_f32_32x32x2_f32).
// 256-thread workgroups (one wave per SIMD), one workgroup per CU; per iteration 4 MFMAs on 4
// accumulators and V independent v_fma_f32, interleaved 1 MFMA : V/4 VALU with
// sched_group_barrier. Prints the time per iteration relative to V = 0.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_inwave.hip -o build/ubench_inwave
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int V, int WPS>
__global__ __launch_bounds__(256 * WPS) void inwave(float* out, int iters, float seed) {
    f32x16 c0 = {seed}, c1 = c0, c2 = c0, c3 = c0;
    const float a = seed + threadIdx.x, b = seed - threadIdx.x;
    float v[V > 0 ? V : 1];
#pragma unroll
    for (int k = 0; k < (V > 0 ? V : 1); ++k) v[k] = seed + k * threadIdx.x;
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c3, 0, 0, 0);
        if constexpr (V > 0) {
#pragma unroll
            for (int k = 0; k < V; ++k) v[k] = fmaf(v[k], a, b);
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);      // 1 MFMA
                __builtin_amdgcn_sched_group_barrier(0x2, V / 4, 0);  // V/4 VALU
            }
        }
    }
    float r = c0[0] + c1[1] + c2[2] + c3[3];
#pragma unroll
    for (int k = 0; k < (V > 0 ? V : 1); ++k) r += v[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int V, int WPS>
static float run(float* d, int cus, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    inwave<V, WPS><<<cus, 256 * WPS>>>(d, iters, 1.f);
    (void)hipEventRecord(e0);
    for (int it = 0; it < 5; ++it) inwave<V, WPS><<<cus, 256 * WPS>>>(d, iters, 1.f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5 * 1e3f;
}

template <int WPS>
static void sweep(float* d, int cus) {
    const int iters = 4096 / WPS;
    const float t0 = run<0, WPS>(d, cus, iters);
    const float ideal = (float)iters * WPS * 4 * 64 / 2.4e3f;  // us at 2.4 GHz, 64 cyc per MFMA
    printf("waves/SIMD=%d  V=0: %.1f us (ideal %.1f at 2.4 GHz)\n", WPS, t0, ideal);
    float t;
    t = run<4, WPS>(d, cus, iters);  printf("  V=4  %.1f us  x%.3f\n", t, t / t0);
    t = run<8, WPS>(d, cus, iters);  printf("  V=8  %.1f us  x%.3f\n", t, t / t0);
    t = run<16, WPS>(d, cus, iters); printf("  V=16 %.1f us  x%.3f\n", t, t / t0);
    t = run<32, WPS>(d, cus, iters); printf("  V=32 %.1f us  x%.3f\n", t, t / t0);
    t = run<48, WPS>(d, cus, iters); printf("  V=48 %.1f us  x%.3f\n", t, t / t0);
    t = run<64, WPS>(d, cus, iters); printf("  V=64 %.1f us  x%.3f\n", t, t / t0);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* d;
    (void)hipMalloc(&d, (size_t)cus * 1024 * sizeof(float));
    sweep<1>(d, cus);
    sweep<2>(d, cus);
    (void)hipFree(d);
    return 0;
}
