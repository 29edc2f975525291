// Micro-benchmark: can fp32 MFMA (v_mfma_f32_32x32x2_f32) and fp32 VALU overlap on one SIMD?
// 512-thread workgroups (2 waves per SIMD), one workgroup per CU. Waves 0-3 run an MFMA stream,
// waves 4-7 a VALU FMA stream; each side can be switched off. If the two pipes co-execute,
// time(both) ~ max(time(mfma), time(valu)); if they share issue/datapath, ~ the sum.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_coexec.hip -o /tmp/ubench_coexec
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int MODE>  // 0 = f32 32x32x2, 1 = bf16 32x32x16, 2 = f32 16x16x4
__global__ __launch_bounds__(512) void coexec(float* out, int n_mfma, int n_valu, float seed) {
    const int wave = threadIdx.x >> 6;
    float r = 0.f;
    if (wave < 4) {
        if (MODE == 2) {
            f32x4 c0 = {seed, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
            const float a = seed + threadIdx.x, b = seed - threadIdx.x;
            for (int i = 0; i < n_mfma; i += 4) {
                c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
                c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
            }
            r = c0[0] + c1[1] + c2[2] + c3[3];
        } else if (MODE == 1) {
            f32x16 c0 = {seed}, c1 = c0, c2 = c0, c3 = c0;
            bf16x8 a, b;
            for (int k = 0; k < 8; ++k) { a[k] = (__bf16)(seed + k); b[k] = (__bf16)(seed - k); }
            for (int i = 0; i < n_mfma; i += 4) {
                c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
                c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
            }
            r = c0[0] + c1[1] + c2[2] + c3[3];
        } else {
            f32x16 c0 = {seed}, c1 = c0, c2 = c0, c3 = c0;
            const float a = seed + threadIdx.x, b = seed - threadIdx.x;
            for (int i = 0; i < n_mfma; i += 4) {
                c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c2, 0, 0, 0);
                c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c3, 0, 0, 0);
            }
            r = c0[0] + c1[1] + c2[2] + c3[3];
        }
    } else {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = seed + k * threadIdx.x;
        for (int i = 0; i < n_valu; i += 8) {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = fmaf(v[k], 1.0001f, 0.5f);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) r += v[k];
    }
    out[blockIdx.x * 512 + threadIdx.x] = r;
}

template <int MODE>
static float run(float* d, int cus, int nm, int nv) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    coexec<MODE><<<cus, 512>>>(d, nm, nv, 1.f);
    hipEventRecord(e0);
    for (int it = 0; it < 5; ++it) coexec<MODE><<<cus, 512>>>(d, nm, nv, 1.f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5 * 1e3f;  // us
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* d;
    hipMalloc(&d, (size_t)cus * 512 * sizeof(float));
    const char* names[3] = {"f32_32x32x2", "bf16_32x32x16", "f32_16x16x4"};
    for (int mode = 0; mode < 3; ++mode) {
        const int nm = mode == 2 ? 32768 : 16384;
        const int nv = 65536 * 2;
        float tm, tv, tb;
        if (mode == 0) { tm = run<0>(d, cus, nm, 0); tv = run<0>(d, cus, 0, nv); tb = run<0>(d, cus, nm, nv); }
        else if (mode == 1) { tm = run<1>(d, cus, nm, 0); tv = run<1>(d, cus, 0, nv); tb = run<1>(d, cus, nm, nv); }
        else { tm = run<2>(d, cus, nm, 0); tv = run<2>(d, cus, 0, nv); tb = run<2>(d, cus, nm, nv); }
        printf("%-14s mfma-only %8.1f us  valu-only %8.1f us  both %8.1f us  (sum %8.1f, max %8.1f)\n",
               names[mode], tm, tv, tb, tm + tv, tm > tv ? tm : tv);
    }
    hipFree(d);
    return 0;
}
