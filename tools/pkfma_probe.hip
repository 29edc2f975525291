// Issue-rate probe: v_pk_fma_f32 (two fp32 FMAs per lane) against v_fmac_f32 on gfx950, with
// 8 independent accumulator chains per lane (no dependency stalls) and 1 / 2 / 4 waves per SIMD.
//   hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 tools/pkfma_probe.hip -o /tmp/pkfma_probe && /tmp/pkfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <bool PK>
__global__ __launch_bounds__(256) void probe(float* out, int iters, float a, float b) {
    float s[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) s[i] = threadIdx.x * 1e-7f + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if constexpr (PK) {
#pragma unroll
                for (int i = 0; i < 16; i += 2) {
                    f32x2 v = __builtin_elementwise_fma(f32x2{s[i], s[i + 1]}, f32x2{a, a}, f32x2{b, b});
                    s[i] = v.x;
                    s[i + 1] = v.y;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) s[i] = __builtin_fmaf(s[i], a, b);
            }
        }
    }
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += s[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

int main() {
    int dev = 0, ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    float* out;
    const int iters = 4096;
    hipMalloc(&out, sizeof(float) * 256 * ncu * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int wps = 1; wps <= 4; wps *= 2) {  // waves per SIMD: blocks of 4 waves, wps blocks per CU
        const int grid = ncu * wps;
        for (int pk = 0; pk < 2; ++pk) {
            auto k = pk ? probe<true> : probe<false>;
            k<<<grid, 256>>>(out, 16, 1.0001f, 1e-6f);
            hipEventRecord(e0);
            k<<<grid, 256>>>(out, iters, 1.0001f, 1e-6f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0.f;
            hipEventElapsedTime(&ms, e0, e1);
            const double fmas = (double)grid * 256 * iters * 8 * 16;
            printf("{\"waves_per_simd\": %d, \"form\": \"%s\", \"ms\": %.4f, \"tflops\": %.2f}\n", wps,
                   pk ? "v_pk_fma_f32" : "v_fmac_f32", ms, 2.0 * fmas / (ms * 1e-3) / 1e12);
        }
    }
    hipFree(out);
    return 0;
}
