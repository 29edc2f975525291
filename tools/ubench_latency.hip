// Micro-benchmark: latency of dependent instruction chains for ONE wave (a single 64-thread
// workgroup), the regime of the sequential MADE kernel's per-round chain (made_seqs_kernel):
// fp32 FMA, packed FMA, DPP adds (quad_perm, row_ror, row_newbcast), a 4-stage 16-lane
// all-reduce, exp2, v_readlane round trips through a scalar register, ballot, LDS read chains
// (pointer chasing) and LDS write -> read round trips.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/ubench_latency.hip -o build/ubench_latency
// Prints cycles per dependent step (clock64 deltas inside the kernel, shader clock).
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

enum { K_FMA, K_PKFMA, K_DPP_QUAD, K_DPP_ROR8, K_DPP_BCAST, K_ALLSUM16, K_EXP2, K_READLANE, K_BALLOT, K_LDS_CHASE,
       K_LDS_WR_RD, K_N };
static const char* kNames[K_N] = {"v_fma_f32", "v_pk_fma_f32", "dpp add quad_perm", "dpp add row_ror:8",
                                  "dpp mov row_newbcast + add", "16-lane all-reduce (4 dpp adds)", "v_exp_f32",
                                  "v_readlane -> s -> v", "ballot -> s_ff1 -> v", "ds_read_b32 pointer chase",
                                  "ds_write_b32 -> ds_read_b32"};

template <int KIND>
__global__ __launch_bounds__(64) void chain(float* out, long long* cyc, int n, float seed) {
    __shared__ float lds[1024];
    const int lane = threadIdx.x;
    for (int i = lane; i < 1024; i += 64) lds[i] = __int_as_float(((i * 7 + 3) & 1023));  // chase table
    __syncthreads();
    float a = seed + lane * 1e-3f, b = 0.999f, c = 1e-4f;
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    f32x2 p = {a, a + 1.f};
    int idx = lane;
    const long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if constexpr (KIND == K_FMA) a = fmaf(a, b, c);
            if constexpr (KIND == K_PKFMA) p = __builtin_elementwise_fma(p, f32x2{b, b}, f32x2{c, c});
            if constexpr (KIND == K_DPP_QUAD) a = a * b + dpp<0xB1>(a);
            if constexpr (KIND == K_DPP_ROR8) a = a * b + dpp<0x128>(a);
            if constexpr (KIND == K_DPP_BCAST) a = a * b + dpp<0x150 + 3>(a);
            if constexpr (KIND == K_ALLSUM16) {
                a = a + dpp<0xB1>(a);
                a = a + dpp<0x4E>(a);
                a = a + dpp<0x141>(a);
                a = (a + dpp<0x140>(a)) * 0.0625f;
            }
            if constexpr (KIND == K_EXP2) a = __builtin_amdgcn_exp2f(a) * 0.5f;
            if constexpr (KIND == K_READLANE)
                a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a), (i + u) & 63)) * b + c;
            if constexpr (KIND == K_BALLOT) {
                const unsigned long long m = __ballot(a > 0.5f);
                a = a * b + (float)(__builtin_ffsll(m) & 1);
            }
            if constexpr (KIND == K_LDS_CHASE) idx = __float_as_int(lds[idx]);
            if constexpr (KIND == K_LDS_WR_RD) {
                lds[lane] = a;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                a = lds[lane ^ 1] * b + c;
            }
        }
    }
    const long long t1 = clock64();
    out[lane] = a + p.x + p.y + (float)idx;
    if (lane == 0) *cyc = t1 - t0;
}

template <int KIND>
static double run(float* d, long long* dc, int n) {
    chain<KIND><<<1, 64>>>(d, dc, n, 0.3f);
    long long c = 0;
    (void)hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);
    return (double)c / (8.0 * n);
}

int main() {
    float* d;
    long long* dc;
    (void)hipMalloc(&d, 64 * sizeof(float));
    (void)hipMalloc(&dc, sizeof(long long));
    const int n = 20000;
    double r[K_N] = {run<K_FMA>(d, dc, n),         run<K_PKFMA>(d, dc, n),     run<K_DPP_QUAD>(d, dc, n),
                     run<K_DPP_ROR8>(d, dc, n),    run<K_DPP_BCAST>(d, dc, n), run<K_ALLSUM16>(d, dc, n),
                     run<K_EXP2>(d, dc, n),        run<K_READLANE>(d, dc, n),  run<K_BALLOT>(d, dc, n),
                     run<K_LDS_CHASE>(d, dc, n),   run<K_LDS_WR_RD>(d, dc, n)};
    for (int k = 0; k < K_N; ++k) printf("%-34s %7.1f clock64 ticks per dependent step\n", kNames[k], r[k]);
    return 0;
}
