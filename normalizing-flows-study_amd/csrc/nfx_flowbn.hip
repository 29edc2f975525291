// Between-layer BatchNorm of NormalizingFlowModel as an invertible flow layer.
//
// Reference: src/models/normalizing_flow_model.py:67-128 (used by forward :35-44 and inverse
// :55-60 when batch_norm_between_layers=True). The affine always uses the RUNNING statistics:
//   forward  y = (x - rm) / sqrt(rv + eps) * g + b          (:81-85)
//   inverse  x = (y - b) / g * sqrt(rv + eps) + rm          (:115-128)
//   log|det| = sum_j log|g_j| - 0.5 log(rv_j + eps), one scalar for the batch (:87-108),
//              added to every sample's log-det in forward, subtracted in inverse.
// In train mode the forward first folds the batch moments into the running statistics
// (:74-79: momentum update with the biased batch variance) and then applies the affine with
// the UPDATED statistics.
//
// Kernels (all HBM-bound elementwise / reduction work, no MFMA):
//   flowbn_apply_kernel     one pass over [B, d]: the affine (op-for-op rounding of the torch
//                           expression, contraction off) and log_det[i] +-= c. Per-feature
//                           constants staged in LDS; float4 loads/stores along the flat array.
//   flowbn_moments_kernel   train mode: per-feature shifted float64 sums (shift = row 0, so
//                           every block and every rank uses a consistent origin) -> per-block
//                           partials; flowbn_moments_finish -> (n, mean, M2) triples, the format
//                           nfs_amd.distributed.merge_bn_stats merges over ranks (SyncBN).
//   flowbn_update_kernel    running-stat momentum update from the triples, fp32 like :77-79.
//   flowbn_backward_kernel  autograd of the affine + scalar log-det w.r.t. x, g, b (the running
//                           statistics are buffers): grad_in elementwise plus per-feature
//                           float64 partial sums; flowbn_backward_finish assembles dg, db.
#include <math.h>

#include "nfx_common.h"

namespace nfx {

constexpr int kBnThreads = 256;
constexpr int kBnMaxD = 1024;       // per-feature constants staged in LDS (4 x 4 KB)
constexpr int kBnMaxBlocks = 1024;  // partial-sum blocks of the reductions

// Per-feature constants in LDS + the scalar log-det (wave 0 reduces, fixed order).
struct BnShared {
    float m[kBnMaxD], s[kBnMaxD], g[kBnMaxD], b[kBnMaxD];
    float c;
};

__device__ __forceinline__ void bn_stage(BnShared& sh, const float* __restrict__ gamma, const float* __restrict__ beta,
                                         const float* __restrict__ rm, const float* __restrict__ rv, float eps,
                                         int d) {
#pragma clang fp contract(off)
    for (int j = threadIdx.x; j < d; j += kBnThreads) {
        sh.m[j] = rm[j];
        sh.s[j] = sqrtf(rv[j] + eps);
        sh.g[j] = gamma[j];
        sh.b[j] = beta[j];
    }
    if (threadIdx.x < 64) {
        // log|det| terms: lane l sums j = l, l + 64, ... in order, then a fixed xor tree (every
        // lane ends with the same value)
        float part = 0.f;
        for (int j = threadIdx.x; j < d; j += 64)
            part = part + (logf(fabsf(gamma[j])) - 0.5f * logf(rv[j] + eps));
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) part = part + __shfl_xor(part, off, 64);
        if (threadIdx.x == 0) sh.c = part;
    }
    __syncthreads();
}

template <int DIR>
__global__ __launch_bounds__(kBnThreads) void flowbn_apply_kernel(
    const float* __restrict__ in, float* __restrict__ out, float* __restrict__ log_det,
    const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ rm,
    const float* __restrict__ rv, float eps, int64_t B, int d) {
#pragma clang fp contract(off)
    __shared__ BnShared sh;
    bn_stage(sh, gamma, beta, rm, rv, eps, d);
    const int64_t n = B * (int64_t)d;
    const int64_t nthreads = (int64_t)gridDim.x * kBnThreads;
    const int64_t tid = (int64_t)blockIdx.x * kBnThreads + threadIdx.x;
    auto f = [&](float v, int j) -> float {
        if constexpr (DIR > 0) {
            return (v - sh.m[j]) / sh.s[j] * sh.g[j] + sh.b[j];
        } else {
            return (v - sh.b[j]) / sh.g[j] * sh.s[j] + sh.m[j];
        }
    };
    // float4 body when the array is 16-byte aligned (torch allocations are), scalar tail
    const bool vec = ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
    int64_t done = 0;
    if (vec) {
        const int64_t n4 = n >> 2;
        const f32x4* in4 = reinterpret_cast<const f32x4*>(in);
        f32x4* out4 = reinterpret_cast<f32x4*>(out);
        for (int64_t q = tid; q < n4; q += nthreads) {
            f32x4 v = __builtin_nontemporal_load(in4 + q);
            int j = (int)((q * 4) % d);
            f32x4 r;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                r[k] = f(v[k], j);
                j = (j + 1 == d) ? 0 : j + 1;
            }
            __builtin_nontemporal_store(r, out4 + q);
        }
        done = n4 << 2;
    }
    for (int64_t e = done + tid; e < n; e += nthreads) out[e] = f(in[e], (int)(e % d));
    const float c = sh.c;
    for (int64_t i = tid; i < B; i += nthreads) {
        if constexpr (DIR > 0)
            log_det[i] = log_det[i] + c;
        else
            log_det[i] = log_det[i] - c;
    }
}

// Shifted float64 moments: block (bx, by) owns rows r = bx*4 + ry (+ 4*gridDim.x k) and the
// features f = by*64 + fx. part[(bx * d + f) * 2 + {0, 1}] = sum (x - x0), sum (x - x0)^2.
__global__ __launch_bounds__(kBnThreads) void flowbn_moments_kernel(const float* __restrict__ x,
                                                                    double* __restrict__ part, int64_t B,
                                                                    int d) {
    __shared__ double red[4][64][2];
    const int fx = threadIdx.x & 63, ry = threadIdx.x >> 6;
    const int f = blockIdx.y * 64 + fx;
    double s1 = 0.0, s2 = 0.0;
    if (f < d && B > 0) {
        const double c = (double)x[f];
        for (int64_t r = (int64_t)blockIdx.x * 4 + ry; r < B; r += (int64_t)gridDim.x * 4) {
            const double v = (double)x[r * d + f] - c;
            s1 += v;
            s2 += v * v;
        }
    }
    red[ry][fx][0] = s1;
    red[ry][fx][1] = s2;
    __syncthreads();
    if (ry == 0 && f < d) {
        for (int k = 1; k < 4; ++k) {
            s1 += red[k][fx][0];
            s2 += red[k][fx][1];
        }
        part[((int64_t)blockIdx.x * d + f) * 2 + 0] = s1;
        part[((int64_t)blockIdx.x * d + f) * 2 + 1] = s2;
    }
}

// stats[f] = (n, mean, M2) from the shifted sums of nb blocks (fixed block order).
__global__ __launch_bounds__(kBnThreads) void flowbn_moments_finish(const float* __restrict__ x,
                                                                    const double* __restrict__ part, int nb,
                                                                    double* __restrict__ stats, int64_t B,
                                                                    int d) {
    for (int f = blockIdx.x * kBnThreads + threadIdx.x; f < d; f += gridDim.x * kBnThreads) {
        double s1 = 0.0, s2 = 0.0;
        for (int k = 0; k < nb; ++k) {
            s1 += part[((int64_t)k * d + f) * 2 + 0];
            s2 += part[((int64_t)k * d + f) * 2 + 1];
        }
        const double n = (double)B;
        const double c = B > 0 ? (double)x[f] : 0.0;
        stats[3 * f + 0] = n;
        stats[3 * f + 1] = c + s1 / n;               // B = 0: NaN, as torch's mean of no rows
        double m2 = s2 - s1 * (s1 / n);
        stats[3 * f + 2] = m2 < 0.0 ? 0.0 : m2;
    }
}

// running = running * (1 - momentum) + momentum * batch, fp32 op by op (:77-79), biased var.
__global__ void flowbn_update_kernel(const double* __restrict__ stats, float* __restrict__ rm,
                                     float* __restrict__ rv, float keep, float mom, int d) {
#pragma clang fp contract(off)
    for (int f = blockIdx.x * blockDim.x + threadIdx.x; f < d; f += gridDim.x * blockDim.x) {
        const double n = stats[3 * f + 0];
        const float mean = (float)stats[3 * f + 1];
        const float var = (float)(stats[3 * f + 2] / n);
        rm[f] = rm[f] * keep + mom * mean;
        rv[f] = rv[f] * keep + mom * var;
    }
}

// Backward of one between-layer BatchNorm call.
//   forward (DIR=+1): q = (x - m)/s;  gx = (gy * g)/s;  sums: A = sum gy*q, Bs = sum gy
//   inverse (DIR=-1): t = y - b;  gu = gy * s (grad of u = t/g);  gx = gu/g;
//                     sums: A = sum gu*t, Bs = sum gu
// plus Gld = sum_i gld_i (the scalar log-det's upstream gradient). Block layout as the moments
// kernel; part[(bx * d + f) * 2 + {0,1}] = (A, Bs), gpart[bx] = Gld partial of block bx (by = 0).
template <int DIR>
__global__ __launch_bounds__(kBnThreads) void flowbn_backward_kernel(
    const float* __restrict__ x, const float* __restrict__ gy, const float* __restrict__ gld,
    float* __restrict__ gx, const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ rm, const float* __restrict__ rv, float eps, double* __restrict__ part,
    double* __restrict__ gpart, int64_t B, int d) {
#pragma clang fp contract(off)
    __shared__ double red[4][64][2];
    const int fx = threadIdx.x & 63, ry = threadIdx.x >> 6;
    const int f = blockIdx.y * 64 + fx;
    double a = 0.0, bs = 0.0;
    if (f < d) {
        const float m = rm[f], s = sqrtf(rv[f] + eps), g = gamma[f], b = beta[f];
        for (int64_t r = (int64_t)blockIdx.x * 4 + ry; r < B; r += (int64_t)gridDim.x * 4) {
            const int64_t e = r * d + f;
            const float go = gy ? gy[e] : 0.f;
            if constexpr (DIR > 0) {
                const float q = (x[e] - m) / s;
                gx[e] = (go * g) / s;
                a += (double)go * (double)q;
                bs += (double)go;
            } else {
                const float t = x[e] - b;
                const float gu = go * s;
                gx[e] = gu / g;
                a += (double)gu * (double)t;
                bs += (double)gu;
            }
        }
    }
    red[ry][fx][0] = a;
    red[ry][fx][1] = bs;
    __syncthreads();
    if (ry == 0 && f < d) {
        for (int k = 1; k < 4; ++k) {
            a += red[k][fx][0];
            bs += red[k][fx][1];
        }
        part[((int64_t)blockIdx.x * d + f) * 2 + 0] = a;
        part[((int64_t)blockIdx.x * d + f) * 2 + 1] = bs;
    }
    if (blockIdx.y == 0) {
        double gl = 0.0;
        if (gld)
            for (int64_t r = (int64_t)blockIdx.x * kBnThreads + threadIdx.x; r < B;
                 r += (int64_t)gridDim.x * kBnThreads)
                gl += (double)gld[r];
        gl = block_sum_f64<kBnThreads>(gl);
        if (threadIdx.x == 0) gpart[blockIdx.x] = gl;
    }
}

// dg, db (fp32, parameters() order of BatchNorm1d: weight then bias) from the partials.
//   forward: dg = A + Gld * sgn(g)/|g|          db = Bs
//   inverse: dg = -A/(g*g) - Gld * sgn(g)/|g|   db = -Bs/g
template <int DIR>
__global__ __launch_bounds__(kBnThreads) void flowbn_backward_finish(const double* __restrict__ part,
                                                                     const double* __restrict__ gpart, int nb,
                                                                     const float* __restrict__ gamma,
                                                                     float* __restrict__ dg,
                                                                     float* __restrict__ db, int d) {
    double gl = 0.0;
    for (int k = 0; k < nb; ++k) gl += gpart[k];
    for (int f = blockIdx.x * kBnThreads + threadIdx.x; f < d; f += gridDim.x * kBnThreads) {
        double a = 0.0, bs = 0.0;
        for (int k = 0; k < nb; ++k) {
            a += part[((int64_t)k * d + f) * 2 + 0];
            bs += part[((int64_t)k * d + f) * 2 + 1];
        }
        const double g = (double)gamma[f];
        const double dlog = (g > 0.0 ? 1.0 : (g < 0.0 ? -1.0 : 0.0)) / fabs(g);
        if constexpr (DIR > 0) {
            dg[f] = (float)(a + gl * dlog);
            db[f] = (float)bs;
        } else {
            dg[f] = (float)(-a / (g * g) - gl * dlog);
            db[f] = (float)(-bs / g);
        }
    }
}

static int bn_row_blocks(int64_t B, int d) {
    const int fchunks = (d + 63) / 64;
    int64_t want = (B + 255) / 256;  // >= 64 rows per thread-row-group at most blocks
    int64_t cap = kBnMaxBlocks / fchunks;
    if (cap < 1) cap = 1;
    if (want > cap) want = cap;
    return (int)(want < 1 ? 1 : want);
}

}  // namespace nfx

using namespace nfx;

extern "C" size_t nfx_flowbn_workspace_bytes(int64_t B, int d) {
    const int nb = bn_row_blocks(B, d > 0 ? d : 1);
    return ((size_t)nb * (size_t)(d > 0 ? d : 1) * 2 + (size_t)nb) * sizeof(double);
}

extern "C" int nfx_flowbn_apply(const float* in, float* out, float* log_det, const float* gamma,
                                const float* beta, const float* running_mean, const float* running_var,
                                float eps, int64_t B, int d, int direction, void* stream) {
    if (B < 0 || d <= 0) return set_error(NFX_EINVAL, "flowbn_apply: bad shape B=%lld d=%d", (long long)B, d);
    if (d > kBnMaxD) return set_error(NFX_EUNSUPPORTED, "flowbn_apply: d=%d > %d", d, kBnMaxD);
    if (direction != NFX_FORWARD && direction != NFX_INVERSE)
        return set_error(NFX_EINVAL, "flowbn_apply: direction %d", direction);
    if (!gamma || !beta || !running_mean || !running_var)
        return set_error(NFX_EINVAL, "flowbn_apply: null BatchNorm parameter");
    if (B == 0) return NFX_OK;
    if (!in || !out || !log_det) return set_error(NFX_EINVAL, "flowbn_apply: null in/out/log_det");
    hipStream_t s = (hipStream_t)stream;
    const int64_t n4 = (B * (int64_t)d + 3) / 4;
    int64_t grid = (n4 + kBnThreads - 1) / kBnThreads;
    const int64_t cap = 8 * (int64_t)num_cus();
    if (grid > cap) grid = cap;
    if (direction > 0)
        flowbn_apply_kernel<1><<<(int)grid, kBnThreads, 0, s>>>(in, out, log_det, gamma, beta, running_mean,
                                                                running_var, eps, B, d);
    else
        flowbn_apply_kernel<-1><<<(int)grid, kBnThreads, 0, s>>>(in, out, log_det, gamma, beta, running_mean,
                                                                 running_var, eps, B, d);
    return check_launch("flowbn_apply_kernel");
}

extern "C" int nfx_flowbn_moments(const float* x, int64_t B, int d, double* stats, void* workspace,
                                  void* stream) {
    if (B < 0 || d <= 0) return set_error(NFX_EINVAL, "flowbn_moments: bad shape B=%lld d=%d", (long long)B, d);
    if (!stats || !workspace || (B > 0 && !x)) return set_error(NFX_EINVAL, "flowbn_moments: null pointer");
    hipStream_t s = (hipStream_t)stream;
    const int nb = bn_row_blocks(B, d);
    double* part = reinterpret_cast<double*>(workspace);
    dim3 grid(nb, (d + 63) / 64);
    flowbn_moments_kernel<<<grid, kBnThreads, 0, s>>>(x, part, B, d);
    int rc = check_launch("flowbn_moments_kernel");
    if (rc) return rc;
    flowbn_moments_finish<<<(d + kBnThreads - 1) / kBnThreads, kBnThreads, 0, s>>>(x, part, nb, stats, B, d);
    return check_launch("flowbn_moments_finish");
}

extern "C" int nfx_flowbn_update_running(const double* stats, float* running_mean, float* running_var,
                                         double momentum, int d, void* stream) {
    if (d <= 0 || !stats || !running_mean || !running_var)
        return set_error(NFX_EINVAL, "flowbn_update_running: bad arguments");
    hipStream_t s = (hipStream_t)stream;
    flowbn_update_kernel<<<(d + 255) / 256, 256, 0, s>>>(stats, running_mean, running_var,
                                                          (float)(1.0 - momentum), (float)momentum, d);
    return check_launch("flowbn_update_kernel");
}

extern "C" int nfx_flowbn_backward(const float* in, const float* grad_out, const float* grad_log_det,
                                   float* grad_in, const float* gamma, const float* beta,
                                   const float* running_mean, const float* running_var, float eps,
                                   float* grad_gamma, float* grad_beta, int64_t B, int d, int direction,
                                   void* workspace, void* stream) {
    if (B < 0 || d <= 0) return set_error(NFX_EINVAL, "flowbn_backward: bad shape B=%lld d=%d", (long long)B, d);
    if (direction != NFX_FORWARD && direction != NFX_INVERSE)
        return set_error(NFX_EINVAL, "flowbn_backward: direction %d", direction);
    if (!gamma || !beta || !running_mean || !running_var || !grad_gamma || !grad_beta || !workspace)
        return set_error(NFX_EINVAL, "flowbn_backward: null pointer");
    if (B > 0 && (!in || !grad_in)) return set_error(NFX_EINVAL, "flowbn_backward: null in/grad_in");
    hipStream_t s = (hipStream_t)stream;
    const int nb = bn_row_blocks(B, d);
    double* part = reinterpret_cast<double*>(workspace);
    double* gpart = part + (size_t)nb * d * 2;
    dim3 grid(nb, (d + 63) / 64);
    if (direction > 0)
        flowbn_backward_kernel<1><<<grid, kBnThreads, 0, s>>>(in, grad_out, grad_log_det, grad_in, gamma, beta,
                                                              running_mean, running_var, eps, part, gpart, B, d);
    else
        flowbn_backward_kernel<-1><<<grid, kBnThreads, 0, s>>>(in, grad_out, grad_log_det, grad_in, gamma, beta,
                                                               running_mean, running_var, eps, part, gpart, B, d);
    int rc = check_launch("flowbn_backward_kernel");
    if (rc) return rc;
    const int fb = (d + kBnThreads - 1) / kBnThreads;
    if (direction > 0)
        flowbn_backward_finish<1><<<fb, kBnThreads, 0, s>>>(part, gpart, nb, gamma, grad_gamma, grad_beta, d);
    else
        flowbn_backward_finish<-1><<<fb, kBnThreads, 0, s>>>(part, gpart, nb, gamma, grad_gamma, grad_beta, d);
    return check_launch("flowbn_backward_finish");
}
