// Train-mode affine coupling layer (RealNVP CouplingLayer, BatchNorm with batch statistics)
// and its backward, for gfx950. SURVEY.md §8(f) items 1 and 2.
//
// Reference: src/flows/coupling/coupling_layer.py
//   nets :18-35  Linear(d,H) BatchNorm1d(H) ReLU Linear(H,H) BatchNorm1d(H) ReLU Linear(H,d)
//   forward :40-68 / inverse :70-96, clamps :50-51/:79-80, guards :61-66/:89-94
// In train mode (model.train(), the reference's training loops: README.md:107-117,
// plots/_common.py:194-211) each BatchNorm1d normalises with the statistics of the whole batch
// and updates its running statistics (momentum 0.1, unbiased variance).
//
// Pass structure of one layer (all on the caller's stream, no host synchronisation):
//   forward   STATS1  per-feature (n, mean, M2) of h1 = W1 xa + b1 (both nets)
//             STATS2  h2 = W2 relu(BN1(h1)) + b2 statistics           (layer 1 folded with STATS1)
//             fold    eval-layout pack with the batch statistics -> the streaming eval kernel
//                     produces (y, log_det); running statistics updated
//   backward  BWD1    recompute, epilogue backward, g_y2 = relu'(.) W3^T delta3:
//                     sums for BN2 backward (sum g, sum g x^), dW3, db3; gx (direct term)
//             BWD2    recompute + e2 = gamma2 (g_y2 - k1 - x^2 k2): dW2 = r2 sum e2 a1^T (MFMA
//                     over the sample dimension), db2, g_y1 = relu'(.) W2^T dh2 (MFMA) -> HBM,
//                     sums for BN1 backward
//             BWD3    e1 = gamma1 (g_y1 - k1 - x^1 k2): dW1, db1, gx += m * W1^T dh1
//             assemble the parameter gradients (fp32, the module's parameters() order)
// Under SyncBN (data-parallel training) the host all-reduces the statistics after STATS1/STATS2
// and the BN-backward sums after BWD1/BWD2 (nfs_amd.distributed), which makes the sharded step
// equal to the full-batch step.
#include <cmath>

#include "nfx_affine_kernel.h"
#include "nfx_affine_train_kernel.h"
#include "nfx_affine_trainw_kernel.h"
#include "nfx_pack.h"

namespace nfx {

// BatchNorm fold of layer `layer` (0 or 1) of net P from float64 statistics triples
// [Hp][3] = (n, mean, M2): r = 1/sqrt(var + eps), var = M2 / n (biased, as BatchNorm1d
// normalises). stats == nullptr -> identity (mean 0, r 1). A triple with n < 0 carries RUNNING
// statistics (eval-mode BatchNorm, nfx_affine_eval_stats): (-1, running_mean, -running_var), so
// var = M2 / n = running_var exactly and the backward drops the batch-coupling terms.
struct BnFold {
    double mean, r;
};
__device__ inline BnFold bn_fold(const double* stats, int Hp, int net, int row, double eps) {
    if (!stats) return {0.0, 1.0};
    const double* q = stats + ((size_t)net * Hp + row) * 3;
    const double var = q[0] != 0.0 ? q[2] / q[0] : 0.0;
    return {q[1], 1.0 / sqrt(var + eps)};
}

__device__ inline float raw_w(const NfxMlpRaw& P, int layer, int in_dim, int row, int col) {
    return P.w[layer][(size_t)row * in_dim + col];
}
__device__ inline float raw_b(const NfxMlpRaw& P, int layer, int row) { return P.b[layer] ? P.b[layer][row] : 0.f; }
__device__ inline float raw_g(const NfxMlpRaw& P, int layer, int row) { return P.bn_w[layer] ? P.bn_w[layer][row] : 1.f; }
__device__ inline float raw_be(const NfxMlpRaw& P, int layer, int row) { return P.bn_b[layer] ? P.bn_b[layer][row] : 0.f; }

__global__ void affine_train_pack_kernel(NfxMlpRaw s_net, NfxMlpRaw b_net, const float* mask,
                                         const double* stats1, const double* stats2, int d, int D, int H,
                                         float* tpack, float* epack) {
    const int HT = (H + 31) / 32, Hp = 32 * HT;
    const TrainLayout L = train_layout(D, HT);
    const double eps = s_net.bn_eps;
    const int gstride = gridDim.x * blockDim.x;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < L.total; i += gstride) {
        float v = 0.f;
        if (i >= L.mask) {
            const int j = i - L.mask;
            v = j < d ? mask[j] : 1.f;
        } else {
            const int net = i / L.net;
            const NfxMlpRaw& P = net ? b_net : s_net;
            const int o = i - net * L.net;
            if (o < L.c1) {  // w1 [HT][KS1][64]
                const int t = o - L.w1, lane = t & 63, ks = (t >> 6) % L.KS1, ht = (t >> 6) / L.KS1;
                const int row = 32 * ht + (lane & 31), c = 2 * ks + (lane >> 5);
                if (row < H && c < d) v = (float)(bn_fold(stats1, Hp, net, row, eps).r * (double)raw_w(P, 0, d, row, c));
            } else if (o < L.w2) {  // c1, g1, e1 [HT][32] accumulator order
                const int which = (o - L.c1) / (HT * 32), t = (o - L.c1) % (HT * 32);
                const int row = 32 * (t >> 5) + crow(t & 15, (t >> 4) & 1);
                if (row < H) {
                    if (which == 0) {
                        const BnFold f = bn_fold(stats1, Hp, net, row, eps);
                        v = (float)(f.r * ((double)raw_b(P, 0, row) - f.mean));
                    } else {
                        v = which == 1 ? raw_g(P, 0, row) : raw_be(P, 0, row);
                    }
                }
            } else if (o < L.c2) {  // w2 [o][kt][rq][lane][rr]
                const int t = o - L.w2, rr = t & 3, lane = (t >> 2) & 63, rq = (t >> 8) & 3;
                const int kt = (t >> 10) % HT, ot = (t >> 10) / HT;
                const int row = 32 * ot + (lane & 31), c = 32 * kt + crow(4 * rq + rr, lane >> 5);
                if (row < H && c < H) v = (float)(bn_fold(stats2, Hp, net, row, eps).r * (double)raw_w(P, 1, H, row, c));
            } else if (o < L.w3) {  // c2, g2, e2
                const int which = (o - L.c2) / (HT * 32), t = (o - L.c2) % (HT * 32);
                const int row = 32 * (t >> 5) + crow(t & 15, (t >> 4) & 1);
                if (row < H) {
                    if (which == 0) {
                        const BnFold f = bn_fold(stats2, Hp, net, row, eps);
                        v = (float)(f.r * ((double)raw_b(P, 1, row) - f.mean));
                    } else {
                        v = which == 1 ? raw_g(P, 1, row) : raw_be(P, 1, row);
                    }
                }
            } else if (o < L.b3) {  // w3 [D][HT][32]
                const int t = o - L.w3, j = t / (HT * 32), a = t % (HT * 32);
                const int c = 32 * (a >> 5) + crow(a & 15, (a >> 4) & 1);
                if (j < d && c < H) v = raw_w(P, 2, H, j, c);
            } else if (o < L.w2t) {
                const int j = o - L.b3;
                if (j < d) v = raw_b(P, 2, j);
            } else if (o < L.w1c) {  // w2t [kt][o][rq][lane][rr]: A[i][k] = W2r[32 o + k][32 kt + i]
                const int t = o - L.w2t, rr = t & 3, lane = (t >> 2) & 63, rq = (t >> 8) & 3;
                const int ot = (t >> 10) % HT, kt = (t >> 10) / HT;
                const int row = 32 * ot + crow(4 * rq + rr, lane >> 5), c = 32 * kt + (lane & 31);
                if (row < H && c < H) v = (float)(bn_fold(stats2, Hp, net, row, eps).r * (double)raw_w(P, 1, H, row, c));
            } else if (o < L.m2) {  // w1c [D][HT][32]: (diag(r1) W1)[row][j]
                const int t = o - L.w1c, j = t / (HT * 32), a = t % (HT * 32);
                const int row = 32 * (a >> 5) + crow(a & 15, (a >> 4) & 1);
                if (j < d && row < H) v = (float)(bn_fold(stats1, Hp, net, row, eps).r * (double)raw_w(P, 0, d, row, j));
            } else {  // m2, r2 [HT][32]: BN2 mean and 1/sqrt(var + eps), accumulator order
                const int which = (o - L.m2) / (HT * 32), t = (o - L.m2) % (HT * 32);
                const int row = 32 * (t >> 5) + crow(t & 15, (t >> 4) & 1);
                if (row < H) {
                    const BnFold f = bn_fold(stats2, Hp, net, row, eps);
                    v = (float)(which == 0 ? f.mean : f.r);
                }
            }
        }
        tpack[i] = v;
    }
    if (!epack) return;
    // eval-layout pack of the streaming kernel, BatchNorm folded with the batch statistics
    const AffineLayout E = affine_layout(d, HT);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < E.s; i += gstride) {  // (split tail: affine_split_pack)
        float v = 0.f;
        if (i >= E.mask) {
            const int j = i - E.mask;
            v = j < d ? mask[j] : 0.f;
        } else {
            const int net = i / E.net;
            const NfxMlpRaw& P = net ? b_net : s_net;
            const int o = i - net * E.net;
            auto wfold = [&](int layer, int in_dim, const double* st, int row, int c) {
                const BnFold f = bn_fold(st, Hp, net, row, eps);
                const double a = (double)raw_g(P, layer, row) * f.r;
                return (float)(a * (double)raw_w(P, layer, in_dim, row, c));
            };
            auto bfold = [&](int layer, const double* st, int row) {
                const BnFold f = bn_fold(st, Hp, net, row, eps);
                const double a = (double)raw_g(P, layer, row) * f.r;
                return (float)(a * ((double)raw_b(P, layer, row) - f.mean) + (double)raw_be(P, layer, row));
            };
            if (o < E.b1) {
                const int t = o - E.w1, lane = t & 63, ks = (t >> 6) % E.KS1, ht = (t >> 6) / E.KS1;
                const int row = 32 * ht + (lane & 31), c = 2 * ks + (lane >> 5);
                if (row < H && c < d) v = wfold(0, d, stats1, row, c);
            } else if (o < E.w2) {
                const int t = o - E.b1, r = t & 15, hh = (t >> 4) & 1, ht = t >> 5;
                const int row = 32 * ht + crow(r, hh);
                if (row < H) v = bfold(0, stats1, row);
            } else if (o < E.b2) {
                const int t = o - E.w2, rr = t & 3, lane = (t >> 2) & 63, rq = (t >> 8) & 3;
                const int kt = (t >> 10) % HT, hto = (t >> 10) / HT;
                const int row = 32 * hto + (lane & 31), c = 32 * kt + crow(4 * rq + rr, lane >> 5);
                if (row < H && c < H) v = wfold(1, H, stats2, row, c);
            } else if (o < E.w3) {
                const int t = o - E.b2, r = t & 15, hh = (t >> 4) & 1, ht = t >> 5;
                const int row = 32 * ht + crow(r, hh);
                if (row < H) v = bfold(1, stats2, row);
            } else if (o < E.b3) {
                const int t = o - E.w3, r = t & 15, hh = (t >> 4) & 1, ht = (t >> 5) % HT, j = (t >> 5) / HT;
                const int c = 32 * ht + crow(r, hh);
                if (c < H) v = raw_w(P, 2, H, j, c);
            } else {
                const int j = o - E.b3;
                if (j < d) v = raw_b(P, 2, j);
            }
        }
        epack[i] = v;
    }
}

// stats[net][row][3] = Chan merge of the per-workgroup triples: one wave per feature, lane l
// merges workgroups l, l + 64, ... in order, then a fixed pairwise tree over the 64 lanes
// (deterministic; the 16-thread serial version took 17 us at 512 workgroups).
__global__ __launch_bounds__(256) void affine_train_stats_finish(const double* part, int nw, int Hp, double* stats) {
    const int l = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);  // net * Hp + row
    if (i >= 2 * Hp) return;                             // whole waves
    double n = 0.0, mean = 0.0, m2 = 0.0;
    for (int w = l; w < nw; w += 64) {
        const double* q = part + ((size_t)w * 2 * Hp + i) * 3;
        if (n == 0.0) {
            n = q[0]; mean = q[1]; m2 = q[2];
        } else {
            chan_merge(n, mean, m2, q[0], q[1], q[2]);
        }
    }
    for (int off = 1; off < 64; off <<= 1) {
        const double nb = __shfl_down(n, off, 64), mb = __shfl_down(mean, off, 64), qb = __shfl_down(m2, off, 64);
        if ((l & (2 * off - 1)) == 0) {
            if (n == 0.0) {
                n = nb; mean = mb; m2 = qb;
            } else {
                chan_merge(n, mean, m2, nb, mb, qb);
            }
        }
    }
    if (l == 0) {
        stats[i * 3 + 0] = n;
        stats[i * 3 + 1] = mean;
        stats[i * 3 + 2] = m2;
    }
}

// out[i] = sum_w part[w * len + i] in float64: 16 threads per element over workgroups g, g+16, ...,
// then the 16 partial sums in order (deterministic).
__global__ __launch_bounds__(256) void affine_train_sum_finish(const float* part, int nw, int len, double* out) {
    __shared__ double red[16][17];
    const int e = threadIdx.x & 15, g = threadIdx.x >> 4;
    const int i = blockIdx.x * 16 + e;
    double a = 0.0;
    if (i < len) {
#pragma unroll 4
        for (int w = g; w < nw; w += 16) a += (double)part[(size_t)w * len + i];
    }
    red[g][e] = a;
    __syncthreads();
    if (g == 0 && i < len) {
        for (int k = 1; k < 16; ++k) a += red[k][e];
        out[i] = a;
    }
}

// Parameter gradients in CouplingLayer.parameters() order, per net (s_net then b_net):
//   0.weight [H,d] 0.bias [H] 1.weight [H] 1.bias [H] 3.weight [H,H] 3.bias [H]
//   4.weight [H] 4.bias [H] 6.weight [d,H] 6.bias [d]
__global__ void affine_train_assemble_kernel(const double* G, const double* stats1, const double* stats2,
                                             int d, int D, int H, double eps, float* grads) {
    const int HT = (H + 31) / 32, Hp = 32 * HT;
    const TrainGrad GL = train_grad_layout(D, HT);
    const int per_net = H * d + H + 2 * H + H * H + H + 2 * H + d * H + d;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 2 * per_net; i += gridDim.x * blockDim.x) {
        const int net = i / per_net;
        int o = i % per_net;
        double v;
        if (o < H * d) {  // 0.weight: r1 * sum e1 xa^T
            const int row = o / d, j = o % d;
            v = bn_fold(stats1, Hp, net, row, eps).r * G[GL.g3w + net * (D * Hp + Hp) + j * Hp + row];
        } else if ((o -= H * d) < H) {  // 0.bias
            v = bn_fold(stats1, Hp, net, o, eps).r * G[GL.g3w + net * (D * Hp + Hp) + D * Hp + o];
        } else if ((o -= H) < H) {  // 1.weight (gamma1) = sum g_y1 x^1
            v = G[GL.g2s + (net * 2 + 1) * Hp + o];
        } else if ((o -= H) < H) {  // 1.bias (beta1) = sum g_y1
            v = G[GL.g2s + (net * 2 + 0) * Hp + o];
        } else if ((o -= H) < H * H) {  // 3.weight: r2 * sum e2 a1^T
            const int row = o / H, c = o % H;
            v = bn_fold(stats2, Hp, net, row, eps).r * G[GL.g2w + net * (Hp * Hp + Hp) + row * Hp + c];
        } else if ((o -= H * H) < H) {  // 3.bias
            v = bn_fold(stats2, Hp, net, o, eps).r * G[GL.g2w + net * (Hp * Hp + Hp) + Hp * Hp + o];
        } else if ((o -= H) < H) {  // 4.weight (gamma2)
            v = G[GL.g1s + (net * 2 + 1) * Hp + o];
        } else if ((o -= H) < H) {  // 4.bias (beta2)
            v = G[GL.g1s + (net * 2 + 0) * Hp + o];
        } else if ((o -= H) < d * H) {  // 6.weight [d, H]
            const int j = o / H, c = o % H;
            v = G[GL.g1w + net * (D * Hp + D) + j * Hp + c];
        } else {  // 6.bias
            o -= d * H;
            v = G[GL.g1w + net * (D * Hp + D) + D * Hp + o];
        }
        grads[i] = (float)v;
    }
}

// BatchNorm1d running statistics (train mode, momentum m): running_mean = m mean + (1-m) rm,
// running_var = m var_unbiased + (1-m) rv, in double then rounded (ATen's CPU kernel order).
struct NfxBnPtrs {
    float* rm[4];
    float* rv[4];
    int64_t* nbt[4];  // num_batches_tracked (null: not counted here)
};
__global__ void affine_train_running_kernel(const double* stats1, const double* stats2, NfxBnPtrs p, int H,
                                            int Hp, double momentum) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;  // (net * 2 + layer) * H + row
    if (i >= 4 * H) return;
    if (i < 4 && p.nbt[i]) p.nbt[i][0] += 1;  // the 4 BatchNorms' num_batches_tracked
    const int k = i / H, row = i % H, net = k >> 1, layer = k & 1;
    const double* q = (layer ? stats2 : stats1) + ((size_t)net * Hp + row) * 3;
    const double n = q[0];
    const double var_u = n > 1.0 ? q[2] / (n - 1.0) : NAN;
    if (p.rm[k]) p.rm[k][row] = (float)(momentum * q[1] + (1.0 - momentum) * (double)p.rm[k][row]);
    if (p.rv[k]) p.rv[k][row] = (float)(momentum * var_u + (1.0 - momentum) * (double)p.rv[k][row]);
}

// Eval-mode statistics triples from the running statistics of the 4 BatchNorms
// (s_net.1, s_net.4, b_net.1, b_net.4): stats{1,2}[net][row] = (-1, running_mean, -running_var).
__global__ void affine_eval_stats_kernel(NfxBnPtrs p, int H, int Hp, double* stats1, double* stats2) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;  // (net * 2 + layer) * Hp + row
    if (i >= 4 * Hp) return;
    const int k = i / Hp, row = i % Hp, net = k >> 1, layer = k & 1;
    double* q = (layer ? stats2 : stats1) + ((size_t)net * Hp + row) * 3;
    const bool live = row < H;
    q[0] = -1.0;
    q[1] = live ? (double)p.rm[k][row] : 0.0;
    q[2] = live ? -(double)p.rv[k][row] : -1.0;
}

int train_sum_finish(const float* part, int nw, int len, double* out, hipStream_t s) {
    affine_train_sum_finish<<<(len + 15) / 16, 256, 0, s>>>(part, nw, len, out);
    return check_launch("affine_train_sum_finish");
}

// Wide path (nfx_affine_trainw_kernel.h): per-net compact partials part[net][w][len] -> G.
// Element i of net n goes to a0 + n * astride + i (i < seg) or b0 + n * bstride + (i - seg).
// 16 threads per element over workgroups w, w+16, ..., then the 16 partials in order.
__global__ __launch_bounds__(256) void affine_trainw_finish(const float* part, int nwx, int len, int seg, int a0,
                                                            int astride, int b0, int bstride, double* G) {
    __shared__ double red[16][17];
    const int e = threadIdx.x & 15, g = threadIdx.x >> 4, n = blockIdx.y;
    const int i = blockIdx.x * 16 + e;
    double a = 0.0;
    if (i < len) {
        const float* p = part + (size_t)n * nwx * len + i;
#pragma unroll 4
        for (int w = g; w < nwx; w += 16) a += (double)p[(size_t)w * len];
    }
    red[g][e] = a;
    __syncthreads();
    if (g == 0 && i < len) {
        for (int k = 1; k < 16; ++k) a += red[k][e];
        G[i < seg ? a0 + n * astride + i : b0 + n * bstride + (i - seg)] = a;
    }
}

static int pad_d(int d) { return d <= 2 ? 2 : (d <= 4 ? 4 : (d <= 8 ? 8 : 0)); }
static size_t train_dl_bytes(int64_t B, int D) { return ((size_t)B * 2 * D * sizeof(float) + 255) & ~(size_t)255; }

static affine_trainw_kernel_t pick_trainw(int HT, int D, int stage) {
    switch (HT) {
        case 3: return affine_trainw_pick_ht<3>(D, stage);
        case 4: return affine_trainw_pick_ht<4>(D, stage);
        default: return nullptr;
    }
}

// Workgroups along x of a wide-path pass (deterministic, host-computable: the workspace is
// sized with it): per-net passes <= one workgroup per CU per net, BWD3 <= two per CU.
static int64_t trainw_gx(int64_t ntiles, int stage) {
    const bool both = trainw_both_nets(stage);
    const int64_t work = both ? ntiles : (ntiles + kTWGroups - 1) / kTWGroups;
    const int64_t cap = (int64_t)num_cus() * (both ? 2 : 1);
    const int64_t g = work < cap ? work : cap;
    return g < 1 ? 1 : g;
}

extern "C" size_t nfx_affine_train_workspace_bytes(int64_t B, int d, int H);

// Wide-path backward stage: 1 = OUT + BWD1, 2 = BWD2 (incl. the BN1-backward sums), 3 = BWD3.
static int trainw_backward(const float* tpack, const float* x, const float* gy, const float* gld, float* gx,
                           int64_t B, int d, int D, int HT, int direction, int stage, const double* stats2, double* G,
                           void* workspace, hipStream_t s) {
    const int Hp = 32 * HT;
    const TrainGrad GL = train_grad_layout(D, HT);
    const int64_t ntiles = (B + 31) / 32;
    const size_t full = nfx_affine_train_workspace_bytes(B, d, 32 * HT);
    const size_t obytes = (size_t)2 * B * D * sizeof(float);
    const size_t gbytes = ((size_t)ntiles * 2 * HT * 1024 * sizeof(float) + 255) & ~(size_t)255;
    char* ws = reinterpret_cast<char*>(workspace);
    float* obuf = reinterpret_cast<float*>(ws + (full - obytes));
    float* gbuf = reinterpret_cast<float*>(ws + (full - obytes - gbytes));
    auto launch = [&](int st) -> int {
        affine_trainw_kernel_t k = pick_trainw(HT, D, st);
        if (!k) return set_error(NFX_EUNSUPPORTED, "affine_train_backward: no wide kernel for HT=%d D=%d", HT, D);
        const size_t lds = (size_t)trainw_lds(D, HT, st).total * sizeof(float);
        int rc = prepare_lds((const void*)k, lds);
        if (rc) return rc;
        const int64_t gxn = trainw_gx(ntiles, st);
        const unsigned ny = trainw_both_nets(st) ? 1 : 2;
        k<<<dim3((unsigned)gxn, ny), trainw_waves(HT, st) * 64, lds, s>>>(tpack, x, gy, gld, gx, gbuf, obuf, G, stats2,
                                                                           workspace, B, d, direction, ntiles);
        if ((rc = check_launch("affine_trainw_kernel"))) return rc;
        if (st == TW_OUT) return NFX_OK;
        if (st == TW_BWD3) {
            affine_train_sum_finish<<<(GL.len3 + 15) / 16, 256, 0, s>>>(reinterpret_cast<const float*>(workspace),
                                                                         (int)gxn, GL.len3, G + GL.g3w);
            return check_launch("affine_train_sum_finish");
        }
        const int len = trainw_len(D, HT, st);
        if (st == TW_BWD1)
            affine_trainw_finish<<<dim3((len + 15) / 16, 2), 256, 0, s>>>(
                reinterpret_cast<const float*>(workspace), (int)gxn, len, 2 * Hp, GL.g1s, 2 * Hp, GL.g1w, D * Hp + D, G);
        else
            affine_trainw_finish<<<dim3((len + 15) / 16, 2), 256, 0, s>>>(
                reinterpret_cast<const float*>(workspace), (int)gxn, len, 2 * Hp, GL.g2s, 2 * Hp, GL.g2w, Hp * Hp + Hp,
                G);
        return check_launch("affine_trainw_finish");
    };
    int rc;
    if (stage == 1) {
        if ((rc = launch(TW_OUT))) return rc;
        return launch(TW_BWD1);
    }
    return launch(stage == 2 ? TW_BWD2 : TW_BWD3);
}

static affine_train_kernel_t pick_train(int HT, int D, int stage) {
    switch (HT) {
        case 1: return affine_train_pick_ht<1>(D, stage);
        case 2: return affine_train_pick_ht<2>(D, stage);
        default: return nullptr;
    }
}

static int train_check(int d, int H, const char* what) {
    if (d <= 0 || H <= 0) return set_error(NFX_EINVAL, "%s: bad shape d=%d H=%d", what, d, H);
    if (!pad_d(d) || H > 128)
        return set_error(NFX_EUNSUPPORTED, "%s: d=%d H=%d outside the compiled train-mode family (d<=8, H<=128)",
                         what, d, H);
    return NFX_OK;
}

struct TrainGrid {
    int grid;
    int64_t nwaves, ntiles;
};

static TrainGrid train_grid(affine_train_kernel_t k, size_t lds, int64_t B) {
    TrainGrid g;
    g.ntiles = (B + 31) / 32;
    g.grid = resident_grid((const void*)k, 256, lds, (g.ntiles + 3) / 4);
    if (g.grid > 2 * num_cus()) g.grid = 2 * num_cus();  // the workspace is sized for <= 2 WGs per CU
    g.nwaves = (int64_t)g.grid * 4;
    return g;
}

}  // namespace nfx

using namespace nfx;

extern "C" size_t nfx_affine_train_pack_floats(int d, int H) {
    const int D = pad_d(d);
    if (!D || H <= 0 || H > 128) return 0;
    return (size_t)((train_layout(D, (H + 31) / 32).total + 3) & ~3);
}

extern "C" size_t nfx_affine_train_stats_doubles(int H) {
    if (H <= 0) return 0;
    return (size_t)2 * 32 * ((H + 31) / 32) * 3;
}

extern "C" size_t nfx_affine_train_grad_doubles(int d, int H) {
    const int D = pad_d(d);
    if (!D || H <= 0 || H > 128) return 0;
    return (size_t)train_grad_layout(D, (H + 31) / 32).total;
}

extern "C" size_t nfx_affine_train_param_floats(int d, int H) {
    if (d <= 0 || H <= 0) return 0;
    return (size_t)2 * (H * d + H + 2 * H + H * H + H + 2 * H + d * H + d);
}

// Workspace: per-wave partials (max over passes) + the g_y1 tiles BWD2 hands to BWD3
// (+ on the wide path, HT > 2, the raw net outputs [2][B][D] of the OUT pass).
extern "C" size_t nfx_affine_train_workspace_bytes(int64_t B, int d, int H) {
    const int D = pad_d(d);
    if (!D || H <= 0 || H > 128 || B < 0) return 0;
    const int HT = (H + 31) / 32, Hp = 32 * HT;
    const TrainGrad GL = train_grad_layout(D, HT);
    const int64_t ntiles = (B + 31) / 32;
    if (HT > 2) {
        size_t partials = 0;
        for (int st = TW_STATS1; st <= TW_BWD3; ++st) {
            const int64_t gx = trainw_gx(ntiles, st);
            size_t bytes;
            if (st == TW_STATS1 || st == TW_STATS2) bytes = (size_t)2 * gx * 2 * Hp * 3 * sizeof(double);
            else if (st == TW_BWD3) bytes = (size_t)gx * GL.len3 * sizeof(float);
            else bytes = (size_t)2 * gx * trainw_len(D, HT, st) * sizeof(float);
            if (bytes > partials) partials = bytes;
        }
        partials = (partials + 255) & ~(size_t)255;
        const size_t gbytes = ((size_t)ntiles * 2 * HT * 1024 * sizeof(float) + 255) & ~(size_t)255;
        return partials + gbytes + (size_t)2 * B * D * sizeof(float);
    }
    int64_t nw = 4 * (int64_t)num_cus() * 2;  // upper bound on resident waves (<= 2 WGs/CU)
    const int64_t cap = 4 * ((ntiles + 3) / 4);
    if (nw > cap) nw = cap < 4 ? 4 : cap;
    size_t per_wave = (size_t)GL.len2 * sizeof(float);
    const size_t st = (size_t)2 * Hp * 3 * sizeof(double);
    if ((size_t)GL.len1 * sizeof(float) > per_wave) per_wave = (size_t)GL.len1 * sizeof(float);
    if ((size_t)GL.len3 * sizeof(float) > per_wave) per_wave = (size_t)GL.len3 * sizeof(float);
    if (st > per_wave) per_wave = st;
    const size_t partials = ((size_t)nw * per_wave + 255) & ~(size_t)255;
    // + the delta3 rows BWD1K hands to BWD2K ([B][2][D]), then the g_y1 tiles (BWD2 -> BWD3)
    return partials + train_dl_bytes(B, D) + (size_t)ntiles * 2 * HT * 1024 * sizeof(float);
}

extern "C" int nfx_affine_train_pack(const NfxMlpRaw* s_net, const NfxMlpRaw* b_net, const float* mask,
                                     const double* stats1, const double* stats2, int d, int H, float* tpack,
                                     float* epack, void* stream) {
    int rc = train_check(d, H, "affine_train_pack");
    if (rc) return rc;
    if (!s_net || !b_net || !mask || !tpack) return set_error(NFX_EINVAL, "affine_train_pack: null pointer");
    if (epack && (!stats1 || !stats2)) return set_error(NFX_EINVAL, "affine_train_pack: eval pack needs both statistics");
    const NfxMlpRaw* nets[2] = {s_net, b_net};
    for (int n = 0; n < 2; ++n)
        for (int l = 0; l < 3; ++l)
            if (!nets[n]->w[l]) return set_error(NFX_EINVAL, "affine_train_pack: net %d layer %d weight is null", n, l);
    const int D = pad_d(d);
    const int total = (int)nfx_affine_train_pack_floats(d, H);
    int blocks = (total + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    affine_train_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(*s_net, *b_net, mask, stats1, stats2, d, D, H,
                                                                      tpack, epack);
    rc = check_launch("affine_train_pack_kernel");
    return rc || !epack ? rc : affine_split_pack(epack, d, H, (hipStream_t)stream);
}

// Floats of the kept layer-2 pre-activations (nfx_affine_train_stats_keep /
// nfx_affine_train_backward_keep): 2 nets x Hp per sample in 32-sample tiles; 0 where the pass
// family does not keep them (HT > 2: the wide path recomputes).
extern "C" size_t nfx_affine_train_keep_floats(int64_t B, int d, int H) {
    if (!pad_d(d) || H <= 0 || H > 64 || B < 1) return 0;
    const int HT = (H + 31) / 32;
    return (size_t)((B + 31) / 32) * 2 * HT * 1024;
}

extern "C" int nfx_affine_train_stats(const float* tpack, const float* x, int64_t B, int d, int H, int layer,
                                      double* stats, void* workspace, void* stream) {
    return nfx_affine_train_stats_keep(tpack, x, B, d, H, layer, stats, workspace, nullptr, stream);
}

extern "C" int nfx_affine_train_stats_keep(const float* tpack, const float* x, int64_t B, int d, int H, int layer,
                                           double* stats, void* workspace, float* keep, void* stream) {
    int rc = train_check(d, H, "affine_train_stats");
    if (rc) return rc;
    if (layer != 1 && layer != 2) return set_error(NFX_EINVAL, "affine_train_stats: layer must be 1 or 2");
    if (B < 1) return set_error(NFX_EINVAL, "affine_train_stats: batch statistics need B >= 1 (B=%lld)", (long long)B);
    if (!tpack || !x || !stats || !workspace) return set_error(NFX_EINVAL, "affine_train_stats: null pointer");
    const int D = pad_d(d), HT = (H + 31) / 32, Hp = 32 * HT;
    if (keep && (layer != 2 || HT > 2))
        return set_error(NFX_EINVAL, "affine_train_stats: keep needs layer 2 and H <= 64 (H=%d)", H);
    if (HT > 2) {  // wide path: one net per workgroup (blockIdx.y)
        const int st = layer == 1 ? TW_STATS1 : TW_STATS2;
        affine_trainw_kernel_t kw = pick_trainw(HT, D, st);
        const size_t lds = (size_t)trainw_lds(D, HT, st).total * sizeof(float);
        if ((rc = prepare_lds((const void*)kw, lds))) return rc;
        const int64_t ntiles = (B + 31) / 32, gx = trainw_gx(ntiles, st);
        hipStream_t s = (hipStream_t)stream;
        kw<<<dim3((unsigned)gx, 2), trainw_waves(HT, st) * 64, lds, s>>>(tpack, x, nullptr, nullptr, nullptr, nullptr,
                                                                          nullptr, nullptr, nullptr, workspace, B, d, 1,
                                                                          ntiles);
        if ((rc = check_launch("affine_trainw_kernel(stats)"))) return rc;
        affine_train_stats_finish<<<(2 * Hp + 3) / 4, 256, 0, s>>>(reinterpret_cast<const double*>(workspace),
                                                                     (int)(2 * gx), Hp, stats);
        return check_launch("affine_train_stats_finish");
    }
    const int ts = layer == 1 ? TS_STATS1 : TS_STATS2;
    affine_train_kernel_t k = pick_train(HT, D, ts);
    const size_t lds = affine_train_lds(D, HT, ts);
    if ((rc = prepare_lds((const void*)k, lds))) return rc;
    const TrainGrid g = train_grid(k, lds, B);
    hipStream_t s = (hipStream_t)stream;
    k<<<g.grid, 256, lds, s>>>(tpack, x, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, workspace, keep,
                               nullptr, B, d, 1, g.ntiles);
    if ((rc = check_launch("affine_train_kernel(stats)"))) return rc;
    affine_train_stats_finish<<<(2 * Hp + 3) / 4, 256, 0, s>>>(reinterpret_cast<const double*>(workspace),
                                                                 g.grid, Hp, stats);
    return check_launch("affine_train_stats_finish");
}

// The train-mode layer's output (y, log_det) from the kept layer-2 pre-activations and the pack
// folded with both statistics: replaces nfx_affine_coupling(epack) in a forward that keeps them.
extern "C" int nfx_affine_train_output(const float* tpack, const float* x, const float* keep, float* y,
                                       float* log_det, int64_t B, int d, int H, int direction, void* stream) {
    int rc = train_check(d, H, "affine_train_output");
    if (rc) return rc;
    if (direction != NFX_FORWARD && direction != NFX_INVERSE)
        return set_error(NFX_EINVAL, "affine_train_output: direction must be +1 or -1");
    if (B < 1) return set_error(NFX_EINVAL, "affine_train_output: B >= 1 required");
    if (!tpack || !x || !keep || !y || !log_det) return set_error(NFX_EINVAL, "affine_train_output: null pointer");
    const int D = pad_d(d), HT = (H + 31) / 32;
    if (HT > 2) return set_error(NFX_EINVAL, "affine_train_output: kept activations need H <= 64 (H=%d)", H);
    affine_train_kernel_t k = pick_train(HT, D, TS_OUTK);
    const size_t lds = affine_train_lds(D, HT, TS_OUTK);
    if ((rc = prepare_lds((const void*)k, lds))) return rc;
    // no per-workgroup partials: the grid is every resident workgroup (not capped at 2 per CU)
    TrainGrid g;
    g.ntiles = (B + 31) / 32;
    g.grid = resident_grid((const void*)k, 256, lds, (g.ntiles + 3) / 4);
    k<<<g.grid, 256, lds, (hipStream_t)stream>>>(tpack, x, nullptr, nullptr, y, nullptr, nullptr, nullptr, nullptr,
                                                 const_cast<float*>(keep), log_det, B, d, direction, g.ntiles);
    return check_launch("affine_train_kernel(output)");
}

extern "C" int nfx_affine_train_update_running(const double* stats1, const double* stats2, float* const* running_mean,
                                               float* const* running_var, int H, double momentum, void* stream) {
    return nfx_affine_train_update_running_counted(stats1, stats2, running_mean, running_var, nullptr, H, momentum,
                                                   stream);
}

// + num_batches_tracked += 1 of the 4 BatchNorms in the same launch (BatchNorm1d.forward in train
// mode; one torch launch per layer otherwise)
extern "C" int nfx_affine_train_update_running_counted(const double* stats1, const double* stats2,
                                                       float* const* running_mean, float* const* running_var,
                                                       int64_t* const* num_batches_tracked, int H, double momentum,
                                                       void* stream) {
    if (!stats1 || !stats2 || !running_mean || !running_var || H <= 0)
        return set_error(NFX_EINVAL, "affine_train_update_running: bad arguments");
    NfxBnPtrs p{};
    for (int k = 0; k < 4; ++k) {
        p.rm[k] = running_mean[k];
        p.rv[k] = running_var[k];
        p.nbt[k] = num_batches_tracked ? num_batches_tracked[k] : nullptr;
    }
    const int Hp = 32 * ((H + 31) / 32);
    affine_train_running_kernel<<<(4 * H + 255) / 256, 256, 0, (hipStream_t)stream>>>(stats1, stats2, p, H, Hp, momentum);
    return check_launch("affine_train_running_kernel");
}

extern "C" int nfx_affine_eval_stats(float* const* running_mean, float* const* running_var, int H, double* stats1,
                                     double* stats2, void* stream) {
    if (!stats1 || !stats2 || !running_mean || !running_var || H <= 0)
        return set_error(NFX_EINVAL, "affine_eval_stats: bad arguments");
    NfxBnPtrs p{};
    for (int k = 0; k < 4; ++k) {
        if (!running_mean[k] || !running_var[k]) return set_error(NFX_EINVAL, "affine_eval_stats: null running stats");
        p.rm[k] = running_mean[k];
        p.rv[k] = running_var[k];
    }
    const int Hp = 32 * ((H + 31) / 32);
    affine_eval_stats_kernel<<<(4 * Hp + 255) / 256, 256, 0, (hipStream_t)stream>>>(p, H, Hp, stats1, stats2);
    return check_launch("affine_eval_stats_kernel");
}

extern "C" int nfx_affine_train_backward(const float* tpack, const float* x, const float* gy, const float* gld,
                                         float* gx, int64_t B, int d, int H, int direction, int stage,
                                         const double* stats2, double* G, void* workspace, void* stream) {
    return nfx_affine_train_backward_keep(tpack, x, gy, gld, gx, B, d, H, direction, stage, stats2, G, workspace,
                                          nullptr, stream);
}

extern "C" int nfx_affine_train_backward_keep(const float* tpack, const float* x, const float* gy, const float* gld,
                                              float* gx, int64_t B, int d, int H, int direction, int stage,
                                              const double* stats2, double* G, void* workspace, const float* keep,
                                              void* stream) {
    int rc = train_check(d, H, "affine_train_backward");
    if (rc) return rc;
    if (stage < 1 || stage > 3) return set_error(NFX_EINVAL, "affine_train_backward: stage must be 1, 2 or 3");
    if (direction != NFX_FORWARD && direction != NFX_INVERSE)
        return set_error(NFX_EINVAL, "affine_train_backward: direction must be +1 or -1");
    if (B < 1) return set_error(NFX_EINVAL, "affine_train_backward: B >= 1 required");
    if (!tpack || !x || !gx || !G || !workspace || !stats2 || (stage < 3 && (!gy || !gld)))
        return set_error(NFX_EINVAL, "affine_train_backward: null pointer");
    const int D = pad_d(d), HT = (H + 31) / 32;
    const TrainGrad GL = train_grad_layout(D, HT);
    if (keep && HT > 2) return set_error(NFX_EINVAL, "affine_train_backward: keep needs H <= 64 (H=%d)", H);
    if (HT > 2) return trainw_backward(tpack, x, gy, gld, gx, B, d, D, HT, direction, stage, stats2, G, workspace,
                                       (hipStream_t)stream);
    const int ts = stage == 1 ? (keep ? TS_BWD1K : TS_BWD1) : (stage == 2 ? (keep ? TS_BWD2K : TS_BWD2) : TS_BWD3);
    affine_train_kernel_t k = pick_train(HT, D, ts);
    const size_t lds = affine_train_lds(D, HT, ts);
    if ((rc = prepare_lds((const void*)k, lds))) return rc;
    const TrainGrid g = train_grid(k, lds, B);
    // partials first, then the delta3 rows and the g_y1 tiles (offsets as in
    // nfx_affine_train_workspace_bytes)
    const size_t full = nfx_affine_train_workspace_bytes(B, d, H);
    const size_t gbytes = (size_t)g.ntiles * 2 * HT * 1024 * sizeof(float);
    char* ws = reinterpret_cast<char*>(workspace);
    float* gbuf = reinterpret_cast<float*>(ws + (full - gbytes));
    float* dlb = reinterpret_cast<float*>(ws + (full - gbytes - train_dl_bytes(B, D)));
    hipStream_t s = (hipStream_t)stream;
    // BWD2K: one net per workgroup (blockIdx.y), the resident workgroups split between the nets
    const int ny = train_stage_nets(ts) == 1 ? 2 : 1, gxn = ny == 2 ? (g.grid + 1) / 2 : g.grid;
    k<<<dim3(gxn, ny), 256, lds, s>>>(tpack, x, gy, gld, gx, gbuf, G, stats2, workspace, const_cast<float*>(keep),
                                      dlb, B, d, direction, g.ntiles);
    if ((rc = check_launch("affine_train_kernel(backward)"))) return rc;
    const int off = stage == 1 ? GL.g1s : (stage == 2 ? GL.g2s : GL.g3w);
    const int len = stage == 1 ? GL.len1 : (stage == 2 ? GL.len2 : GL.len3);
    affine_train_sum_finish<<<(len + 15) / 16, 256, 0, s>>>(reinterpret_cast<const float*>(workspace), gxn * ny,
                                                            len, G + off);
    return check_launch("affine_train_sum_finish");
}

extern "C" int nfx_affine_train_assemble(const double* G, const double* stats1, const double* stats2, int d, int H,
                                         float eps, float* grads, void* stream) {
    int rc = train_check(d, H, "affine_train_assemble");
    if (rc) return rc;
    if (!G || !stats1 || !stats2 || !grads) return set_error(NFX_EINVAL, "affine_train_assemble: null pointer");
    const int n = (int)nfx_affine_train_param_floats(d, H);
    int blocks = (n + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    affine_train_assemble_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(G, stats1, stats2, d, pad_d(d), H,
                                                                          (double)eps, grads);
    return check_launch("affine_train_assemble_kernel");
}
