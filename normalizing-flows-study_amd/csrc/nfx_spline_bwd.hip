// Spline coupling backward: pack + C-ABI (kernel: nfx_spline_bwd_kernel.h). SURVEY.md §8(f) 1.
//
// nfx_spline_coupling_backward(direction, ...) computes, for one SplineCouplingLayer call
// y, ld = forward/inverse(x) (src/flows/spline/spline_coupling_layer.py:96-180), dL/dx and the
// gradients of param_net.{0,2,4}.{weight,bias} from dL/dy and dL/dld — what autograd produces for
// the reference's composite — in one fused kernel, a fixed-order reduction over workgroups and an
// assembly into the module's parameters() order.
#include "nfx_pack.h"
#include "nfx_spline_bwd_kernel.h"

namespace nfx {

__device__ inline int spline_bwd_tdim(const float* mask, int d, int t) {
    int n = 0;
    for (int j = 0; j < d; ++j) {
        if (mask[j] == 0.f) {
            if (n == t) return j;
            ++n;
        }
    }
    return -1;
}

__global__ void spline_bwd_pack_kernel(NfxMlpRaw net, const float* mask, int d, int H, int K, float* packed) {
    const int HT = (H + 31) / 32;
    const int NTM = spline_bwd_ntmax(HT);
    const SplineBwdLayout BL = spline_bwd_layout(HT, NTM);
    const SplineLayout L = BL.F;
    const int P = 3 * K - 1;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < BL.total; i += gridDim.x * blockDim.x) {
        float v = 0.f;
        if (i < L.b1) {
            int t = i - L.w1, lane = t & 63, ks = (t >> 6) & 3, ht = t >> 8;
            int row = 32 * ht + (lane & 31), col = 2 * ks + (lane >> 5);
            v = (row < H && col < d) ? mlp_weight(net, 0, d, row, col) : 0.f;
        } else if (i < L.w2) {
            int t = i - L.b1, r = t & 15, h = (t >> 4) & 1, ht = t >> 5;
            int row = 32 * ht + crow(r, h);
            v = row < H ? mlp_bias(net, 0, row) : 0.f;
        } else if (i < L.b2) {
            int t = i - L.w2, rr = t & 3, lane = (t >> 2) & 63, rq = (t >> 8) & 3;
            int kt = (t >> 10) % HT, hto = (t >> 10) / HT;
            int row = 32 * hto + (lane & 31), col = 32 * kt + crow(4 * rq + rr, lane >> 5);
            v = (row < H && col < H) ? mlp_weight(net, 1, H, row, col) : 0.f;
        } else if (i < L.w3) {
            int t = i - L.b2, r = t & 15, h = (t >> 4) & 1, ht = t >> 5;
            int row = 32 * ht + crow(r, h);
            v = row < H ? mlp_bias(net, 1, row) : 0.f;
        } else if (i < L.b3) {
            int t = i - L.w3, rr = t & 3, lane = (t >> 2) & 63, rq = (t >> 8) & 3;
            int kt = (t >> 10) % HT, tile = (t >> 10) / HT;
            int dt = spline_bwd_tdim(mask, d, tile), p = lane & 31;
            int col = 32 * kt + crow(4 * rq + rr, lane >> 5);
            v = (dt >= 0 && p < P && col < H) ? mlp_weight(net, 2, H, dt * P + p, col) : 0.f;
        } else if (i < L.mask) {
            int t = i - L.b3, r = t & 15, h = (t >> 4) & 1, tile = t >> 5;
            int dt = spline_bwd_tdim(mask, d, tile), p = crow(r, h);
            v = (dt >= 0 && p < P) ? mlp_bias(net, 2, dt * P + p) : 0.f;
        } else if (i < L.tdim) {
            int j = i - L.mask;
            v = j < d ? mask[j] : 0.f;
        } else if (i < L.meta) {
            v = (float)spline_bwd_tdim(mask, d, i - L.tdim);
        } else if (i < L.total) {
            int nt = 0;
            for (int j = 0; j < d; ++j) nt += mask[j] == 0.f ? 1 : 0;
            v = (i == L.meta) ? (float)nt : 0.f;
        } else if (i < BL.w3t) {  // w2t [kt][o][rq][lane][rr]: A[i][k] = W2[32 o + k][32 kt + i]
            int t = i - BL.w2t, rr = t & 3, lane = (t >> 2) & 63, rq = (t >> 8) & 3;
            int ot = (t >> 10) % HT, kt = (t >> 10) / HT;
            int row = 32 * ot + crow(4 * rq + rr, lane >> 5), col = 32 * kt + (lane & 31);
            v = (row < H && col < H) ? mlp_weight(net, 1, H, row, col) : 0.f;
        } else if (i < BL.w1c) {  // w3t [kt][tile][rq][lane][rr]: A[i][k] = W3[dt P + k][32 kt + i]
            int t = i - BL.w3t, rr = t & 3, lane = (t >> 2) & 63, rq = (t >> 8) & 3;
            int tile = (t >> 10) % NTM, kt = (t >> 10) / NTM;
            int dt = spline_bwd_tdim(mask, d, tile), p = crow(4 * rq + rr, lane >> 5);
            int col = 32 * kt + (lane & 31);
            v = (dt >= 0 && p < P && col < H) ? mlp_weight(net, 2, H, dt * P + p, col) : 0.f;
        } else if (i < BL.w1c + 8 * HT * 32) {  // w1c [8][HT][32]: W1[row][j]
            int t = i - BL.w1c, j = t / (HT * 32), a = t % (HT * 32);
            int row = 32 * (a >> 5) + crow(a & 15, (a >> 4) & 1);
            v = (j < d && row < H) ? mlp_weight(net, 0, d, row, j) : 0.f;
        }
        packed[i] = v;
    }
}

// G (float64, the spline_grad_layout sums) -> fp32 gradients of param_net.{0,2,4}.{weight,bias}
// in parameters() order: 0.weight [H,d] 0.bias [H] 2.weight [H,H] 2.bias [H] 4.weight [d P,H]
// 4.bias [d P] (rows of conditioning dimensions are unused by the layer: zero gradient).
__global__ void spline_bwd_assemble_kernel(const double* G, const float* mask, int d, int H, int K, float* grads) {
    const int HT = (H + 31) / 32, Hp = 32 * HT, P = 3 * K - 1;
    const SplineGrad GL = spline_grad_layout(HT, spline_bwd_ntmax(HT));
    const int n = H * d + H + H * H + H + d * P * H + d * P;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        int o = i;
        double v = 0.0;
        if (o < H * d) {
            v = G[GL.w1 + (o % d) * Hp + o / d];
        } else if ((o -= H * d) < H) {
            v = G[GL.b1 + o];
        } else if ((o -= H) < H * H) {
            v = G[GL.w2 + (o / H) * Hp + o % H];
        } else if ((o -= H * H) < H) {
            v = G[GL.b2 + o];
        } else if ((o -= H) < d * P * H) {
            const int row = o / H, col = o % H, dt = row / P, p = row % P;
            int t = 0;
            for (int j = 0; j < dt; ++j) t += mask[j] == 0.f ? 1 : 0;
            v = mask[dt] == 0.f ? G[GL.w3 + (t * 32 + p) * Hp + col] : 0.0;
        } else {
            o -= d * P * H;
            const int dt = o / P, p = o % P;
            int t = 0;
            for (int j = 0; j < dt; ++j) t += mask[j] == 0.f ? 1 : 0;
            v = mask[dt] == 0.f ? G[GL.b3 + t * 32 + p] : 0.0;
        }
        grads[i] = (float)v;
    }
}

static int spline_bwd_check(int d, int H, int K, int nt, const char* what) {
    if (d <= 0 || H <= 0 || K < 2) return set_error(NFX_EINVAL, "%s: bad shape d=%d H=%d K=%d", what, d, H, K);
    const int HT = (H + 31) / 32;
    if (d > 8 || H > 64 || K > 11 || (nt >= 0 && nt > spline_bwd_ntmax(HT)))
        return set_error(NFX_EUNSUPPORTED,
                         "%s: d=%d H=%d K=%d (%d transformed dims) outside the fused backward family "
                         "(d<=8, H<=64, K<=11, <=%d transformed dims at this H)", what, d, H, K, nt,
                         spline_bwd_ntmax(HT));
    return NFX_OK;
}

static spline_bwd_kernel_t pick_spline_bwd(int HT, int K, int inv) {
    switch (HT) {
        case 1: return spline_bwd_pick_ht<1>(K, inv);
        case 2: return spline_bwd_pick_ht<2>(K, inv);
        default: return nullptr;
    }
}

}  // namespace nfx

using namespace nfx;

extern "C" size_t nfx_spline_backward_packed_floats(int d, int H, int K) {
    if (spline_bwd_check(d, H, K, -1, "spline_backward_packed_floats")) return 0;
    const int HT = (H + 31) / 32;
    return (size_t)spline_bwd_layout(HT, spline_bwd_ntmax(HT)).total;
}

extern "C" size_t nfx_spline_backward_param_floats(int d, int H, int K) {
    if (d <= 0 || H <= 0 || K < 2) return 0;
    const int P = 3 * K - 1;
    return (size_t)(H * d + H + H * H + H + d * P * H + d * P);
}

extern "C" size_t nfx_spline_backward_workspace_bytes(int64_t B, int d, int H, int K) {
    if (spline_bwd_check(d, H, K, -1, "spline_backward_workspace_bytes") || B < 0) return 0;
    const int HT = (H + 31) / 32;
    const SplineGrad GL = spline_grad_layout(HT, spline_bwd_ntmax(HT));
    const int64_t ntiles = (B + 31) / 32;
    int64_t nwg = 2 * (int64_t)num_cus();
    const int64_t cap = (ntiles + 3) / 4;
    if (nwg > cap) nwg = cap < 1 ? 1 : cap;
    return (((size_t)nwg * GL.total * sizeof(float) + 255) & ~(size_t)255) + (size_t)GL.total * sizeof(double);
}

extern "C" int nfx_spline_pack_backward(const NfxMlpRaw* net, const float* mask, int d, int H, int K, float* packed,
                                        void* stream) {
    int rc = spline_bwd_check(d, H, K, -1, "spline_pack_backward");
    if (rc) return rc;
    if (!net || !mask || !packed) return set_error(NFX_EINVAL, "spline_pack_backward: null pointer");
    for (int l = 0; l < 3; ++l)
        if (!net->w[l]) return set_error(NFX_EINVAL, "spline_pack_backward: layer %d weight is null", l);
    const int total = (int)nfx_spline_backward_packed_floats(d, H, K);
    int blocks = (total + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    spline_bwd_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(*net, mask, d, H, K, packed);
    return check_launch("spline_bwd_pack_kernel");
}

extern "C" int nfx_spline_coupling_backward(const float* packed, const float* mask, const float* in,
                                            const float* grad_out, const float* grad_log_det, float* grad_in,
                                            float* grads, void* workspace, int64_t B, int d, int H, int K,
                                            int n_transformed, float bound, float min_bin_width,
                                            float min_bin_height, float min_derivative, int direction,
                                            void* stream) {
    int rc = spline_bwd_check(d, H, K, n_transformed, "spline_coupling_backward");
    if (rc) return rc;
    if (direction != NFX_FORWARD && direction != NFX_INVERSE)
        return set_error(NFX_EINVAL, "spline_coupling_backward: direction must be +1 or -1");
    if (B < 1) return set_error(NFX_EINVAL, "spline_coupling_backward: B >= 1 required");
    if (!packed || !mask || !in || !grad_out || !grad_log_det || !grad_in || !grads || !workspace)
        return set_error(NFX_EINVAL, "spline_coupling_backward: null pointer");
    const int HT = (H + 31) / 32;
    spline_bwd_kernel_t k = pick_spline_bwd(HT, K, direction < 0);
    if (!k) return set_error(NFX_EUNSUPPORTED, "spline_coupling_backward: no kernel for H=%d K=%d", H, K);
    SplineConsts C;
    C.bound = bound;
    C.two_bound = (float)(2.0 * (double)bound);
    C.min_w = min_bin_width;
    C.cw = (float)(1.0 - (double)min_bin_width * K);
    C.min_h = min_bin_height;
    C.ch = (float)(1.0 - (double)min_bin_height * K);
    C.min_d = min_derivative;
    C.rescale = 0;
    C.rs_lo = 0.f;
    C.rs_to_scale = C.rs_from_scale = 1.f;
    const size_t lds = spline_bwd_lds(HT);
    if ((rc = prepare_lds((const void*)k, lds))) return rc;
    const int64_t ntiles = (B + 31) / 32;
    int grid = resident_grid((const void*)k, 256, lds, (ntiles + 3) / 4);
    if (grid > 2 * num_cus()) grid = 2 * num_cus();  // the workspace holds <= 2 partials per CU
    const SplineGrad GL = spline_grad_layout(HT, spline_bwd_ntmax(HT));
    const size_t full = nfx_spline_backward_workspace_bytes(B, d, H, K);
    float* part = reinterpret_cast<float*>(workspace);
    double* G = reinterpret_cast<double*>(reinterpret_cast<char*>(workspace) + full - (size_t)GL.total * sizeof(double));
    hipStream_t s = (hipStream_t)stream;
    k<<<grid, 256, lds, s>>>(packed, in, grad_out, grad_log_det, grad_in, part, B, d, C, ntiles);
    if ((rc = check_launch("spline_bwd_kernel"))) return rc;
    if ((rc = train_sum_finish(part, grid, GL.total, G, s))) return rc;
    const int n = (int)nfx_spline_backward_param_floats(d, H, K);
    int blocks = (n + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    spline_bwd_assemble_kernel<<<blocks, 256, 0, s>>>(G, mask, d, H, K, grads);
    return check_launch("spline_bwd_assemble_kernel");
}
