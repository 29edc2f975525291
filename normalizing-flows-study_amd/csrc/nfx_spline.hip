// Spline coupling: weight pack + C-ABI entry points (kernel: nfx_spline_kernel.h).
#include <math.h>

#include "nfx_pack.h"
#include "nfx_spline_kernel.h"

namespace nfx {

// t-th transformed dimension (mask == 0), or -1.
__device__ inline int spline_tdim(const float* mask, int d, int t) {
    int n = 0;
    for (int j = 0; j < d; ++j) {
        if (mask[j] == 0.f) {
            if (n == t) return j;
            ++n;
        }
    }
    return -1;
}

__global__ void spline_pack_kernel(NfxMlpRaw net, const float* mask, int d, int H, int K, float* packed) {
    const int HT = (H + 31) / 32;
    const SplineLayout L = spline_layout(HT, d);
    const int P = 3 * K - 1;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < L.total; i += gridDim.x * blockDim.x) {
        float v = 0.f;
        if (i < L.b1) {
            const int KS = spline_ks1(d);
            int t = i - L.w1, lane = t & 63, ks = (t >> 6) % KS, ht = (t >> 6) / KS;
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
            int dt = spline_tdim(mask, d, tile), p = lane & 31;
            int col = 32 * kt + crow(4 * rq + rr, lane >> 5);
            v = (dt >= 0 && p < P && col < H) ? mlp_weight(net, 2, H, dt * P + p, col) : 0.f;
        } else if (i < L.mask) {
            int t = i - L.b3, r = t & 15, h = (t >> 4) & 1, tile = t >> 5;
            int dt = spline_tdim(mask, d, tile), p = crow(r, h);
            v = (dt >= 0 && p < P) ? mlp_bias(net, 2, dt * P + p) : 0.f;
        } else if (i < L.tdim) {
            int j = i - L.mask;
            v = j < d ? mask[j] : 0.f;
        } else if (i < L.meta) {
            int t = i - L.tdim;
            v = (float)spline_tdim(mask, d, t);
        } else {
            int nt = 0;
            for (int j = 0; j < d; ++j) nt += mask[j] == 0.f ? 1 : 0;
            v = (i == L.meta) ? (float)nt : 0.f;
        }
        packed[i] = v;
    }
}

static spline_kernel_t pick_spline(int HT, int K, int dir, bool logp, int d) {
    if (d > 8) {
        switch (HT) {
            case 1: return spline_wide_pick_ht<1>(K, dir, logp);
            case 2: return spline_wide_pick_ht<2>(K, dir, logp);
            case 3: return spline_wide_pick_ht<3>(K, dir, logp);
            case 4: return spline_wide_pick_ht<4>(K, dir, logp);
            default: return nullptr;
        }
    }
    if (d == 2) {
        switch (HT) {
            case 1: return spline_pick_ht<1, 2>(K, dir, logp);
            case 2: return spline_pick_ht<2, 2>(K, dir, logp);
            case 3: return spline_pick_ht<3, 2>(K, dir, logp);
            case 4: return spline_pick_ht<4, 2>(K, dir, logp);
            default: return nullptr;
        }
    }
    switch (HT) {
        case 1: return spline_pick_ht<1, 0>(K, dir, logp);
        case 2: return spline_pick_ht<2, 0>(K, dir, logp);
        case 3: return spline_pick_ht<3, 0>(K, dir, logp);
        case 4: return spline_pick_ht<4, 0>(K, dir, logp);
        default: return nullptr;
    }
}

}  // namespace nfx

using namespace nfx;

extern "C" size_t nfx_spline_packed_floats(int d, int H, int K) {
    if (d <= 0 || H <= 0 || K <= 1) return 0;
    return (size_t)spline_layout((H + 31) / 32, d).total;
}

extern "C" int nfx_spline_pack(const NfxMlpRaw* net, const float* mask, int d, int H, int K,
                               float* packed, void* stream) {
    if (!net || !mask || !packed) return set_error(NFX_EINVAL, "spline_pack: null pointer");
    if (d <= 0 || d > 64 || H <= 0 || H > 128 || K < 2 || K > 11)
        return set_error(NFX_EUNSUPPORTED, "spline_pack: d=%d H=%d K=%d outside d<=64, H<=128, 2<=K<=11", d, H, K);
    for (int l = 0; l < 3; ++l)
        if (!net->w[l]) return set_error(NFX_EINVAL, "spline_pack: layer %d weight is null", l);
    const int total = (int)nfx_spline_packed_floats(d, H, K);
    int blocks = (total + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    spline_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(*net, mask, d, H, K, packed);
    return check_launch("spline_pack_kernel");
}

static int spline_launch(const float* packed, const float* in, float* out, float* log_det, int64_t B,
                         int d, int H, int K, float bound, float min_bin_width, float min_bin_height,
                         float min_derivative, int rescale, float data_min, float data_max,
                         int direction, int accumulate, float* logp, double* sums, void* workspace,
                         hipStream_t stream) {
    const bool fused = sums != nullptr;
    if (B < 0 || d <= 0 || H <= 0) return set_error(NFX_EINVAL, "spline_coupling: bad shape");
    if (direction != NFX_FORWARD && direction != NFX_INVERSE)
        return set_error(NFX_EINVAL, "spline_coupling: direction must be +1 or -1");
    if (d > 64 || H > 128 || K < 2 || K > 11)
        return set_error(NFX_EUNSUPPORTED, "spline_coupling: d=%d H=%d K=%d outside d<=64, H<=128, 2<=K<=11", d, H, K);
    if (fused && B > 0 && (!logp || !workspace)) return set_error(NFX_EINVAL, "spline_coupling_logprob: null logp/workspace");
    if (B == 0) return fused ? gauss_finish(reinterpret_cast<double*>(workspace), 0, sums, 0, stream) : NFX_OK;
    if (!packed || !in || !out || !log_det) return set_error(NFX_EINVAL, "spline_coupling: null pointer");
    if (in == out) return set_error(NFX_EINVAL, "spline_coupling: in and out must not alias");
    const int HT = (H + 31) / 32;
    spline_kernel_t k = pick_spline(HT, K, direction, fused, d);
    if (!k) return set_error(NFX_EUNSUPPORTED, "spline_coupling: no kernel for H=%d K=%d", H, K);
    const SplineConsts C =
        spline_consts(K, bound, min_bin_width, min_bin_height, min_derivative, rescale, data_min, data_max);
    if (d > 8) {  // wide kernel: 32-sample tiles, weights from L2
        const size_t ldsw = (size_t)kSplineWideWaves * 32 * (d | 1) * sizeof(float);
        const int64_t ntiles = (B + 31) / 32;
        int gw = resident_grid((const void*)k, 64 * kSplineWideWaves, ldsw,
                               (ntiles + kSplineWideWaves - 1) / kSplineWideWaves);
        if (gw > kMaxPartials) gw = kMaxPartials;
        double* pw = reinterpret_cast<double*>(workspace);
        k<<<gw, 64 * kSplineWideWaves, ldsw, stream>>>(packed, in, out, log_det, B, d, C, accumulate, ntiles, logp, pw,
                                                        sums, gauss_const(d));
        return check_launch("spline_wide_kernel");
    }
    const size_t lds = (size_t)spline_layout(HT, d).total * sizeof(float);
    int rc = prepare_lds((const void*)k, lds);
    if (rc) return rc;
    const int64_t nchunks = (B + 63) / 64;
    // up to one 32-sample half chunk per wave at small batches (as nfx_affine.hip)
    int grid = resident_grid((const void*)k, 256, lds, ((B + 31) / 32 + 3) / 4);
    if (grid > kMaxPartials) grid = kMaxPartials;
    double* partials = reinterpret_cast<double*>(workspace);
    k<<<grid, 256, lds, stream>>>(packed, in, out, log_det, B, d, C, accumulate, nchunks, logp, partials, sums,
                                  gauss_const(d));
    return check_launch("spline_coupling_kernel");
}

extern "C" int nfx_spline_coupling(const float* packed, const float* in, float* out, float* log_det,
                                   int64_t B, int d, int H, int K, float bound, float min_bin_width,
                                   float min_bin_height, float min_derivative, int rescale,
                                   float data_min, float data_max, int direction, int accumulate,
                                   void* stream) {
    return spline_launch(packed, in, out, log_det, B, d, H, K, bound, min_bin_width, min_bin_height,
                         min_derivative, rescale, data_min, data_max, direction, accumulate, nullptr,
                         nullptr, nullptr, (hipStream_t)stream);
}

extern "C" int nfx_spline_coupling_logprob(const float* packed, const float* in, float* out,
                                           float* log_det, float* logp, double* sums, void* workspace,
                                           int64_t B, int d, int H, int K, float bound,
                                           float min_bin_width, float min_bin_height,
                                           float min_derivative, int rescale, float data_min,
                                           float data_max, int accumulate, void* stream) {
    if (!sums) return set_error(NFX_EINVAL, "spline_coupling_logprob: null sums");
    return spline_launch(packed, in, out, log_det, B, d, H, K, bound, min_bin_width, min_bin_height,
                         min_derivative, rescale, data_min, data_max, NFX_INVERSE, accumulate, logp,
                         sums, workspace, (hipStream_t)stream);
}
