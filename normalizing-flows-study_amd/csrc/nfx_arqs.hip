// ARQS — autoregressive rational-quadratic spline flow (src/flows/spline/arqs.py:7-114).
//
// The reference runs d sequential steps in both directions (forward :44-80, inverse :82-114):
// step i evaluates the full MADE(d, H, R = 3K-1) on the partially filled state (columns < i
// set, the rest zero), views the output as [B, d, R] and feeds row i's R parameters to the
// unit-interval spline (rational_quadratic_spline) of input column i. The view does NOT follow
// MADE's output order (output unit o = k*d + i' belongs to MADE dimension i' = o mod d), so
// step i's parameters can depend on state columns >= i that are still zero: unlike MAF.forward
// the steps cannot be collapsed into one MADE pass. This kernel reproduces that exactly.
//
// One launch runs all d steps for every sample: a workgroup of HT waves walks 32-sample tiles;
// per step only the R output rows of the step are computed (one MFMA tile instead of the
// reference's R*d rows), layer 1 is a rank-1 update of register-resident pre-activations with
// the one new state column, layers 2-3 are MFMA tiles with each wave's weight rows held in
// registers for the whole kernel, and the spline runs on 32 threads per step. MFMA work per
// sample and step: 2*(2*Hp^2 + 32*Hp) flops; HBM traffic: the x row in, the y row and the
// log-det out (weights are L2-resident after the first tiles).
#include <climits>

#include "nfx_arqs_kernel.h"
#include "nfx_pack.h"

namespace nfx {

__global__ void arqs_pack_kernel(NfxMlpRaw net, int d, int H, int K, float* packed) {
    const int HT = (H + 31) / 32, R = 3 * K - 1;
    const ArqsLayout L = arqs_layout(d, HT, R);
    for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < L.total; o += gridDim.x * blockDim.x) {
        float v = 0.f;
        if (o < L.b1) {  // w2 / w3 A operands
            const int layer = o < L.w3 ? 1 : 2;
            const int t = o - (layer == 1 ? L.w2 : L.w3);
            const int rr = t & 3, lane = (t >> 2) & 63, rq = (t >> 8) & 3;
            const int kt = (t >> 10) % HT, hto = (t >> 10) / HT;
            const int row = 32 * hto + (lane & 31), col = 32 * kt + crow(4 * rq + rr, lane >> 5);
            v = (row < H && col < H) ? mlp_weight(net, layer, H, row, col) : 0.f;
        } else if (o < L.w1t) {  // b1 b2 b3
            const int layer = (o - L.b1) / (HT * 32);
            const int t = (o - L.b1) % (HT * 32);
            const int r = t & 15, h = (t >> 4) & 1, ht = t >> 5;
            const int row = 32 * ht + crow(r, h);
            v = row < H ? mlp_bias(net, layer, row) : 0.f;
        } else if (o < L.w4) {  // w1t
            const int t = o - L.w1t;
            const int r = t & 15, h = (t >> 4) & 1, ht = (t >> 5) % HT, j = (t >> 5) / HT;
            const int row = 32 * ht + crow(r, h);
            v = row < H ? mlp_weight(net, 0, d, row, j) : 0.f;
        } else if (o < L.b4) {  // w4: the R rows of step i
            const int t = o - L.w4;
            const int rr = t & 3, lane = (t >> 2) & 63, rq = (t >> 8) & 3;
            const int kt = (t >> 10) % HT, i = (t >> 10) / HT;
            const int m = lane & 31, col = 32 * kt + crow(4 * rq + rr, lane >> 5);
            v = (m < R && col < H) ? mlp_weight(net, 3, H, i * R + m, col) : 0.f;
        } else {  // b4
            const int t = o - L.b4;
            const int r = t & 15, h = (t >> 4) & 1, i = t >> 5;
            const int m = crow(r, h);
            v = m < R ? mlp_bias(net, 3, i * R + m) : 0.f;
        }
        packed[o] = v;
    }
}

static arqs_kernel_t pick_arqs(int HT, int K, int inverse) {
    switch (HT) {
        case 1: return arqs_pick_ht<1>(K, inverse);
        case 2: return arqs_pick_ht<2>(K, inverse);
        case 3: return arqs_pick_ht<3>(K, inverse);
        case 4: return arqs_pick_ht<4>(K, inverse);
        default: return nullptr;
    }
}

}  // namespace nfx

using namespace nfx;

extern "C" size_t nfx_arqs_packed_floats(int d, int H, int K) {
    if (d <= 0 || H <= 0 || K < 2) return 0;
    return (size_t)arqs_layout(d, (H + 31) / 32, 3 * K - 1).total;
}

extern "C" int nfx_arqs_pack(const NfxMlpRaw* made, int d, int H, int K, float* packed, void* stream) {
    if (!made || !packed) return set_error(NFX_EINVAL, "arqs_pack: null pointer");
    if (d <= 0 || H <= 0 || K < 2) return set_error(NFX_EINVAL, "arqs_pack: bad shape d=%d H=%d K=%d", d, H, K);
    if (H > 128 || K > 11) return set_error(NFX_EUNSUPPORTED, "arqs: H=%d K=%d outside the compiled family (H<=128, K<=11)", H, K);
    if (made->n_layers != 4) return set_error(NFX_EINVAL, "arqs_pack: MADE has 4 masked linears, got %d", made->n_layers);
    const int total = (int)nfx_arqs_packed_floats(d, H, K);
    int blocks = (total + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    arqs_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(*made, d, H, K, packed);
    return check_launch("arqs_pack_kernel");
}

extern "C" int nfx_arqs(const float* packed, const float* in, float* out, float* log_det, int64_t B,
                        int d, int H, int K, float min_bin_width, float min_bin_height,
                        float min_derivative, int rescale, double data_min, double data_max,
                        int direction, int accumulate, void* stream) {
    if (B < 0 || d <= 0 || H <= 0 || K < 2) return set_error(NFX_EINVAL, "arqs: bad shape B=%lld d=%d H=%d K=%d", (long long)B, d, H, K);
    if (direction != NFX_FORWARD && direction != NFX_INVERSE) return set_error(NFX_EINVAL, "arqs: direction must be +1 or -1");
    const int HT = (H + 31) / 32;
    arqs_kernel_t k = pick_arqs(HT, K, direction == NFX_INVERSE);
    if (!k) return set_error(NFX_EUNSUPPORTED, "arqs: H=%d K=%d outside the compiled family (H<=128, K<=11)", H, K);
    if (B == 0) return NFX_OK;
    if (!packed || !in || !out || !log_det) return set_error(NFX_EINVAL, "arqs: null pointer");
    if (in == out) return set_error(NFX_EINVAL, "arqs: in and out must not alias");
    ArqsArgs A{};
    A.packed = packed;
    A.in = in;
    A.out = out;
    A.logdet = log_det;
    A.B = B;
    A.ntiles = (B + 31) / 32;
    A.d = d;
    A.accumulate = accumulate;
    A.rescale = rescale ? 1 : 0;
    A.lo = (float)data_min;                 // x - data_min: the scalar is cast to fp32 (arqs.py:34)
    A.span = (float)(data_max - data_min);  // Python-float difference, then fp32
    A.min_w = min_bin_width;
    A.cw = (float)(1.0 - (double)min_bin_width * K);
    A.min_h = min_bin_height;
    A.ch = (float)(1.0 - (double)min_bin_height * K);
    A.min_d = min_derivative;
    const int grid = resident_grid((const void*)k, 64 * HT, 0, A.ntiles);
    k<<<grid, 64 * HT, 0, (hipStream_t)stream>>>(A);
    return check_launch("arqs_kernel");
}
