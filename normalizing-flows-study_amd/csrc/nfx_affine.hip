// Fused affine-coupling layer (RealNVP CouplingLayer) for gfx950.
//
// Reference: src/flows/coupling/coupling_layer.py
//   forward :40-68   x = z*m + (1-m)*(z*exp(s)+b),  ld = sum((1-m)*s)
//   inverse :70-96   z = x*m + (1-m)*((x-b)*exp(-s)), ld = sum((1-m)*(-s))
//   s = clamp(s_net(x*m), -10, 10), b = clamp(b_net(x*m), -10, 10)   (:50-51, :79-80)
//   s_net/b_net: Linear(d,H) BN ReLU Linear(H,H) BN ReLU Linear(H,d)   (:18-35)
//   guards: non-finite outputs -> 0, non-finite ld -> 0                 (:61-66, :89-94)
//
// One kernel = one layer, fully fused: conditioner MLPs on fp32 MFMA (32x32x2, activations
// kept in accumulator registers between layers, weights staged once per workgroup in LDS),
// the 64->d output layer on VALU with a v_permlane32_swap half-wave combine, the affine
// transform, the NaN/Inf guards and the per-sample log-det accumulate. HBM traffic is the
// x row in, the y row out and the log-det read-modify-write: 8d+8 bytes per sample.
//
// Work decomposition: a wave owns 64-sample chunks (two 32-sample MFMA column tiles);
// after the output layer lane l holds sample (chunk*64 + l) for the epilogue, so x/y/log_det
// accesses are fully coalesced. Waves grid-stride over chunks so the LDS weight image is
// loaded once per workgroup. Small batches go to the latency-oriented variant in
// nfx_affine_small_kernel.h instead (see affine_policy).
#include <atomic>
#include <climits>
#include <cstdlib>

#include "nfx_affine_kernel.h"
#include "nfx_affine_small_kernel.h"
#include "nfx_pack.h"

namespace nfx {


__global__ void affine_pack_kernel(NfxMlpRaw s_net, NfxMlpRaw b_net, const float* mask, int d,
                                   int H, float* packed) {
    const int HT = (H + 31) / 32;
    const AffineLayout L = affine_layout(d, HT);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < L.s; i += gridDim.x * blockDim.x) {
        float v = 0.f;
        if (i >= L.mask) {
            int j = i - L.mask;
            v = j < d ? mask[j] : 0.f;
        } else {
            const int net = i / L.net;
            const NfxMlpRaw& P = net ? b_net : s_net;
            const int o = i - net * L.net;
            if (o < L.b1) {
                int t = o - L.w1, lane = t & 63, ks = (t >> 6) % L.KS1, ht = (t >> 6) / L.KS1;
                int row = 32 * ht + (lane & 31), col = 2 * ks + (lane >> 5);
                v = (row < H && col < d) ? mlp_weight(P, 0, d, row, col) : 0.f;
            } else if (o < L.w2) {
                int t = o - L.b1, r = t & 15, h = (t >> 4) & 1, ht = t >> 5;
                int row = 32 * ht + crow(r, h);
                v = row < H ? mlp_bias(P, 0, row) : 0.f;
            } else if (o < L.b2) {
                int t = o - L.w2, rr = t & 3, lane = (t >> 2) & 63, rq = (t >> 8) & 3;
                int kt = (t >> 10) % HT, hto = (t >> 10) / HT;
                int row = 32 * hto + (lane & 31), col = 32 * kt + crow(4 * rq + rr, lane >> 5);
                v = (row < H && col < H) ? mlp_weight(P, 1, H, row, col) : 0.f;
            } else if (o < L.w3) {
                int t = o - L.b2, r = t & 15, h = (t >> 4) & 1, ht = t >> 5;
                int row = 32 * ht + crow(r, h);
                v = row < H ? mlp_bias(P, 1, row) : 0.f;
            } else if (o < L.b3 && d > 8) {  // MFMA A-operand tiles of the output layer
                int t = o - L.w3, rr = t & 3, lane = (t >> 2) & 63, rq = (t >> 8) & 3;
                int kt = (t >> 10) % HT, j = (t >> 10) / HT;
                int row = 32 * j + (lane & 31), col = 32 * kt + crow(4 * rq + rr, lane >> 5);
                v = (row < d && col < H) ? mlp_weight(P, 2, H, row, col) : 0.f;
            } else if (o < L.b3) {
                int t = o - L.w3, r = t & 15, h = (t >> 4) & 1, ht = (t >> 5) % HT, j = (t >> 5) / HT;
                int col = 32 * ht + crow(r, h);
                v = col < H ? mlp_weight(P, 2, H, j, col) : 0.f;
            } else if (d > 8) {  // output bias in accumulator order
                int t = o - L.b3, r = t & 15, h = (t >> 4) & 1, j = t >> 5;
                int row = 32 * j + crow(r, h);
                v = row < d ? mlp_bias(P, 2, row) : 0.f;
            } else {
                int j = o - L.b3;
                v = j < d ? mlp_bias(P, 2, j) : 0.f;
            }
        }
        packed[i] = v;
    }
}

// The split tail of an affine image (affine_split, nfx_affine_kernel.h), derived from the fp32
// image written before it on the same stream: copies of w1 b1 b2 w3 b3 and the mask, W2's three
// round-to-nearest bf16 pieces in v_mfma_f32_32x32x16_bf16 A-operand order, and the safety words (W2 finite
// and |w| <= 1e6; xsafe = (1e30 - max|b1|) / max_row sum|w1|). One workgroup: the two maxima
// are reductions and the tail is ~14k floats.
__global__ __launch_bounds__(1024) void affine_split_pack_kernel(float* packed, int d, int H) {
    const int HT = (H + 31) / 32, KS1 = (d + 1) / 2;
    const AffineLayout L = affine_layout(d, HT);
    const AffineSplit S = affine_split(d, HT);
    float* out = packed + L.s;
    __shared__ int w2_bad;
    __shared__ float rowsum[2 * 64], bmax[2 * 64];
    if (threadIdx.x == 0) w2_bad = 0;
    __syncthreads();
    bool bad = false;
    for (int i = threadIdx.x; i < S.total; i += blockDim.x) {
        const int net = i < S.mask ? i / S.net : 0;
        const int o = i - net * S.net;
        const float* P = packed + net * L.net;
        uint32_t v = 0;
        if (i >= S.ok) {
            continue;  // the safety words: below, after the reductions
        } else if (i >= S.mask) {
            v = __float_as_uint(packed[L.mask + (i - S.mask)]);
        } else if (o < S.b1) {
            v = __float_as_uint(P[L.w1 + (o - S.w1)]);
        } else if (o < S.b2) {
            v = __float_as_uint(P[L.b1 + (o - S.b1)]);
        } else if (o < S.w3) {
            v = __float_as_uint(P[L.b2 + (o - S.b2)]);
        } else if (o < S.b3) {
            v = __float_as_uint(P[L.w3 + (o - S.w3)]);
        } else if (o < S.w2s) {
            v = __float_as_uint(P[L.b3 + (o - S.b3)]);
        } else {
            // dword t: [out tile hto][k block kb][piece p][lane][q], elements 2q, 2q + 1
            const int t = o - S.w2s, q = t & 3, lane = (t >> 2) & 63, g = t >> 8;
            const int p = g % 3, kb = (g / 3) % (2 * HT), hto = (g / 3) / (2 * HT);
            const int kt = kb >> 1;
            uint32_t half[2];
            for (int e = 0; e < 2; ++e) {
                const int r = 8 * (kb & 1) + 2 * q + e;  // accumulator register of the B operand
                const float w = P[L.w2 + ((hto * HT + kt) * 4 + (r >> 2)) * 256 + lane * 4 + (r & 3)];
                if (!(fabsf(w) <= 1e6f)) bad = true;
                // round-to-nearest pieces (random signs: unbiased dropped products, split_block)
                const uint32_t u0 = __builtin_bit_cast(uint16_t, (__bf16)w);
                const float r1 = w - __uint_as_float(u0 << 16);
                const uint32_t u1 = __builtin_bit_cast(uint16_t, (__bf16)r1);
                const uint32_t u2 = __builtin_bit_cast(uint16_t, (__bf16)(r1 - __uint_as_float(u1 << 16)));
                half[e] = p == 0 ? u0 : p == 1 ? u1 : u2;
            }
            v = half[0] | (half[1] << 16);
        }
        out[i] = __uint_as_float(v);
    }
    if (bad) atomicOr(&w2_bad, 1);
    // layer-1 bound: row sums of |w1| (rows 32 ht + c of net n) and |b1|
    for (int i = threadIdx.x; i < 2 * 64; i += blockDim.x) {
        rowsum[i] = 0.f;
        bmax[i] = 0.f;
    }
    __syncthreads();
    if (threadIdx.x < 2 * 32 * HT) {
        const int net = threadIdx.x / (32 * HT), row = threadIdx.x % (32 * HT), ht = row >> 5, c = row & 31;
        const float* P = packed + net * L.net;
        float sum = 0.f;
        for (int ks = 0; ks < KS1; ++ks)
            for (int hh = 0; hh < 2; ++hh) sum += fabsf(P[L.w1 + (ht * KS1 + ks) * 64 + c + 32 * hh]);
        rowsum[net * 64 + row] = sum;
        float b = 0.f;
        for (int r = 0; r < 16; ++r)
            for (int hh = 0; hh < 2; ++hh)
                if (crow(r, hh) == c) b = fabsf(P[L.b1 + ht * 32 + 16 * hh + r]);
        bmax[net * 64 + row] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float n1 = 0.f, c1 = 0.f;
        bool nan = false;
        for (int i = 0; i < 2 * 64; ++i) {
            nan = nan || !(rowsum[i] <= 3e38f) || !(bmax[i] <= 3e38f);
            n1 = fmaxf(n1, rowsum[i]);
            c1 = fmaxf(c1, bmax[i]);
        }
        const float xs = nan ? 0.f : (1e30f - c1) / n1;  // n1 == 0: +inf (no x reaches layer 1)
        out[S.ok] = w2_bad ? 0.f : 1.f;
        out[S.ok + 1] = xs > 0.f ? xs : 0.f;
        out[S.ok + 2] = 0.f;
        out[S.ok + 3] = 0.f;
    }
}

int affine_split_pack(float* packed, int d, int H, hipStream_t s) {
    if (!affine_has_split(d, (H + 31) / 32)) return NFX_OK;
    affine_split_pack_kernel<<<1, 1024, 0, s>>>(packed, d, H);
    return check_launch("affine_split_pack_kernel");
}

static affine_kernel_t pick_affine(int HT, int d, int dir, bool logp) {
    switch (HT) {
        case 1: return affine_pick_ht<1>(d, dir, logp);
        case 2: return affine_pick_ht<2>(d, dir, logp);
        case 3: return affine_pick_ht<3>(d, dir, logp);
        case 4: return affine_pick_ht<4>(d, dir, logp);
        default: return nullptr;
    }
}

static affine_kernel_t pick_affine_small(int HT, int d, int dir, bool logp) {
    switch (HT) {
        case 1: return affine_small_pick_ht<1>(d, dir, logp);
        case 2: return affine_small_pick_ht<2>(d, dir, logp);
        case 3: return affine_small_pick_ht<3>(d, dir, logp);
        case 4: return affine_small_pick_ht<4>(d, dir, logp);
        default: return nullptr;
    }
}

// Kernel choice (nfx_affine_kernel_policy). AUTO compares MFMA "rounds": the streaming kernel
// runs ceil(chunks / resident waves) 64-sample chunks per wave, each a chain of ~2*HT times the
// MFMAs of one small-kernel 32-sample tile, of which the small kernel runs ceil(tiles /
// resident workgroups) per workgroup. (Measured at RealNVP H=128: small 8 us vs streaming 37 us
// per layer up to 8k samples, break-even near 64k.) Initial policy: $NFX_AFFINE_POLICY or AUTO.
static std::atomic<int>& affine_policy() {
    static std::atomic<int> v{[] {
        const char* e = getenv("NFX_AFFINE_POLICY");
        return e ? atoi(e) : NFX_AFFINE_AUTO;
    }()};
    return v;
}

int affine_policy_get() { return affine_policy().load(std::memory_order_relaxed); }

typedef void (*affine_wide_t)(const float*, const float*, float*, float*, int64_t, int, int, int64_t, float*,
                              double*, double*, float);

template <int HT>
static affine_wide_t wide_pick(int dir, bool logp) {
    if (dir > 0) return affine_wide_kernel<HT, 1, false>;
    return logp ? affine_wide_kernel<HT, -1, true> : affine_wide_kernel<HT, -1, false>;
}

static int affine_wide_launch(const float* packed, const float* in, float* out, float* log_det, int64_t B, int d,
                              int H, int direction, int accumulate, float* logp, double* sums, void* workspace,
                              hipStream_t stream) {
    const bool fused = sums != nullptr;
    const int HT = (H + 31) / 32;
    if (d > 64 || HT > 4)
        return set_error(NFX_EUNSUPPORTED, "affine_coupling: d=%d H=%d outside the compiled family (d<=64, H<=128)", d, H);
    affine_wide_t k = HT == 1 ? wide_pick<1>(direction, fused)
                      : HT == 2 ? wide_pick<2>(direction, fused)
                      : HT == 3 ? wide_pick<3>(direction, fused) : wide_pick<4>(direction, fused);
    if (B == 0) return fused ? gauss_finish(reinterpret_cast<double*>(workspace), 0, sums, 0, stream) : NFX_OK;
    if (!packed || !in || !out || !log_det) return set_error(NFX_EINVAL, "affine_coupling: null pointer");
    if (in == out) return set_error(NFX_EINVAL, "affine_coupling: in and out must not alias");
    const size_t lds = (size_t)kWideWaves * 32 * (d | 1) * sizeof(float);
    const int64_t ntiles = (B + 31) / 32;
    int grid = resident_grid((const void*)k, 64 * kWideWaves, lds, (ntiles + kWideWaves - 1) / kWideWaves);
    if (grid > kMaxPartials) grid = kMaxPartials;
    double* partials = reinterpret_cast<double*>(workspace);
    k<<<grid, 64 * kWideWaves, lds, stream>>>(packed, in, out, log_det, B, d, accumulate, ntiles, logp, partials,
                                              sums, gauss_const(d));
    return check_launch("affine_wide_kernel");  // (LOGP: the last workgroup wrote sums)
}

static int affine_launch(const float* packed, const float* in, float* out, float* log_det, int64_t B,
                         int d, int H, int direction, int accumulate, float* logp, double* sums,
                         void* workspace, hipStream_t stream) {
    const bool fused = sums != nullptr;
    if (B < 0 || d <= 0 || H <= 0) return set_error(NFX_EINVAL, "affine_coupling: bad shape B=%lld d=%d H=%d", (long long)B, d, H);
    if (direction != NFX_FORWARD && direction != NFX_INVERSE)
        return set_error(NFX_EINVAL, "affine_coupling: direction must be +1 or -1");
    if (fused && B > 0 && (!logp || !workspace)) return set_error(NFX_EINVAL, "affine_coupling_logprob: null logp/workspace");
    const int HT = (H + 31) / 32;
    if (d > 8) return affine_wide_launch(packed, in, out, log_det, B, d, H, direction, accumulate, logp, sums,
                                         workspace, stream);
    affine_kernel_t k = pick_affine(HT, d, direction, fused);
    if (!k) return set_error(NFX_EUNSUPPORTED, "affine_coupling: d=%d H=%d outside the compiled family (d<=64, H<=128)", d, H);
    if (B == 0) return fused ? gauss_finish(reinterpret_cast<double*>(workspace), 0, sums, 0, stream) : NFX_OK;
    if (!packed || !in || !out || !log_det) return set_error(NFX_EINVAL, "affine_coupling: null pointer");
    if (in == out) return set_error(NFX_EINVAL, "affine_coupling: in and out must not alias");
    const AffineLayout L = affine_layout(d, HT);
    const size_t lds = (size_t)(affine_has_split(d, HT) ? affine_split(d, HT).total : L.total) * sizeof(float);
    int rc = prepare_lds((const void*)k, lds);
    if (rc) return rc;
    double* partials = reinterpret_cast<double*>(workspace);
    const int64_t nchunks = (B + 63) / 64;
    const int64_t ntiles = (B + 31) / 32;
    const int policy = affine_policy().load(std::memory_order_relaxed);
    affine_kernel_t ks = pick_affine_small(HT, d, direction, fused);
    int grid_small = resident_grid((const void*)ks, 128 * HT, 0, ntiles);
    bool small = policy == NFX_AFFINE_SMALL;
    if (policy == NFX_AFFINE_AUTO) {
        const int64_t waves = 4 * (int64_t)resident_grid((const void*)k, 256, lds, INT64_MAX);
        const int64_t rounds_stream = (nchunks + waves - 1) / waves;
        const int64_t rounds_small = (ntiles + grid_small - 1) / grid_small;
        small = rounds_small < 2 * HT * rounds_stream;
    }
    if (small) {
        if (grid_small > kMaxPartials) grid_small = kMaxPartials;
        ks<<<grid_small, 128 * HT, 0, stream>>>(packed, in, out, log_det, B, accumulate, ntiles, logp,
                                                partials, sums, gauss_const(d));
        return check_launch("affine_small_kernel");
    }
    // Up to one 32-sample half chunk per wave: when the resident waves outnumber the 64-sample
    // chunks (small batches, e.g. a strong-scaled 125k shard), the kernel's split gives every wave
    // a half chunk instead of leaving half the waves idle behind full chunks (the layer time is one
    // wave's chain: 64 -> 32 samples halves it)
    int grid = resident_grid((const void*)k, 256, lds, ((B + 31) / 32 + 3) / 4);
    if (grid > kMaxPartials) grid = kMaxPartials;
    k<<<grid, 256, lds, stream>>>(packed, in, out, log_det, B, accumulate, nchunks, logp, partials, sums,
                                  gauss_const(d));
    return check_launch("affine_coupling_kernel");
}

// Grid: enough resident workgroups to fill every CU (occupancy from the runtime), never more
// than there are 4-chunk groups of work.
int resident_grid(const void* kernel, int threads, size_t lds_bytes, int64_t work_groups) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds_bytes) != hipSuccess ||
        per_cu <= 0)
        per_cu = 1;
    int64_t g = (int64_t)num_cus() * per_cu;
    if (work_groups < g) g = work_groups;
    return (int)(g < 1 ? 1 : g);
}

int prepare_lds(const void* kernel, size_t bytes) {
    if (bytes > 65536) {
        if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) !=
            hipSuccess) {
            (void)hipGetLastError();  // do not leave the error sticky for the caller's next HIP call
            return set_error(NFX_ELAUNCH, "hipFuncSetAttribute(dynamic LDS %zu B) failed", bytes);
        }
    }
    return NFX_OK;
}

}  // namespace nfx

using namespace nfx;

extern "C" size_t nfx_affine_packed_floats(int d, int H) {
    if (d <= 0 || H <= 0) return 0;
    return (size_t)affine_layout(d, (H + 31) / 32).total;
}

extern "C" int nfx_affine_pack(const NfxMlpRaw* s_net, const NfxMlpRaw* b_net, const float* mask,
                               int d, int H, float* packed, void* stream) {
    if (!s_net || !b_net || !mask || !packed) return set_error(NFX_EINVAL, "affine_pack: null pointer");
    if (d <= 0 || H <= 0) return set_error(NFX_EINVAL, "affine_pack: bad shape d=%d H=%d", d, H);
    const NfxMlpRaw* nets[2] = {s_net, b_net};
    for (int n = 0; n < 2; ++n)
        for (int l = 0; l < 3; ++l)
            if (!nets[n]->w[l]) return set_error(NFX_EINVAL, "affine_pack: net %d layer %d weight is null", n, l);
    const int total = (int)nfx_affine_packed_floats(d, H);
    int blocks = (total + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    affine_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(*s_net, *b_net, mask, d, H, packed);
    const int rc = check_launch("affine_pack_kernel");
    return rc ? rc : affine_split_pack(packed, d, H, (hipStream_t)stream);
}

extern "C" int nfx_affine_coupling(const float* packed, const float* in, float* out, float* log_det,
                                   int64_t B, int d, int H, int direction, int accumulate,
                                   void* stream) {
    return affine_launch(packed, in, out, log_det, B, d, H, direction, accumulate, nullptr, nullptr,
                         nullptr, (hipStream_t)stream);
}

extern "C" int nfx_affine_kernel_policy(int policy) {
    if (policy < 0) return affine_policy().load();
    if (policy > NFX_AFFINE_SMALL) return set_error(NFX_EINVAL, "affine_kernel_policy: unknown policy %d", policy);
    return affine_policy().exchange(policy);
}

extern "C" int nfx_affine_coupling_logprob(const float* packed, const float* in, float* out,
                                           float* log_det, float* logp, double* sums, void* workspace,
                                           int64_t B, int d, int H, int accumulate, void* stream) {
    if (!sums) return set_error(NFX_EINVAL, "affine_coupling_logprob: null sums");
    return affine_launch(packed, in, out, log_det, B, d, H, NFX_INVERSE, accumulate, logp, sums,
                         workspace, (hipStream_t)stream);
}
