// Streaming spline chain: launch + C-ABI (kernel: nfx_spline_schain_kernel.h).
#include "nfx_spline_schain_kernel.h"

#include <cstdlib>

namespace nfx {

static int spline_schain_wpad_rt(int HT) { return (spline_layout(HT, 2).total + 255) & ~255; }

// Chunks of rows one workgroup can hold next to the two weight images.
static int64_t spline_schain_slice_cap(int HT) {
    const size_t w = 2 * (size_t)spline_schain_wpad_rt(HT) * sizeof(float);
    const size_t lds = 160 * 1024, stat = 1024;
    if (w + stat >= lds) return 0;
    return (int64_t)((lds - stat - w) / (64 * 3 * sizeof(float)));
}

static bool spline_chain_supported(int64_t B, int d, int H, int K) {
    const int HT = (H + 31) / 32;
    return B >= 0 && d == 2 && HT >= 1 && HT <= 2 && K >= 2 && K <= 11 && spline_schain_slice_cap(HT) >= 1;
}

static int spline_chain_launch(const float* const* packs, int nl, const float* in, float* out, float* log_det,
                               int64_t B, int d, int H, int K, float bound, float min_w, float min_h, float min_d,
                               int direction, int accumulate, float* logp, double* sums, void* workspace,
                               hipStream_t s, uint64_t* rng = nullptr, uint64_t seed = 0, float* zout = nullptr) {
    const bool fused = sums != nullptr;
    const bool sample = rng != nullptr;
    if (sample && (direction != NFX_FORWARD || fused || accumulate))
        return set_error(NFX_EINVAL, "spline_chain_sample: forward chains, no accumulate");
    if (nl <= 0 || nl > kChainMax) return set_error(NFX_EINVAL, "spline_chain: 1 <= n_layers <= %d (got %d)", kChainMax, nl);
    if (direction != NFX_FORWARD && direction != NFX_INVERSE)
        return set_error(NFX_EINVAL, "spline_chain: direction must be +1 or -1");
    if (fused && direction != NFX_INVERSE) return set_error(NFX_EINVAL, "spline_chain_logprob: inverse chains only");
    if (B < 0) return set_error(NFX_EINVAL, "spline_chain: B < 0");
    if (!spline_chain_supported(B, d, H, K))
        return set_error(NFX_EUNSUPPORTED, "spline_chain: d=%d H=%d K=%d outside d = 2, H <= 64, 2 <= K <= 11", d, H, K);
    if (B == 0) return fused ? gauss_finish(reinterpret_cast<double*>(workspace), 0, sums, 0, s) : NFX_OK;
    if (!packs || (!in && !sample) || !out || !log_det || (fused && (!logp || !workspace)))
        return set_error(NFX_EINVAL, "spline_chain: null pointer");
    if (in == out && !sample) return set_error(NFX_EINVAL, "spline_chain: in and out must not alias");
    if (sample && zout == out) return set_error(NFX_EINVAL, "spline_chain_sample: z and x must not alias");
    NfxChainPacks P{};
    for (int l = 0; l < nl; ++l) {
        if (!packs[l]) return set_error(NFX_EINVAL, "spline_chain: layer %d pack is null", l);
        P.p[l] = packs[l];
    }
    const int HT = (H + 31) / 32;
    const SplineConsts C = spline_consts(K, bound, min_w, min_h, min_d, 0, 0.f, 0.f);
    const int64_t nchunks = (B + 63) / 64;
    int64_t grid = num_cus();
    if (grid > nchunks) grid = nchunks;
    if (grid > kMaxPartials) grid = kMaxPartials;
    const int64_t per_wg = (nchunks + grid - 1) / grid;
    // $NFX_SCHAIN_WAVES=8 / 12 forces one kernel (A/B measurements)
    static const int force = [] {
        const char* e = getenv("NFX_SCHAIN_WAVES");
        return e ? atoi(e) : 0;
    }();
    const bool small = force ? force == kSplineSchainWavesSmall : per_wg <= kSplineSchainWavesSmall;
    const int nw = small ? kSplineSchainWavesSmall : kSplineSchainWaves;
    spline_schain_t k = HT == 1 ? spline_schain_pick_ht<1>(K, direction, fused, small)
                                : spline_schain_pick_ht<2>(K, direction, fused, small);
    if (!k) return set_error(NFX_EUNSUPPORTED, "spline_chain: no kernel for K=%d", K);
    const int64_t cap = spline_schain_slice_cap(HT);
    const int64_t nslices = (per_wg + cap - 1) / cap;
    const int64_t slice = (per_wg + nslices - 1) / nslices;
    const size_t lds = (2 * (size_t)spline_schain_wpad_rt(HT) + (size_t)slice * 64 * 3) * sizeof(float);
    int rc = prepare_lds((const void*)k, lds);
    if (rc) return rc;
    k<<<(unsigned)grid, 64 * nw, lds, s>>>(P, nl, in, out, log_det, B, C, accumulate, nchunks,
                                                            (int)slice, logp, reinterpret_cast<double*>(workspace),
                                                            sums, gauss_const(d), seed, rng, zout);
    return check_launch("spline_schain_kernel");
}

}  // namespace nfx

using namespace nfx;

extern "C" int nfx_spline_chain_supported(int64_t B, int d, int H, int K) {
    return spline_chain_supported(B, d, H, K) ? 1 : 0;
}

extern "C" int nfx_spline_chain(const float* const* packs, int n_layers, const float* in, float* out, float* log_det,
                                int64_t B, int d, int H, int K, float bound, float min_bin_width, float min_bin_height,
                                float min_derivative, int direction, int accumulate, void* stream) {
    return spline_chain_launch(packs, n_layers, in, out, log_det, B, d, H, K, bound, min_bin_width, min_bin_height,
                               min_derivative, direction, accumulate, nullptr, nullptr, nullptr, (hipStream_t)stream);
}

extern "C" int nfx_spline_chain_logprob(const float* const* packs, int n_layers, const float* in, float* out,
                                        float* log_det, float* logp, double* sums, void* workspace, int64_t B, int d,
                                        int H, int K, float bound, float min_bin_width, float min_bin_height,
                                        float min_derivative, int accumulate, void* stream) {
    if (!sums) return set_error(NFX_EINVAL, "spline_chain_logprob: null sums");
    return spline_chain_launch(packs, n_layers, in, out, log_det, B, d, H, K, bound, min_bin_width, min_bin_height,
                               min_derivative, NFX_INVERSE, accumulate, logp, sums, workspace, (hipStream_t)stream);
}

extern "C" int nfx_spline_chain_sample(const float* const* packs, int n_layers, uint64_t seed, uint64_t* rng_state,
                                       float* z, float* x, float* log_det, int64_t B, int d, int H, int K, float bound,
                                       float min_bin_width, float min_bin_height, float min_derivative, void* stream) {
    if (!rng_state) return set_error(NFX_EINVAL, "spline_chain_sample: null rng_state");
    return spline_chain_launch(packs, n_layers, nullptr, x, log_det, B, d, H, K, bound, min_bin_width, min_bin_height,
                               min_derivative, NFX_FORWARD, 0, nullptr, nullptr, nullptr, (hipStream_t)stream,
                               rng_state, seed, z);
}
