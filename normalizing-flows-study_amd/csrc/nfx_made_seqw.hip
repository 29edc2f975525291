// Instantiations of the wave-per-sample sequential MADE kernel (nfx_made_seqw_kernel.h) and its
// launcher, used by nfx_made.hip for MAF.forward / IAF.inverse with H <= 64.
#include "nfx_made_seqw_kernel.h"

namespace nfx {

template <int HT, int NWV>
static made_seqw_kernel_t seqw_pick_nwv(int variant, bool logp) {
    if (variant == NFX_MAF_FORWARD) return made_seqw_kernel<HT, NFX_MAF_FORWARD, false, NWV>;
    return logp ? made_seqw_kernel<HT, NFX_IAF_INVERSE, true, NWV> : made_seqw_kernel<HT, NFX_IAF_INVERSE, false, NWV>;
}

template <int HT>
static made_seqw_kernel_t seqw_pick(int variant, bool logp, int nwv) {
    switch (nwv) {
        case 4: return seqw_pick_nwv<HT, 4>(variant, logp);
        default: return seqw_pick_nwv<HT, 8>(variant, logp);
    }
}

// Waves (= samples) per workgroup: 8 once that still gives every CU a workgroup (one fits a CU:
// the two staged 64-step blocks take ~100 KB of LDS), else 4. Not 16: the kernel holds two
// chunks' operands in registers (~150 VGPRs), more than 4 waves per SIMD leave room for.
static int seqw_waves(int64_t B) {
    const int64_t cus = num_cus();
    if ((B + 7) / 8 >= cus) return 8;
    return 4;
}

int made_seqw_launch(const float* packed, const float* in, float* out, float* log_det, int64_t B, int d, int H,
                     int variant, int accumulate, float* logp, double* partials, double* sums, bool fused,
                     int* grid_out, hipStream_t s) {
    const int HT = (H + 31) / 32;
    const int nwv = seqw_waves(B);
    made_seqw_kernel_t k = HT == 1 ? seqw_pick<1>(variant, fused, nwv) : seqw_pick<2>(variant, fused, nwv);
    const size_t lds = (size_t)seqw_lds_floats(32 * HT, nwv) * sizeof(float);
    int rc = prepare_lds((const void*)k, lds);
    if (rc) return rc;
    int64_t grid = (B + nwv - 1) / nwv;
    if (grid > kMaxPartials) grid = kMaxPartials;
    k<<<(unsigned)grid, (nwv + 1) * 64, lds, s>>>(packed, in, out, log_det, B, d, H, accumulate, logp, partials,
                                           sums, gauss_const(d));
    *grid_out = (int)grid;
    return check_launch("made_seqw_kernel");
}

}  // namespace nfx
