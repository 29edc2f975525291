// Instantiations of the parallel MADE-affine kernel (MAF.inverse / IAF.forward):
// hidden tiles HT = 1..4, weights LDS-resident or L2-streamed.
#include "nfx_made_kernel.h"
#include "nfx_made_wide_kernel.h"

namespace nfx {

template <int HT, bool WLDS>
static made_par_kernel_t par_var(int variant) {
    return variant == NFX_MAF_INVERSE ? made_parallel_kernel<HT, WLDS, NFX_MAF_INVERSE>
                                      : made_parallel_kernel<HT, WLDS, NFX_IAF_FORWARD>;
}

template <int HT>
made_par_kernel_t made_pick_ht(bool wlds, int variant) {
    return wlds ? par_var<HT, true>(variant) : par_var<HT, false>(variant);
}
template made_par_kernel_t made_pick_ht<1>(bool, int);
template made_par_kernel_t made_pick_ht<2>(bool, int);
template made_par_kernel_t made_pick_ht<3>(bool, int);
template made_par_kernel_t made_pick_ht<4>(bool, int);

template <int HT, bool WLDS>
static made_par_kernel_t tile_var(int variant, bool logp) {
    if (variant != NFX_MAF_INVERSE) return made_tile_kernel<HT, WLDS, NFX_IAF_FORWARD, false>;
    return logp ? made_tile_kernel<HT, WLDS, NFX_MAF_INVERSE, true> : made_tile_kernel<HT, WLDS, NFX_MAF_INVERSE, false>;
}

template <int HT>
made_par_kernel_t made_tile_pick_ht(bool wlds, int variant, bool logp) {
    return wlds ? tile_var<HT, true>(variant, logp) : tile_var<HT, false>(variant, logp);
}
template made_par_kernel_t made_tile_pick_ht<1>(bool, int, bool);
template made_par_kernel_t made_tile_pick_ht<2>(bool, int, bool);
template made_par_kernel_t made_tile_pick_ht<3>(bool, int, bool);
template made_par_kernel_t made_tile_pick_ht<4>(bool, int, bool);

template <int HT, int NW>
static made_par_kernel_t made_wide_pick_nw(int variant, bool logp) {
    if (variant != NFX_MAF_INVERSE) return made_wide_kernel<HT, NFX_IAF_FORWARD, false, NW>;
    return logp ? made_wide_kernel<HT, NFX_MAF_INVERSE, true, NW> : made_wide_kernel<HT, NFX_MAF_INVERSE, false, NW>;
}
template <int HT>
made_par_kernel_t made_wide_pick_ht(int variant, bool logp, int nw) {
    return nw == 4 ? made_wide_pick_nw<HT, 4>(variant, logp) : made_wide_pick_nw<HT, 8>(variant, logp);
}
template made_par_kernel_t made_wide_pick_ht<1>(int, bool, int);
template made_par_kernel_t made_wide_pick_ht<2>(int, bool, int);

}  // namespace nfx
