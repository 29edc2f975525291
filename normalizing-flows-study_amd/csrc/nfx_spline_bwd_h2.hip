// Explicit instantiations of the spline-coupling backward kernel for hidden tiles HT = 2
// (K = 2..11 bins, both directions). One TU per HT for a parallel build.
#include "nfx_spline_bwd_kernel.h"

namespace nfx {

template <int K>
static spline_bwd_kernel_t pick_k2(int inv) {
    constexpr int NTM = spline_bwd_ntmax(2);
    return inv ? spline_bwd_kernel<2, K, NTM, true> : spline_bwd_kernel<2, K, NTM, false>;
}

template <>
spline_bwd_kernel_t spline_bwd_pick_ht<2>(int K, int inv) {
    switch (K) {
        case 2: return pick_k2<2>(inv);
        case 3: return pick_k2<3>(inv);
        case 4: return pick_k2<4>(inv);
        case 5: return pick_k2<5>(inv);
        case 6: return pick_k2<6>(inv);
        case 7: return pick_k2<7>(inv);
        case 8: return pick_k2<8>(inv);
        case 9: return pick_k2<9>(inv);
        case 10: return pick_k2<10>(inv);
        case 11: return pick_k2<11>(inv);
        default: return nullptr;
    }
}

}  // namespace nfx
