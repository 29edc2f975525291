// Explicit instantiations of the spline-coupling backward kernel for hidden tiles HT = 1
// (K = 2..11 bins, both directions). One TU per HT for a parallel build.
#include "nfx_spline_bwd_kernel.h"

namespace nfx {

template <int K>
static spline_bwd_kernel_t pick_k1(int inv) {
    constexpr int NTM = spline_bwd_ntmax(1);
    return inv ? spline_bwd_kernel<1, K, NTM, true> : spline_bwd_kernel<1, K, NTM, false>;
}

template <>
spline_bwd_kernel_t spline_bwd_pick_ht<1>(int K, int inv) {
    switch (K) {
        case 2: return pick_k1<2>(inv);
        case 3: return pick_k1<3>(inv);
        case 4: return pick_k1<4>(inv);
        case 5: return pick_k1<5>(inv);
        case 6: return pick_k1<6>(inv);
        case 7: return pick_k1<7>(inv);
        case 8: return pick_k1<8>(inv);
        case 9: return pick_k1<9>(inv);
        case 10: return pick_k1<10>(inv);
        case 11: return pick_k1<11>(inv);
        default: return nullptr;
    }
}

}  // namespace nfx
