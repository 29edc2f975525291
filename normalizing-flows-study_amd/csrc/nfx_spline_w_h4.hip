// Explicit instantiations of the wide spline-coupling kernel (8 < d <= 64) for hidden tiles
// HT = 4: K = 2..11, both directions + the fused-log_prob inverse (one TU per HT: parallel build).
#include "nfx_spline_kernel.h"

namespace nfx {

template <int K>
static spline_kernel_t wpick_4(int dir, bool logp) {
    if (dir > 0) return spline_wide_kernel<4, K, 1, false>;
    return logp ? spline_wide_kernel<4, K, -1, true> : spline_wide_kernel<4, K, -1, false>;
}

template <>
spline_kernel_t spline_wide_pick_ht<4>(int K, int dir, bool logp) {
    switch (K) {
        case 2: return wpick_4<2>(dir, logp);
        case 3: return wpick_4<3>(dir, logp);
        case 4: return wpick_4<4>(dir, logp);
        case 5: return wpick_4<5>(dir, logp);
        case 6: return wpick_4<6>(dir, logp);
        case 7: return wpick_4<7>(dir, logp);
        case 8: return wpick_4<8>(dir, logp);
        case 9: return wpick_4<9>(dir, logp);
        case 10: return wpick_4<10>(dir, logp);
        case 11: return wpick_4<11>(dir, logp);
        default: return nullptr;
    }
}

}  // namespace nfx
