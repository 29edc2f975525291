// Explicit instantiations of the spline-coupling kernel for hidden tiles HT = 3, runtime d <= 8
// (K = 2..11, both directions + the fused-log_prob inverse; one TU per (HT, d class) for a
// parallel build).
#include "nfx_spline_kernel.h"

namespace nfx {

template <int K>
static spline_kernel_t pick_3_0(int dir, bool logp) {
    if (dir > 0) return spline_coupling_kernel<3, K, 1, false, 0>;
    return logp ? spline_coupling_kernel<3, K, -1, true, 0> : spline_coupling_kernel<3, K, -1, false, 0>;
}

template <>
spline_kernel_t spline_pick_ht<3, 0>(int K, int dir, bool logp) {
    switch (K) {
        case 2: return pick_3_0<2>(dir, logp);
        case 3: return pick_3_0<3>(dir, logp);
        case 4: return pick_3_0<4>(dir, logp);
        case 5: return pick_3_0<5>(dir, logp);
        case 6: return pick_3_0<6>(dir, logp);
        case 7: return pick_3_0<7>(dir, logp);
        case 8: return pick_3_0<8>(dir, logp);
        case 9: return pick_3_0<9>(dir, logp);
        case 10: return pick_3_0<10>(dir, logp);
        case 11: return pick_3_0<11>(dir, logp);
        default: return nullptr;
    }
}

}  // namespace nfx
