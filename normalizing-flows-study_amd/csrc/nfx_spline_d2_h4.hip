// Explicit instantiations of the spline-coupling kernel for hidden tiles HT = 4, d = 2 (compile-time)
// (K = 2..11, both directions + the fused-log_prob inverse; one TU per (HT, d class) for a
// parallel build).
#include "nfx_spline_kernel.h"

namespace nfx {

template <int K>
static spline_kernel_t pick_4_2(int dir, bool logp) {
    if (dir > 0) return spline_coupling_kernel<4, K, 1, false, 2>;
    return logp ? spline_coupling_kernel<4, K, -1, true, 2> : spline_coupling_kernel<4, K, -1, false, 2>;
}

template <>
spline_kernel_t spline_pick_ht<4, 2>(int K, int dir, bool logp) {
    switch (K) {
        case 2: return pick_4_2<2>(dir, logp);
        case 3: return pick_4_2<3>(dir, logp);
        case 4: return pick_4_2<4>(dir, logp);
        case 5: return pick_4_2<5>(dir, logp);
        case 6: return pick_4_2<6>(dir, logp);
        case 7: return pick_4_2<7>(dir, logp);
        case 8: return pick_4_2<8>(dir, logp);
        case 9: return pick_4_2<9>(dir, logp);
        case 10: return pick_4_2<10>(dir, logp);
        case 11: return pick_4_2<11>(dir, logp);
        default: return nullptr;
    }
}

}  // namespace nfx
