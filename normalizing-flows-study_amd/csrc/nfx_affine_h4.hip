// Explicit instantiations of the affine-coupling kernel for hidden tiles HT = 4
// (d = 1..8, both directions, + the fused-log_prob inverse; one TU per HT for a parallel build).
#include "nfx_affine_kernel.h"

namespace nfx {

template <int D>
static affine_kernel_t pick_4(int dir, bool logp) {
    if (dir > 0) return affine_coupling_kernel<4, D, 1, false>;
    return logp ? affine_coupling_kernel<4, D, -1, true> : affine_coupling_kernel<4, D, -1, false>;
}

template <>
affine_kernel_t affine_pick_ht<4>(int d, int dir, bool logp) {
    switch (d) {
        case 1: return pick_4<1>(dir, logp);
        case 2: return pick_4<2>(dir, logp);
        case 3: return pick_4<3>(dir, logp);
        case 4: return pick_4<4>(dir, logp);
        case 5: return pick_4<5>(dir, logp);
        case 6: return pick_4<6>(dir, logp);
        case 7: return pick_4<7>(dir, logp);
        case 8: return pick_4<8>(dir, logp);
        default: return nullptr;
    }
}

}  // namespace nfx
