// Explicit instantiations of the affine-coupling kernel for hidden tiles HT = 1
// (d = 1..8, both directions, + the fused-log_prob inverse; one TU per HT for a parallel build).
#include "nfx_affine_kernel.h"

namespace nfx {

template <int D>
static affine_kernel_t pick_1(int dir, bool logp) {
    if (dir > 0) return affine_coupling_kernel<1, D, 1, false>;
    return logp ? affine_coupling_kernel<1, D, -1, true> : affine_coupling_kernel<1, D, -1, false>;
}

template <>
affine_kernel_t affine_pick_ht<1>(int d, int dir, bool logp) {
    switch (d) {
        case 1: return pick_1<1>(dir, logp);
        case 2: return pick_1<2>(dir, logp);
        case 3: return pick_1<3>(dir, logp);
        case 4: return pick_1<4>(dir, logp);
        case 5: return pick_1<5>(dir, logp);
        case 6: return pick_1<6>(dir, logp);
        case 7: return pick_1<7>(dir, logp);
        case 8: return pick_1<8>(dir, logp);
        default: return nullptr;
    }
}

}  // namespace nfx
