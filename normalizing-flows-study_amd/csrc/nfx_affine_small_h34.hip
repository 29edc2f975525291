// Explicit instantiations of the small-batch affine kernel (nfx_affine_small_kernel.h) for
// HT = 3 and 4 (d = 1..8, both directions, + the fused-log_prob inverse).
#include "nfx_affine_small_kernel.h"

namespace nfx {

template <int D>
static affine_kernel_t small_pick_3(int dir, bool logp) {
    if (dir > 0) return affine_small_kernel<3, D, 1, false>;
    return logp ? affine_small_kernel<3, D, -1, true> : affine_small_kernel<3, D, -1, false>;
}

template <>
affine_kernel_t affine_small_pick_ht<3>(int d, int dir, bool logp) {
    switch (d) {
        case 1: return small_pick_3<1>(dir, logp);
        case 2: return small_pick_3<2>(dir, logp);
        case 3: return small_pick_3<3>(dir, logp);
        case 4: return small_pick_3<4>(dir, logp);
        case 5: return small_pick_3<5>(dir, logp);
        case 6: return small_pick_3<6>(dir, logp);
        case 7: return small_pick_3<7>(dir, logp);
        case 8: return small_pick_3<8>(dir, logp);
        default: return nullptr;
    }
}

template <int D>
static affine_kernel_t small_pick_4(int dir, bool logp) {
    if (dir > 0) return affine_small_kernel<4, D, 1, false>;
    return logp ? affine_small_kernel<4, D, -1, true> : affine_small_kernel<4, D, -1, false>;
}

template <>
affine_kernel_t affine_small_pick_ht<4>(int d, int dir, bool logp) {
    switch (d) {
        case 1: return small_pick_4<1>(dir, logp);
        case 2: return small_pick_4<2>(dir, logp);
        case 3: return small_pick_4<3>(dir, logp);
        case 4: return small_pick_4<4>(dir, logp);
        case 5: return small_pick_4<5>(dir, logp);
        case 6: return small_pick_4<6>(dir, logp);
        case 7: return small_pick_4<7>(dir, logp);
        case 8: return small_pick_4<8>(dir, logp);
        default: return nullptr;
    }
}

}  // namespace nfx
