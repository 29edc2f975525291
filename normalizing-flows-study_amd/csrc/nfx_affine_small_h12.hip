// Explicit instantiations of the small-batch affine kernel (nfx_affine_small_kernel.h) for
// HT = 1 and 2 (d = 1..8, both directions, + the fused-log_prob inverse).
#include "nfx_affine_small_kernel.h"

namespace nfx {

template <int D>
static affine_kernel_t small_pick_1(int dir, bool logp) {
    if (dir > 0) return affine_small_kernel<1, D, 1, false>;
    return logp ? affine_small_kernel<1, D, -1, true> : affine_small_kernel<1, D, -1, false>;
}

template <>
affine_kernel_t affine_small_pick_ht<1>(int d, int dir, bool logp) {
    switch (d) {
        case 1: return small_pick_1<1>(dir, logp);
        case 2: return small_pick_1<2>(dir, logp);
        case 3: return small_pick_1<3>(dir, logp);
        case 4: return small_pick_1<4>(dir, logp);
        case 5: return small_pick_1<5>(dir, logp);
        case 6: return small_pick_1<6>(dir, logp);
        case 7: return small_pick_1<7>(dir, logp);
        case 8: return small_pick_1<8>(dir, logp);
        default: return nullptr;
    }
}

template <int D>
static affine_kernel_t small_pick_2(int dir, bool logp) {
    if (dir > 0) return affine_small_kernel<2, D, 1, false>;
    return logp ? affine_small_kernel<2, D, -1, true> : affine_small_kernel<2, D, -1, false>;
}

template <>
affine_kernel_t affine_small_pick_ht<2>(int d, int dir, bool logp) {
    switch (d) {
        case 1: return small_pick_2<1>(dir, logp);
        case 2: return small_pick_2<2>(dir, logp);
        case 3: return small_pick_2<3>(dir, logp);
        case 4: return small_pick_2<4>(dir, logp);
        case 5: return small_pick_2<5>(dir, logp);
        case 6: return small_pick_2<6>(dir, logp);
        case 7: return small_pick_2<7>(dir, logp);
        case 8: return small_pick_2<8>(dir, logp);
        default: return nullptr;
    }
}

}  // namespace nfx
