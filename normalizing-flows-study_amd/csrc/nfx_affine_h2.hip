// Explicit instantiations of the affine-coupling kernel for hidden tiles HT = 2
// (one translation unit per HT so the build compiles them in parallel).
#include "nfx_affine_kernel.h"

namespace nfx {

template <int HT, int D>
static affine_kernel_t pick_dir(int dir) {
    return dir < 0 ? affine_coupling_kernel<HT, D, -1> : affine_coupling_kernel<HT, D, 1>;
}

template <>
affine_kernel_t affine_pick_ht<2>(int d, int dir) {
    switch (d) {
        case 1: return pick_dir<2, 1>(dir);
        case 2: return pick_dir<2, 2>(dir);
        case 3: return pick_dir<2, 3>(dir);
        case 4: return pick_dir<2, 4>(dir);
        case 5: return pick_dir<2, 5>(dir);
        case 6: return pick_dir<2, 6>(dir);
        case 7: return pick_dir<2, 7>(dir);
        case 8: return pick_dir<2, 8>(dir);
        default: return nullptr;
    }
}

}  // namespace nfx
