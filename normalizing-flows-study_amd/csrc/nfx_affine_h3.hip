// Explicit instantiations of the affine-coupling kernel for hidden tiles HT = 3
// (one translation unit per HT so the build compiles them in parallel).
#include "nfx_affine_kernel.h"

namespace nfx {

template <int HT, int D>
static affine_kernel_t pick_dir(int dir) {
    return dir < 0 ? affine_coupling_kernel<HT, D, -1> : affine_coupling_kernel<HT, D, 1>;
}

template <>
affine_kernel_t affine_pick_ht<3>(int d, int dir) {
    switch (d) {
        case 1: return pick_dir<3, 1>(dir);
        case 2: return pick_dir<3, 2>(dir);
        case 3: return pick_dir<3, 3>(dir);
        case 4: return pick_dir<3, 4>(dir);
        case 5: return pick_dir<3, 5>(dir);
        case 6: return pick_dir<3, 6>(dir);
        case 7: return pick_dir<3, 7>(dir);
        case 8: return pick_dir<3, 8>(dir);
        default: return nullptr;
    }
}

}  // namespace nfx
