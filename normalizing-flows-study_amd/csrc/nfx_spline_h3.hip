// Explicit instantiations of the spline-coupling kernel for hidden tiles HT = 3
// (K = 2..11, both directions; one translation unit per HT for a parallel build).
#include "nfx_spline_kernel.h"

namespace nfx {

template <int K>
static spline_kernel_t pick_dir_3(int dir) {
    return dir < 0 ? spline_coupling_kernel<3, K, -1> : spline_coupling_kernel<3, K, 1>;
}

template <>
spline_kernel_t spline_pick_ht<3>(int K, int dir) {
    switch (K) {
        case 2: return pick_dir_3<2>(dir);
        case 3: return pick_dir_3<3>(dir);
        case 4: return pick_dir_3<4>(dir);
        case 5: return pick_dir_3<5>(dir);
        case 6: return pick_dir_3<6>(dir);
        case 7: return pick_dir_3<7>(dir);
        case 8: return pick_dir_3<8>(dir);
        case 9: return pick_dir_3<9>(dir);
        case 10: return pick_dir_3<10>(dir);
        case 11: return pick_dir_3<11>(dir);
        default: return nullptr;
    }
}

}  // namespace nfx
