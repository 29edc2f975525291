// Explicit instantiations of the wide train-mode affine-coupling kernels for hidden tiles
// HT = 3 (padded d = 2, 4, 8; the six passes of nfx_affine_trainw_kernel.h). One TU per HT.
#include "nfx_affine_trainw_kernel.h"

namespace nfx {

template <int D>
static affine_trainw_kernel_t pickw_3(int stage) {
    switch (stage) {
        case TW_STATS1: return affine_trainw_kernel<3, D, TW_STATS1>;
        case TW_STATS2: return affine_trainw_kernel<3, D, TW_STATS2>;
        case TW_OUT: return affine_trainw_kernel<3, D, TW_OUT>;
        case TW_BWD1: return affine_trainw_kernel<3, D, TW_BWD1>;
        case TW_BWD2: return affine_trainw_kernel<3, D, TW_BWD2>;
        case TW_BWD3: return affine_trainw_kernel<3, D, TW_BWD3>;
        default: return nullptr;
    }
}

template <>
affine_trainw_kernel_t affine_trainw_pick_ht<3>(int D, int stage) {
    switch (D) {
        case 2: return pickw_3<2>(stage);
        case 4: return pickw_3<4>(stage);
        case 8: return pickw_3<8>(stage);
        default: return nullptr;
    }
}

}  // namespace nfx
