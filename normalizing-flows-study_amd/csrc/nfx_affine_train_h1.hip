// Explicit instantiations of the train-mode affine-coupling kernels for hidden tiles HT = 1
// (padded d = 2, 4, 8; the five passes of nfx_affine_train.hip). One TU per HT for a parallel build.
#include "nfx_affine_train_kernel.h"

namespace nfx {

template <int D>
static affine_train_kernel_t pick_1(int stage) {
    switch (stage) {
        case TS_STATS1: return affine_train_kernel<1, D, TS_STATS1>;
        case TS_STATS2: return affine_train_kernel<1, D, TS_STATS2>;
        case TS_BWD1: return affine_train_kernel<1, D, TS_BWD1>;
        case TS_BWD2: return affine_train_kernel<1, D, TS_BWD2>;
        case TS_BWD3: return affine_train_kernel<1, D, TS_BWD3>;
        case TS_BWD1K: return affine_train_kernel<1, D, TS_BWD1K>;
        case TS_BWD2K: return affine_train_kernel<1, D, TS_BWD2K>;
        case TS_OUTK: return affine_train_kernel<1, D, TS_OUTK>;
        default: return nullptr;
    }
}

template <>
affine_train_kernel_t affine_train_pick_ht<1>(int D, int stage) {
    switch (D) {
        case 2: return pick_1<2>(stage);
        case 4: return pick_1<4>(stage);
        case 8: return pick_1<8>(stage);
        default: return nullptr;
    }
}

}  // namespace nfx
