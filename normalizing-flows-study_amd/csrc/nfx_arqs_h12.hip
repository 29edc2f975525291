// Explicit instantiations of the ARQS kernel (nfx_arqs_kernel.h) for HT = 1 and 2, K = 2..11.
#include "nfx_arqs_kernel.h"

namespace nfx {

template <int K>
static arqs_kernel_t arqs_dir_1(int inverse) {
    return inverse ? arqs_kernel<1, K, true> : arqs_kernel<1, K, false>;
}

template <>
arqs_kernel_t arqs_pick_ht<1>(int K, int inverse) {
    switch (K) {
        case 2: return arqs_dir_1<2>(inverse);
        case 3: return arqs_dir_1<3>(inverse);
        case 4: return arqs_dir_1<4>(inverse);
        case 5: return arqs_dir_1<5>(inverse);
        case 6: return arqs_dir_1<6>(inverse);
        case 7: return arqs_dir_1<7>(inverse);
        case 8: return arqs_dir_1<8>(inverse);
        case 9: return arqs_dir_1<9>(inverse);
        case 10: return arqs_dir_1<10>(inverse);
        case 11: return arqs_dir_1<11>(inverse);
        default: return nullptr;
    }
}

template <int K>
static arqs_kernel_t arqs_dir_2(int inverse) {
    return inverse ? arqs_kernel<2, K, true> : arqs_kernel<2, K, false>;
}

template <>
arqs_kernel_t arqs_pick_ht<2>(int K, int inverse) {
    switch (K) {
        case 2: return arqs_dir_2<2>(inverse);
        case 3: return arqs_dir_2<3>(inverse);
        case 4: return arqs_dir_2<4>(inverse);
        case 5: return arqs_dir_2<5>(inverse);
        case 6: return arqs_dir_2<6>(inverse);
        case 7: return arqs_dir_2<7>(inverse);
        case 8: return arqs_dir_2<8>(inverse);
        case 9: return arqs_dir_2<9>(inverse);
        case 10: return arqs_dir_2<10>(inverse);
        case 11: return arqs_dir_2<11>(inverse);
        default: return nullptr;
    }
}

}  // namespace nfx
