// Explicit instantiations of the ARQS kernel (nfx_arqs_kernel.h) for HT = 3 and 4, K = 2..11.
#include "nfx_arqs_kernel.h"

namespace nfx {

template <int K>
static arqs_kernel_t arqs_dir_3(int inverse) {
    return inverse ? arqs_kernel<3, K, true> : arqs_kernel<3, K, false>;
}

template <>
arqs_kernel_t arqs_pick_ht<3>(int K, int inverse) {
    switch (K) {
        case 2: return arqs_dir_3<2>(inverse);
        case 3: return arqs_dir_3<3>(inverse);
        case 4: return arqs_dir_3<4>(inverse);
        case 5: return arqs_dir_3<5>(inverse);
        case 6: return arqs_dir_3<6>(inverse);
        case 7: return arqs_dir_3<7>(inverse);
        case 8: return arqs_dir_3<8>(inverse);
        case 9: return arqs_dir_3<9>(inverse);
        case 10: return arqs_dir_3<10>(inverse);
        case 11: return arqs_dir_3<11>(inverse);
        default: return nullptr;
    }
}

template <int K>
static arqs_kernel_t arqs_dir_4(int inverse) {
    return inverse ? arqs_kernel<4, K, true> : arqs_kernel<4, K, false>;
}

template <>
arqs_kernel_t arqs_pick_ht<4>(int K, int inverse) {
    switch (K) {
        case 2: return arqs_dir_4<2>(inverse);
        case 3: return arqs_dir_4<3>(inverse);
        case 4: return arqs_dir_4<4>(inverse);
        case 5: return arqs_dir_4<5>(inverse);
        case 6: return arqs_dir_4<6>(inverse);
        case 7: return arqs_dir_4<7>(inverse);
        case 8: return arqs_dir_4<8>(inverse);
        case 9: return arqs_dir_4<9>(inverse);
        case 10: return arqs_dir_4<10>(inverse);
        case 11: return arqs_dir_4<11>(inverse);
        default: return nullptr;
    }
}

}  // namespace nfx
