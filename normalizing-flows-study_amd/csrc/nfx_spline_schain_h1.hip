// Streaming spline chain instances, HT = 1 (H <= 32): nfx_spline_schain_kernel.h.
#include "nfx_spline_schain_kernel.h"

namespace nfx {

template <int K, int NW>
static spline_schain_t pick_kw(int dir, bool logp) {
    if (dir > 0) return spline_schain_kernel<1, K, 1, false, NW>;
    return logp ? spline_schain_kernel<1, K, -1, true, NW> : spline_schain_kernel<1, K, -1, false, NW>;
}

template <int K>
static spline_schain_t pick_k(int dir, bool logp, bool small) {
    return small ? pick_kw<K, kSplineSchainWavesSmall>(dir, logp) : pick_kw<K, kSplineSchainWaves>(dir, logp);
}

template <>
spline_schain_t spline_schain_pick_ht<1>(int K, int dir, bool logp, bool small) {
    switch (K) {
        case 2: return pick_k<2>(dir, logp, small);
        case 3: return pick_k<3>(dir, logp, small);
        case 4: return pick_k<4>(dir, logp, small);
        case 5: return pick_k<5>(dir, logp, small);
        case 6: return pick_k<6>(dir, logp, small);
        case 7: return pick_k<7>(dir, logp, small);
        case 8: return pick_k<8>(dir, logp, small);
        case 9: return pick_k<9>(dir, logp, small);
        case 10: return pick_k<10>(dir, logp, small);
        case 11: return pick_k<11>(dir, logp, small);
        default: return nullptr;
    }
}

}  // namespace nfx
