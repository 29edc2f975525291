// Streaming spline chain instances, HT = 1 (H <= 32): nfx_spline_schain_kernel.h.
#include "nfx_spline_schain_kernel.h"

namespace nfx {

template <int K>
static spline_schain_t pick_k(int dir, bool logp) {
    if (dir > 0) return spline_schain_kernel<1, K, 1, false, kSplineSchainWaves>;
    return logp ? spline_schain_kernel<1, K, -1, true, kSplineSchainWaves> : spline_schain_kernel<1, K, -1, false, kSplineSchainWaves>;
}

template <>
spline_schain_t spline_schain_pick_ht<1>(int K, int dir, bool logp) {
    switch (K) {
        case 2: return pick_k<2>(dir, logp);
        case 3: return pick_k<3>(dir, logp);
        case 4: return pick_k<4>(dir, logp);
        case 5: return pick_k<5>(dir, logp);
        case 6: return pick_k<6>(dir, logp);
        case 7: return pick_k<7>(dir, logp);
        case 8: return pick_k<8>(dir, logp);
        case 9: return pick_k<9>(dir, logp);
        case 10: return pick_k<10>(dir, logp);
        case 11: return pick_k<11>(dir, logp);
        default: return nullptr;
    }
}

}  // namespace nfx
