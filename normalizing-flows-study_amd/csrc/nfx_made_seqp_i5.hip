// Instantiations of made_seqp_kernel (nfx_made_seqp_kernel.h) for S = 5 .. 8 slots (a shard of
// nfx_made_seqp.hip's dispatch, split for parallel compilation).
#include "nfx_made_seqp_kernel.h"

namespace nfx {

template <int HT, int S>
static made_seqp_kernel_t pick_v(int variant, bool logp) {
    if (variant == NFX_MAF_FORWARD) return made_seqp_kernel<HT, NFX_MAF_FORWARD, false, S>;
    return logp ? made_seqp_kernel<HT, NFX_IAF_INVERSE, true, S> : made_seqp_kernel<HT, NFX_IAF_INVERSE, false, S>;
}

template <int HT>
static made_seqp_kernel_t pick_s(int S, int variant, bool logp) {
    switch (S) {
        case 5: return pick_v<HT, 5>(variant, logp);
        case 6: return pick_v<HT, 6>(variant, logp);
        case 7: return pick_v<HT, 7>(variant, logp);
        case 8: return pick_v<HT, 8>(variant, logp);
        default: return nullptr;
    }
}

made_seqp_kernel_t made_seqp_pick_5(int HT, int S, int variant, bool logp) {
    return HT == 1 ? pick_s<1>(S, variant, logp) : pick_s<2>(S, variant, logp);
}

}  // namespace nfx
