// made_seqp_kernel (nfx_made_seqp_kernel.h): its pack-time images and chunk schedule, the
// instantiations (S = ceil(d / 64) slots, 1..16) and the launcher used by nfx_made.hip for
// MAF.forward / IAF.inverse with H <= 64, d <= 1024.
#include "nfx_made_seqp_kernel.h"

namespace nfx {

// The push images, from the unit-order copies and the degree tables made_live_kernel wrote
// (s_deg: [unit degree | degrees by rank | unit by rank]). Units by completion rank.
template <int HT>
__global__ __launch_bounds__(256) void made_seqp_image_kernel(float* __restrict__ packed, int d, int H) {
    constexpr int Hp = 32 * HT;
    const MadeLayout L = made_layout(d, HT);
    const int S = L.ps;
    const float* P = packed;
    const float* ordD = P + L.s_deg + Hp;
    const float* ordU = P + L.s_deg + 2 * Hp;
    const int tid = blockIdx.x * 256 + threadIdx.x, nth = gridDim.x * 256;
    const int S2 = (S + 1) / 2, S4 = (S + 3) / 4;
    // pw4 [g][j][l][4]: unit g's (mu, alpha) output weights for steps 64 s + l, s = 2j, 2j + 1
    for (int e = tid; e < Hp * S2 * 256; e += nth) {
        const int cc = e & 3, l = (e >> 2) & 63, j = (e >> 8) % S2, g = (e >> 8) / S2;
        const int sl = 2 * j + (cc >> 1), h = cc & 1, i = 64 * sl + l;
        packed[L.pw4 + e] = (sl < S && i < d) ? P[L.s_w4 + (size_t)(h * d + i) * Hp + (int)ordU[g]] : 0.f;
    }
    // pw1 [g][j][l][4]: unit g's layer-1 weights of inputs 64 s + l, s = 4j .. 4j + 3 (masked)
    for (int e = tid; e < Hp * S4 * 256; e += nth) {
        const int cc = e & 3, l = (e >> 2) & 63, j = (e >> 8) % S4, g = (e >> 8) / S4;
        const int sl = 4 * j + cc, i = 64 * sl + l;
        packed[L.pw1 + e] = (sl < S && i < d) ? P[L.s_w1t + (size_t)i * Hp + (int)ordU[g]] : 0.f;
    }
    // pb4 [s][l][2]
    for (int e = tid; e < S * 128; e += nth) {
        const int h = e & 1, i = e >> 1;
        packed[L.pb4 + e] = i < d ? P[L.s_b4 + h * d + i] : 0.f;
    }
    // pw23 [g][p][2] = (W2, W3)[rank p][rank g]
    for (int e = tid; e < 2 * Hp * Hp; e += nth) {
        const int h = e & 1, p = (e >> 1) % Hp, g = (e >> 1) / Hp, a = (int)ordU[p], b = (int)ordU[g];
        packed[L.pw23 + e] = P[(h ? L.s_w3 : L.s_w2) + a * Hp + b];
    }
    for (int p = tid; p < Hp; p += nth) {
        const int a = (int)ordU[p];
        packed[L.ptb + p] = P[L.s_b1 + a];
        packed[L.ptb + Hp + p] = P[L.s_b2 + a];
        packed[L.ptb + 2 * Hp + p] = P[L.s_b3 + a];
        packed[L.ptb + 3 * Hp + p] = ordD[p];
    }
}

// The chunk schedule (one lane, serially). A chunk ends with the completion of the next unit
// (the step of its degree) when that falls in its slot, or in the next slot short of that slot's
// last step and of the last step (a crossing chunk: the tail of slot K + the head of slot K + 1);
// otherwise it ends with its slot (or the last step) and completes nothing. Entry layout and
// flags: nfx_made_seqp_kernel.h. Runs after made_seqp_image_kernel (reads its tables).
template <int HT>
__global__ __launch_bounds__(64) void made_seqp_chunk_kernel(float* __restrict__ packed, int d, int H) {
    constexpr int Hp = 32 * HT;
    const MadeLayout L = made_layout(d, HT);
    __shared__ int deg[Hp], gend[Hp];
    __shared__ float b1[Hp], wd2[Hp], wd3[Hp];
    const float* P = packed;
    for (int p = threadIdx.x; p < Hp; p += 64) {
        deg[p] = p < H ? (int)P[L.ptb + 3 * Hp + p] : 0x7FFFFFFF;
        b1[p] = P[L.ptb + p];
        wd2[p] = P[L.pw23 + 2 * (p * Hp + p)];
        wd3[p] = P[L.pw23 + 2 * (p * Hp + p) + 1];
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int p = 0; p < Hp; ++p) {
        int q = p + 1;
        while (q < H && deg[q] == deg[p]) ++q;
        gend[p] = q;
    }
    auto bits = [](int lo, int hi) -> uint64_t {  // lanes lo..hi (inclusive) of a slot
        const int n = hi - lo + 1;
        return (n >= 64 ? ~0ull : ((1ull << n) - 1ull)) << lo;
    };
    uint32_t* tab = reinterpret_cast<uint32_t*>(packed + L.ptab);
    const int cap = seqp_max_chunks(d, Hp) - 1;
    int k = 0;
    const int S2 = (L.ps + 1) / 2, S4 = (L.ps + 3) / 4;
    // one entry: masks, flags, units g / u, the three scalars, which layers' results count
    auto emit = [&](uint64_t m, int n2, uint32_t fl, int g, int u, float eb1, float ew2, float ew3, bool l1,
                    bool l2, bool l3) {
        if (k >= cap) return;  // (cannot happen: cap bounds the schedule)
        uint32_t* en = tab + 16 * k;
        g = g < Hp ? g : Hp - 1;
        u = u < Hp ? u : Hp - 1;
        en[0] = (uint32_t)m;
        en[1] = (uint32_t)(m >> 32);
        en[2] = en[3] = l1 ? 0xFFFFFFFFu : 0u;
        en[4] = fl | (uint32_t)g << 8 | (uint32_t)n2 << 16;
        en[5] = (uint32_t)(4 * (L.pw4 + g * S2 * 256));
        en[6] = (uint32_t)(4 * (L.pw1 + u * S4 * 256));
        en[7] = (uint32_t)(4 * (L.pw23 + u * Hp * 2));
        en[8] = __float_as_uint(eb1);
        en[9] = __float_as_uint(ew2);
        en[10] = en[11] = l2 ? 0xFFFFFFFFu : 0u;
        en[12] = en[13] = l3 ? 0xFFFFFFFFu : 0u;
        en[14] = __float_as_uint(ew3);
        en[15] = 0u;
        ++k;
    };
    int gi = 0, i = 0;
    while (i < d && k < cap) {
        const int nd = gi < H ? deg[gi] : 0x7FFFFFFF;
        const int slast = i | 63;
        int e;
        uint64_t m = 0;
        int n2 = 0;
        bool completes = false, cross = false;
        if (nd < i) {  // a unit of degree < 0 (no inputs): completes before step 0, empty chunk
            e = i - 1;
            completes = true;
        } else if (nd <= slast && nd <= d - 1) {
            e = nd;
            m = bits(i & 63, nd & 63);
            completes = true;
        } else if (nd > slast && nd < slast + 64 && nd < d - 1) {
            e = nd;
            m = bits(i & 63, 63);
            n2 = (nd & 63) + 1;
            completes = cross = true;
        } else {
            e = slast < d - 1 ? slast : d - 1;
            m = bits(i & 63, e & 63);
        }
        const bool slot_end = cross || (m != 0 && (e == slast || e == d - 1));
        uint32_t fl = (slot_end ? kSpSlotEnd : 0u) | (cross ? kSpCross : 0u);
        const int q = completes ? gend[gi] : gi;
        // (b2, b3 start the running sums; the entries carry b1 and the diagonal weights)
        if (!completes) {
            emit(m, n2, fl, gi, gi, 0.f, 0.f, 0.f, false, false, false);
        } else if (q == gi + 1) {
            emit(m, n2, fl, gi, q, b1[gi], wd2[gi], wd3[gi], true, true, true);
        } else if (e == d - 1) {
            // a group at the last step feeds no later step: nothing to complete
            emit(m, n2, fl, gi, q, 0.f, 0.f, 0.f, false, false, false);
        } else {
            // group gi..q-1: layer 1 of gi with the steps, then the empty chunks (their units'
            // layer-2 / layer-3 values are the running sums alone: diagonal weight 0)
            emit(m, n2, fl, gi, gi + 1, b1[gi], 0.f, 0.f, true, false, false);
            for (int p = gi + 1; p < q; ++p) emit(0, 0, 0, p, p + 1 < q ? p + 1 : gi, b1[p], 0.f, 0.f, true, false, false);
            for (int p = gi; p < q; ++p) emit(0, 0, 0, p, p + 1 < q ? p + 1 : gi, 0.f, 0.f, 0.f, false, true, false);
            for (int p = gi; p < q; ++p) emit(0, 0, 0, p, p + 1 < q ? gi : q, 0.f, 0.f, 0.f, false, false, true);
        }
        if (completes) gi = q;
        i = e + 1;
    }
    // sentinels up to the table's end: empty slot-ending chunks with valid offsets, so that a
    // wave can never run past the table (the kernel clamps its entry index to the last one)
    for (; k <= cap; ++k) {
        uint32_t* en = tab + 16 * k;
        for (int j = 0; j < 16; ++j) en[j] = 0u;
        en[4] = kSpSlotEnd;
        en[5] = (uint32_t)(4 * L.pw4);
        en[6] = (uint32_t)(4 * L.pw1);
        en[7] = (uint32_t)(4 * L.pw23);
    }
}

int made_pack_seqp(int d, int H, float* packed, hipStream_t s) {
    const int HT = (H + 31) / 32;
    if (seqp_slots(d, HT) == 0) return NFX_OK;
    if (HT == 1) made_seqp_image_kernel<1><<<64, 256, 0, s>>>(packed, d, H);
    else made_seqp_image_kernel<2><<<64, 256, 0, s>>>(packed, d, H);
    int rc = check_launch("made_seqp_image_kernel");
    if (rc) return rc;
    if (HT == 1) made_seqp_chunk_kernel<1><<<1, 64, 0, s>>>(packed, d, H);
    else made_seqp_chunk_kernel<2><<<1, 64, 0, s>>>(packed, d, H);
    return check_launch("made_seqp_chunk_kernel");
}

// instantiation shards (nfx_made_seqp_i*.hip): slots S in [S0, S0 + 3]
made_seqp_kernel_t made_seqp_pick_1(int HT, int S, int variant, bool logp);
made_seqp_kernel_t made_seqp_pick_5(int HT, int S, int variant, bool logp);
made_seqp_kernel_t made_seqp_pick_9(int HT, int S, int variant, bool logp);
made_seqp_kernel_t made_seqp_pick_13(int HT, int S, int variant, bool logp);

static made_seqp_kernel_t seqp_pick(int HT, int S, int variant, bool logp) {
    if (S >= 1 && S <= 4) return made_seqp_pick_1(HT, S, variant, logp);
    if (S >= 5 && S <= 8) return made_seqp_pick_5(HT, S, variant, logp);
    if (S >= 9 && S <= 12) return made_seqp_pick_9(HT, S, variant, logp);
    if (S >= 13 && S <= 16) return made_seqp_pick_13(HT, S, variant, logp);
    return nullptr;
}

int made_seqp_launch(const float* packed, const float* in, float* out, float* log_det, int64_t B, int d, int H,
                     int variant, int accumulate, float* logp, double* partials, double* sums, bool fused,
                     hipStream_t s) {
    const int HT = (H + 31) / 32;
    const int S = seqp_slots(d, HT);
    made_seqp_kernel_t k = seqp_pick(HT, S, variant, fused);
    if (!k) return set_error(NFX_EUNSUPPORTED, "made_seqp: d=%d H=%d outside H <= 64, d <= 1024", d, H);
    const size_t lds = (size_t)seqp_lds_floats(S) * sizeof(float);
    int rc = prepare_lds((const void*)k, lds);
    if (rc) return rc;
    int64_t grid = (B + kSeqpWaves - 1) / kSeqpWaves;
    const int64_t res = resident_grid((const void*)k, kSeqpThreads, lds, grid);
    if (grid > res) grid = res;
    if (grid > kMaxPartials) grid = kMaxPartials;
    k<<<(unsigned)grid, kSeqpThreads, lds, s>>>(packed, in, out, log_det, B, d, H, accumulate, logp, partials, sums,
                                                gauss_const(d));
    return check_launch("made_seqp_kernel");
}

}  // namespace nfx
