// A whole chain of affine coupling layers (NormalizingFlowModel / RealNVP / SequentialFlow of
// CouplingLayers, eval mode) in ONE launch, for small and medium batches: the reference's
// sampling throughput runs (RealNVP(2, 10, 128).forward on n = 4,000, plots/_common.py:264-274)
// and the per-GPU shards of a strong-scaled log_prob.
//
// Per layer the arithmetic is exactly affine_small_kernel's (nfx_affine_small_kernel.h: a
// workgroup of 2*HT waves per 32-sample tile, wave = (net, layer-2 output tile), the output-layer
// partials meet in LDS, 32 threads finish the affine map, guards and log-det) — same roundings,
// so the chain equals the per-layer kernels bit for bit. What changes is the loop order: a
// workgroup owns a contiguous set of tiles and carries their rows x [32][D] and running log-det
// in LDS through ALL layers (layer l+1 reads what layer l's epilogue wrote), loading each layer's
// weights once per workgroup. No [B, d] intermediate ever goes to HBM, and a 10-layer chain is
// one launch instead of 10 (each ~8 us at n = 4,000, most of it launch and ramp).
// The log-det accumulates in the reference's order: ld = ((0 + ld_first) + ...) + ld_last (or
// starts from the caller's log-det when accumulate = 1); the last layer of an inverse chain can
// add the fused Gaussian log-density and float64 NLL partials (LOGP), as nfx_*_logprob do.
#include "nfx_chain.h"

namespace nfx {

// SAMPLE (forward chains): the rows are not read from `in` but drawn on the device — z ~ N(0, I)
// from Philox4x32-10 keyed by `seed` at the counter offset rng[0] (base_draw, nfx_chain.h),
// written to `zout` when non-null — and the LAST workgroup to finish advances rng[0] past this
// launch's draws (arrival count in rng[1]), so a replayed graph draws fresh values every time.
template <int HT, int D, int DIR, bool LOGP, bool SAMPLE = false>
__global__ __launch_bounds__(128 * HT) void affine_chain_kernel(NfxChainPacks packs, int nl, const float* __restrict__ in,
                                                                float* __restrict__ out, float* __restrict__ logdet,
                                                                int64_t B, int accumulate, int64_t ntiles, int tpw,
                                                                float* __restrict__ logp, double* __restrict__ partials, double* __restrict__ sums,
                                                                float cgauss, uint64_t seed = 0, uint64_t* rng = nullptr,
                                                                float* __restrict__ zout = nullptr) {
    constexpr AffineLayout L = affine_layout(D, HT);
    constexpr int KS1 = L.KS1;
    constexpr int NB1 = HT * 32;
    constexpr int NTAIL = L.net - L.b2;
    constexpr int NPN = NB1 + NTAIL;
    constexpr int NTHR = 128 * HT;
    __shared__ __attribute__((aligned(16))) float sw[2 * NPN + up4(D)];
    __shared__ float part[2][2][HT][D][32];
    extern __shared__ float st[];  // [tpw][32][D] rows, then [tpw][32] running log-det
    float* sx = st;
    float* sld = st + (size_t)tpw * 32 * D;

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int net = wave / HT, hto = wave % HT;
    const int lane = lane_id(), h = lane >> 5, col = lane & 31;
    const int64_t t0 = (int64_t)blockIdx.x * tpw;
    const int nt = (int)(ntiles - t0 < tpw ? ntiles - t0 : tpw);
    const int64_t r0 = t0 * 32;
    if constexpr (SAMPLE) {
        const uint64_t off = __hip_atomic_load(rng, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int e = threadIdx.x; e < nt * 32; e += NTHR) {
            const int64_t row = r0 + e;
            float z[D];
            base_draw<D>(row, seed, off, z);
#pragma unroll
            for (int j = 0; j < D; ++j) sx[e * D + j] = row < B ? z[j] : 0.f;
            if (zout && row < B) {
#pragma unroll
                for (int j = 0; j < D; ++j) zout[row * D + j] = z[j];
            }
        }
    } else {
        for (int e = threadIdx.x; e < nt * 32 * D; e += NTHR) sx[e] = r0 + e / D < B ? in[r0 * D + e] : 0.f;
    }
    for (int e = threadIdx.x; e < nt * 32; e += NTHR) sld[e] = (accumulate && r0 + e < B) ? logdet[r0 + e] : 0.f;

    for (int li = 0; li < nl; ++li) {
        const float* packed = packs.p[DIR > 0 ? li : nl - 1 - li];
        __syncthreads();  // every reader of the previous layer's sw (and state) is done
        for (int i = threadIdx.x; i < 2 * NPN + up4(D); i += NTHR) {
            float v;
            if (i >= 2 * NPN) {
                v = packed[L.mask + i - 2 * NPN];
            } else {
                const int n2 = i / NPN, o = i - n2 * NPN;
                v = packed[n2 * L.net + (o < NB1 ? L.b1 + o : L.b2 + o - NB1)];
            }
            sw[i] = v;
        }
        const float* P = packed + net * L.net;
        float w1r[HT][KS1];
#pragma unroll
        for (int ht = 0; ht < HT; ++ht)
#pragma unroll
            for (int ks = 0; ks < KS1; ++ks) w1r[ht][ks] = P[L.w1 + (ht * KS1 + ks) * 64 + lane];
        f32x4 w2r[HT][4];
        {
            const f32x4* wg = reinterpret_cast<const f32x4*>(P + L.w2) + lane;
#pragma unroll
            for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                for (int rq = 0; rq < 4; ++rq) w2r[kt][rq] = wg[((hto * HT + kt) * 4 + rq) * 64];
        }
        __syncthreads();
        const float* sb1 = sw + net * NPN;
        const float* sb2 = sb1 + NB1;
        const float* sw3 = sb2 + (L.w3 - L.b2);
        float mkb[KS1];
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks) mkb[ks] = (2 * ks + h < D) ? sw[2 * NPN + 2 * ks + h] : 0.f;
        for (int tt = 0; tt < nt; ++tt) {
            const int buf = tt & 1;
            const float* row = sx + (size_t)(tt * 32 + col) * D;
            float xcur[KS1];
#pragma unroll
            for (int ks = 0; ks < KS1; ++ks) {
                const int k = 2 * ks + h;
                xcur[ks] = k < D ? row[k] : 0.f;
            }
            f32x16 h1[HT];
#pragma unroll
            for (int ht = 0; ht < HT; ++ht) {
                f32x16 a = load_bias16(sb1 + ht * 32, h);
#pragma unroll
                for (int ks = 0; ks < KS1; ++ks) a = mfma32(w1r[ht][ks], xcur[ks] * mkb[ks], a);
#pragma unroll
                for (int r = 0; r < 16; ++r) a[r] = trelu(a[r]);
                h1[ht] = a;
            }
            f32x16 a = load_bias16(sb2 + hto * 32, h);
#pragma unroll
            for (int kt = 0; kt < HT; ++kt)
#pragma unroll
                for (int rq = 0; rq < 4; ++rq)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) a = mfma32(w2r[kt][rq][rr], h1[kt][4 * rq + rr], a);
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const f32x16 w3 = load_bias16(sw3 + (j * HT + hto) * 32, h);
                float p = 0.f;
#pragma unroll
                for (int r = 0; r < 16; ++r) p = fmaf(w3[r], trelu(a[r]), p);
                p = halves_sum(p, p);
                if (lane < 32) part[buf][net][hto][j][col] = p;
            }
            __syncthreads();
            if (wave == 0 && lane < 32) {
#pragma clang fp contract(off)  // separate mul/add roundings, as affine_small_kernel / the reference
                float* rw = sx + (size_t)(tt * 32 + col) * D;
                const float* sb3s = sw + NB1 + (L.b3 - L.b2);
                const float* sb3b = sb3s + NPN;
                float y[D];
                float ld = 0.f;
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    float ps = part[buf][0][0][j][col], pb = part[buf][1][0][j][col];
#pragma unroll
                    for (int ht = 1; ht < HT; ++ht) {
                        ps = ps + part[buf][0][ht][j][col];
                        pb = pb + part[buf][1][ht][j][col];
                    }
                    const float sv = tclamp(ps + sb3s[j], -10.f, 10.f);
                    const float bv = tclamp(pb + sb3b[j], -10.f, 10.f);
                    const float m = sw[2 * NPN + j], om = 1.f - m;
                    const float xj = rw[j];
                    const float xa = xj * m;
                    float tv;
                    if constexpr (DIR < 0) {
                        tv = (xj - bv) * exp_fast(-sv);
                        ld = ld + om * (-sv);
                    } else {
                        tv = xj * exp_fast(sv) + bv;
                        ld = ld + om * sv;
                    }
                    const float v = xa + om * tv;
                    y[j] = nonfinite(v) ? 0.f : v;
                }
#pragma unroll
                for (int j = 0; j < D; ++j) rw[j] = y[j];
                if (nonfinite(ld)) ld = 0.f;
                sld[tt * 32 + col] = sld[tt * 32 + col] + ld;
            }
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < nt * 32 * D; e += NTHR)
        if (r0 + e / D < B) out[r0 * D + e] = sx[e];
    double lpacc = 0.0;
    for (int e = threadIdx.x; e < nt * 32; e += NTHR) {
        const int64_t s = r0 + e;
        if (s >= B) continue;
        const float ldt = sld[e];
        logdet[s] = ldt;
        if constexpr (LOGP) {
            const float* rw = sx + (size_t)e * D;
            float m = gauss_sq0(rw[0]);
#pragma unroll
            for (int j = 1; j < D; ++j) m = gauss_sq(m, rw[j]);
            const float lp = gauss_lp(m, cgauss, ldt);
            logp[s] = lp;
            lpacc += (double)lp;
        }
    }
    if constexpr (LOGP) {
        logp_commit<NTHR>(lpacc, partials, sums, B);
    }
    if constexpr (SAMPLE) {
        // every workgroup read rng[0] in its prologue; the last one to get here moves it on
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            uint64_t* cnt = rng + 1;
            const uint64_t prev = __hip_atomic_fetch_add(cnt, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (prev == (uint64_t)gridDim.x - 1) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                __hip_atomic_store(rng, __hip_atomic_load(rng, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(cnt, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

typedef void (*affine_chain_t)(NfxChainPacks, int, const float*, float*, float*, int64_t, int, int64_t, int, float*,
                               double*, double*, float, uint64_t, uint64_t*, float*);

template <int HT, int D>
static affine_chain_t chain_pick_d(int dir, bool logp) {
    if (dir > 0) return affine_chain_kernel<HT, D, 1, false>;
    return logp ? affine_chain_kernel<HT, D, -1, true> : affine_chain_kernel<HT, D, -1, false>;
}

template <int HT>
static affine_chain_t chain_pick_ht(int d, int dir, bool logp) {
    if (d <= 2) return chain_pick_d<HT, 2>(dir, logp);
    if (d <= 4) return chain_pick_d<HT, 4>(dir, logp);
    return chain_pick_d<HT, 8>(dir, logp);
}

template <int HT>
static affine_chain_t sample_pick_ht(int d) {
    if (d <= 2) return affine_chain_kernel<HT, 2, 1, false, true>;
    if (d <= 4) return affine_chain_kernel<HT, 4, 1, false, true>;
    return affine_chain_kernel<HT, 8, 1, false, true>;
}

static int chain_pad_d(int d) { return d <= 2 ? 2 : (d <= 4 ? 4 : 8); }

// Rows of state one workgroup may carry: tiles * 32 * (D + 1) floats of dynamic LDS <= 64 KiB.
static int64_t chain_max_tpw(int D) { return 65536 / (32 * (D + 1) * 4); }

// Largest batch the small-batch chain fits (min(4 x CUs, kMaxPartials) workgroups of
// chain_max_tpw tiles).
static int64_t small_chain_max_b(int D) {
    const int64_t cap = 4 * (int64_t)num_cus() < (int64_t)kMaxPartials ? 4 * (int64_t)num_cus() : (int64_t)kMaxPartials;
    return cap * chain_max_tpw(D) * 32;
}

bool chain_supported(int64_t B, int d, int H) {
    if (d != 2 && d != 4 && d != 8) return false;
    if (H <= 0 || H > 128 || B < 0) return false;
    const int pol = affine_policy_get();
    const bool want_stream = pol == NFX_AFFINE_STREAMING || (pol == NFX_AFFINE_AUTO && B > kSmallChainMaxB);
    if (want_stream && schain_supported(B, d, H)) return true;
    return B <= small_chain_max_b(d);
}

static int chain_launch(const float* const* packs, int nl, const float* in, float* out, float* log_det, int64_t B,
                        int d, int H, int direction, int accumulate, float* logp, double* sums, void* workspace,
                        hipStream_t s, uint64_t* rng = nullptr, uint64_t seed = 0, float* zout = nullptr) {
    const bool fused = sums != nullptr;
    const bool sample = rng != nullptr;
    if (nl <= 0 || nl > kChainMax) return set_error(NFX_EINVAL, "affine_chain: 1 <= n_layers <= %d (got %d)", kChainMax, nl);
    if (d <= 0 || d > 8 || H <= 0 || H > 128)
        return set_error(NFX_EUNSUPPORTED, "affine_chain: d=%d H=%d outside d<=8, H<=128", d, H);
    if (direction != NFX_FORWARD && direction != NFX_INVERSE)
        return set_error(NFX_EINVAL, "affine_chain: direction must be +1 or -1");
    if (fused && direction != NFX_INVERSE) return set_error(NFX_EINVAL, "affine_chain_logprob: inverse chains only");
    if (B < 0) return set_error(NFX_EINVAL, "affine_chain: B < 0");
    if (B == 0) return fused ? gauss_finish(reinterpret_cast<double*>(workspace), 0, sums, 0, s) : NFX_OK;
    if (!packs || (!in && !sample) || !out || !log_det || (fused && (!logp || !workspace)))
        return set_error(NFX_EINVAL, "affine_chain: null pointer");
    if (in == out && !sample) return set_error(NFX_EINVAL, "affine_chain: in and out must not alias");
    if (sample && (direction != NFX_FORWARD || fused || accumulate))
        return set_error(NFX_EINVAL, "affine_chain_sample: forward chains, no accumulate");
    if (sample && zout == out) return set_error(NFX_EINVAL, "affine_chain_sample: z and x must not alias");
    NfxChainPacks P{};
    for (int l = 0; l < nl; ++l) {
        if (!packs[l]) return set_error(NFX_EINVAL, "affine_chain: layer %d pack is null", l);
        P.p[l] = packs[l];
    }
    const int HT = (H + 31) / 32, D = chain_pad_d(d);
    if (d != D) return set_error(NFX_EUNSUPPORTED, "affine_chain: d=%d must be 2, 4 or 8 (row layout)", d);
    // Layout: the streaming chain (nfx_affine_schain.hip, the per-layer streaming kernel's
    // arithmetic) for large batches, the small-batch chain below otherwise; the affine kernel
    // policy forces either (tests compare each with its per-layer kernel bit for bit).
    const int pol = affine_policy_get();
    const bool want_stream = pol == NFX_AFFINE_STREAMING || (pol == NFX_AFFINE_AUTO && B > kSmallChainMaxB);
    if (want_stream && schain_supported(B, d, H) && !sample)
        return schain_launch(P, nl, in, out, log_det, B, d, H, direction, accumulate, logp, sums, workspace, s);
    if (sample && B > small_chain_max_b(D))
        return set_error(NFX_EUNSUPPORTED, "affine_chain_sample: B=%lld above the small-batch chain", (long long)B);
    affine_chain_t k = sample ? (HT == 1 ? sample_pick_ht<1>(d) : HT == 2 ? sample_pick_ht<2>(d)
                                 : HT == 3 ? sample_pick_ht<3>(d) : sample_pick_ht<4>(d))
                       : HT == 1 ? chain_pick_ht<1>(d, direction, fused)
                       : HT == 2 ? chain_pick_ht<2>(d, direction, fused)
                       : HT == 3 ? chain_pick_ht<3>(d, direction, fused) : chain_pick_ht<4>(d, direction, fused);
    const int64_t ntiles = (B + 31) / 32;
    // one tile per workgroup while that fits ~4 workgroups per CU; beyond, each workgroup carries
    // several tiles (every workgroup re-reads each layer's weights from L2 once, so fewer, fuller
    // workgroups cut that traffic)
    const int64_t cap = 4 * (int64_t)num_cus() < (int64_t)kMaxPartials ? 4 * (int64_t)num_cus() : (int64_t)kMaxPartials;
    int64_t grid = ntiles < cap ? ntiles : cap;
    int64_t tpw = (ntiles + grid - 1) / grid;
    if (tpw > chain_max_tpw(D)) return set_error(NFX_EUNSUPPORTED, "affine_chain: B=%lld too large", (long long)B);
    grid = (ntiles + tpw - 1) / tpw;
    const size_t lds = (size_t)tpw * 32 * (D + 1) * sizeof(float);
    int rc = prepare_lds((const void*)k, lds);
    if (rc) return rc;
    k<<<(unsigned)grid, 128 * HT, lds, s>>>(P, nl, in, out, log_det, B, accumulate, ntiles, (int)tpw, logp,
                                            reinterpret_cast<double*>(workspace), sums, gauss_const(d), seed, rng, zout);
    return check_launch("affine_chain_kernel");
}

}  // namespace nfx

using namespace nfx;

extern "C" int nfx_affine_chain(const float* const* packs, int n_layers, const float* in, float* out,
                                float* log_det, int64_t B, int d, int H, int direction, int accumulate,
                                void* stream) {
    return chain_launch(packs, n_layers, in, out, log_det, B, d, H, direction, accumulate, nullptr, nullptr, nullptr,
                        (hipStream_t)stream);
}

extern "C" int nfx_affine_chain_supported(int64_t B, int d, int H) { return chain_supported(B, d, H) ? 1 : 0; }

extern "C" int nfx_affine_chain_logprob(const float* const* packs, int n_layers, const float* in, float* out,
                                        float* log_det, float* logp, double* sums, void* workspace, int64_t B,
                                        int d, int H, int accumulate, void* stream) {
    if (!sums) return set_error(NFX_EINVAL, "affine_chain_logprob: null sums");
    return chain_launch(packs, n_layers, in, out, log_det, B, d, H, NFX_INVERSE, accumulate, logp, sums, workspace,
                        (hipStream_t)stream);
}

extern "C" int nfx_affine_chain_sample(const float* const* packs, int n_layers, uint64_t seed, uint64_t* rng_state,
                                       float* z, float* x, float* log_det, int64_t B, int d, int H, void* stream) {
    if (!rng_state) return set_error(NFX_EINVAL, "affine_chain_sample: null rng_state");
    return chain_launch(packs, n_layers, nullptr, x, log_det, B, d, H, NFX_FORWARD, 0, nullptr, nullptr, nullptr,
                        (hipStream_t)stream, rng_state, seed, z);
}
