// MADE affine flows: weight pack, sequential-kernel instantiations and the C-ABI.
// Kernels: nfx_made_kernel.h (parallel instantiations in nfx_made_par.hip).
#include "nfx_made_kernel.h"
#include "nfx_made_wide_kernel.h"
#include <atomic>
#include <cstdlib>

#include "nfx_made_seqs_kernel.h"
#include "nfx_pack.h"

namespace nfx {

__global__ void made_pack_kernel(NfxMlpRaw net, int d, int H, float* packed) {
    const int HT = (H + 31) / 32;
    const MadeLayout L = made_layout(d, HT);
    const int Hp = L.Hp, G1 = 4 * L.NKC;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < L.total; i += gridDim.x * blockDim.x) {
        if (i >= L.s_deg) continue;  // degree tables: made_live_kernel
        float v = 0.f;
        if (i < L.b1) {
            int t = i - L.w1, rr = t & 3, lane = (t >> 2) & 63, g = (t >> 8) % G1, ht = (t >> 8) / G1;
            int row = 32 * ht + (lane & 31), col = 2 * (4 * g + rr) + (lane >> 5);
            v = (row < H && col < d) ? mlp_weight(net, 0, d, row, col) : 0.f;
        } else if (i < L.w2) {
            int t = i - L.b1, r = t & 15, h = (t >> 4) & 1, ht = t >> 5, row = 32 * ht + crow(r, h);
            v = row < H ? mlp_bias(net, 0, row) : 0.f;
        } else if (i < L.b2 || (i >= L.w3 && i < L.b3)) {
            const int layer = i < L.b2 ? 1 : 2;
            int t = i - (layer == 1 ? L.w2 : L.w3), rr = t & 3, lane = (t >> 2) & 63, rq = (t >> 8) & 3;
            int kt = (t >> 10) % HT, hto = (t >> 10) / HT;
            int row = 32 * hto + (lane & 31), col = 32 * kt + crow(4 * rq + rr, lane >> 5);
            v = (row < H && col < H) ? mlp_weight(net, layer, H, row, col) : 0.f;
        } else if (i < L.w3 || (i >= L.b3 && i < L.w4)) {
            const int layer = i < L.w3 ? 1 : 2;
            int t = i - (layer == 1 ? L.b2 : L.b3), r = t & 15, h = (t >> 4) & 1, ht = t >> 5;
            int row = 32 * ht + crow(r, h);
            v = row < H ? mlp_bias(net, layer, row) : 0.f;
        } else if (i < L.b4) {
            int t = i - L.w4, rr = t & 3, lane = (t >> 2) & 63, rq = (t >> 8) & 3;
            int kt = (t >> 10) % HT, jw = (t >> 10) / HT, which = jw & 1, j = jw >> 1;
            int orow = 32 * j + (lane & 31), col = 32 * kt + crow(4 * rq + rr, lane >> 5);
            v = (orow < d && col < H) ? mlp_weight(net, 3, H, which * d + orow, col) : 0.f;
        } else if (i < L.par_total) {
            int t = i - L.b4, r = t & 15, h = (t >> 4) & 1, jw = t >> 5, which = jw & 1, j = jw >> 1;
            int orow = 32 * j + crow(r, h);
            v = orow < d ? mlp_bias(net, 3, which * d + orow) : 0.f;
        } else if (i < L.s_b1) {
            int t = i - L.s_w1t, ii = t / Hp, a = t % Hp;
            v = (ii < d && a < H) ? mlp_weight(net, 0, d, a, ii) : 0.f;
        } else if (i < L.s_w2) {
            int a = i - L.s_b1;
            v = a < H ? mlp_bias(net, 0, a) : 0.f;
        } else if (i < L.s_b2 || (i >= L.s_w3 && i < L.s_b3)) {
            const int layer = i < L.s_b2 ? 1 : 2;
            int t = i - (layer == 1 ? L.s_w2 : L.s_w3), a = t / Hp, b = t % Hp;
            v = (a < H && b < H) ? mlp_weight(net, layer, H, a, b) : 0.f;
        } else if (i < L.s_w3 || (i >= L.s_b3 && i < L.s_w4)) {
            const int layer = i < L.s_w3 ? 1 : 2;
            int a = i - (layer == 1 ? L.s_b2 : L.s_b3);
            v = a < H ? mlp_bias(net, layer, a) : 0.f;
        } else if (i < L.s_b4) {
            int t = i - L.s_w4, row = t / Hp, a = t % Hp;
            v = (row < 2 * d && a < H) ? mlp_weight(net, 3, H, row, a) : 0.f;
        } else if (i < L.s_deg) {
            int row = i - L.s_b4;
            v = row < 2 * d ? mlp_bias(net, 3, row) : 0.f;
        }
        packed[i] = v;
    }
}

// Structural zeros of the packed parallel image + the overflow-safe input bound (one block).
// The MADE masks zero whole 32 x 32 weight blocks (hidden units of low degree never see
// high-degree inputs); the tile kernel stops each output tile's k-loop after its last nonzero
// block when the tile's 32 input rows are all finite with max|x| <= tsafe. Every activation is
// finite then, so a skipped block would only have added exact zeros (a + 0*b == a for finite b,
// and relu maps -0 to +0): bit-identical to the dense product. Rows failing the test
// (non-finite or huge inputs, where the reference's 0*inf = NaN contamination matters) run the
// dense product. tsafe: with n_l = max row sum |W'_l| and c_l = max |b'_l|, every partial sum
// of layer l is bounded by A_l = n_l*A_{l-1} + c_l (A_0 = max|x|); tsafe is the largest A_0
// keeping every A_l <= 1e37 (0 when a weight is non-finite: dense path always).
constexpr int kLiveThreads = 1024;  // made_live_kernel: one block, 8 threads per weight row

__global__ __launch_bounds__(kLiveThreads) void made_live_kernel(NfxMlpRaw net, int d, int H, float* packed) {
    const int HT = (H + 31) / 32;
    const MadeLayout L = made_layout(d, HT);
    // hidden-unit degrees (M1[a][j] = (j <= deg(a)), made.py:56: row sums of the input mask - 1)
    // and the stable by-degree completion
    // order of the sequential kernels: s_deg [unit degree | degrees in order | units in order]
    {
        __shared__ int deg[256];
        const int Hp = L.Hp;
        // 16 lanes per unit (64 units per pass of the block), each counting a strided slice of the
        // unit's mask row with its loads independent, then a 16-lane sum: the serial row walk per
        // thread was most of this kernel's time at every training step's re-pack
        for (int a0 = 0; a0 < Hp; a0 += kLiveThreads / 16) {
            const int a = a0 + (threadIdx.x >> 4), q = threadIdx.x & 15;
            int n = 0;
            if (a < H && net.mask[0]) {
                const float* row = net.mask[0] + (size_t)a * d;
#pragma unroll 4
                for (int j = q; j < d; j += 16) n += row[j] != 0.f ? 1 : 0;
            }
            n += __shfl_xor(n, 1);
            n += __shfl_xor(n, 2);
            n += __shfl_xor(n, 4);
            n += __shfl_xor(n, 8);
            if (q == 0 && a < Hp) deg[a] = a < H ? (net.mask[0] ? n - 1 : 0) : 1000000000;
        }
        __syncthreads();
        for (int a = threadIdx.x; a < Hp; a += kLiveThreads) {
            const int da = deg[a];
            int rank = 0;
            for (int b = 0; b < Hp; ++b) rank += (deg[b] < da || (deg[b] == da && b < a)) ? 1 : 0;
            packed[L.s_deg + a] = (float)da;
            packed[L.s_deg + Hp + rank] = (float)da;
            packed[L.s_deg + 2 * Hp + rank] = (float)a;
        }
    }
    // the extent words (made_extent_kernel, launched next, max-es into them)
    int* nk = reinterpret_cast<int*>(packed);
    for (int i = threadIdx.x; i < 3 * HT + L.NJ; i += kLiveThreads) nk[L.nk1 + i] = 0;
    // overflow bound
    __shared__ double red[256];
    const int rows[4] = {H, H, H, 2 * d}, cols[4] = {d, H, H, H};
    const double tsafe = block_mlp_tsafe(net, 4, rows, cols, 1.0e37, red);
    if (threadIdx.x == 0) packed[L.tsafe] = (float)fmin(tsafe, 3.0e38);
}

// The k-block extents of the packed parallel image (made_live_kernel's structural zeros): one
// wave per 256-float weight group (32 rows x 8 k-steps), one float4 per lane and a ballot, the
// group's extent max-ed into its tile's word (zeroed by made_live_kernel, launched before).
__global__ __launch_bounds__(256) void made_extent_kernel(int d, int H, float* packed) {
    const int HT = (H + 31) / 32;
    const MadeLayout L = made_layout(d, HT);
    int* nk = reinterpret_cast<int*>(packed);
    const int n1 = HT * 4 * L.NKC, n23 = HT * HT * 4, n4 = L.NJ * 2 * HT * 4;
    const int lane = lane_id();
    for (int gi = blockIdx.x * 4 + (threadIdx.x >> 6); gi < n1 + 2 * n23 + n4; gi += gridDim.x * 4) {
        int off, word, ext;  // 256-float weight group (32 rows x 8 k-steps) -> its k-block extent
        if (gi < n1) {
            const int ht = gi / (4 * L.NKC), g = gi % (4 * L.NKC);
            off = L.w1 + gi * 256;
            word = L.nk1 + ht;
            ext = g / 4 + 1;
        } else if (gi < n1 + 2 * n23) {
            const int t = (gi - n1) % n23, layer = (gi - n1) / n23;
            off = (layer == 0 ? L.w2 : L.w3) + t * 256;
            word = (layer == 0 ? L.nk2 : L.nk3) + t / (HT * 4);
            ext = (t % (HT * 4)) / 4 + 1;
        } else {
            const int t = gi - n1 - 2 * n23;
            off = L.w4 + t * 256;
            word = L.nk4 + t / (2 * HT * 4);
            ext = (t % (HT * 4)) / 4 + 1;
        }
        const f32x4 v = *reinterpret_cast<const f32x4*>(packed + off + 4 * lane);
        const bool nzl = v[0] != 0.f || v[1] != 0.f || v[2] != 0.f || v[3] != 0.f;  // NaN != 0: kept
        if (__ballot(nzl) != 0 && lane == 0) atomicMax(&nk[word], ext);
    }
}

template <int HT>
made_seqs_kernel_t made_seqs_pick_ht(int variant, bool logp) {
    if (variant == NFX_MAF_FORWARD) return made_seqs_kernel<HT, NFX_MAF_FORWARD, false>;
    return logp ? made_seqs_kernel<HT, NFX_IAF_INVERSE, true> : made_seqs_kernel<HT, NFX_IAF_INVERSE, false>;
}
template made_seqs_kernel_t made_seqs_pick_ht<1>(int, bool);
template made_seqs_kernel_t made_seqs_pick_ht<2>(int, bool);

template <int HT, int VAR>
static made_seq_kernel_t seq_var() {
    return made_seq_kernel<HT, VAR>;
}

template <int HT>
made_seq_kernel_t made_seq_pick_ht(int variant) {
    return variant == NFX_MAF_FORWARD ? seq_var<HT, NFX_MAF_FORWARD>() : seq_var<HT, NFX_IAF_INVERSE>();
}
template made_seq_kernel_t made_seq_pick_ht<1>(int);
template made_seq_kernel_t made_seq_pick_ht<2>(int);
template made_seq_kernel_t made_seq_pick_ht<3>(int);
template made_seq_kernel_t made_seq_pick_ht<4>(int);

static made_par_kernel_t pick_par(int HT, bool wlds, int variant) {
    switch (HT) {
        case 1: return made_pick_ht<1>(wlds, variant);
        case 2: return made_pick_ht<2>(wlds, variant);
        case 3: return made_pick_ht<3>(wlds, variant);
        case 4: return made_pick_ht<4>(wlds, variant);
        default: return nullptr;
    }
}

static made_par_kernel_t pick_tile(int HT, bool wlds, int variant, bool logp) {
    switch (HT) {
        case 1: return made_tile_pick_ht<1>(wlds, variant, logp);
        case 2: return made_tile_pick_ht<2>(wlds, variant, logp);
        case 3: return made_tile_pick_ht<3>(wlds, variant, logp);
        case 4: return made_tile_pick_ht<4>(wlds, variant, logp);
        default: return nullptr;
    }
}

static made_seq_kernel_t pick_seq(int HT, int variant) {
    switch (HT) {
        case 1: return made_seq_pick_ht<1>(variant);
        case 2: return made_seq_pick_ht<2>(variant);
        case 3: return made_seq_pick_ht<3>(variant);
        case 4: return made_seq_pick_ht<4>(variant);
        default: return nullptr;
    }
}

int made_big_launch(const float* packed, const float* in, float* out, float* log_det, int64_t B, int d, int H,
                    int variant, int accumulate, hipStream_t s);

constexpr size_t kLdsBytes = 160 * 1024;
constexpr int kTileMaxD = 64;  // made_tile_kernel: whole [32 x d] x tile per wave in LDS

}  // namespace nfx

using namespace nfx;

extern "C" size_t nfx_made_packed_floats(int d, int H) {
    if (d <= 0 || H <= 0) return 0;
    return (size_t)made_layout(d, (H + 31) / 32).total;
}

namespace nfx {
int made_pack_seqp(int d, int H, float* packed, hipStream_t s);
// the sequential directions' part of a pack (HT <= 2): the rank-ordered image and the chunk
// schedule, from the degree tables made_live_kernel wrote
static int made_pack_seq(int d, int H, float* packed, hipStream_t s) {
    const int HT = (H + 31) / 32;
    if (HT > 2) return NFX_OK;
    if (HT == 1) made_seqs_image_kernel<1><<<64, 256, 0, s>>>(packed, d, H);
    else made_seqs_image_kernel<2><<<64, 256, 0, s>>>(packed, d, H);
    int rc = check_launch("made_seqs_image_kernel");
    if (rc) return rc;
    if (HT == 1) made_seqs_chunk_kernel<1><<<1, 64, 0, s>>>(packed, d, H);
    else made_seqs_chunk_kernel<2><<<1, 64, 0, s>>>(packed, d, H);
    rc = check_launch("made_seqs_chunk_kernel");
    if (rc) return rc;
    return made_pack_seqp(d, H, packed, s);
}
}  // namespace nfx

extern "C" int nfx_made_pack_parallel(const NfxMlpRaw* net, int d, int H, float* packed, void* stream) {
    if (!net || !packed) return set_error(NFX_EINVAL, "made_pack: null pointer");
    if (d <= 0 || d > 4096 || H <= 0 || H > 256)
        return set_error(NFX_EUNSUPPORTED, "made_pack: d=%d H=%d outside d<=4096, H<=256", d, H);
    if (net->n_layers != 4) return set_error(NFX_EINVAL, "made_pack: MADE has 4 masked layers (got %d)", net->n_layers);
    for (int l = 0; l < 4; ++l)
        if (!net->w[l]) return set_error(NFX_EINVAL, "made_pack: layer %d weight is null", l);
    const int total = (int)nfx_made_packed_floats(d, H);
    int blocks = (total + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    made_pack_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(*net, d, H, packed);
    int rc = check_launch("made_pack_kernel");
    if (rc) return rc;
    made_live_kernel<<<1, kLiveThreads, 0, (hipStream_t)stream>>>(*net, d, H, packed);
    rc = check_launch("made_live_kernel");
    if (rc) return rc;
    {
        const int HT = (H + 31) / 32;
        const MadeLayout L = made_layout(d, HT);
        const int groups = HT * 4 * L.NKC + 2 * HT * HT * 4 + L.NJ * 2 * HT * 4;
        made_extent_kernel<<<(groups + 3) / 4, 256, 0, (hipStream_t)stream>>>(d, H, packed);
    }
    return check_launch("made_extent_kernel");
}

extern "C" int nfx_made_pack_sequential(int d, int H, float* packed, void* stream) {
    if (!packed) return set_error(NFX_EINVAL, "made_pack_sequential: null pointer");
    if (d <= 0 || d > 4096 || H <= 0 || H > 256)
        return set_error(NFX_EUNSUPPORTED, "made_pack_sequential: d=%d H=%d outside d<=4096, H<=256", d, H);
    return made_pack_seq(d, H, packed, (hipStream_t)stream);
}

extern "C" int nfx_made_pack(const NfxMlpRaw* net, int d, int H, float* packed, void* stream) {
    const int rc = nfx_made_pack_parallel(net, d, H, packed, stream);
    if (rc) return rc;
    return made_pack_seq(d, H, packed, (hipStream_t)stream);
}

namespace nfx {
int made_seqw_launch(const float* packed, const float* in, float* out, float* log_det, int64_t B, int d, int H,
                     int variant, int accumulate, float* logp, double* partials, double* sums, bool fused,
                     int* grid_out, hipStream_t s);
int made_seqp_launch(const float* packed, const float* in, float* out, float* log_det, int64_t B, int d, int H,
                     int variant, int accumulate, float* logp, double* partials, double* sums, bool fused,
                     hipStream_t s);
}  // namespace nfx

// Sequential-direction kernel choice (nfx_made_seq_policy): NFX_MADE_SEQ_AUTO (default, or
// $NFX_MADE_SEQ_POLICY), NFX_MADE_SEQ_SEGMENT (made_seqs_kernel: 16 lanes per sample) or
// NFX_MADE_SEQ_WAVE (made_seqw_kernel: a wave per sample).
static std::atomic<int>& made_seq_policy() {
    static std::atomic<int> v{[] {
        const char* e = getenv("NFX_MADE_SEQ_POLICY");
        return e ? atoi(e) : NFX_MADE_SEQ_AUTO;
    }()};
    return v;
}

namespace nfx {
int made_seq_policy_get() { return made_seq_policy().load(std::memory_order_relaxed); }
}  // namespace nfx

static int made_launch(const float* packed, const float* in, float* out, float* log_det, int64_t B,
                       int d, int H, int variant, int accumulate, float* logp, double* sums,
                       void* workspace, hipStream_t s) {
    const bool fused = sums != nullptr;
    if (B < 0 || d <= 0 || H <= 0) return set_error(NFX_EINVAL, "made_affine: bad shape");
    if (d > 4096 || H > 256) return set_error(NFX_EUNSUPPORTED, "made_affine: d=%d H=%d outside d<=4096, H<=256", d, H);
    if (variant < NFX_MAF_INVERSE || variant > NFX_IAF_INVERSE)
        return set_error(NFX_EINVAL, "made_affine: unknown variant %d", variant);
    const int HT = (H + 31) / 32;
    if (HT > 4) {  // 128 < H <= 256: nfx_made_big.hip (no fused log_prob epilogue)
        if (fused) return set_error(NFX_EUNSUPPORTED, "made_affine_logprob: no fused log_prob for H=%d > 128", H);
        if (B == 0) return NFX_OK;
        if (!packed || !in || !out || !log_det) return set_error(NFX_EINVAL, "made_affine: null pointer");
        if (in == out) return set_error(NFX_EINVAL, "made_affine: in and out must not alias");
        return made_big_launch(packed, in, out, log_det, B, d, H, variant, accumulate, s);
    }
    const MadeLayout L = made_layout(d, HT);
    const bool parallel = variant == NFX_MAF_INVERSE || variant == NFX_IAF_FORWARD;
    const size_t wide_lds_bytes = (size_t)wide_lds(L, HT).total * sizeof(float);
    const bool wide = parallel && d > kTileMaxD && HT <= 2 && wide_lds_bytes <= kLdsBytes;
    const bool seqs = (variant == NFX_MAF_FORWARD || variant == NFX_IAF_INVERSE) && HT <= 2;
    if (fused && !((variant == NFX_MAF_INVERSE && (d <= kTileMaxD || wide)) || (variant == NFX_IAF_INVERSE && seqs)))
        return set_error(NFX_EUNSUPPORTED,
                         "made_affine_logprob: fused log_prob needs MAF inverse with d <= %d or H <= 64, "
                         "or IAF inverse with H <= 64", kTileMaxD);
    if (fused && B > 0 && (!logp || !workspace)) return set_error(NFX_EINVAL, "made_affine_logprob: null logp/workspace");
    if (B == 0) return fused ? gauss_finish(reinterpret_cast<double*>(workspace), 0, sums, 0, s) : NFX_OK;
    if (!packed || !in || !out || !log_det) return set_error(NFX_EINVAL, "made_affine: null pointer");
    if (in == out) return set_error(NFX_EINVAL, "made_affine: in and out must not alias");
    double* partials = reinterpret_cast<double*>(workspace);
    if (wide) {
        const int64_t nchunks = (B + 63) / 64;
        // 8 waves per workgroup share each staged weight slice; when that leaves CUs idle (fewer
        // than one 8-chunk round per CU, e.g. a 64Ki per-GPU shard), 4-wave workgroups spread
        // the chunks over twice as many CUs
        const int nw = nchunks < (int64_t)kWideWaves * num_cus() ? 4 : kWideWaves;
        const size_t lds_nw = (size_t)wide_lds(L, HT, nw).total * sizeof(float);
        made_par_kernel_t k = HT == 1 ? made_wide_pick_ht<1>(variant, fused, nw) : made_wide_pick_ht<2>(variant, fused, nw);
        int rc = prepare_lds((const void*)k, lds_nw);
        if (rc) return rc;
        int grid = resident_grid((const void*)k, 64 * nw, lds_nw, (nchunks + nw - 1) / nw);
        if (grid > kMaxPartials) grid = kMaxPartials;
        k<<<grid, 64 * nw, lds_nw, s>>>(packed, in, out, log_det, B, d, accumulate, nchunks, logp, partials,
                                        sums, gauss_const(d));
        return check_launch("made_wide_kernel");  // (LOGP: the last workgroup wrote sums)
    }
    if ((variant == NFX_MAF_INVERSE || variant == NFX_IAF_FORWARD) && d <= kTileMaxD) {
        const int64_t ntiles = (B + 31) / 32;
        // 8 waves per workgroup (two per SIMD) while the batch fills the chip. Below that (no
        // fused log_prob) as few waves per workgroup as spread the tiles one wave per SIMD, the
        // weights read through L2 rather than staged per workgroup: 6x IAF(2, 64) sampling at
        // n = 4,000 112 -> 73 us; staging the weights per workgroup measured no better at d = 63
        // (profiles/r06_tile/)
        int nw = 8;
        if (!fused && ntiles < 4 * (int64_t)num_cus()) nw = (int)((ntiles + num_cus() - 1) / num_cus());
        const size_t wbytes = (size_t)L.par_total * sizeof(float);
        const size_t tiles = nw * 32 * (size_t)kTileStride * sizeof(float);
        const bool wlds = nw == 8 && wbytes + tiles <= kLdsBytes;
        made_par_kernel_t k = pick_tile(HT, wlds, variant, fused);
        if (!k) return set_error(NFX_EUNSUPPORTED, "made_affine: no kernel for H=%d", H);
        const size_t lds = (wlds ? wbytes : 0) + tiles;
        int rc = prepare_lds((const void*)k, lds);
        if (rc) return rc;
        int grid = resident_grid((const void*)k, 64 * nw, lds, (ntiles + nw - 1) / nw);
        if (grid > kMaxPartials) grid = kMaxPartials;
        k<<<grid, 64 * nw, lds, s>>>(packed, in, out, log_det, B, d, accumulate, ntiles, logp, partials, sums,
                                     gauss_const(d));
        return check_launch("made_tile_kernel");
    }
    if (variant == NFX_MAF_INVERSE || variant == NFX_IAF_FORWARD) {
        const size_t wbytes = (size_t)L.par_total * sizeof(float);
        const size_t stage8 = 8 * (size_t)kStageFloats * sizeof(float);
        const bool wlds = wbytes + stage8 <= kLdsBytes;
        made_par_kernel_t k = pick_par(HT, wlds, variant);
        if (!k) return set_error(NFX_EUNSUPPORTED, "made_affine: no kernel for H=%d", H);
        const int threads = wlds ? 512 : 256;
        const size_t lds = wlds ? wbytes + stage8 : 4 * (size_t)kStageFloats * sizeof(float);
        int rc = prepare_lds((const void*)k, lds);
        if (rc) return rc;
        const int64_t nchunks = (B + 63) / 64;
        const int nw = threads / 64;
        const int grid = resident_grid((const void*)k, threads, lds, (nchunks + nw - 1) / nw);
        k<<<grid, threads, lds, s>>>(packed, in, out, log_det, B, d, accumulate, nchunks, nullptr, nullptr, nullptr,
                                     0.f);
        return check_launch("made_parallel_kernel");
    }
    // AUTO: the wave-per-sample kernel while the batch leaves the segment kernel's 4-sample waves
    // short of 2 per SIMD (measured, IAF(784, 64): 74.8 vs 107.9 us at 1,024; 116 vs 138 us at
    // 4,096 for the segment kernel, profiles/r03i_seqw_sweep.jsonl)
    const int seq_pol = made_seq_policy().load(std::memory_order_relaxed);
    // AUTO: the push kernel while it leads (IAF(784, 64) + log_prob: 31.9 vs 53.5 / 92.7 us at 1,024,
    // 82.7 vs 137.5 / 94.9 us at 4,096 for the wave / segment kernels; the segment kernel from
    // 8,192, gpurun_out/r05a/sweep.jsonl) — for d > 32 only: at d <= 32 it trails the wave and
    // segment kernels at every batch up to 4,000 (MAF(32, 64) at 1,024: 48.4 vs 35.6 / 52.6 us;
    // MAF(2, 64) at 4,000: 39.6 vs 36.1 / 30.2 us, profiles/r06_tile/seq.jsonl)
    const bool push_auto = seq_pol == NFX_MADE_SEQ_AUTO && d > 32 && B <= 4096 * (int64_t)num_cus() / 256;
    if (seqs && (seq_pol == NFX_MADE_SEQ_PUSH || push_auto) && L.ps > 0)
        return made_seqp_launch(packed, in, out, log_det, B, d, H, variant, accumulate, logp, partials, sums, fused, s);
    if (seqs && (seq_pol == NFX_MADE_SEQ_PUSH || seq_pol == NFX_MADE_SEQ_WAVE || (seq_pol == NFX_MADE_SEQ_AUTO && B <= 2048 * (int64_t)num_cus() / 256))) {
        int grid = 0;
        return made_seqw_launch(packed, in, out, log_det, B, d, H, variant, accumulate, logp, partials, sums, fused,
                                &grid, s);
    }
    if (seqs) {
        made_seqs_kernel_t k = HT == 1 ? made_seqs_pick_ht<1>(variant, fused) : made_seqs_pick_ht<2>(variant, fused);
        const size_t lds = (size_t)seqs_lds(L.Hp).total * sizeof(float);
        int rc = prepare_lds((const void*)k, lds);
        if (rc) return rc;
        const int threads = kSeqsThreads;
        int grid = resident_grid((const void*)k, threads, lds, (B + 4 * kSeqsWaves - 1) / (4 * kSeqsWaves));
        if (grid > kMaxPartials) grid = kMaxPartials;
        k<<<grid, threads, lds, s>>>(packed, in, out, log_det, B, d, H, accumulate, logp, partials, sums,
                                     gauss_const(d));
        return check_launch("made_seqs_kernel");
    }
    made_seq_kernel_t k = pick_seq(HT, variant);
    if (!k) return set_error(NFX_EUNSUPPORTED, "made_affine: no sequential kernel for H=%d", H);
    const size_t lds = 2 * 64 * (size_t)(L.Hp + 4) * sizeof(float);
    int rc = prepare_lds((const void*)k, lds);
    if (rc) return rc;
    const int64_t grid = (B + 63) / 64;
    k<<<(unsigned)grid, 64, lds, s>>>(packed, in, out, log_det, B, d, H, accumulate);
    return check_launch("made_seq_kernel");
}

extern "C" int nfx_made_seq_policy(int policy) {
    if (policy < 0) return made_seq_policy().load();
    if (policy > NFX_MADE_SEQ_PUSH) return set_error(NFX_EINVAL, "made_seq_policy: unknown policy %d", policy);
    return made_seq_policy().exchange(policy);
}

extern "C" int nfx_made_affine(const float* packed, const float* in, float* out, float* log_det,
                               int64_t B, int d, int H, int variant, int accumulate, void* stream) {
    return made_launch(packed, in, out, log_det, B, d, H, variant, accumulate, nullptr, nullptr, nullptr,
                       (hipStream_t)stream);
}

extern "C" int nfx_made_affine_logprob(const float* packed, const float* in, float* out, float* log_det,
                                       float* logp, double* sums, void* workspace, int64_t B, int d,
                                       int H, int variant, int accumulate, void* stream) {
    if (!sums) return set_error(NFX_EINVAL, "made_affine_logprob: null sums");
    return made_launch(packed, in, out, log_det, B, d, H, variant, accumulate, logp, sums, workspace,
                       (hipStream_t)stream);
}
