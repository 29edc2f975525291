// MADE weight gradients as sample contractions on fp32 MFMA — the parameter half of the MADE
// backward: for every MaskedLinear of the conditioner
//   dW = (δ · aᵀ) ⊙ mask,  db = Σ_samples δ
// (the gradient of F.linear(a, W * mask, b), masked_linear.py:14-18, made.py:81-134), with δ the
// layer's output gradient and a its input, both per sample. The backward kernels
// (nfx_made_bwd.hip, nfx_made_seqbwd.hip) write δ and a FEATURE-MAJOR, [rows x P] with a
// sample pitch P = nfx_made_factor_pitch(B) = B:
//   D4 (2d) | D3 (H) | D2 (H) | D1 (H) | H3 (H+1) | H2 (H+1) | H1 (H+1) | X1 (d+1)
// (the +1 rows are unused here; the bias gradients are row sums of δ).
//
// Contraction kernel: the sample dimension is the MFMA k dimension. A task = (sample chunk,
// 32x32 output tile of one layer); lane (i, kh) of the wave loads 16 consecutive samples of
// δ row i and of a row i (four 16-byte reads when the pitch keeps rows 16-byte aligned, i.e.
// B % 4 == 0, else sixteen 4-byte reads; with the other lane half they cover the step's
// 128-byte segment) and feeds them as 16 v_mfma_f32_32x32x2_f32 k-steps — the k index of an
// MFMA is a sample, and both operands agree on which, so no transpose is ever needed. The bias
// sums ride along as lane-local adds of the δ values the tile already holds (column tile 0).
// Tasks of one chunk are numbered consecutively and their workgroups are placed on ONE XCD
// (blockIdx -> XCD round robin undone), so the rows a chunk's tiles share are fetched from HBM
// once into that XCD's L2. Per-chunk fp32 partials are reduced in float64 in a fixed order
// (train_sum_finish) and assembled into the module's parameters() order with the masks applied:
// deterministic run to run.
#include "nfx_common.h"

namespace nfx {

struct WgLayer {
    const float* dm;  // δ rows [M x P]
    const float* am;  // input rows [N x P]
    const float* mask;  // [M x N] row-major (the MaskedLinear buffer), or nullptr
    float* gw;        // weight gradient [M x N] (row-major, nn.Linear layout)
    float* gb;        // bias gradient [M] (nullptr: no bias)
    int M, N, tm, tn, tile0, btile0;  // tiles: tm x tn starting at tile0; row blocks at btile0
};
struct WgArgs {
    WgLayer l[4];
    int nl, T, NBT;  // layers, total tiles, total bias row blocks
};

constexpr int kWgWaves = 4;
constexpr int kWgTs = 36;  // LDS transpose tile row stride (floats)

__device__ __forceinline__ int wg_layer_of(const WgArgs& a, int t) {
    int k = 0;
#pragma unroll
    for (int j = 1; j < 4; ++j)
        if (j < a.nl && t >= a.l[j].tile0) k = j;
    return k;
}

template <bool VEC4>
__global__ __launch_bounds__(64 * kWgWaves) void made_wgrad_kernel(WgArgs a, int64_t B, int64_t P, int64_t chunk,
                                                                   int64_t ntasks, int blocks_per_xcd, float* part) {
    __shared__ float wg_lds[kWgWaves * 32 * kWgTs];
    // undo the hardware's round robin of consecutive workgroups over the 8 XCDs
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: descriptors stay scalar
    const int64_t task = ((int64_t)xcd * blocks_per_xcd + slot) * kWgWaves + wave;
    if (task >= ntasks) return;
    const int T = a.T;
    const int64_t c = task / T;
    const int t = (int)(task % T);
    const int k = wg_layer_of(a, t);
    // field by field with constant kernarg indices: a dynamic index would copy the struct to
    // scratch and turn every descriptor below into a VGPR (waterfall loops around each load)
#define WGF(f) (k == 0 ? a.l[0].f : (k == 1 ? a.l[1].f : (k == 2 ? a.l[2].f : a.l[3].f)))
    const float* Ldm = WGF(dm);
    const float* Lam = WGF(am);
    const bool has_b = WGF(gb) != nullptr;
    const int LM = WGF(M), LN = WGF(N), Ltn = WGF(tn), Ltile0 = WGF(tile0), Lbt0 = WGF(btile0);
#undef WGF
    const int lt = t - Ltile0, tmi = lt / Ltn, tni = lt % Ltn;
    const int lane = lane_id(), i = lane & 31, kh = lane >> 5;
    // descriptors based at the tile's first row: rows past M / N read as 0 (range check)
    const int rowsD = LM - 32 * tmi < 32 ? LM - 32 * tmi : 32;
    const int rowsA = LN - 32 * tni < 32 ? LN - 32 * tni : 32;
    const auto rd = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Ldm) + (int64_t)32 * tmi * P, 0,
                                                      (int)(rowsD * P * 4), 0x00020000);
    const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Lam) + (int64_t)32 * tni * P, 0,
                                                      (int)(rowsA * P * 4), 0x00020000);
    const bool bias = tni == 0 && has_b;
    f32x16 acc{};
    float bsum = 0.f;
    // Rows arrive COALESCED — lane l reads samples 4 (l & 7) .. + 3 of row 8q + (l >> 3), so one
    // load instruction covers eight whole 128-byte row segments (16 cache accesses instead of the
    // 64 of a lane-per-row read: the texture-address stage was 82 % busy with those) — and are
    // turned into MFMA operand order (lane (i, kh): row i, samples 16 kh + 4q .. + 3) through a
    // wave-private LDS tile. Same MFMA operands in the same order as a lane-per-row read.
    float* tl = wg_lds + wave * (32 * kWgTs);  // [32 rows][kWgTs], δ then a (LDS keeps a wave's order)
    const int cr = lane >> 3, cc = 4 * (lane & 7);
    const int gvo = (int)((cr * P + cc) * 4);
    auto stage = [&](const __amdgpu_buffer_rsrc_t& r, int64_t st, f32x4 (&g)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int so = (int)((st + (int64_t)8 * q * P) * 4);
            if constexpr (VEC4) {
                const auto u = __builtin_amdgcn_raw_buffer_load_b128(r, gvo, so, 0);
                g[q] = f32x4{__uint_as_float(u[0]), __uint_as_float(u[1]), __uint_as_float(u[2]), __uint_as_float(u[3])};
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) g[q][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, gvo, so + 4 * e, 0));
            }
        }
    };
    auto xpose = [&](const f32x4 (&gd)[4], const f32x4 (&ga)[4], f32x4 (&dv)[4], f32x4 (&av)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q) *reinterpret_cast<f32x4*>(tl + (8 * q + cr) * kWgTs + cc) = gd[q];
#pragma unroll
        for (int q = 0; q < 4; ++q) dv[q] = *reinterpret_cast<const f32x4*>(tl + i * kWgTs + 16 * kh + 4 * q);
        asm volatile("" ::: "memory");  // (the tile is rewritten with a only after δ's reads, in LDS order)
#pragma unroll
        for (int q = 0; q < 4; ++q) *reinterpret_cast<f32x4*>(tl + (8 * q + cr) * kWgTs + cc) = ga[q];
#pragma unroll
        for (int q = 0; q < 4; ++q) av[q] = *reinterpret_cast<const f32x4*>(tl + i * kWgTs + 16 * kh + 4 * q);
    };
    auto step_mfma = [&](const f32x4 (&dv)[4], const f32x4 (&av)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                acc = mfma32(dv[q][e], av[q][e], acc);
                if (bias) bsum += dv[q][e];
            }
    };
    // Chunk c takes the 32-sample steps c, c + nch, c + 2 nch, ... (steps dealt round-robin over
    // the chunks, so at any moment the chunks read one window of nch consecutive steps).
    const int64_t nch = (B + chunk - 1) / chunk;
    const int64_t nfs = B / 32;  // full steps of the batch
    const int64_t nfull = nfs > c ? (nfs - c + nch - 1) / nch : 0;  // this chunk's full steps
    auto step_at = [&](int64_t k) { return 32 * (c + nch * k); };
    if (nfull > 0) {
        // two register sets of global rows: the next step's rows are in flight while this step
        // goes through the LDS tile and its 16 MFMAs (past the last step the prefetch re-reads it)
        f32x4 gdA[4], gaA[4], gdB[4], gaB[4], dv[4], av[4];
        int64_t k = 0;
        stage(rd, step_at(0), gdA);
        stage(ra, step_at(0), gaA);
        for (;;) {
            int64_t sn = step_at(k + 1 < nfull ? k + 1 : k);
            stage(rd, sn, gdB);
            stage(ra, sn, gaB);
            xpose(gdA, gaA, dv, av);
            step_mfma(dv, av);
            if (++k >= nfull) break;
            sn = step_at(k + 1 < nfull ? k + 1 : k);
            stage(rd, sn, gdA);
            stage(ra, sn, gaA);
            xpose(gdB, gaB, dv, av);
            step_mfma(dv, av);
            if (++k >= nfull) break;
        }
    }
    if (B % 32 != 0 && nfs % nch == c) {  // the batch's ragged last step: samples >= B hold pitch padding -> 0
        const int64_t st = 32 * nfs;
        f32x4 gd[4], ga[4], dv[4], av[4];
        stage(rd, st, gd);
        stage(ra, st, ga);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const bool ok = st + cc + e < B;
                gd[q][e] = ok ? gd[q][e] : 0.f;
                ga[q][e] = ok ? ga[q][e] : 0.f;
            }
        xpose(gd, ga, dv, av);
        step_mfma(dv, av);
    }
    const int64_t len = (int64_t)T * 1024 + (int64_t)a.NBT * 32;
    float* out = part + c * len + (int64_t)t * 1024 + lane * 16;
#pragma unroll
    for (int q = 0; q < 4; ++q)
        *reinterpret_cast<f32x4*>(out + 4 * q) = f32x4{acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
    if (bias) {
        const float other = __shfl_xor(bsum, 32, 64);
        if (kh == 0) part[c * len + (int64_t)T * 1024 + (int64_t)(Lbt0 + tmi) * 32 + i] = bsum + other;
    }
}

// sums[T*1024 + NBT*32] (float64, accumulator order) -> parameter gradients, masks applied.
__global__ void made_wgrad_assemble_kernel(WgArgs a, const double* sums) {
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < a.T * 1024 + a.NBT * 32; e += gridDim.x * blockDim.x) {
        if (e < a.T * 1024) {
            const int t = e >> 10, lane = (e >> 4) & 63, r = e & 15;
            const WgLayer& L = a.l[wg_layer_of(a, t)];
            const int lt = t - L.tile0, tmi = lt / L.tn, tni = lt % L.tn;
            const int row = 32 * tmi + crow(r, lane >> 5), col = 32 * tni + (lane & 31);
            if (row < L.M && col < L.N) {
                const size_t o = (size_t)row * L.N + col;
                const float g = (float)sums[e];
                L.gw[o] = L.mask ? g * L.mask[o] : g;
            }
        } else {
            const int b = e - a.T * 1024, bt = b >> 5, i = b & 31;
            int k = 0;
            for (int j = 1; j < a.nl; ++j)
                if (bt >= a.l[j].btile0) k = j;
            const WgLayer& L = a.l[k];
            const int row = 32 * (bt - L.btile0) + i;
            if (L.gb && row < L.M) L.gb[row] = (float)sums[e];
        }
    }
}

static int64_t wg_chunk(int64_t B, int T) {
    // about 6144 tasks (6 waves per SIMD in one round: 84 VGPRs, 4.6 KB of LDS each), chunks of
    // >= 1024 samples, 32-aligned
    int64_t c = (B * T + 6143) / 6144;
    if (c < 1024) c = 1024;
    return (c + 31) & ~(int64_t)31;
}

static WgArgs wg_args(const float* factors, int64_t P, int d, int H, const float* const* masks, float* grads) {
    WgArgs a{};
    const float* D4 = factors;
    const float* D3 = D4 + (int64_t)2 * d * P;
    const float* D2 = D3 + (int64_t)H * P;
    const float* D1 = D2 + (int64_t)H * P;
    const float* H3 = D1 + (int64_t)H * P;
    const float* H2 = H3 + (int64_t)(H + 1) * P;
    const float* H1 = H2 + (int64_t)(H + 1) * P;
    const float* X1 = H1 + (int64_t)(H + 1) * P;
    const float* dm[4] = {D1, D2, D3, D4};
    const float* am[4] = {X1, H1, H2, H3};
    const int M[4] = {H, H, H, 2 * d}, N[4] = {d, H, H, H};
    // parameters() order: net.0.weight, net.0.bias, net.2.*, net.4.*, net.6.*
    int64_t off = 0, tile = 0, bt = 0;
    for (int k = 0; k < 4; ++k) {
        WgLayer& L = a.l[k];
        L.dm = dm[k];
        L.am = am[k];
        L.mask = masks ? masks[k] : nullptr;
        L.M = M[k];
        L.N = N[k];
        L.tm = (M[k] + 31) / 32;
        L.tn = (N[k] + 31) / 32;
        L.tile0 = (int)tile;
        L.btile0 = (int)bt;
        tile += L.tm * L.tn;
        bt += L.tm;
        L.gw = grads + off;
        off += (int64_t)M[k] * N[k];
        L.gb = grads + off;
        off += M[k];
    }
    a.nl = 4;
    a.T = (int)tile;
    a.NBT = (int)bt;
    return a;
}

}  // namespace nfx

using namespace nfx;

extern "C" int64_t nfx_made_factor_pitch(int64_t B) { return B <= 0 ? 0 : B; }

extern "C" size_t nfx_made_wgrad_workspace_bytes(int64_t B, int d, int H) {
    if (B <= 0 || d <= 0 || H <= 0) return 0;
    const int64_t T = ((H + 31) / 32) * (((d + 31) / 32) + 2 * ((H + 31) / 32)) + ((2 * d + 31) / 32) * ((H + 31) / 32);
    const int64_t NBT = 3 * ((H + 31) / 32) + (2 * d + 31) / 32;
    const int64_t len = T * 1024 + NBT * 32;
    const int64_t chunk = wg_chunk(B, (int)T);
    const int64_t nch = (B + chunk - 1) / chunk;
    return (size_t)(nch * len * sizeof(float) + len * sizeof(double) + 256);
}

extern "C" size_t nfx_made_param_floats(int d, int H) {
    if (d <= 0 || H <= 0) return 0;
    return (size_t)(H * d + H + 2 * (H * H + H) + 2 * d * H + 2 * d);
}

extern "C" int nfx_made_backward_weights(const float* factors, int64_t B, int d, int H, const float* const* masks,
                                         float* grads, void* workspace, void* stream) {
    if (B < 0 || d <= 0 || H <= 0 || d > 4096 || H > 256)
        return set_error(NFX_EINVAL, "made_backward_weights: bad shape B=%lld d=%d H=%d", (long long)B, d, H);
    if (!grads) return set_error(NFX_EINVAL, "made_backward_weights: null grads");
    hipStream_t s = (hipStream_t)stream;
    const int64_t P = nfx_made_factor_pitch(B);
    if (B == 0) {
        const hipError_t e = hipMemsetAsync(grads, 0, nfx_made_param_floats(d, H) * sizeof(float), s);
        return e == hipSuccess ? NFX_OK : set_error(NFX_ELAUNCH, "made_backward_weights: memset failed");
    }
    if (!factors || !workspace) return set_error(NFX_EINVAL, "made_backward_weights: null pointer");
    if ((int64_t)32 * P * 4 >= ((int64_t)1 << 31))
        return set_error(NFX_EUNSUPPORTED, "made_backward_weights: B=%lld too large for 32-bit row offsets", (long long)B);
    const WgArgs a = wg_args(factors, P, d, H, masks, grads);
    const int64_t len = (int64_t)a.T * 1024 + (int64_t)a.NBT * 32;
    const int64_t chunk = wg_chunk(B, a.T);
    const int64_t nch = (B + chunk - 1) / chunk;
    const int64_t ntasks = nch * a.T;
    const int64_t wgs = (ntasks + kWgWaves - 1) / kWgWaves;
    const int bpx = (int)((wgs + 7) / 8);
    float* part = reinterpret_cast<float*>(workspace);
    double* sums = reinterpret_cast<double*>(
        reinterpret_cast<char*>(workspace) + ((nch * len * sizeof(float) + 255) & ~(size_t)255));
    if (P % 4 == 0)
        made_wgrad_kernel<true><<<8 * bpx, 64 * kWgWaves, 0, s>>>(a, B, P, chunk, ntasks, bpx, part);
    else
        made_wgrad_kernel<false><<<8 * bpx, 64 * kWgWaves, 0, s>>>(a, B, P, chunk, ntasks, bpx, part);
    int rc = check_launch("made_wgrad_kernel");
    if (rc) return rc;
    if ((rc = train_sum_finish(part, (int)nch, (int)len, sums, s))) return rc;
    made_wgrad_assemble_kernel<<<(int)((len + 255) / 256), 256, 0, s>>>(a, sums);
    return check_launch("made_wgrad_assemble_kernel");
}
