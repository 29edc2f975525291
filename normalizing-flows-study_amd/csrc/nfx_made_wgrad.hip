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
    int nrs, ncs, task0;              // workgroup tasks: super blocks of <= 4 x 4 tiles
};
struct WgArgs {
    WgLayer l[4];
    int nl, T, NBT, TPC;  // layers, total tiles, total bias row blocks, workgroup tasks per chunk
};


__device__ __forceinline__ int wg_layer_of(const WgArgs& a, int t) {
    int k = 0;
#pragma unroll
    for (int j = 1; j < 4; ++j)
        if (j < a.nl && t >= a.l[j].tile0) k = j;
    return k;
}

// One workgroup = (sample chunk, layer, super block of <= 4 x 4 output tiles). Per 32-sample step
// the rows its tiles need — <= 128 δ rows and <= 128 input rows, 128 bytes each — are read from
// HBM ONCE (coalesced 16-byte loads, 8 per row segment) into a double-buffered LDS stage (row
// stride 36 floats: the 16-byte operand reads of 32 different rows are conflict-free), the next
// step's loads in flight while the 4 waves run their tiles' MFMAs from LDS (each wave <= 4 tiles,
// 16 MFMAs per tile per step: lane (i, kh) feeds samples 16 kh .. 16 kh + 15 of row i).
constexpr int kWgRS = 36;              // LDS row stride (floats)
constexpr int kWgStage = 256 * kWgRS;  // one buffer: <= 128 δ rows + <= 128 input rows

template <bool VEC4>
__global__ __launch_bounds__(256) void made_wgrad_kernel(WgArgs a, int64_t B, int64_t P, int64_t chunk,
                                                         int64_t ntasks, float* part) {
    extern __shared__ f32x4 lds4[];
    float* lds = reinterpret_cast<float*>(lds4);
    const int64_t task = blockIdx.x;
    if (task >= ntasks) return;
    const int T = a.T;
    const int64_t c = task / a.TPC;
    const int tk = (int)(task % a.TPC);
    int k = 0;
#pragma unroll
    for (int j = 1; j < 4; ++j)
        if (j < a.nl && tk >= a.l[j].task0) k = j;
#define WGF(f) (k == 0 ? a.l[0].f : (k == 1 ? a.l[1].f : (k == 2 ? a.l[2].f : a.l[3].f)))
    const float* Ldm = WGF(dm);
    const float* Lam = WGF(am);
    const bool has_b = WGF(gb) != nullptr;
    const int LM = WGF(M), LN = WGF(N), Ltn = WGF(tn), Ltm = WGF(tm), Ltile0 = WGF(tile0), Lbt0 = WGF(btile0);
    const int Lncs = WGF(ncs), Ltask0 = WGF(task0);
#undef WGF
    const int lt = tk - Ltask0, rs = lt / Lncs, cs = lt % Lncs;
    const int rb0 = 4 * rs, cb0 = 4 * cs;
    const int nrb = Ltm - rb0 < 4 ? Ltm - rb0 : 4, ncb = Ltn - cb0 < 4 ? Ltn - cb0 : 4;
    const int R = 32 * nrb, NR = R + 32 * ncb;  // staged rows: δ rows [0, R), input rows [R, NR)
    const int64_t s0 = c * chunk, s1 = (s0 + chunk < B) ? s0 + chunk : B;
    const int nsteps = (int)((s1 - s0 + 31) / 32);
    const int lane = lane_id(), i = lane & 31, kh = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nt = nrb * ncb;

    // staging: item = (row, 16-byte piece q) for items threadIdx.x + 256 j
    // two register sets: step s + 2 is loaded while step s computes and step s + 1 waits in
    // registers for its LDS buffer (HBM latency covered by two steps of MFMA work)
    auto load = [&](int step, f32x4 (&st)[8]) {
        const int64_t sb = s0 + 32 * (int64_t)step;
        const bool tail = sb + 32 > s1;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int item = threadIdx.x + 256 * j, row = item >> 3, q = item & 7;
            f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
            if (row < NR) {
                const bool dside = row < R;
                const int grow = dside ? 32 * rb0 + row : 32 * cb0 + row - R;
                if (grow < (dside ? LM : LN)) {
                    const float* src = (dside ? Ldm : Lam) + (int64_t)grow * P + sb + 4 * q;
                    if (VEC4 && !tail) {
                        v = *reinterpret_cast<const f32x4*>(src);
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = sb + 4 * q + e < s1 ? src[e] : 0.f;
                    }
                }
            }
            st[j] = v;
        }
    };
    auto stash = [&](int buf, const f32x4 (&st)[8]) {
        float* dst = lds + buf * kWgStage;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int item = threadIdx.x + 256 * j, row = item >> 3, q = item & 7;
            if (row < NR) *reinterpret_cast<f32x4*>(dst + row * kWgRS + 4 * q) = st[j];
        }
    };

    f32x16 acc[4];
    float bsum[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        acc[u] = f32x16{};
        bsum[u] = 0.f;
    }
    auto compute = [&](int step) {
        const float* buf = lds + (step & 1) * kWgStage;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int ti = wave + 4 * u;
            if (ti < nt) {
                const int ta = ti / ncb, tb = ti % ncb;
                const float* ar = buf + (32 * ta + i) * kWgRS + 16 * kh;
                const float* br = buf + (R + 32 * tb + i) * kWgRS + 16 * kh;
                const bool bias = has_b && cs == 0 && tb == 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const f32x4 av = *reinterpret_cast<const f32x4*>(ar + 4 * q);
                    const f32x4 bv = *reinterpret_cast<const f32x4*>(br + 4 * q);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        acc[u] = mfma32(av[e], bv[e], acc[u]);
                        if (bias) bsum[u] += av[e];
                    }
                }
            }
        }
    };
    f32x4 sa[8], sb2[8];
    load(0, sa);
    stash(0, sa);
    if (nsteps > 1) load(1, sa);
    __syncthreads();
    for (int step = 0; step < nsteps; step += 2) {
        // even step: sa holds step + 1
        if (step + 2 < nsteps) load(step + 2, sb2);
        compute(step);
        if (step + 1 < nsteps) stash((step + 1) & 1, sa);
        __syncthreads();
        if (step + 1 >= nsteps) break;
        // odd step: sb2 holds step + 2
        if (step + 3 < nsteps) load(step + 3, sa);
        compute(step + 1);
        if (step + 2 < nsteps) stash((step + 2) & 1, sb2);
        __syncthreads();
    }
    const int64_t len = (int64_t)T * 1024 + (int64_t)a.NBT * 32;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int ti = wave + 4 * u;
        if (ti < nt) {
            const int ta = ti / ncb, tb = ti % ncb;
            const int gt = Ltile0 + (rb0 + ta) * Ltn + cb0 + tb;
            float* o = part + c * len + (int64_t)gt * 1024 + lane * 16;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *reinterpret_cast<f32x4*>(o + 4 * q) = f32x4{acc[u][4 * q], acc[u][4 * q + 1], acc[u][4 * q + 2], acc[u][4 * q + 3]};
            if (has_b && cs == 0 && tb == 0) {
                const float other = __shfl_xor(bsum[u], 32, 64);
                if (kh == 0) part[c * len + (int64_t)T * 1024 + (int64_t)(Lbt0 + rb0 + ta) * 32 + i] = bsum[u] + other;
            }
        }
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

static int64_t wg_chunk(int64_t B, int TPC) {
    // about 1024 workgroups (4 per CU, one round at 2 resident per CU... 72 KB LDS each), chunks of
    // >= 512 samples, 32-aligned
    int64_t c = (B * TPC + 1023) / 1024;
    if (c < 512) c = 512;
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
    int64_t off = 0, tile = 0, bt = 0, task = 0;
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
        L.nrs = (L.tm + 3) / 4;
        L.ncs = (L.tn + 3) / 4;
        L.task0 = (int)task;
        task += L.nrs * L.ncs;
        L.gw = grads + off;
        off += (int64_t)M[k] * N[k];
        L.gb = grads + off;
        off += M[k];
    }
    a.nl = 4;
    a.T = (int)tile;
    a.NBT = (int)bt;
    a.TPC = (int)task;
    return a;
}

}  // namespace nfx

using namespace nfx;

extern "C" int64_t nfx_made_factor_pitch(int64_t B) { return B <= 0 ? 0 : B; }

extern "C" size_t nfx_made_wgrad_workspace_bytes(int64_t B, int d, int H) {
    if (B <= 0 || d <= 0 || H <= 0) return 0;
    const WgArgs a = wg_args(nullptr, B, d, H, nullptr, nullptr);
    const int64_t len = (int64_t)a.T * 1024 + (int64_t)a.NBT * 32;
    const int64_t chunk = wg_chunk(B, a.TPC);
    const int64_t nch = (B + chunk - 1) / chunk;
    return (size_t)(((nch * len * sizeof(float) + 255) & ~(size_t)255) + len * sizeof(double));
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
    const int64_t chunk = wg_chunk(B, a.TPC);
    const int64_t nch = (B + chunk - 1) / chunk;
    const int64_t ntasks = nch * a.TPC;
    float* part = reinterpret_cast<float*>(workspace);
    double* sums = reinterpret_cast<double*>(
        reinterpret_cast<char*>(workspace) + ((nch * len * sizeof(float) + 255) & ~(size_t)255));
    const size_t lds = 2 * (size_t)kWgStage * sizeof(float);
    const void* kp = P % 4 == 0 ? (const void*)made_wgrad_kernel<true> : (const void*)made_wgrad_kernel<false>;
    if (int rcl = prepare_lds(kp, lds)) return rcl;
    if (ntasks > 0x7fffffff) return set_error(NFX_EUNSUPPORTED, "made_backward_weights: too many tasks");
    if (P % 4 == 0)
        made_wgrad_kernel<true><<<(unsigned)ntasks, 256, lds, s>>>(a, B, P, chunk, ntasks, part);
    else
        made_wgrad_kernel<false><<<(unsigned)ntasks, 256, lds, s>>>(a, B, P, chunk, ntasks, part);
    int rc = check_launch("made_wgrad_kernel");
    if (rc) return rc;
    if ((rc = train_sum_finish(part, (int)nch, (int)len, sums, s))) return rc;
    made_wgrad_assemble_kernel<<<(int)((len + 255) / 256), 256, 0, s>>>(a, sums);
    return check_launch("made_wgrad_assemble_kernel");
}
