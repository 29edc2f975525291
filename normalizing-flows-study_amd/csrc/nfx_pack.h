// Device-side weight folding shared by the *_pack kernels.
#pragma once
#include "nfx_common.h"

namespace nfx {

// Folded weight W'[row][col] of layer `layer` (0-based) of an MLP:
// MaskedLinear mask (w*m, masked_linear.py:18) then eval BatchNorm scale gamma/sqrt(rv+eps).
__device__ inline float mlp_weight(const NfxMlpRaw& net, int layer, int in_dim, int row, int col) {
    size_t idx = (size_t)row * in_dim + col;
    float w = net.w[layer][idx];
    if (net.mask[layer]) w = w * net.mask[layer][idx];
    if (layer < 3 && net.bn_w[layer]) {
        double a = (double)net.bn_w[layer][row] / sqrt((double)net.bn_rv[layer][row] + (double)net.bn_eps);
        return (float)(a * (double)w);
    }
    return w;
}

__device__ inline float mlp_bias(const NfxMlpRaw& net, int layer, int row) {
    float b = net.b[layer] ? net.b[layer][row] : 0.f;
    if (layer < 3 && net.bn_w[layer]) {
        double a = (double)net.bn_w[layer][row] / sqrt((double)net.bn_rv[layer][row] + (double)net.bn_eps);
        return (float)(a * ((double)b - (double)net.bn_rm[layer][row]) + (double)net.bn_b[layer][row]);
    }
    return b;
}

// Overflow-safe input bound of an MLP, computed by one block of up to 1024 threads (every thread
// gets the result; 8 threads per weight row). With n_l = max row sum |W'_l| and c_l = max |b'_l|, every partial sum of layer l is
// bounded by A_l = n_l*A_{l-1} + c_l (A_0 = max|x|): returns the largest A_0 keeping every
// A_l <= lim (0 when a weight or bias is non-finite). ReLU/clamps only shrink magnitudes, so
// inputs within the bound produce finite activations everywhere.
__device__ inline double block_mlp_tsafe(const NfxMlpRaw& net, int nl, const int* rows, const int* cols,
                                         double lim, double* red /* [>= 2 * waves] shared */) {
    double alpha = 1.0, beta = 0.0, tsafe = 3.0e38;
    for (int l = 0; l < nl; ++l) {
        double nmax = 0.0, cmax = 0.0;
        // 8 threads per row, each over a strided slice of the columns: independent loads in
        // flight instead of one serial row walk per thread
        for (int r0 = 0; r0 < rows[l]; r0 += (int)(blockDim.x >> 3)) {
            const int r = r0 + (threadIdx.x >> 3), q = threadIdx.x & 7;
            double sum = 0.0;
            if (r < rows[l])
                for (int c = q; c < cols[l]; c += 8) sum += fabs((double)mlp_weight(net, l, cols[l], r, c));
            sum += __shfl_xor(sum, 1);
            sum += __shfl_xor(sum, 2);
            sum += __shfl_xor(sum, 4);
            if (r < rows[l]) {
                nmax = (sum > nmax || sum != sum) ? sum : nmax;
                const double b = fabs((double)mlp_bias(net, l, r));
                cmax = (b > cmax || b != b) ? b : cmax;
            }
        }
        // NaN-propagating max over the block: within each wave by shuffles, then the 4 wave
        // results through LDS (two barriers instead of one per tree level)
        auto nmaxd = [](double a, double b) { return (b > a || b != b) ? b : a; };
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            nmax = nmaxd(nmax, __shfl_xor(nmax, o));
            cmax = nmaxd(cmax, __shfl_xor(cmax, o));
        }
        const int wv = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) {
            red[2 * wv] = nmax;
            red[2 * wv + 1] = cmax;
        }
        __syncthreads();
        nmax = red[0];
        cmax = red[1];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
            nmax = nmaxd(nmax, red[2 * w]);
            cmax = nmaxd(cmax, red[2 * w + 1]);
        }
        __syncthreads();
        alpha = nmax * alpha;
        beta = nmax * beta + cmax;
        if (!(beta < lim) || !(alpha < 1e300)) tsafe = 0.0;
        else if (alpha > 0.0) tsafe = fmin(tsafe, (lim - beta) / alpha);
    }
    return tsafe;
}

}  // namespace nfx
