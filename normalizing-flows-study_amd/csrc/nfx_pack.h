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

}  // namespace nfx
