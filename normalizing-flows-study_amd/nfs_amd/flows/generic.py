"""Any-shape path for conditioner MLPs (csrc/nfx_generic.hip).

The fused layer kernels cover bounded shape families (a whole conditioner held in registers and
LDS). A layer beyond them runs its conditioner one nn.Linear at a time through the gfx950 GEMM
kernels (`nfx_linear_*`, fp32 MFMA) with HBM-resident activations, plus the layer's element
kernel. These helpers are the host side of that sequence; every call is a HIP launch.
"""
import torch

from .. import _lib


def linear_forward(x, lin, in_scale=None, relu=False, wmask=None, post=None):
    """relu?(((x * in_scale) @ (lin.weight * wmask).T + lin.bias) * post[0] + post[1]) — one
    nn.Linear / MaskedLinear (+ folded eval BatchNorm, + ReLU) on MFMA."""
    M, K = x.shape
    N = lin.out_features
    y = torch.empty(M, N, device=x.device, dtype=torch.float32)
    w = lin.weight.detach()
    b = None if lin.bias is None else lin.bias.detach()
    ps, pt = (None, None) if post is None else post
    _lib.check(_lib.lib().nfx_linear_forward(_lib.ptr(x), _lib.ptr(w), _lib.ptr(wmask), _lib.ptr(b),
                                             _lib.ptr(in_scale), _lib.ptr(ps), _lib.ptr(pt), _lib.ptr(y),
                                             M, K, N, int(bool(relu)), _lib.stream_of(x)), "nfx_linear_forward")
    return y


def linear_backward_data(gy, lin, act=None, out_scale=None, out=None, wmask=None):
    """(gy @ (lin.weight * wmask)) * out_scale, masked where act <= 0 (the ReLU feeding this
    Linear); added into `out` when given."""
    M, N = gy.shape
    K = lin.in_features
    acc = out is not None
    if out is None:
        out = torch.empty(M, K, device=gy.device, dtype=torch.float32)
    _lib.check(_lib.lib().nfx_linear_backward_data(_lib.ptr(gy), _lib.ptr(lin.weight.detach()), _lib.ptr(wmask),
                                                   _lib.ptr(act), _lib.ptr(out_scale), _lib.ptr(out), M, N, K,
                                                   int(acc), _lib.stream_of(gy)), "nfx_linear_backward_data")
    return out


def linear_backward_weight(gy, x, lin, in_scale=None, wmask=None):
    """(dL/dweight, dL/dbias) of one nn.Linear / MaskedLinear: (gy^T (x * in_scale)) * wmask,
    column sums of gy."""
    M, N = gy.shape
    K = lin.in_features
    L = _lib.lib()
    gw = torch.empty(N, K, device=gy.device, dtype=torch.float32)
    gb = None if lin.bias is None else torch.empty(N, device=gy.device, dtype=torch.float32)
    ws = torch.empty(max(1, L.nfx_linear_workspace_bytes(M, N, K)), device=gy.device, dtype=torch.uint8)
    _lib.check(L.nfx_linear_backward_weight(_lib.ptr(gy), _lib.ptr(x), _lib.ptr(in_scale), _lib.ptr(wmask),
                                            _lib.ptr(gw), _lib.ptr(gb), M, N, K, _lib.ptr(ws), _lib.stream_of(gy)),
               "nfx_linear_backward_weight")
    return gw, gb


def mlp3_forward(x, l1, l2, l3, in_scale):
    """Linear -> ReLU -> Linear -> ReLU -> Linear on (x * in_scale): (h1, h2, out)."""
    h1 = linear_forward(x, l1, in_scale, relu=True)
    h2 = linear_forward(h1, l2, relu=True)
    return h1, h2, linear_forward(h2, l3)


def mlp3_backward(x, l1, l2, l3, in_scale, h1, h2, g3, gx, out_scale=None):
    """Backward of mlp3_forward given dL/dout = g3: parameter gradients in parameters() order
    (l1.weight, l1.bias, l2.weight, l2.bias, l3.weight, l3.bias); dL/dx (times out_scale, default
    in_scale) is added into gx."""
    gw3, gb3 = linear_backward_weight(g3, h2, l3)
    g2 = linear_backward_data(g3, l3, act=h2)
    gw2, gb2 = linear_backward_weight(g2, h1, l2)
    g1 = linear_backward_data(g2, l2, act=h1)
    gw1, gb1 = linear_backward_weight(g1, x, l1, in_scale)
    linear_backward_data(g1, l1, out_scale=in_scale if out_scale is None else out_scale, out=gx)
    return [gw1, gb1, gw2, gb2, gw3, gb3]


def made_forward(x, lins, masks, posts):
    """MADE conditioner (made.py:136-140): MaskedLinear (+ eval BatchNorm) + ReLU three times, then
    the output MaskedLinear. Returns (h1, h2, h3, params [B, 2d])."""
    h1 = linear_forward(x, lins[0], relu=True, wmask=masks[0], post=posts[0])
    h2 = linear_forward(h1, lins[1], relu=True, wmask=masks[1], post=posts[1])
    h3 = linear_forward(h2, lins[2], relu=True, wmask=masks[2], post=posts[2])
    return h1, h2, h3, linear_forward(h3, lins[3], wmask=masks[3])


def made_input_vjp(gp, lins, masks, h1, h2, h3, out):
    """dL/d(MADE input) for dL/dparams = gp (no BatchNorm), added into `out`."""
    g = linear_backward_data(gp, lins[3], act=h3, wmask=masks[3])
    g = linear_backward_data(g, lins[2], act=h2, wmask=masks[2])
    g = linear_backward_data(g, lins[1], act=h1, wmask=masks[1])
    return linear_backward_data(g, lins[0], wmask=masks[0], out=out)


def made_backward(x, lins, masks, h1, h2, h3, gp, gx):
    """Backward of made_forward (no BatchNorm) given dL/dparams = gp: parameter gradients in
    parameters() order; dL/dx is added into gx (skipped when gx is None)."""
    g4 = linear_backward_weight(gp, h3, lins[3], wmask=masks[3])
    g = linear_backward_data(gp, lins[3], act=h3, wmask=masks[3])
    g3 = linear_backward_weight(g, h2, lins[2], wmask=masks[2])
    g = linear_backward_data(g, lins[2], act=h2, wmask=masks[2])
    g2 = linear_backward_weight(g, h1, lins[1], wmask=masks[1])
    g = linear_backward_data(g, lins[1], act=h1, wmask=masks[1])
    g1 = linear_backward_weight(g, x, lins[0], wmask=masks[0])
    if gx is not None:
        linear_backward_data(g, lins[0], wmask=masks[0], out=gx)
    return [*g1, *g2, *g3, *g4]


class _LinRows:
    """Output rows [r0, r1) of an nn.Linear / MaskedLinear (contiguous views of weight and bias)."""

    def __init__(self, lin, r0, r1):
        self.weight = lin.weight[r0:r1]
        self.bias = None if lin.bias is None else lin.bias[r0:r1]
        self.in_features = lin.in_features
        self.out_features = r1 - r0


def made_backward_rows(x, lins, masks, h1, h2, h3, gp_rows, r0, r1, gx, grads=None):
    """made_backward for a dL/dparams that is zero outside output columns [r0, r1) (gp_rows: those
    columns, contiguous [B, r1 - r0]; e.g. one ARQS step's spline row): the output layer's weight
    and data gradients run on its rows [r0, r1) only, not on all of them. The parameter gradients
    are accumulated into `grads` (parameters() order, full shapes; created when None) and
    returned; dL/dx is added into gx."""
    l4 = _LinRows(lins[3], r0, r1)
    m4 = masks[3][r0:r1]
    gw4, gb4 = linear_backward_weight(gp_rows, h3, l4, wmask=m4)
    g = linear_backward_data(gp_rows, l4, act=h3, wmask=m4)
    g3 = linear_backward_weight(g, h2, lins[2], wmask=masks[2])
    g = linear_backward_data(g, lins[2], act=h2, wmask=masks[2])
    g2 = linear_backward_weight(g, h1, lins[1], wmask=masks[1])
    g = linear_backward_data(g, lins[1], act=h1, wmask=masks[1])
    g1 = linear_backward_weight(g, x, lins[0], wmask=masks[0])
    linear_backward_data(g, lins[0], wmask=masks[0], out=gx)
    if grads is None:
        grads = [*g1, *g2, *g3, torch.zeros_like(lins[3].weight, dtype=torch.float32),
                 None if lins[3].bias is None else torch.zeros_like(lins[3].bias, dtype=torch.float32)]
    else:
        for a, b in zip(grads[:6], [*g1, *g2, *g3]):
            if a is not None:
                a.add_(b)
    grads[6][r0:r1].add_(gw4)
    if gb4 is not None:
        grads[7][r0:r1].add_(gb4)
    return grads


# ---- MADE with BatchNorm1d (use_batch_norm=True): activations kept pre- and post-BatchNorm ------
def bn_apply_relu(z, t):
    """relu(z * scale + shift) with t = [mean, invstd, scale, shift] (nfx_bn_prepare)."""
    h = torch.empty_like(z)
    _lib.check(_lib.lib().nfx_bn_apply_relu(_lib.ptr(z), _lib.ptr(t[2]), _lib.ptr(t[3]), _lib.ptr(h), z.shape[0],
                                            z.shape[1], _lib.stream_of(z)), "nfx_bn_apply_relu")
    return h


def bn_backward(g, z, t, gamma, train, count, sums_hook=None):
    """dL/dz of BatchNorm + (dL/dgamma, dL/dbeta) as float64 sums; train: batch-statistics terms
    with the global sample count (device float64 pointer `count`), sums passed to `sums_hook`
    (SyncBN all-reduce) first."""
    L = _lib.lib()
    M, N = g.shape
    st = _lib.stream_of(g)
    sums = torch.empty(2, N, device=g.device, dtype=torch.float64)
    ws = torch.empty(max(1, L.nfx_bn_workspace_bytes(M, N)), device=g.device, dtype=torch.uint8)
    _lib.check(L.nfx_bn_backward_sums(_lib.ptr(g), _lib.ptr(z), _lib.ptr(t[0]), _lib.ptr(t[1]), _lib.ptr(sums), M, N,
                                      _lib.ptr(ws), st), "nfx_bn_backward_sums")
    if train and sums_hook is not None:
        sums_hook(sums)
    gz = torch.empty_like(g)
    _lib.check(L.nfx_bn_backward_apply(_lib.ptr(g), _lib.ptr(z), _lib.ptr(t[0]), _lib.ptr(t[1]), _lib.ptr(gamma),
                                       _lib.ptr(sums), _lib.ptr(count) if train else None, int(train), _lib.ptr(gz),
                                       M, N, st), "nfx_bn_backward_apply")
    return gz, sums


def made_bn_forward(x, lins, masks, bnp):
    """MADE with BatchNorm given each BatchNorm's [mean, invstd, scale, shift]: the pre-BatchNorm
    z and post-ReLU h of the three hidden layers, and the params."""
    acts, h = [], x
    for i in range(3):
        z = linear_forward(h, lins[i], wmask=masks[i])
        h = bn_apply_relu(z, bnp[i])
        acts.append((z, h))
    return acts, linear_forward(h, lins[3], wmask=masks[3])


def made_bn_backward(x, lins, masks, bns, bnp, acts, gp, gx, train=False, counts=None, sums_hook=None):
    """Backward of made_bn_forward given dL/dparams = gp: parameter gradients in parameters()
    order (Linear, BatchNorm per hidden layer, then the output Linear); dL/dx added into gx
    (skipped when None)."""
    w4 = linear_backward_weight(gp, acts[2][1], lins[3], wmask=masks[3])
    g = linear_backward_data(gp, lins[3], act=acts[2][1], wmask=masks[3])
    per = [None, None, None]
    for i in (2, 1, 0):
        z = acts[i][0]
        gz, sums = bn_backward(g, z, bnp[i], bns[i].weight.detach(), train, counts[i] if train else None, sums_hook)
        hin = x if i == 0 else acts[i - 1][1]
        wl = linear_backward_weight(gz, hin, lins[i], wmask=masks[i])
        if i > 0:
            g = linear_backward_data(gz, lins[i], act=hin, wmask=masks[i])
        elif gx is not None:
            linear_backward_data(gz, lins[0], wmask=masks[0], out=gx)
        per[i] = [wl[0], wl[1], sums[1].float(), sums[0].float()]
    return [*per[0], *per[1], *per[2], *w4]


def made_bn_input_vjp(gp, lins, masks, bns, bnp, acts, out):
    """dL/d(MADE input) through eval-mode BatchNorm (a fixed per-feature scale), added into out."""
    g = linear_backward_data(gp, lins[3], act=acts[2][1], wmask=masks[3])
    for i in (2, 1, 0):
        gz, _ = bn_backward(g, acts[i][0], bnp[i], bns[i].weight.detach(), False, None)
        if i > 0:
            g = linear_backward_data(gz, lins[i], act=acts[i - 1][1], wmask=masks[i])
        else:
            linear_backward_data(gz, lins[0], wmask=masks[0], out=out)
    return out
