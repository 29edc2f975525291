"""CPU oracle of the reference hot path (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

Every function restates one reference routine op for op, on a state dict `sd` keyed exactly
like the reference module's state_dict (prefix = the module's path). All citations are to
/root/reference (itxtx/normalizing-flows-study).
"""
import math

import torch
import torch.nn.functional as F

__all__ = [
    "made_degrees", "made_masks", "coupling", "spline_coupling", "rqs_unit", "made", "made_bn", "maf", "iaf", "arqs",
    "flow_model", "sequential_flow", "gauss_log_prob", "nll_f64", "realnvp_spec", "spline_model_spec", "maf_spec",
]


# ---------------------------------------------------------------------------------------------
# MADE degrees / masks — src/flows/autoregressive/made.py:24-41 (degrees), :47-79 (masks)
# ---------------------------------------------------------------------------------------------
def made_degrees(d, H):
    """m[0] of MADE (made.py:28-39) with numpy's float64 linspace written out:
    y_i = i * ((d-1)/(H-1)) (float64), y_{H-1} = d-1, degree = floor(y_i)."""
    if d <= 1:
        return [0] * H
    if d == 2:
        return ([0, 0, 1, 1] * (H // 4 + 1))[:H]
    if H == 1:
        return [0]
    step = float(d - 1) / float(H - 1)
    deg = [math.floor(float(i) * step) for i in range(H)]
    deg[-1] = d - 1
    return deg


def made_masks(d, H, mult=2):
    """(M1 [H,d], Mhh [H,H], M2 [mult*d, H]) as uint8 (made.py:56, :63, :72-78)."""
    m0 = torch.tensor(made_degrees(d, H), dtype=torch.int64)
    mi = torch.arange(d)
    m1 = (mi[None, :] <= m0[:, None]).to(torch.uint8)
    mhh = (m0[None, :] <= m0[:, None]).to(torch.uint8)
    m2 = (m0[None, :] < mi[:, None]).to(torch.uint8).repeat(mult, 1)
    return m1, mhh, m2


# ---------------------------------------------------------------------------------------------
# Affine coupling — src/flows/coupling/coupling_layer.py:40-96
# ---------------------------------------------------------------------------------------------
def _coupling_net(sd, p, x, training=False):
    """Linear -> BatchNorm1d -> ReLU -> Linear -> BatchNorm1d -> ReLU -> Linear
    (coupling_layer.py:18-35). Eval: BatchNorm uses running statistics. training=True: batch
    statistics, and the running statistics in `sd` are updated in place (momentum 0.1), as
    nn.BatchNorm1d does in train mode."""
    h = F.linear(x, sd[p + "0.weight"], sd[p + "0.bias"])
    h = F.batch_norm(h, sd[p + "1.running_mean"], sd[p + "1.running_var"], sd[p + "1.weight"],
                     sd[p + "1.bias"], training, 0.1, 1e-5)
    h = F.relu(h)
    h = F.linear(h, sd[p + "3.weight"], sd[p + "3.bias"])
    h = F.batch_norm(h, sd[p + "4.running_mean"], sd[p + "4.running_var"], sd[p + "4.weight"],
                     sd[p + "4.bias"], training, 0.1, 1e-5)
    h = F.relu(h)
    return F.linear(h, sd[p + "6.weight"], sd[p + "6.bias"])


def coupling(sd, p, x, direction, training=False):
    m = sd[p + "mask"]
    xa = x * m
    s = torch.clamp(_coupling_net(sd, p + "s_net.", xa, training), min=-10.0, max=10.0)   # :50, :79
    b = torch.clamp(_coupling_net(sd, p + "b_net.", xa, training), min=-10.0, max=10.0)   # :51, :80
    if direction > 0:
        y = xa + (1 - m) * (x * torch.exp(s) + b)                                # :55
        ld = ((1 - m) * s).sum(dim=1)                                             # :58
    else:
        y = xa + (1 - m) * ((x - b) * torch.exp(-s))                             # :83
        ld = ((1 - m) * -s).sum(dim=1)                                            # :86
    y = torch.where(torch.isnan(y) | torch.isinf(y), torch.zeros_like(y), y)     # :61, :89
    ld = torch.where(torch.isnan(ld) | torch.isinf(ld), torch.zeros_like(ld), ld)
    return y, ld


# ---------------------------------------------------------------------------------------------
# RQ spline coupling — src/flows/spline/spline_coupling_layer.py:96-309
# ---------------------------------------------------------------------------------------------
def _knots(v, bound):
    c = F.pad(torch.cumsum(v, dim=-1), pad=(1, 0), mode="constant", value=0.0)    # :208-210
    c = (2 * bound) * c + (-bound)                                                 # :211
    c[..., 0] = -bound                                                             # :212
    c[..., -1] = bound                                                             # :213
    return c


def _rqs_bounded(x, uw, uh, ud, inverse, K, bound, min_w, min_h, min_d):
    eps = 1e-8                                                                     # :189
    inside = (x >= -bound) & (x <= bound)                                          # :192
    outputs = torch.where(~inside, x, torch.zeros_like(x))
    logabsdet = torch.zeros_like(x)
    if not inside.any():                                                           # :200
        return outputs, logabsdet
    w = torch.clamp(min_w + (1 - min_w * K) * F.softmax(uw, dim=-1), min=eps)      # :204-206
    cw = _knots(w, bound)
    w = torch.clamp(cw[..., 1:] - cw[..., :-1], min=eps)                           # :214-215
    h = torch.clamp(min_h + (1 - min_h * K) * F.softmax(uh, dim=-1), min=eps)      # :217-219
    ch = _knots(h, bound)
    h = torch.clamp(ch[..., 1:] - ch[..., :-1], min=eps)                           # :227-228
    dv = torch.clamp(min_d + F.softplus(ud), min=eps)                              # :230-231
    dv = F.pad(dv, pad=(1, 1), mode="constant", value=1.0)                         # :232
    fx = x.contiguous().view(-1)
    bnd = (ch if inverse else cw).contiguous().view(-1, K + 1)                     # :236-239
    k = torch.clamp(torch.searchsorted(bnd, fx.unsqueeze(-1), right=True).squeeze(-1) - 1, 0, K - 1)

    def g(t, idx):
        return torch.gather(t.contiguous().view(-1, t.shape[-1]), 1, idx.unsqueeze(-1)).squeeze(-1)

    w_k, z_k, h_k, y_k = g(w, k), g(cw, k), g(h, k), g(ch, k)                      # :254-257
    d_k = g(dv, k)
    d_k1 = g(dv, (k + 1).clamp(max=dv.shape[-1] - 1))                               # :259
    s_k = h_k / torch.clamp(w_k, min=eps)                                          # :260
    if inverse:                                                                    # :263-281
        a = (fx - y_k) * (d_k + d_k1 - 2 * s_k) + h_k * (s_k - d_k)
        b = h_k * d_k - (fx - y_k) * (d_k + d_k1 - 2 * s_k)
        c = -s_k * (fx - y_k)
        disc = torch.clamp(b.pow(2) - 4 * a * c, min=0.0)
        den = -b - torch.sqrt(disc)
        den = torch.where(den.abs() < eps, torch.full_like(den, eps), den)
        xi = torch.clamp((2 * c) / den, 0, 1)
        out = xi * w_k + z_k
        dld = s_k + (d_k1 + d_k - 2 * s_k) * xi * (1 - xi)
        nld = s_k.pow(2) * (d_k1 * xi.pow(2) + 2 * s_k * xi * (1 - xi) + d_k * (1 - xi).pow(2))
        lad = -torch.log(torch.clamp(nld, min=eps)) + 2 * torch.log(torch.clamp(dld, min=eps))
    else:                                                                          # :282-293
        xi = torch.clamp((fx - z_k) / torch.clamp(w_k, min=eps), 0, 1)
        den = torch.clamp(s_k + (d_k1 + d_k - 2 * s_k) * xi * (1 - xi), min=eps)
        out = y_k + h_k * (s_k * xi.pow(2) + d_k * xi * (1 - xi)) / den
        nd = s_k.pow(2) * (d_k1 * xi.pow(2) + 2 * s_k * xi * (1 - xi) + d_k * (1 - xi).pow(2))
        lad = torch.log(torch.clamp(nd / torch.clamp(den.pow(2), min=eps), min=eps))
    sel = inside.view(-1)                                                          # :298-303
    o = outputs.clone().view(-1)
    l = logabsdet.clone().view(-1)
    o[sel] = out[sel]
    l[sel] = lad[sel]
    o = o.view_as(x)
    l = l.view_as(x)
    o = torch.where(torch.isnan(o) | torch.isinf(o), x, o)                         # :306
    l = torch.where(torch.isnan(l) | torch.isinf(l), torch.zeros_like(l), l)       # :307
    return o, l


def spline_coupling(sd, p, x, direction, K=10, bound=5.0, min_w=1e-3, min_h=1e-3, min_d=1e-3,
                    data_min=None, data_max=None):
    d = x.shape[1]
    m = sd[p + "mask"]
    xr = x if data_min is None else (2 * bound) / (data_max - data_min) * (x - data_min) - bound
    h = F.relu(F.linear(xr * m, sd[p + "param_net.0.weight"], sd[p + "param_net.0.bias"]))
    h = F.relu(F.linear(h, sd[p + "param_net.2.weight"], sd[p + "param_net.2.bias"]))
    par = F.linear(h, sd[p + "param_net.4.weight"], sd[p + "param_net.4.bias"]).view(-1, d, 3 * K - 1)
    uw, uh, ud = torch.split(par, [K, K, K - 1], dim=-1)                           # :71-75
    sel = m == 0
    yb, lb = _rqs_bounded(xr[:, sel], uw[:, sel], uh[:, sel], ud[:, sel], direction < 0, K, bound,
                          min_w, min_h, min_d)
    if data_min is not None:
        yb = (yb + bound) * ((data_max - data_min) / (2 * bound)) + data_min
    y = x.clone()
    y[:, sel] = yb                                                                 # :125-126
    ld = lb.sum(dim=1)
    y = torch.where(torch.isnan(y) | torch.isinf(y), torch.zeros_like(y), y)      # :130
    ld = torch.where(torch.isnan(ld) | torch.isinf(ld), torch.zeros_like(ld), ld)
    return y, ld


# ---------------------------------------------------------------------------------------------
# Unit-interval RQS — src/flows/spline/rational_quadratic_spline.py:4-104
# ---------------------------------------------------------------------------------------------
def rqs_unit(x, uw, uh, ud, inverse=False, min_w=1e-3, min_h=1e-3, min_d=1e-3):
    eps = 1e-6                                                                     # :19
    K = uw.shape[-1]
    w = torch.clamp(min_w + (1 - min_w * K) * F.softmax(uw, dim=-1), min=eps)      # :22-28
    h = torch.clamp(min_h + (1 - min_h * K) * F.softmax(uh, dim=-1), min=eps)
    dv = torch.clamp(F.softplus(ud) + min_d, min=eps)                              # :32-33
    xk = F.pad(torch.cumsum(w, dim=-1), (1, 0), "constant", 0.0)                   # :36
    yk = F.pad(torch.cumsum(h, dim=-1), (1, 0), "constant", 0.0)                   # :37
    dv = F.pad(dv, (1, 1), "constant", 1.0)                                        # :40
    k = torch.searchsorted((yk if inverse else xk).contiguous(), x.unsqueeze(-1), right=True) - 1
    k = torch.clamp(k, 0, K - 1)                                                   # :56
    x_k, y_k = torch.gather(xk, -1, k), torch.gather(yk, -1, k)
    w_k, h_k = torch.gather(w, -1, k), torch.gather(h, -1, k)
    d_k, d_k1 = torch.gather(dv, -1, k), torch.gather(dv, -1, k + 1)
    s_k = h_k / torch.clamp(w_k, min=eps)                                          # :66
    u = x.unsqueeze(-1)
    if inverse:                                                                    # :70-87
        t1 = (u - y_k) * (d_k + d_k1 - 2 * s_k)
        a = h_k * (s_k - d_k) + t1
        b = h_k * d_k - t1
        c = -s_k * (u - y_k)
        disc = torch.clamp(b.pow(2) - 4 * a * c, min=0)
        th = torch.clamp((2 * c) / (-b - torch.sqrt(disc)), 0, 1)
        out = th * w_k + x_k
        tt = th * (1 - th)
        num = s_k.pow(2) * (d_k1 * th.pow(2) + 2 * s_k * tt + d_k * (1 - th).pow(2))
        den = (s_k + (d_k + d_k1 - 2 * s_k) * tt).pow(2)
        ld = -torch.log(torch.clamp(num / torch.clamp(den, min=eps), min=eps))
    else:                                                                          # :89-102
        th = torch.clamp((u - x_k) / torch.clamp(w_k, min=eps), 0, 1)
        tt = th * (1 - th)
        num = h_k * (s_k * th.pow(2) + d_k * tt)
        den = s_k + (d_k + d_k1 - 2 * s_k) * tt
        out = y_k + num / torch.clamp(den, min=eps)
        nd = s_k.pow(2) * (d_k1 * th.pow(2) + 2 * s_k * tt + d_k * (1 - th).pow(2))
        ld = torch.log(torch.clamp(nd / torch.clamp(den.pow(2), min=eps), min=eps))
    return out.squeeze(-1), ld.squeeze(-1)


# ---------------------------------------------------------------------------------------------
# MADE / MAF / IAF — made.py:81-140, masked_linear.py:14-18,
# masked_autoregressive_flow.py:18-78, inverse_autoregressive_flow.py:30-103
# ---------------------------------------------------------------------------------------------
def made(sd, p, x):
    """MaskedLinear x4 with ReLU between (use_batch_norm=False, made.py:87-114);
    each MaskedLinear is F.linear(x, W * mask, b) (masked_linear.py:18)."""
    h = x
    for i, idx in enumerate((0, 2, 4, 6)):
        q = f"{p}net.{idx}."
        h = F.linear(h, sd[q + "weight"] * sd[q + "mask"].to(sd[q + "weight"].dtype), sd[q + "bias"])
        if i < 3:
            h = F.relu(h)
    return h


def _net(batch_norm, training):
    """The MADE conditioner: made (use_batch_norm=False) or made_bn (eval / train mode)."""
    if not batch_norm:
        return made
    return lambda sd, p, x: made_bn(sd, p, x, training)


def maf(sd, p, x, direction, batch_norm=False, training=False):
    d = x.shape[1]
    made = _net(batch_norm, training)  # noqa: F823 - the conditioner of this layer
    if direction < 0:                                                              # :18-44
        mu, alpha = made(sd, p + "conditioner.", x).chunk(2, dim=1)
        alpha = torch.clamp(alpha, min=-3, max=3)
        z = (x - mu) * torch.exp(torch.clamp(-alpha, min=-5, max=5))
        ld = -torch.sum(alpha, dim=1)
        z = torch.where(torch.isnan(z) | torch.isinf(z), torch.zeros_like(z), z)
    else:                                                                          # :46-78
        z = torch.zeros_like(x)
        ld = torch.zeros(x.shape[0], dtype=x.dtype)
        for i in range(d):
            mu, alpha = made(sd, p + "conditioner.", z).chunk(2, dim=1)
            alpha = torch.clamp(alpha, min=-3, max=3)
            zn = z.clone()
            zn[:, i] = x[:, i] * torch.exp(torch.clamp(alpha[:, i], min=-5, max=5)) + mu[:, i]
            z = zn
            ld += alpha[:, i]
        z = torch.where(torch.isnan(z) | torch.isinf(z), torch.zeros_like(z), z)
    ld = torch.where(torch.isnan(ld) | torch.isinf(ld), torch.zeros_like(ld), ld)
    return z, torch.clamp(ld, min=-100, max=100)


def iaf(sd, p, x, direction, batch_norm=False, training=False):
    d = x.shape[1]
    made = _net(batch_norm, training)  # noqa: F823 - the conditioner of this layer
    if direction > 0:                                                              # :30-63
        mu, alpha = made(sd, p + "conditioner.", x).chunk(2, dim=1)
        alpha = torch.clamp(alpha, min=-2, max=2)
        mu = torch.clamp(mu, min=-10, max=10)
        y = x * torch.exp(torch.clamp(alpha, min=-3, max=3)) + mu
        ld = torch.sum(alpha, dim=1)
    else:                                                                          # :65-103
        y = torch.zeros_like(x)
        ld = torch.zeros(x.shape[0], dtype=x.dtype)
        for i in range(d):
            mu, alpha = made(sd, p + "conditioner.", y).chunk(2, dim=1)
            alpha = torch.clamp(alpha, min=-2, max=2)
            mu = torch.clamp(mu, min=-10, max=10)
            yn = y.clone()
            yn[:, i] = (x[:, i] - mu[:, i]) * torch.exp(torch.clamp(-alpha[:, i], min=-3, max=3))
            y = yn
            ld -= alpha[:, i]
    y = torch.where(torch.isnan(y) | torch.isinf(y), x, y)
    ld = torch.where(torch.isnan(ld) | torch.isinf(ld), torch.zeros_like(ld), ld)
    return y, torch.clamp(ld, min=-50, max=50)


# ---------------------------------------------------------------------------------------------
# ARQS — src/flows/spline/arqs.py:7-114 (MADE(d, H, 3K-1) conditioner + unit RQS, sequential)
# ---------------------------------------------------------------------------------------------
def made_bn(sd, p, x, training=False):
    """MADE with use_batch_norm=True: MaskedLinear -> BatchNorm1d -> ReLU (made.py:87-114). Eval:
    running statistics; training=True: batch statistics, and the running statistics in `sd`
    updated in place (momentum 0.1, unbiased variance), once per call as nn.BatchNorm1d does."""
    h = x
    idx = 0
    for i in range(4):
        q = f"{p}net.{idx}."
        h = F.linear(h, sd[q + "weight"] * sd[q + "mask"].to(sd[q + "weight"].dtype), sd[q + "bias"])
        idx += 1
        if i < 3:
            b = f"{p}net.{idx}."
            h = F.batch_norm(h, sd[b + "running_mean"], sd[b + "running_var"], sd[b + "weight"],
                             sd[b + "bias"], training, 0.1, 1e-5)
            h = F.relu(h)
            idx += 2
    return h


def arqs(sd, p, x, direction, K=8, data_min=None, data_max=None, batch_norm=False, training=False):
    B, d = x.shape
    R = 3 * K - 1
    net = _net(batch_norm, training)
    rescale = data_min is not None and data_max is not None
    xr = (x - data_min) / (data_max - data_min) if rescale else x                   # :28-34
    state = torch.zeros_like(xr)                                                    # :49 / :87
    ld = torch.zeros(B)                                                             # :50 / :88
    for i in range(d):                                                              # :52 / :90
        prm = net(sd, p + "conditioner.", state).view(B, d, R)                      # :54-58
        o, l = rqs_unit(xr[:, i], prm[:, i, :K], prm[:, i, K:2 * K], prm[:, i, 2 * K:],
                        inverse=direction < 0)                                       # :64-70
        sn = state.clone()                                                          # :72-74
        sn[:, i] = o
        state = sn
        ld += l
    out = state * (data_max - data_min) + data_min if rescale else state            # :36-42
    return out, ld


# ---------------------------------------------------------------------------------------------
# Model chaining — src/models/normalizing_flow_model.py:25-65 (batch_norm_between_layers=False)
# spec: list of (kind, prefix, kwargs); kind in {"coupling", "spline", "maf", "iaf"}
# ---------------------------------------------------------------------------------------------
_LAYER = {"coupling": coupling, "spline": spline_coupling, "maf": maf, "iaf": iaf, "arqs": arqs}


def flow_model(sd, spec, x, direction, bn_prefix=None, training=False):
    """NormalizingFlowModel.forward/inverse (src/models/normalizing_flow_model.py:25-65).

    bn_prefix (e.g. "flow.batch_norms.") enables the between-layer BatchNorm of layers
    i < n-1 (:35-44, :55-60, :67-128); training=True updates its running statistics in `sd` in
    place before the forward affine (:74-79)."""
    log_det_sum = 0                                   # :30 / :53 — python int, then f32 tensor
    n = len(spec)
    order = range(n) if direction > 0 else reversed(range(n))
    for i in order:
        kind, p, kw = spec[i]
        if direction < 0 and bn_prefix is not None and i < n - 1:
            q = f"{bn_prefix}{i}."
            x = _bn_inverse(sd, q, x)                                       # :58
            log_det_sum -= _bn_log_det(sd, q)                                # :60
        x, ld = _LAYER[kind](sd, p, x, direction, **kw)
        log_det_sum += ld
        if direction > 0 and bn_prefix is not None and i < n - 1:
            q = f"{bn_prefix}{i}."
            x = _bn_apply(sd, q, x, training)                               # :43
            log_det_sum += _bn_log_det(sd, q)                                # :44
    return x, log_det_sum


def _bn_apply(sd, q, x, training, momentum=0.1, eps=1e-5):
    """normalizing_flow_model.py:67-85: running-stat update in train mode, then the affine with
    the (updated) running statistics."""
    if training:
        with torch.no_grad():
            sd[q + "running_mean"].mul_(1 - momentum).add_(momentum * x.mean(dim=0))
            sd[q + "running_var"].mul_(1 - momentum).add_(momentum * x.var(dim=0, unbiased=False))
    gamma, beta = sd[q + "weight"].view(1, -1), sd[q + "bias"].view(1, -1)
    mean, var = sd[q + "running_mean"].view(1, -1), sd[q + "running_var"].view(1, -1)
    return (x - mean) / torch.sqrt(var + eps) * gamma + beta


def _bn_log_det(sd, q, eps=1e-5):
    """normalizing_flow_model.py:87-108: sum_j log|g_j| - 0.5 log(rv_j + eps) (a scalar)."""
    return (torch.log(torch.abs(sd[q + "weight"])) - 0.5 * torch.log(sd[q + "running_var"] + eps)).sum()


def _bn_inverse(sd, q, y, eps=1e-5):
    """normalizing_flow_model.py:110-128."""
    gamma, beta = sd[q + "weight"].view(1, -1), sd[q + "bias"].view(1, -1)
    mean, var = sd[q + "running_mean"].view(1, -1), sd[q + "running_var"].view(1, -1)
    return (y - beta) / gamma * torch.sqrt(var + eps) + mean


def sequential_flow(sd, spec, x, direction):
    """SequentialFlow.forward/inverse (src/flows/flow/sequential_flow.py:15-34): the accumulator
    is torch.zeros(B) (f32), layers in order (forward) or reverse order (inverse)."""
    total = torch.zeros(x.size(0))
    layers = spec if direction > 0 else list(reversed(spec))
    for kind, p, kw in layers:
        x, ld = _LAYER[kind](sd, p, x, direction, **kw)
        total += ld
    return x, total


def realnvp_spec(n_layers, prefix="flow.flows.", training=False):
    kw = {"training": True} if training else {}
    return [("coupling", f"{prefix}{i}.", kw) for i in range(n_layers)]


def spline_model_spec(n_layers, K=10, prefix="flow.flows."):
    return [("spline", f"{prefix}{i}.", {"K": K}) for i in range(n_layers)]


def maf_spec(n_layers, prefix="flows."):
    return [("maf", f"{prefix}{i}.", {}) for i in range(n_layers)]


# ---------------------------------------------------------------------------------------------
# log_prob glue — MultivariateNormal(0, I).log_prob(z) + log_det (README.md:113-114;
# src/utils.py:39-55; src/flows/flow/flow.py:67-73)
# ---------------------------------------------------------------------------------------------
def gauss_log_prob(z, ld):
    d = z.shape[1]
    return -0.5 * (d * math.log(2 * math.pi) + z.pow(2).sum(-1)) + ld


def nll_f64(logp):
    return -float(logp.double().mean())
