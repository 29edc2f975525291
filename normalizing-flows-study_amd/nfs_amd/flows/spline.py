"""Rational-quadratic spline coupling — drop-in for src/flows/spline/spline_coupling_layer.py.

`SplineCouplingLayer` keeps the reference constructor (spline_coupling_layer.py:13-23),
attributes, `param_net` (Linear -> ReLU -> Linear -> ReLU -> Linear, no BatchNorm, :56-62),
initialisation (:311-323) and state_dict keys. On a ROCm device it runs as ONE fused gfx950
kernel per call (csrc/nfx_spline*.hip): param MLP on fp32 MFMA, softmax/softplus/knots,
bin search, the RQ spline (forward or citardauq inverse), guards and log-det.

`rational_quadratic_spline` is the stand-alone unit-interval spline of
src/flows/spline/rational_quadratic_spline.py:4-104 (elementwise kernel nfx_rqs_unit on GPU).
"""
import ctypes
import os

import torch
import torch.nn as nn
from torch.nn import functional as F

from .. import _lib
from . import generic as _generic
from .flow import HipFlow, STATS

MAX_K = 11        # 3K-1 <= 32: one MFMA row tile of spline parameters per transformed dim
MAX_D = 64        # spline_coupling_kernel (d <= 8) / spline_wide_kernel (d <= 64)
MAX_D_BWD = 8     # fused backward
MAX_H = 128
MAX_H_BWD = 64    # fused backward: dW accumulators of <= 2 (H <= 32) / 1 (H <= 64) transformed dims
# Tests: route every call through the any-shape path (GEMM conditioner + element kernels,
# csrc/nfx_generic.hip) even where a fused kernel exists, to pin it against the same fixtures.
FORCE_GENERIC = False
# (kernel-name, start-event, end-event) of every fused backward while a list is installed here
# (bench.py roofline timing); None = no events.
BACKWARD_EVENTS = None


def _cum_knots(w, bound):
    """Prepend 0 to cumsum(w) along bins, map to [-bound, bound], pin the ends
    (spline_coupling_layer.py:208-213)."""
    c = F.pad(torch.cumsum(w, dim=-1), pad=(1, 0), mode="constant", value=0.0)
    c = (2 * bound) * c + (-bound)
    c = torch.cat([torch.full_like(c[..., :1], -bound), c[..., 1:-1], torch.full_like(c[..., :1], bound)], dim=-1)
    return c


def rq_spline_bounded(inputs, uw, uh, ud, inverse, num_bins, bound, min_w, min_h, min_d):
    """Composite form of SplineCouplingLayer._rational_quadratic_spline (:182-309).

    inputs [B, n]; uw/uh [B, n, K]; ud [B, n, K-1] -> (outputs [B, n], logabsdet [B, n])."""
    eps = 1e-8
    inside = (inputs >= -bound) & (inputs <= bound)
    outputs = torch.where(~inside, inputs, torch.zeros_like(inputs))
    logabsdet = torch.zeros_like(inputs)
    if not bool(inside.any()):
        return outputs, logabsdet

    w = torch.clamp(min_w + (1 - min_w * num_bins) * F.softmax(uw, dim=-1), min=eps)
    cw = _cum_knots(w, bound)
    w = torch.clamp(cw[..., 1:] - cw[..., :-1], min=eps)
    h = torch.clamp(min_h + (1 - min_h * num_bins) * F.softmax(uh, dim=-1), min=eps)
    ch = _cum_knots(h, bound)
    h = torch.clamp(ch[..., 1:] - ch[..., :-1], min=eps)
    dv = torch.clamp(min_d + F.softplus(ud), min=eps)
    dv = F.pad(dv, pad=(1, 1), mode="constant", value=1.0)

    flat = inputs.contiguous().view(-1)
    knots = (ch if inverse else cw).contiguous().view(-1, num_bins + 1)
    k = torch.searchsorted(knots, flat.unsqueeze(-1), right=True).squeeze(-1) - 1
    k = torch.clamp(k, 0, num_bins - 1)

    def pick(t, idx):
        return torch.gather(t.contiguous().view(-1, t.shape[-1]), 1, idx.unsqueeze(-1)).squeeze(-1)

    w_k, x_k, h_k, y_k = pick(w, k), pick(cw, k), pick(h, k), pick(ch, k)
    d_k = pick(dv, k)
    d_k1 = pick(dv, (k + 1).clamp(max=dv.shape[-1] - 1))
    s_k = h_k / torch.clamp(w_k, min=eps)

    if inverse:
        dy = flat - y_k
        a = dy * (d_k + d_k1 - 2 * s_k) + h_k * (s_k - d_k)
        b = h_k * d_k - dy * (d_k + d_k1 - 2 * s_k)
        c = -s_k * dy
        disc = torch.clamp(b.pow(2) - 4 * a * c, min=0.0)
        den = -b - torch.sqrt(disc)
        den = torch.where(den.abs() < eps, torch.full_like(den, eps), den)
        xi = torch.clamp((2 * c) / den, 0, 1)
        out = xi * w_k + x_k
        den_ld = s_k + (d_k1 + d_k - 2 * s_k) * xi * (1 - xi)
        num_ld = s_k.pow(2) * (d_k1 * xi.pow(2) + 2 * s_k * xi * (1 - xi) + d_k * (1 - xi).pow(2))
        lad = -torch.log(torch.clamp(num_ld, min=eps)) + 2 * torch.log(torch.clamp(den_ld, min=eps))
    else:
        xi = torch.clamp((flat - x_k) / torch.clamp(w_k, min=eps), 0, 1)
        den = torch.clamp(s_k + (d_k1 + d_k - 2 * s_k) * xi * (1 - xi), min=eps)
        out = y_k + h_k * (s_k * xi.pow(2) + d_k * xi * (1 - xi)) / den
        num_d = s_k.pow(2) * (d_k1 * xi.pow(2) + 2 * s_k * xi * (1 - xi) + d_k * (1 - xi).pow(2))
        lad = torch.log(torch.clamp(num_d / torch.clamp(den.pow(2), min=eps), min=eps))

    sel = inside.view(-1)
    outputs = outputs.clone().view(-1)
    logabsdet = logabsdet.clone().view(-1)
    outputs[sel] = out[sel]
    logabsdet[sel] = lad[sel]
    outputs = outputs.view_as(inputs)
    logabsdet = logabsdet.view_as(inputs)
    outputs = torch.where(torch.isnan(outputs) | torch.isinf(outputs), inputs, outputs)
    logabsdet = torch.where(torch.isnan(logabsdet) | torch.isinf(logabsdet), torch.zeros_like(logabsdet), logabsdet)
    return outputs, logabsdet


class SplineCouplingLayer(HipFlow):
    def __init__(self, data_dim, hidden_dim, mask, num_bins=10, bound=5.0, min_bin_width=1e-3,
                 min_bin_height=1e-3, min_derivative=1e-3, data_min=None, data_max=None):
        super().__init__()
        self.data_dim = data_dim
        self.num_bins = num_bins
        self.bound = bound
        self.min_bin_width = min_bin_width
        self.min_bin_height = min_bin_height
        self.min_derivative = min_derivative
        self.data_min = data_min
        self.data_max = data_max
        self.register_buffer("mask", mask)
        self.param_net = nn.Sequential(
            nn.Linear(data_dim, hidden_dim), nn.ReLU(),
            nn.Linear(hidden_dim, hidden_dim), nn.ReLU(),
            nn.Linear(hidden_dim, data_dim * (3 * num_bins - 1)))
        self._initialize_weights()

    def _initialize_weights(self):
        for layer in self.param_net[:-1]:
            if isinstance(layer, nn.Linear):
                nn.init.xavier_normal_(layer.weight, gain=1.0)
                if layer.bias is not None:
                    nn.init.zeros_(layer.bias)
        final = self.param_net[-1]
        nn.init.zeros_(final.weight)
        if final.bias is not None:
            nn.init.zeros_(final.bias)

    def _get_spline_params(self, z_a):
        params = self.param_net(z_a).view(-1, self.data_dim, 3 * self.num_bins - 1)
        return torch.split(params, [self.num_bins, self.num_bins, self.num_bins - 1], dim=-1)

    def _rescale_to_spline(self, x):
        if self.data_min is None or self.data_max is None:
            return x
        scale = (2 * self.bound) / (self.data_max - self.data_min)
        return scale * (x - self.data_min) - self.bound

    def _rescale_from_spline(self, x):
        if self.data_min is None or self.data_max is None:
            return x
        scale = (self.data_max - self.data_min) / (2 * self.bound)
        return (x + self.bound) * scale + self.data_min

    def _rational_quadratic_spline(self, inputs, unnormalized_widths, unnormalized_heights,
                                   unnormalized_derivatives, inverse=False):
        return rq_spline_bounded(inputs, unnormalized_widths, unnormalized_heights,
                                 unnormalized_derivatives, inverse, self.num_bins, self.bound,
                                 self.min_bin_width, self.min_bin_height, self.min_derivative)

    # -- composite path (spline_coupling_layer.py:96-180) -------------------------------------
    def _torch_call(self, x, direction):
        xr = self._rescale_to_spline(x)
        uw, uh, ud = self._get_spline_params(xr * self.mask)
        sel = self.mask == 0
        yb, ldb = self._rational_quadratic_spline(xr[:, sel], uw[:, sel], uh[:, sel], ud[:, sel],
                                                  inverse=direction < 0)
        yb = self._rescale_from_spline(yb)
        y = x.clone()
        y[:, sel] = yb
        ld = ldb.sum(dim=1)
        y = torch.where(torch.isnan(y) | torch.isinf(y), torch.zeros_like(y), y)
        ld = torch.where(torch.isnan(ld) | torch.isinf(ld), torch.zeros_like(ld), ld)
        return y, ld

    # -- HIP path -------------------------------------------------------------------------------
    def _hidden(self):
        return self.param_net[0].out_features

    def _rescale_scalars(self):
        if self.data_min is None or self.data_max is None:
            return 0, 0.0, 0.0
        lo, hi = self.data_min, self.data_max
        if torch.is_tensor(lo):
            if lo.numel() != 1:
                return None
            lo = float(lo)
        if torch.is_tensor(hi):
            if hi.numel() != 1:
                return None
            hi = float(hi)
        return 1, float(lo), float(hi)

    def _hip_supported(self, x):
        d, H, K = self.data_dim, self._hidden(), self.num_bins
        if x.dim() != 2 or x.shape[1] != d:
            return False, f"input shape {tuple(x.shape)} vs data_dim={d}"
        if self._fused_family() or self._generic_ok():
            return True, ""
        return False, (f"d={d} H={H} K={K}: fused kernels need d <= {MAX_D}, H <= {MAX_H}, K <= {MAX_K}; "
                       f"the any-shape path needs 2 <= K <= {MAX_K} and scalar or [d] data_min/data_max")

    def _fused_family(self):
        """Shapes of the fused eval kernels (spline_coupling_kernel / spline_wide_kernel): scalar
        bounds only (per-dimension ones take the any-shape path)."""
        return (not FORCE_GENERIC and self.data_dim <= MAX_D and self._hidden() <= MAX_H
                and 1 <= self.num_bins <= MAX_K and self._rescale_scalars() is not None)

    def _generic_ok(self):
        """The any-shape path (csrc/nfx_generic.hip): GEMM conditioner + spline element kernels,
        with scalar or per-dimension data_min/data_max bounds (nfx_spline_elem_*_bounded)."""
        if not 2 <= self.num_bins <= MAX_K:
            return False
        if self.data_min is None or self.data_max is None:
            return True
        return all((not torch.is_tensor(t)) or t.numel() in (1, self.data_dim) for t in (self.data_min, self.data_max))

    def _bounds(self, device):
        """[4][d] float32 on the device = data_min | 2B/(max - min) | (max - min)/(2B) | mask * to,
        the first three evaluated exactly as the reference's _rescale_to_spline /
        _rescale_from_spline expressions (python floats in double, tensors in their fp32 ops; rows
        0-2 are nfx_spline_elem_*_bounded's `bounds`, row 3 maps the conditioner's dL/dxr to dL/dx),
        cached with the parameters and buffers (keyed on the bound objects too); None without
        bounds."""
        if self.data_min is None or self.data_max is None:
            return None
        key = (id(self.data_min), id(self.data_max), getattr(self.data_min, "_version", 0),
               getattr(self.data_max, "_version", 0))
        c = self.__dict__.get("_nfx_bounds_key")
        if c != key:
            self.__dict__.pop("_nfx_bounds_pack_cache", None)
            object.__setattr__(self, "_nfx_bounds_key", key)
        return self._packed(device, self._build_bounds, slot="_nfx_bounds_pack_cache")

    def _build_bounds(self, device):
        lo, hi, d = self.data_min, self.data_max, self.data_dim
        cpu = lambda v: v.detach().cpu() if torch.is_tensor(v) else v  # noqa: E731
        lo, hi = cpu(lo), cpu(hi)
        to = (2 * self.bound) / (hi - lo)
        fr = (hi - lo) / (2 * self.bound)
        rows = [torch.as_tensor(v, dtype=torch.float32).reshape(-1).expand(d) for v in (lo, to, fr)]
        rows.append(self.mask.detach().cpu().float() * rows[1])
        return torch.stack(rows).to(device=device).contiguous()

    def _mask_dev(self, device):
        m = self.mask
        return m.detach().to(device=device, dtype=torch.float32).contiguous()

    def _generic_params(self, x, bounds=None):
        """Conditioner recompute on the any-shape path: (mask, conditioner input, h1, h2, params
        [B, d(3K-1)]); with bounds the input is the rescaled x (nfx_spline_rescale)."""
        mask = self._mask_dev(x.device)
        xin = x
        if bounds is not None:
            xin = torch.empty_like(x)
            _lib.check(_lib.lib().nfx_spline_rescale(_lib.ptr(x), _lib.ptr(bounds), _lib.ptr(xin), x.shape[0],
                                                     self.data_dim, float(self.bound), _lib.stream_of(x)),
                       "nfx_spline_rescale")
        h1, h2, prm = _generic.mlp3_forward(xin, self.param_net[0], self.param_net[2], self.param_net[4], mask)
        return mask, xin, h1, h2, prm

    def _spline_scalars(self):
        return (float(self.bound), float(self.min_bin_width), float(self.min_bin_height),
                float(self.min_derivative))

    def _generic_launch(self, x, out, log_det, direction, accumulate):
        bounds = self._bounds(x.device)
        mask, _, _, _, prm = self._generic_params(x, bounds)
        L = _lib.lib()
        if bounds is None:
            _lib.check(L.nfx_spline_elem_forward(
                _lib.ptr(x), _lib.ptr(prm), _lib.ptr(mask), _lib.ptr(out), _lib.ptr(log_det), x.shape[0],
                self.data_dim, self.num_bins, *self._spline_scalars(), int(direction), int(bool(accumulate)),
                _lib.stream_of(x)), "nfx_spline_elem_forward")
        else:
            _lib.check(L.nfx_spline_elem_forward_bounded(
                _lib.ptr(x), _lib.ptr(prm), _lib.ptr(mask), _lib.ptr(bounds), _lib.ptr(out), _lib.ptr(log_det),
                x.shape[0], self.data_dim, self.num_bins, *self._spline_scalars(), int(direction),
                int(bool(accumulate)), _lib.stream_of(x)), "nfx_spline_elem_forward_bounded")

    def _generic_backward(self, x, gy, gld, direction):
        """dL/dx and parameter gradients on the any-shape path: conditioner recompute (GEMMs),
        the spline adjoint per element (nfx_spline_elem_backward), then the conditioner's
        backward GEMMs (data gradient into dL/dx, weight gradients split over the batch)."""
        B, d = x.shape
        bounds = self._bounds(x.device)
        mask, xin, h1, h2, prm = self._generic_params(x, bounds)
        gprm = torch.empty_like(prm)
        gx = torch.empty_like(x)
        L = _lib.lib()
        if bounds is None:
            _lib.check(L.nfx_spline_elem_backward(
                _lib.ptr(x), _lib.ptr(prm), _lib.ptr(mask), _lib.ptr(gy), _lib.ptr(gld), _lib.ptr(gprm),
                _lib.ptr(gx), B, d, self.num_bins, *self._spline_scalars(), int(direction), _lib.stream_of(x)),
                "nfx_spline_elem_backward")
            out_scale = None
        else:
            _lib.check(L.nfx_spline_elem_backward_bounded(
                _lib.ptr(x), _lib.ptr(prm), _lib.ptr(mask), _lib.ptr(bounds), _lib.ptr(gy), _lib.ptr(gld),
                _lib.ptr(gprm), _lib.ptr(gx), B, d, self.num_bins, *self._spline_scalars(), int(direction),
                _lib.stream_of(x)), "nfx_spline_elem_backward_bounded")
            out_scale = bounds[3]
        grads = _generic.mlp3_backward(xin, self.param_net[0], self.param_net[2], self.param_net[4], mask, h1, h2,
                                       gprm, gx, out_scale=out_scale)
        return gx, grads

    def _build_pack(self, device):
        d, H, K = self.data_dim, self._hidden(), self.num_bins
        L = _lib.lib()
        packed = torch.empty(L.nfx_spline_packed_floats(d, H, K), device=device, dtype=torch.float32)
        raw, keep = _lib.mlp_raw([self.param_net[0], self.param_net[2], self.param_net[4]])
        mask = self.mask.detach().to(device=device, dtype=torch.float32).contiguous()
        _lib.check(L.nfx_spline_pack(raw, _lib.ptr(mask), d, H, K, _lib.ptr(packed),
                                     _lib.stream_of(packed)), "nfx_spline_pack")
        packed._nfx_keep = (keep, mask)
        return packed

    # -- fused backward (training) ---------------------------------------
    def _hip_backward_ok(self, x, direction):
        return x.dtype == torch.float32 and (self._fused_backward_ok() or self._generic_ok())

    def _fused_backward_ok(self):
        """Shapes of the fused backward kernel (spline_bwd_kernel); others take the any-shape
        path (_generic_backward)."""
        d, H, K = self.data_dim, self._hidden(), self.num_bins
        nt = self._n_transformed()
        ntmax = 2 if H <= 32 else 1
        return (not FORCE_GENERIC and d <= MAX_D_BWD and H <= MAX_H_BWD and 2 <= K <= MAX_K and nt <= ntmax
                and (self.data_min is None or self.data_max is None))  # bounds: the any-shape path

    def _n_transformed(self):
        """Number of transformed (mask == 0) dimensions, cached per mask version (no sync)."""
        m = self.mask
        key = (m.data_ptr(), m._version)
        c = self.__dict__.get("_nfx_nt")
        if c is None or c[0] != key:
            c = (key, int((m == 0).sum()))
            object.__setattr__(self, "_nfx_nt", c)
        return c[1]

    def _build_bwd_pack(self, device):
        d, H, K = self.data_dim, self._hidden(), self.num_bins
        L = _lib.lib()
        packed = torch.empty(L.nfx_spline_backward_packed_floats(d, H, K), device=device, dtype=torch.float32)
        raw, keep = _lib.mlp_raw([self.param_net[0], self.param_net[2], self.param_net[4]])
        mask = self.mask.detach().to(device=device, dtype=torch.float32).contiguous()
        _lib.check(L.nfx_spline_pack_backward(raw, _lib.ptr(mask), d, H, K, _lib.ptr(packed),
                                              _lib.stream_of(packed)), "nfx_spline_pack_backward")
        packed._nfx_keep = (keep, mask)
        return packed, mask

    def _hip_backward(self, x, gy, gld, direction):
        """dL/dx and the parameter gradients (parameters() order) of one forward/inverse call:
        nfx_spline_coupling_backward (MLP recompute, spline adjoint, data-gradient chain and the
        weight-gradient contractions in one kernel, then a fixed-order workgroup reduction)."""
        x = x.contiguous()
        B, d = x.shape
        H, K = self._hidden(), self.num_bins
        gy = torch.zeros_like(x) if gy is None else gy.contiguous().float()
        gld = torch.zeros(B, device=x.device) if gld is None else gld.contiguous().float()
        if not self._fused_backward_ok():
            return self._generic_backward(x, gy, gld, direction)
        packed, mask = self._packed(x.device, self._build_bwd_pack, slot="_nfx_bwd_pack_cache")
        L = _lib.lib()
        gx = torch.empty_like(x)
        grads = torch.empty(L.nfx_spline_backward_param_floats(d, H, K), device=x.device, dtype=torch.float32)
        ws = torch.empty(L.nfx_spline_backward_workspace_bytes(B, d, H, K), device=x.device, dtype=torch.uint8)
        nt = self._n_transformed()
        ev = BACKWARD_EVENTS
        if ev is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        _lib.check(L.nfx_spline_coupling_backward(
            _lib.ptr(packed), _lib.ptr(mask), _lib.ptr(x), _lib.ptr(gy), _lib.ptr(gld), _lib.ptr(gx),
            _lib.ptr(grads), _lib.ptr(ws), B, d, H, K, nt, float(self.bound), float(self.min_bin_width),
            float(self.min_bin_height), float(self.min_derivative), int(direction), _lib.stream_of(x)),
            "nfx_spline_coupling_backward")
        if ev is not None:
            e1.record()
            ev.append(("spline_bwd_kernel", e0, e1))
        out, o = [], 0
        for prm in self.parameters():
            n = prm.numel()
            out.append(grads[o:o + n].view_as(prm))
            o += n
        grads._nfx_keep = ws
        return gx, out

    def _hip_launch(self, x, out, log_det, direction, accumulate):
        if not self._fused_family():
            return self._generic_launch(x, out, log_det, direction, accumulate)
        packed = self._packed(x.device, self._build_pack)
        rescale, lo, hi = self._rescale_scalars()
        _lib.check(_lib.lib().nfx_spline_coupling(
            _lib.ptr(packed), _lib.ptr(x), _lib.ptr(out), _lib.ptr(log_det), x.shape[0],
            self.data_dim, self._hidden(), self.num_bins, float(self.bound),
            float(self.min_bin_width), float(self.min_bin_height), float(self.min_derivative),
            rescale, lo, hi, int(direction), int(bool(accumulate)), _lib.stream_of(x)),
            "nfx_spline_coupling")

    def _hip_launch_logprob(self, x, out, log_det, logp, sums, workspace, accumulate):
        if not self._fused_family():
            return False
        packed = self._packed(x.device, self._build_pack)
        rescale, lo, hi = self._rescale_scalars()
        _lib.check(_lib.lib().nfx_spline_coupling_logprob(
            _lib.ptr(packed), _lib.ptr(x), _lib.ptr(out), _lib.ptr(log_det), _lib.ptr(logp),
            _lib.ptr(sums), _lib.ptr(workspace), x.shape[0], self.data_dim, self._hidden(),
            self.num_bins, float(self.bound), float(self.min_bin_width),
            float(self.min_bin_height), float(self.min_derivative), rescale, lo, hi,
            int(bool(accumulate)), _lib.stream_of(x)), "nfx_spline_coupling_logprob")
        return True


# One-launch chains of SplineCouplingLayers (nfx_spline_chain, csrc/nfx_spline_schain_kernel.h) run
# every batch of at least this many samples (0 = every batch); NFX_SPLINE_CHAIN_MIN_B overrides,
# tests set CHAIN_ENABLED = False to compare with the per-layer kernels.
CHAIN_ENABLED = True
CHAIN_MIN_B = int(os.environ.get("NFX_SPLINE_CHAIN_MIN_B", "0"))


def chain_ok(flows, x):
    """A run of eval-mode SplineCouplingLayers, d = 2, one (H, K, bound, minimums), no rescale, on
    fp32 ROCm rows that nfx_spline_chain takes."""
    if not CHAIN_ENABLED or FORCE_GENERIC or not flows or len(flows) > 64 or x.shape[0] < max(1, CHAIN_MIN_B):
        return False
    return _chain_key_ok(flows, x)


def chain_launch(flows, x, out, ld, direction, accumulate, logprob=None):
    """All `flows` (module order) in one nfx_spline_chain launch; logprob=(logp, sums, workspace)
    adds the fused Gaussian log-density to an inverse chain."""
    packs = (ctypes.c_void_p * len(flows))(*[_lib.ptr(f._packed(x.device, f._build_pack)) for f in flows])
    f0 = flows[0]
    L = _lib.lib()
    p = _lib.ptr
    consts = (float(f0.bound), float(f0.min_bin_width), float(f0.min_bin_height), float(f0.min_derivative))
    if logprob is not None:
        logp, sums, ws = logprob
        _lib.check(L.nfx_spline_chain_logprob(packs, len(flows), p(x), p(out), p(ld), p(logp), p(sums), p(ws),
                                              x.shape[0], f0.data_dim, f0._hidden(), f0.num_bins, *consts,
                                              int(bool(accumulate)), _lib.stream_of(x)), "nfx_spline_chain_logprob")
    else:
        _lib.check(L.nfx_spline_chain(packs, len(flows), p(x), p(out), p(ld), x.shape[0], f0.data_dim, f0._hidden(),
                                      f0.num_bins, *consts, int(direction), int(bool(accumulate)), _lib.stream_of(x)),
                   "nfx_spline_chain")
    STATS["hip"] += 1


def sample_chain_ok(flows, n, device):
    """chain_ok for the fused sampling pass (nfx_spline_chain_sample): eval-mode d = 2
    SplineCouplingLayers of one (H, K, bound, minimums), no rescale, n rows, a ROCm device."""
    if not CHAIN_ENABLED or FORCE_GENERIC or not flows or len(flows) > 64 or n <= 0:
        return False
    if torch.device(device).type != "cuda" or any(getattr(f, "training", False) for f in flows):
        return False
    probe = torch.empty(n, flows[0].data_dim if hasattr(flows[0], "data_dim") else 0, device="meta")
    return _chain_key_ok(flows, probe)


def _chain_key_ok(flows, x):
    f0 = flows[0]
    if type(f0) is not SplineCouplingLayer:
        return False
    key = (f0.data_dim, f0._hidden(), f0.num_bins, float(f0.bound), float(f0.min_bin_width),
           float(f0.min_bin_height), float(f0.min_derivative))
    if x.dim() != 2 or x.shape[1] != f0.data_dim:
        return False
    for f in flows:
        if type(f) is not SplineCouplingLayer or f._torch_only() or not f._fused_family():
            return False
        if f._rescale_scalars() != (0, 0.0, 0.0):
            return False
        if (f.data_dim, f._hidden(), f.num_bins, float(f.bound), float(f.min_bin_width), float(f.min_bin_height),
                float(f.min_derivative)) != key:
            return False
    return bool(_lib.lib().nfx_spline_chain_supported(x.shape[0], key[0], key[1], key[2]))


def chain_sample(flows, rng_state, seed, z, x, ld):
    """z ~ N(0, I) drawn on the device and x, ld = forward(z) through every flow, one launch
    (nfx_spline_chain_sample); rng_state = the device uint64[2] generator state it advances."""
    packs = (ctypes.c_void_p * len(flows))(*[_lib.ptr(f._packed(x.device, f._build_pack)) for f in flows])
    f0 = flows[0]
    p = _lib.ptr
    _lib.check(_lib.lib().nfx_spline_chain_sample(
        packs, len(flows), int(seed) & ((1 << 64) - 1), p(rng_state), p(z), p(x), p(ld), x.shape[0], f0.data_dim,
        f0._hidden(), f0.num_bins, float(f0.bound), float(f0.min_bin_width), float(f0.min_bin_height),
        float(f0.min_derivative), _lib.stream_of(x)), "nfx_spline_chain_sample")
    STATS["hip"] += 1


def _rqs_unit_torch(inputs, widths, heights, derivatives, inverse, min_bin_width,
                    min_bin_height, min_derivative):
    """Composite of rational_quadratic_spline.py:4-104 (epsilon forced to 1e-6, :19)."""
    eps = 1e-6
    K = widths.shape[-1]
    w = torch.clamp(min_bin_width + (1 - min_bin_width * K) * F.softmax(widths, dim=-1), min=eps)
    h = torch.clamp(min_bin_height + (1 - min_bin_height * heights.shape[-1]) * F.softmax(heights, dim=-1), min=eps)
    dv = torch.clamp(F.softplus(derivatives) + min_derivative, min=eps)
    xk = F.pad(torch.cumsum(w, dim=-1), (1, 0), "constant", 0.0)
    yk = F.pad(torch.cumsum(h, dim=-1), (1, 0), "constant", 0.0)
    dv = F.pad(dv, (1, 1), "constant", 1.0)
    knots = (yk if inverse else xk).contiguous()
    if knots.dim() > 2:
        knots = knots.view(-1, knots.shape[-1])
    idx = torch.clamp(torch.searchsorted(knots, inputs.unsqueeze(-1), right=True) - 1, 0, K - 1)
    x_k, y_k = torch.gather(xk, -1, idx), torch.gather(yk, -1, idx)
    w_k, h_k = torch.gather(w, -1, idx), torch.gather(h, -1, idx)
    d_k, d_k1 = torch.gather(dv, -1, idx), torch.gather(dv, -1, idx + 1)
    s_k = h_k / torch.clamp(w_k, min=eps)
    u = inputs.unsqueeze(-1)
    if inverse:
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
    else:
        th = torch.clamp((u - x_k) / torch.clamp(w_k, min=eps), 0, 1)
        tt = th * (1 - th)
        den = s_k + (d_k + d_k1 - 2 * s_k) * tt
        out = y_k + h_k * (s_k * th.pow(2) + d_k * tt) / torch.clamp(den, min=eps)
        num = s_k.pow(2) * (d_k1 * th.pow(2) + 2 * s_k * tt + d_k * (1 - th).pow(2))
        ld = torch.log(torch.clamp(num / torch.clamp(den.pow(2), min=eps), min=eps))
    return out.squeeze(-1), ld.squeeze(-1)


def rational_quadratic_spline(inputs, widths, heights, derivatives, inverse=False,
                              min_bin_width=1e-3, min_bin_height=1e-3, min_derivative=1e-3,
                              epsilon=1e-6):
    """Unit-interval RQ spline (src/flows/spline/rational_quadratic_spline.py:4-104).

    Elementwise over inputs of any shape S with widths/heights [*S, K] and derivatives
    [*S, K - 1]. fp32 on a ROCm device runs the gfx950 kernels — nfx_rqs_unit forward and, under
    autograd, nfx_rqs_unit_backward (gradients for inputs and all three parameter tensors); CPU
    tensors run the composite. A GPU call outside the kernels (another dtype, K outside 2..16,
    shapes that need broadcasting) raises NotImplementedError / ValueError, as every layer does,
    unless nfs_amd.flows.flow.ALLOW_TORCH_FALLBACK is set."""
    if inputs.device.type != "cuda":
        STATS["torch"] += 1
        return _rqs_unit_torch(inputs, widths, heights, derivatives, inverse, min_bin_width,
                               min_bin_height, min_derivative)
    from . import flow as _flow
    K = widths.shape[-1] if widths.dim() else 0
    S = tuple(inputs.shape)
    why = None
    if any(t.dtype != torch.float32 for t in (inputs, widths, heights, derivatives)):
        why = "fp32 tensors only"
    elif not 2 <= K <= 16:
        why = f"K={K} outside 2..16"
    elif (tuple(widths.shape) != S + (K,) or tuple(heights.shape) != S + (K,)
          or tuple(derivatives.shape) != S + (K - 1,)):
        if not _flow.ALLOW_TORCH_FALLBACK:
            raise ValueError(f"rational_quadratic_spline: inputs {S} need widths/heights {S + (K,)} and "
                             f"derivatives {S + (K - 1,)} (got {tuple(widths.shape)}, {tuple(heights.shape)}, "
                             f"{tuple(derivatives.shape)}; broadcasting is not supported on the GPU)")
        why = "broadcast shapes"
    if why is not None:
        if not _flow.ALLOW_TORCH_FALLBACK:
            raise NotImplementedError(f"rational_quadratic_spline: no gfx950 kernel for this call ({why}); "
                                      f"set nfs_amd.flows.flow.ALLOW_TORCH_FALLBACK=True to run eager PyTorch")
        STATS["torch"] += 1
        return _rqs_unit_torch(inputs, widths, heights, derivatives, inverse, min_bin_width,
                               min_bin_height, min_derivative)
    consts = (float(min_bin_width), float(min_bin_height), float(min_derivative), bool(inverse))
    if torch.is_grad_enabled() and any(t.requires_grad for t in (inputs, widths, heights, derivatives)):
        return _RqsUnitFn.apply(inputs, widths, heights, derivatives, consts)
    out, ld = _rqs_unit_hip(inputs.reshape(-1), widths.reshape(-1, K), heights.reshape(-1, K),
                            derivatives.reshape(-1, K - 1), *consts)
    return out.view(S), ld.view(S)


def _rqs_unit_hip(inputs, widths, heights, derivatives, min_w, min_h, min_d, inverse):
    N = inputs.shape[0]
    K = widths.shape[-1]
    x = inputs.contiguous()
    uw, uh, ud = widths.contiguous(), heights.contiguous(), derivatives.contiguous()
    out = torch.empty_like(x)
    ld = torch.empty_like(x)
    _lib.check(_lib.lib().nfx_rqs_unit(
        _lib.ptr(x), _lib.ptr(uw), _lib.ptr(uh), _lib.ptr(ud), _lib.ptr(out), _lib.ptr(ld), N, K,
        float(min_w), float(min_h), float(min_d), int(bool(inverse)), _lib.stream_of(x)),
        "nfx_rqs_unit")
    STATS["hip"] += 1
    return out, ld


class _RqsUnitFn(torch.autograd.Function):
    """The unit RQ spline under autograd: nfx_rqs_unit forward, nfx_rqs_unit_backward (the
    elementwise adjoint of rational_quadratic_spline.py:4-104) backward."""

    @staticmethod
    def forward(ctx, inputs, widths, heights, derivatives, consts):
        S, K = tuple(inputs.shape), widths.shape[-1]
        x = inputs.reshape(-1).contiguous()
        uw = widths.reshape(-1, K).contiguous()
        uh = heights.reshape(-1, K).contiguous()
        ud = derivatives.reshape(-1, K - 1).contiguous()
        out, ld = _rqs_unit_hip(x, uw, uh, ud, *consts)
        ctx.save_for_backward(x, uw, uh, ud)
        ctx.consts, ctx.S = consts, S
        return out.view(S), ld.view(S)

    @staticmethod
    def backward(ctx, g_out, g_ld):
        x, uw, uh, ud = ctx.saved_tensors
        min_w, min_h, min_d, inverse = ctx.consts
        N, K = x.shape[0], uw.shape[1]
        go = torch.zeros_like(x) if g_out is None else g_out.reshape(-1).contiguous().float()
        gl = torch.zeros_like(x) if g_ld is None else g_ld.reshape(-1).contiguous().float()
        gx, gw, gh, gd = torch.empty_like(x), torch.empty_like(uw), torch.empty_like(uh), torch.empty_like(ud)
        p = _lib.ptr
        _lib.check(_lib.lib().nfx_rqs_unit_backward(
            p(x), p(uw), p(uh), p(ud), p(go), p(gl), p(gx), p(gw), p(gh), p(gd), N, K, min_w, min_h, min_d,
            int(inverse), _lib.stream_of(x)), "nfx_rqs_unit_backward")
        STATS["hip"] += 1
        S = ctx.S
        return gx.view(S), gw.view(S + (K,)), gh.view(S + (K,)), gd.view(S + (K - 1,)), None
