"""ARQS — drop-in for src/flows/spline/arqs.py (autoregressive rational-quadratic spline flow).

Same constructor (:13-26; `layers` is accepted and unused, as in the reference), `conditioner`
= MADE(dim, hidden_dim, 3*num_bins-1, use_batch_norm), `_rescale_to_unit` /
`_rescale_from_unit` (:28-42) and state_dict keys. Both directions are sequential over the d
coordinates exactly as the reference writes them (forward :44-80, inverse :82-114): step i
runs the MADE on the partially filled output vector, views it as [B, d, 3K-1] and feeds row i
to the unit-interval spline of input column i. On a ROCm device the whole d-step loop is ONE
kernel launch (csrc/nfx_arqs*.hip); elsewhere (CPU, float64, train-mode BatchNorm) the same
steps run as torch ops.
"""
import torch
import torch.nn as nn

from .. import _lib
from .. import distributed as _dist
from . import generic as _generic
from .autoregressive import MADE, bn_train_supported, made_bn_eval_params, made_bn_train_call
from .flow import STATS, HipFlow
from .spline import _rqs_unit_torch

MAX_K = 11   # 3K-1 <= 32: one MFMA row tile of spline parameters per step
MAX_H = 128
# Tests: route every call through the any-shape path (csrc/nfx_generic.hip) even where the fused
# ARQS kernel exists, to pin it against the same fixtures.
FORCE_GENERIC = False


class ARQS(HipFlow):
    def __init__(self, dim, hidden_dim=128, num_bins=8, layers=2, data_min=None, data_max=None,
                 use_batch_norm=False):
        super().__init__()
        self.dim = dim
        self.data_dim = dim
        self.num_bins = num_bins
        self.data_min = data_min
        self.data_max = data_max
        self.conditioner = MADE(input_dim=dim, hidden_dim=hidden_dim,
                                output_dim_multiplier=3 * num_bins - 1, use_batch_norm=use_batch_norm)
        # rational_quadratic_spline's defaults (rational_quadratic_spline.py:4-13)
        self.min_bin_width = 1e-3
        self.min_bin_height = 1e-3
        self.min_derivative = 1e-3

    def _rescale_to_unit(self, x):
        if self.data_min is None or self.data_max is None:
            return x
        return (x - self.data_min) / (self.data_max - self.data_min)

    def _rescale_from_unit(self, x):
        if self.data_min is None or self.data_max is None:
            return x
        return x * (self.data_max - self.data_min) + self.data_min

    # -- composite (reference ops) -----------------------------------------------------------
    def _torch_call(self, x, direction):
        xr = self._rescale_to_unit(x)
        state = torch.zeros_like(xr)
        log_det = torch.zeros(x.size(0), device=x.device)  # default dtype, as :50 / :88
        b, d = x.shape
        R = 3 * self.num_bins - 1
        K = self.num_bins
        for i in range(self.dim):
            params = self.conditioner(state).view(b, d, R)
            o, l = _rqs_unit_torch(xr[:, i], params[:, i, :K], params[:, i, K:2 * K], params[:, i, 2 * K:],
                                   direction < 0, self.min_bin_width, self.min_bin_height,
                                   self.min_derivative)
            new = state.clone()
            new[:, i] = o
            state = new
            log_det += l
        return self._rescale_from_unit(state), log_det

    # -- HIP path ----------------------------------------------------------------------------
    def _torch_only(self):
        return any(bn.training for bn in self._batchnorms())

    def _rescale_scalars(self):
        if self.data_min is None or self.data_max is None:
            return 0, 0.0, 0.0
        lo, hi = self.data_min, self.data_max
        for v in (lo, hi):
            if torch.is_tensor(v) and v.numel() != 1:
                return None
        # fp32 tensors: the kernel's fp32(hi - lo) from the exact double difference equals the
        # reference's fp32 tensor subtraction
        return 1, float(lo), float(hi)

    def _hip_supported(self, x):
        d, H, K = self.dim, self.conditioner.hidden_dim, self.num_bins
        if x.dim() != 2 or x.shape[1] != d:
            return False, f"input shape {tuple(x.shape)} vs dim={d}"
        if K > MAX_K or K < 2:
            return False, f"K={K} (2..{MAX_K})"
        if not self._fused_family() and not self._generic_ok():
            return False, "data_min/data_max of a shape other than scalar or [dim]"
        return True, ""

    def _fused_family(self):
        """Shapes of the fused ARQS kernel (nfx_arqs*.hip: H <= 128, scalar bounds)."""
        return not FORCE_GENERIC and self.conditioner.hidden_dim <= MAX_H and self._rescale_scalars() is not None

    def _generic_ok(self):
        """The any-shape path: 2 <= K <= 11, bounds None, scalar or per-dimension."""
        if not 2 <= self.num_bins <= MAX_K:
            return False
        if self.data_min is None or self.data_max is None:
            return True
        return all((not torch.is_tensor(t)) or t.numel() in (1, self.dim) for t in (self.data_min, self.data_max))

    def _bounds(self, device):
        """[2][d] float32 on the device = data_min | data_max - data_min, rounded as the reference's
        _rescale_to_unit / _rescale_from_unit expressions (python floats in double, tensors in
        fp32), cached with the parameters (keyed on the bound objects too); None without bounds."""
        if self.data_min is None or self.data_max is None:
            return None
        key = (id(self.data_min), id(self.data_max), getattr(self.data_min, "_version", 0),
               getattr(self.data_max, "_version", 0))
        if self.__dict__.get("_nfx_bounds_key") != key:
            self.__dict__.pop("_nfx_bounds_pack_cache", None)
            object.__setattr__(self, "_nfx_bounds_key", key)
        return self._packed(device, self._build_bounds, slot="_nfx_bounds_pack_cache")

    def _build_bounds(self, device):
        cpu = lambda v: v.detach().cpu() if torch.is_tensor(v) else v  # noqa: E731
        lo, hi = cpu(self.data_min), cpu(self.data_max)
        rows = [torch.as_tensor(v, dtype=torch.float32).reshape(-1).expand(self.dim) for v in (lo, hi - lo)]
        return torch.stack(rows).to(device=device).contiguous()

    def _map(self, t, bounds, mode):
        out = torch.empty_like(t)
        _lib.check(_lib.lib().nfx_arqs_bounds(_lib.ptr(t), _lib.ptr(bounds), _lib.ptr(out), t.shape[0], self.dim,
                                              mode, _lib.stream_of(t)), "nfx_arqs_bounds")
        return out

    # -- any-shape path (csrc/nfx_generic.hip): the reference's d steps, MADE on MFMA GEMMs --------
    def _generic_pack(self, device):
        lins = self.conditioner.linears()
        masks = [lin.mask.detach().to(device=device, dtype=torch.float32).contiguous() for lin in lins]
        posts = [None, None, None]
        for i, bn in enumerate(self.conditioner.batchnorms()):
            sc = (bn.weight.detach() / torch.sqrt(bn.running_var.detach() + bn.eps)).float().contiguous()
            posts[i] = (sc, (bn.bias.detach() - bn.running_mean.detach() * sc).float().contiguous())
        return masks, posts

    def _generic_made(self, state):
        masks, posts = self._packed(state.device, self._generic_pack, slot="_nfx_generic_pack_cache")
        return masks, _generic.made_forward(state, self.conditioner.linears(), masks, posts)

    def _step(self, xr, prm, state, ld, gld, lam, gprm, gx, i, direction, mode):
        B, d = state.shape
        p = _lib.ptr
        _lib.check(_lib.lib().nfx_arqs_step(p(xr), p(prm), p(state), p(ld), p(gld), p(lam), p(gprm), p(gx), B, d,
                                            self.num_bins, i, int(direction), mode, float(self.min_bin_width),
                                            float(self.min_bin_height), float(self.min_derivative),
                                            _lib.stream_of(state)), "nfx_arqs_step")

    def _generic_forward_state(self, xr, direction, state=None, ld=None):
        """The reference's d steps (arqs.py:51-78 / :89-112) into `state` (zeroed first) with the
        step log-dets added into `ld`: returns (state, ld)."""
        state = torch.zeros_like(xr) if state is None else state.zero_()
        ld = torch.zeros(xr.shape[0], device=xr.device, dtype=torch.float32) if ld is None else ld
        for i in range(self.dim):
            _, (_, _, _, prm) = self._generic_made(state)
            self._step(xr, prm, state, ld, None, None, None, None, i, direction, 0)
        return state, ld

    def _generic_launch(self, x, out, log_det, direction, accumulate):
        bounds = self._bounds(x.device)
        if bounds is None:
            self._generic_forward_state(x, direction, out, log_det if accumulate else log_det.zero_())
            return
        state, _ = self._generic_forward_state(self._map(x, bounds, 0), direction, None,
                                               log_det if accumulate else log_det.zero_())
        _lib.check(_lib.lib().nfx_arqs_bounds(_lib.ptr(state), _lib.ptr(bounds), _lib.ptr(out), x.shape[0], self.dim,
                                              1, _lib.stream_of(x)), "nfx_arqs_bounds")

    # -- train-mode BatchNorm in the MADE: the reference's d calls, each with batch statistics -----
    def _dispatch(self, x, direction):
        if bn_train_supported(self.conditioner, x, self.dim) and self._generic_ok():
            STATS["hip"] += 1
            if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
                return _ArqsTrainFunction.apply(self, direction, x, *list(self.parameters()))
            return self._train_forward(x, direction)[:2]
        return super()._dispatch(x, direction)

    def _train_forward(self, x, direction):
        """Returns (y, ld, state, bnps, counts): each step's MADE call normalises with the batch
        statistics of the partial state and updates the running statistics (d updates)."""
        x = x.detach().contiguous()
        bounds = self._bounds(x.device)
        xr = x if bounds is None else self._map(x, bounds, 0)
        masks, _ = self._packed(x.device, self._generic_pack, slot="_nfx_generic_pack_cache")
        state = torch.zeros_like(xr)
        ld = torch.zeros(x.shape[0], device=x.device, dtype=torch.float32)
        bnps, counts = [], []
        for i in range(self.dim):
            prm, bnp, cnt = made_bn_train_call(self.conditioner, masks, state)
            self._step(xr, prm, state, ld, None, None, None, None, i, direction, 0)
            bnps.append(bnp)
            counts.append(cnt)
        y = state.clone() if bounds is None else self._map(state, bounds, 1)
        return y, ld, state, bnps, counts

    def _build_pack(self, device):
        d, H, K = self.dim, self.conditioner.hidden_dim, self.num_bins
        L = _lib.lib()
        packed = torch.empty(L.nfx_arqs_packed_floats(d, H, K), device=device, dtype=torch.float32)
        lins = self.conditioner.linears()
        bns = self.conditioner.batchnorms() or ()
        raw, keep = _lib.mlp_raw(lins, bns, masks=[lin.mask for lin in lins])
        _lib.check(L.nfx_arqs_pack(raw, d, H, K, _lib.ptr(packed), _lib.stream_of(packed)), "nfx_arqs_pack")
        packed._nfx_keep = keep
        return packed

    # -- backward (training): reverse-mode through the reference's d steps ------------------------
    def _hip_backward_ok(self, x, direction):
        bns = self.conditioner.batchnorms()
        if bns and any(bn.training or not bn.affine or bn.running_mean is None for bn in bns):
            return False  # (train mode runs _ArqsTrainFunction)
        return x.dtype == torch.float32 and self._generic_ok()

    def _hip_backward(self, x, gy, gld, direction, train=None):
        """dL/dx and the parameter gradients (parameters() order) of one call, reverse-mode through
        the reference's d steps: the state before step i is the final state with columns >= i
        zeroed (each column is written once), so step i's MADE is recomputed there (GEMMs; with
        BatchNorm: eval running statistics, or call i's own batch statistics when train =
        (state, bnps, counts) from _train_forward), its spline row differentiated (nfx_arqs_step
        mode 1: rqs_unit_adjoint), the MADE's weight gradients accumulated and its input VJP added
        into the running state adjoint. With bounds, dL/dstate = gy w and dL/dx = dL/dxr / w."""
        x = x.contiguous()
        B, d = x.shape
        gy = torch.zeros_like(x) if gy is None else gy.contiguous().float()
        gld = torch.zeros(B, device=x.device) if gld is None else gld.contiguous().float()
        bounds = self._bounds(x.device)
        xr = x if bounds is None else self._map(x, bounds, 0)
        if train is not None:
            state = train[0].clone()
        else:
            state, _ = self._generic_forward_state(xr, direction)
        lam = gy.clone() if bounds is None else self._map(gy, bounds, 3)
        gx = torch.empty_like(x)
        R = 3 * self.num_bins - 1
        gprm = torch.zeros(B, d * R, device=x.device, dtype=torch.float32)
        lins = self.conditioner.linears()
        bns = self.conditioner.batchnorms()
        if bns:
            masks, _ = self._packed(x.device, self._generic_pack, slot="_nfx_generic_pack_cache")
            eval_bnp = None if train is not None else self._packed(
                x.device, lambda dev: made_bn_eval_params(self.conditioner, dev), slot="_nfx_generic_bn_pack_cache")
        grads = None
        for i in reversed(range(d)):
            self._step(None, None, state, None, None, None, None, None, i, direction, 2)
            if bns:
                bnp = train[1][i] if train is not None else eval_bnp
                acts, prm = _generic.made_bn_forward(state, lins, masks, bnp)
                self._step(xr, prm, state, None, gld, lam, gprm, gx, i, direction, 1)
                gi = _generic.made_bn_backward(state, lins, masks, bns, bnp, acts, gprm, lam, train is not None,
                                               train[2][i] if train is not None else None,
                                               _dist.allreduce_bn_sums if train is not None else None)
            else:
                masks, (h1, h2, h3, prm) = self._generic_made(state)
                self._step(xr, prm, state, None, gld, lam, gprm, gx, i, direction, 1)
                # only step i's R output columns carry a gradient: the output layer's backward on
                # those rows alone (O(d R H B) per call instead of O(d^2 R H B))
                gsl = gprm[:, i * R:(i + 1) * R].contiguous()
                grads = _generic.made_backward_rows(state, lins, masks, h1, h2, h3, gsl, i * R, (i + 1) * R, lam,
                                                    grads)
                continue
            grads = gi if grads is None else [a.add_(b) for a, b in zip(grads, gi)]
        if bounds is not None:
            gx = self._map(gx, bounds, 2)
        return gx, grads

    def _hip_launch(self, x, out, log_det, direction, accumulate):
        if not self._fused_family():
            return self._generic_launch(x, out, log_det, direction, accumulate)
        packed = self._packed(x.device, self._build_pack)
        rescale, lo, hi = self._rescale_scalars()
        _lib.check(_lib.lib().nfx_arqs(
            _lib.ptr(packed), _lib.ptr(x), _lib.ptr(out), _lib.ptr(log_det), x.shape[0], self.dim,
            self.conditioner.hidden_dim, self.num_bins, float(self.min_bin_width),
            float(self.min_bin_height), float(self.min_derivative), rescale, lo, hi, int(direction),
            int(bool(accumulate)), _lib.stream_of(x)), "nfx_arqs")


class _ArqsTrainFunction(torch.autograd.Function):
    """ARQS with train-mode BatchNorm in the MADE: the reference's d calls, each normalising with
    the batch statistics of the partial state (running statistics updated d times), then the
    reverse sweep with each call's own statistics (ARQS._hip_backward(train=...))."""

    @staticmethod
    def forward(ctx, layer, direction, x, *params):
        y, ld, state, bnps, counts = layer._train_forward(x, direction)
        ctx.layer, ctx.direction, ctx.bnps, ctx.counts = layer, direction, bnps, counts
        ctx.save_for_backward(x, state)
        return y, ld

    @staticmethod
    def backward(ctx, gy, gld):
        x, state = ctx.saved_tensors
        gx, grads = ctx.layer._hip_backward(x.detach(), gy, gld, ctx.direction, train=(state, ctx.bnps, ctx.counts))
        STATS["hip"] += 1
        params = list(ctx.layer.parameters())
        return (None, None, gx, *[g if p.requires_grad else None for p, g in zip(params, grads)])
