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
from .autoregressive import MADE
from .flow import HipFlow
from .spline import _rqs_unit_torch

MAX_K = 11   # 3K-1 <= 32: one MFMA row tile of spline parameters per step
MAX_H = 128


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
        if H > MAX_H or K > MAX_K or K < 2:
            return False, f"H={H} (<= {MAX_H}) K={K} (2..{MAX_K})"
        if self._rescale_scalars() is None:
            return False, "per-dimension data_min/data_max tensors"
        return True, ""

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

    def _hip_launch(self, x, out, log_det, direction, accumulate):
        packed = self._packed(x.device, self._build_pack)
        rescale, lo, hi = self._rescale_scalars()
        _lib.check(_lib.lib().nfx_arqs(
            _lib.ptr(packed), _lib.ptr(x), _lib.ptr(out), _lib.ptr(log_det), x.shape[0], self.dim,
            self.conditioner.hidden_dim, self.num_bins, float(self.min_bin_width),
            float(self.min_bin_height), float(self.min_derivative), rescale, lo, hi, int(direction),
            int(bool(accumulate)), _lib.stream_of(x)), "nfx_arqs")
