"""Affine coupling layer (RealNVP) — drop-in for src/flows/coupling/coupling_layer.py.

Same constructor, attributes (`data_dim`, `mask` buffer, `s_net`, `b_net`), initialisation and
state_dict keys as the reference `CouplingLayer` (coupling_layer.py:5-111). On a ROCm device
in eval mode the layer runs as ONE fused gfx950 kernel (csrc/nfx_affine*.hip): both conditioner
MLPs on fp32 MFMA with BatchNorm folded from its running statistics, the affine transform,
the NaN/Inf guards and the log-det.
"""
import torch
import torch.nn as nn

from .. import _lib
from .flow import HipFlow

MAX_D = 8
MAX_H = 128


class CouplingLayer(HipFlow):
    def __init__(self, data_dim, hidden_dim, mask):
        super().__init__()
        self.data_dim = data_dim
        self.register_buffer("mask", mask)
        # coupling_layer.py:18-35
        self.s_net = nn.Sequential(
            nn.Linear(data_dim, hidden_dim), nn.BatchNorm1d(hidden_dim), nn.ReLU(),
            nn.Linear(hidden_dim, hidden_dim), nn.BatchNorm1d(hidden_dim), nn.ReLU(),
            nn.Linear(hidden_dim, data_dim))
        self.b_net = nn.Sequential(
            nn.Linear(data_dim, hidden_dim), nn.BatchNorm1d(hidden_dim), nn.ReLU(),
            nn.Linear(hidden_dim, hidden_dim), nn.BatchNorm1d(hidden_dim), nn.ReLU(),
            nn.Linear(hidden_dim, data_dim))
        self._initialize_weights()

    def _initialize_weights(self):
        # coupling_layer.py:98-111
        for net in [self.s_net, self.b_net]:
            for layer in net[:-1]:
                if isinstance(layer, nn.Linear):
                    nn.init.xavier_normal_(layer.weight, gain=1.0)
                    if layer.bias is not None:
                        nn.init.zeros_(layer.bias)
        nn.init.zeros_(self.s_net[-1].weight)
        nn.init.zeros_(self.s_net[-1].bias)
        nn.init.zeros_(self.b_net[-1].weight)
        nn.init.zeros_(self.b_net[-1].bias)

    # -- composite (autograd / CPU / fp64) path: the reference math -------------------------
    def _torch_call(self, x, direction):
        mask = self.mask
        xa = x * mask
        s = torch.clamp(self.s_net(xa), min=-10.0, max=10.0)
        b = torch.clamp(self.b_net(xa), min=-10.0, max=10.0)
        if direction > 0:  # coupling_layer.py:40-68
            y = xa + (1 - mask) * (x * torch.exp(s) + b)
            ld = ((1 - mask) * s).sum(dim=1)
        else:  # coupling_layer.py:70-96
            y = xa + (1 - mask) * ((x - b) * torch.exp(-s))
            ld = ((1 - mask) * -s).sum(dim=1)
        y = torch.where(torch.isnan(y) | torch.isinf(y), torch.zeros_like(y), y)
        ld = torch.where(torch.isnan(ld) | torch.isinf(ld), torch.zeros_like(ld), ld)
        return y, ld

    # -- HIP path ---------------------------------------------------------------------------
    def _hidden(self):
        return self.s_net[0].out_features

    def _torch_only(self):
        # Train-mode BatchNorm normalises with batch statistics (batch-global), which a
        # per-sample fused kernel cannot reproduce; the eval hot path folds running stats.
        return any(bn.training or bn.running_mean is None for bn in self._batchnorms())

    def _hip_supported(self, x):
        d, H = self.data_dim, self._hidden()
        if x.dim() != 2 or x.shape[1] != d:
            return False, f"input shape {tuple(x.shape)} vs data_dim={d}"
        if d > MAX_D or H > MAX_H:
            return False, f"d={d} (<= {MAX_D}) H={H} (<= {MAX_H})"
        return True, ""

    def _build_pack(self, device):
        d, H = self.data_dim, self._hidden()
        L = _lib.lib()
        n = L.nfx_affine_packed_floats(d, H)
        packed = torch.empty(n, device=device, dtype=torch.float32)
        s_raw, k1 = _lib.mlp_raw([self.s_net[0], self.s_net[3], self.s_net[6]],
                                 [self.s_net[1], self.s_net[4]])
        b_raw, k2 = _lib.mlp_raw([self.b_net[0], self.b_net[3], self.b_net[6]],
                                 [self.b_net[1], self.b_net[4]])
        mask = self.mask.detach().to(device=device, dtype=torch.float32).contiguous()
        _lib.check(L.nfx_affine_pack(s_raw, b_raw, _lib.ptr(mask), d, H, _lib.ptr(packed),
                                     _lib.stream_of(packed)), "nfx_affine_pack")
        packed._nfx_keep = (k1, k2, mask)  # sources stay alive while the pack kernel is queued
        return packed

    def _hip_launch(self, x, out, log_det, direction, accumulate):
        packed = self._packed(x.device, self._build_pack)
        _lib.check(_lib.lib().nfx_affine_coupling(
            _lib.ptr(packed), _lib.ptr(x), _lib.ptr(out), _lib.ptr(log_det), x.shape[0],
            self.data_dim, self._hidden(), int(direction), int(bool(accumulate)),
            _lib.stream_of(x)), "nfx_affine_coupling")

    def _hip_launch_logprob(self, x, out, log_det, logp, sums, workspace, accumulate):
        packed = self._packed(x.device, self._build_pack)
        _lib.check(_lib.lib().nfx_affine_coupling_logprob(
            _lib.ptr(packed), _lib.ptr(x), _lib.ptr(out), _lib.ptr(log_det), _lib.ptr(logp),
            _lib.ptr(sums), _lib.ptr(workspace), x.shape[0], self.data_dim, self._hidden(),
            int(bool(accumulate)), _lib.stream_of(x)), "nfx_affine_coupling_logprob")
        return True
