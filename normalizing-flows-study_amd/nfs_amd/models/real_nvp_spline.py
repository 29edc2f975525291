"""RealNVPSpline — drop-in for src/models/real_nvp_spline.py:6-48 (RQ-spline couplings, K=10)."""
import torch
import torch.nn as nn

from ..flows.spline import SplineCouplingLayer
from .normalizing_flow_model import NormalizingFlowModel


class RealNVPSpline(nn.Module):
    def __init__(self, data_dim, n_layers, hidden_dim, batch_norm_between_layers=False):
        super().__init__()
        assert n_layers % 2 == 0, "Number of layers must be even to ensure all dimensions are transformed."
        layers = []
        mask_a = torch.zeros(data_dim)
        mask_a[:data_dim // 2] = 1
        mask_b = 1 - mask_a
        for i in range(n_layers):
            mask = mask_a if i % 2 == 0 else mask_b
            layers.append(SplineCouplingLayer(data_dim, hidden_dim, mask))
        self.flow = NormalizingFlowModel(layers, batch_norm_between_layers)

    def forward(self, z):
        return self.flow.forward(z)

    def inverse(self, x):
        return self.flow.inverse(x)

    def log_prob(self, x, return_sums=False, workspace=None):
        return self.flow.log_prob(x, return_sums=return_sums, workspace=workspace)

    def nll(self, x):
        return self.flow.nll(x)

    def sample_fused_ok(self, num_samples, device):
        return self.flow.sample_fused_ok(num_samples, device)

    def sample_fused(self, num_samples, device="cuda", out=None):
        return self.flow.sample_fused(num_samples, device, out)
