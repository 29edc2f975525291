"""GPU: fused backward of the MAF density direction (nfx_made_affine_backward, §8(f) item 1).

Gradients (dL/dx and every MADE parameter) of L = <gz, z> + <gld, log_det> through
MaskedAutoregressiveFlow.inverse, against autograd of the same module evaluated in float64 on
the CPU (the reference's ops, masked_autoregressive_flow.py:18-44). The fp32 kernel must be as
close to the float64 gradients as the fp32 composite is (checked side by side), within
  per element |g - g64| <= 1e-5 * (1 + |g64|) for dL/dx, and
  max |g - g64| <= 2e-5 * (1 + max |g64|) for the parameter gradients (sums over the batch).
"""
import copy

import pytest
import torch

import nfs_amd
from nfs_amd.flows.flow import STATS

pytestmark = pytest.mark.gpu


def _maf(d, H, seed):
    torch.manual_seed(seed)
    f = nfs_amd.MaskedAutoregressiveFlow(d, H)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in f.parameters():
            p.add_(0.1 * torch.randn(p.shape, generator=g))
    return f


def _grads(f, x, gz, gld):
    x = x.clone().requires_grad_(True)
    for p in f.parameters():
        p.grad = None
    z, ld = f.inverse(x)
    ((z * gz).sum() + (ld * gld).sum()).backward()
    return x.grad, [p.grad for p in f.parameters()]


def _check(g, ref, tol):
    g, ref = g.double().cpu(), ref.double().cpu()
    err = (g - ref).abs().max().item()
    assert err <= tol * (1 + ref.abs().max().item()), (err, ref.abs().max().item())


@pytest.mark.parametrize("d,H,B", [(5, 16, 1), (5, 16, 77), (33, 32, 1000), (63, 64, 2048), (64, 64, 300),
                                   (2, 64, 500)])
def test_made_backward_vs_float64_autograd(cuda_device, d, H, B):
    f = _maf(d, H, d * 100 + H)
    f64 = copy.deepcopy(f).double()
    x = torch.randn(B, d)
    x[: min(B, 3)] *= 4.0  # some rows saturate the alpha clamp
    gz = torch.randn(B, d)
    gld = torch.randn(B)
    gx64, gp64 = _grads(f64, x.double(), gz.double(), gld.double())
    fg = f.to(cuda_device).train()  # train(): parameters require grad; no BatchNorm in this MADE
    STATS["hip"] = 0
    gx, gp = _grads(fg, x.to(cuda_device), gz.to(cuda_device), gld.to(cuda_device))
    assert STATS["hip"] >= 2  # fused forward + fused backward
    assert ((gx.double().cpu() - gx64).abs() <= 1e-5 * (1 + gx64.abs())).all()
    for g, r in zip(gp, gp64):
        _check(g, r, 2e-5)


def test_made_backward_logdet_clamp_and_training_step(cuda_device):
    """A saturated log-det (|sum alpha| > 100 is impossible at |alpha| <= 3 for d < 34, so use
    d = 63 with large alphas) blocks the log-det gradient exactly like torch.clamp; then one
    full training step through NormalizingFlowModel matches the composite backward."""
    d, H = 63, 64
    f = _maf(d, H, 7)
    with torch.no_grad():
        f.conditioner.linears()[-1].bias[d:] += 5.0  # every alpha clamps at +3 -> ld = -189 -> clamp
    f64 = copy.deepcopy(f).double()
    x = torch.randn(256, d)
    gz, gld = torch.randn(256, d), torch.randn(256)
    gx64, gp64 = _grads(f64, x.double(), gz.double(), gld.double())
    gx, gp = _grads(f.to(cuda_device), x.to(cuda_device), gz.to(cuda_device), gld.to(cuda_device))
    assert ((gx.double().cpu() - gx64).abs() <= 1e-5 * (1 + gx64.abs())).all()
    for g, r in zip(gp, gp64):
        _check(g, r, 2e-5)

    torch.manual_seed(1)
    model = nfs_amd.NormalizingFlowModel([_maf(d, H, 20 + i) for i in range(3)])
    ref = copy.deepcopy(model).double()
    data = torch.randn(1024, d)
    loss64 = -ref.log_prob(data.double()).mean()
    loss64.backward()
    model = model.to(cuda_device).train()
    loss = -model.log_prob(data.to(cuda_device)).mean()
    loss.backward()
    assert abs(loss.item() - loss64.item()) <= 1e-5 * (1 + abs(loss64.item()))
    for p, p64 in zip(model.parameters(), ref.parameters()):
        _check(p.grad, p64.grad, 2e-5)
