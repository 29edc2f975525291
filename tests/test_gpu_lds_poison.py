"""GPU: no kernel reads LDS it did not write.

LDS is not cleared between kernels, so a kernel that read a word it never wrote would see what
the previous kernel on that CU left there: results that depend on the history of the process.
Each case poisons the LDS of every CU (nfx_debug_fill_lds: NaN, +Inf, a huge finite value, zero)
right before the call and requires results bit-identical to the zero-poisoned run.
"""
import pytest
import torch

import nfs_amd
from nfs_amd import _lib

pytestmark = pytest.mark.gpu

PATTERNS = [0x7FC00000, 0x7F800000, 0x7E967699, 0xFFFFFFFF]  # NaN, +Inf, 1e38, NaN (all ones)


def _poison(bits, dev):
    _lib.check(_lib.lib().nfx_debug_fill_lds(bits, _lib.stream_of(torch.empty(1, device=dev))),
               "nfx_debug_fill_lds")


def _perturb(m, sigma, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(sigma * torch.randn(p.shape, generator=g))
    return m


def _alt_mask(d, i):
    m = torch.zeros(d)
    m[(i % 2)::2] = 1
    return m


def _model(kind):
    torch.manual_seed(3)
    if kind == "realnvp":
        return _perturb(nfs_amd.RealNVP(2, 4, 64), 0.1, 1), 2
    if kind == "affine_d16":
        return _perturb(nfs_amd.NormalizingFlowModel(
            [nfs_amd.CouplingLayer(16, 64, _alt_mask(16, i)) for i in range(2)]), 0.1, 2), 16
    if kind == "spline":
        return _perturb(nfs_amd.NormalizingFlowModel(
            [nfs_amd.SplineCouplingLayer(3, 64, _alt_mask(3, i), num_bins=8) for i in range(2)]), 0.1, 3), 3
    if kind == "maf63":
        return _perturb(nfs_amd.NormalizingFlowModel(
            [nfs_amd.MaskedAutoregressiveFlow(63, 64) for _ in range(2)]), 0.02, 4), 63
    if kind == "maf80_wide":
        return _perturb(nfs_amd.NormalizingFlowModel(
            [nfs_amd.MaskedAutoregressiveFlow(80, 64) for _ in range(2)]), 0.02, 5), 80
    if kind == "iaf150":
        return _perturb(nfs_amd.NormalizingFlowModel(
            [nfs_amd.InverseAutoregressiveFlow(150, 64) for _ in range(2)]), 0.02, 6), 150
    if kind == "realnvp_bn_between":
        return _perturb(nfs_amd.RealNVP(2, 4, 64, batch_norm_between_layers=True), 0.1, 7), 2
    if kind == "spline_d16":
        return _perturb(nfs_amd.NormalizingFlowModel(
            [nfs_amd.SplineCouplingLayer(16, 64, _alt_mask(16, i), num_bins=8) for i in range(2)]), 0.1, 8), 16
    if kind == "maf100_h128":
        return _perturb(nfs_amd.NormalizingFlowModel(
            [nfs_amd.MaskedAutoregressiveFlow(100, 128) for _ in range(2)]), 0.02, 9), 100
    if kind == "iaf784":
        return _perturb(nfs_amd.NormalizingFlowModel([nfs_amd.InverseAutoregressiveFlow(784, 64)]), 0.02, 10), 784
    if kind == "arqs":
        return _perturb(nfs_amd.NormalizingFlowModel([nfs_amd.ARQS(6, 64, num_bins=8) for _ in range(2)]), 0.05, 11), 6
    if kind == "made_h256":
        return _perturb(nfs_amd.NormalizingFlowModel(
            [nfs_amd.MaskedAutoregressiveFlow(70, 256), nfs_amd.InverseAutoregressiveFlow(70, 256)]), 0.02, 12), 70
    raise ValueError(kind)


KINDS = ["realnvp", "affine_d16", "spline", "maf63", "maf80_wide", "iaf150", "realnvp_bn_between",
         "spline_d16", "maf100_h128", "iaf784", "arqs", "made_h256"]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("B", [77, 4099])
def test_eval_paths_independent_of_stale_lds(cuda_device, kind, B):
    m, d = _model(kind)
    m = m.to(cuda_device).eval()
    x = (1.5 * torch.randn(B, d, generator=torch.Generator().manual_seed(B))).to(cuda_device)
    outs = {}
    with torch.no_grad():
        for bits in [0] + PATTERNS:
            res = []
            for fn in (lambda: m.log_prob(x), lambda: m.inverse(x), lambda: m.forward(x)):
                _poison(bits, cuda_device)
                r = fn()
                res += list(r) if isinstance(r, tuple) else [r]
            torch.cuda.synchronize()
            outs[bits] = [t.clone() for t in res]
    for bits in PATTERNS:
        for i, (a, b) in enumerate(zip(outs[bits], outs[0])):
            bad = (a != b) & ~(torch.isnan(a) & torch.isnan(b))
            rows = bad.reshape(B, -1).any(dim=1).nonzero().flatten().tolist()
            assert not rows, (hex(bits), i, len(rows), rows[:16])


@pytest.mark.parametrize("kind", ["realnvp", "spline", "maf63", "iaf150", "maf80_wide", "iaf784"])
def test_backward_independent_of_stale_lds(cuda_device, kind):
    m, d = _model(kind)
    m = m.to(cuda_device)
    if kind != "realnvp":
        m.eval()
    B = 4099 if d < 500 else 300
    x = (1.2 * torch.randn(B, d, generator=torch.Generator().manual_seed(11))).to(cuda_device)
    ref = None
    for bits in [0] + PATTERNS:
        m.zero_grad(set_to_none=True)
        xr = x.clone().requires_grad_(True)
        _poison(bits, cuda_device)
        # density direction, and for the IAFs also the sampling direction under autograd
        loss = -m.log_prob(xr).mean()
        if kind.startswith("iaf"):
            loss = loss + m.forward(xr)[0].square().mean()
        _poison(bits, cuda_device)
        loss.backward()
        torch.cuda.synchronize()
        got = [xr.grad.clone()] + [p.grad.clone() for p in m.parameters() if p.grad is not None]
        if ref is None:
            ref = got
            continue
        for i, (a, b) in enumerate(zip(got, ref)):
            assert torch.equal(a, b), (hex(bits), i, (a - b).abs().max().item())
