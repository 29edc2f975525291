"""GPU: the reference's other benchmark-figure models in training (plots/_common.py:157-169,
179-183, 194-211) against the reference's own outputs (G16, tests/golden/make_golden.py:g16):

  spline  RealNVPSpline(2, 8, 64), K = 10, Adam lr 5e-4
  maf     NormalizingFlowModel([MaskedAutoregressiveFlow(2, 64)] * 6), lr 1e-3
  iaf     NormalizingFlowModel([InverseAutoregressiveFlow(2, 64)] * 6), lr 1e-3

full batch on 2,000 two-moons points. The training direction is `inverse` (density): spline
couplings and MAF run their parallel fused backward, IAF its sequential one; every layer's
forward and backward is a HIP launch (STATS["torch"] == 0). The first step's z, log-det, loss
and parameter gradients are compared with the reference's fp32 values and with float64 autograd
of the same module (the reference's own distance from float64 is the yardstick, as in
test_gpu_affine_train.py), then 3 Adam + clip_grad_norm_(5.0) steps: each loss within 5e-5 of
the reference's or 1e-4 of the float64 trajectory.
"""
import copy

import numpy as np
import pytest
import torch

import nfs_amd
from conftest import assert_fp32_parity, load_golden

pytestmark = pytest.mark.gpu


def _build(name):
    if name == "spline":
        return nfs_amd.RealNVPSpline(2, 8, 64), 5e-4
    cls = nfs_amd.MaskedAutoregressiveFlow if name == "maf" else nfs_amd.InverseAutoregressiveFlow
    return nfs_amd.NormalizingFlowModel([cls(2, 64) for _ in range(6)]), 1e-3


def _load(module, g, prefix):
    sd = module.state_dict()
    module.load_state_dict({k: (v if k.endswith("num_batches_tracked") else torch.from_numpy(np.array(g[prefix + k])))
                            for k, v in sd.items()})
    return module


def _loss(z, ld):
    return -(-0.5 * (z.pow(2).sum(1) + 2 * np.log(2 * np.pi)) + ld).mean()


def _gclose(a, b, what, ref32, frac=2e-4):
    """max|a - b| <= max(frac * max|b|, 4 * max|ref32 - b|)."""
    a, b, r = (torch.as_tensor(np.asarray(t.detach().cpu() if torch.is_tensor(t) else t)).double() for t in (a, b, ref32))
    err = (a - b).abs().max().item()
    bound = max(frac * max(b.abs().max().item(), 1e-30), 4 * (r - b).abs().max().item())
    assert err <= bound, f"{what}: max err {err:.3e} > {bound:.3e}"


@pytest.mark.parametrize("name", ["spline", "maf", "iaf"])
def test_figure_model_train_step_vs_reference(cuda_device, name):
    g = load_golden("g16_fig_models.npz")
    m, _ = _build(name)
    m = _load(m, g, name + ".init.")
    m64 = copy.deepcopy(m).double().train()
    gpu = m.to(cuda_device).train()
    x = torch.from_numpy(g["x"])
    nfs_amd.reset_stats()
    z, ld = gpu.inverse(x.to(cuda_device))
    loss = _loss(z, ld)
    loss.backward()
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] > 0, nfs_amd.STATS
    z64, ld64 = m64.inverse(x.double())
    l64 = _loss(z64, ld64)
    l64.backward()
    assert_fp32_parity(z.detach().cpu(), g[name + ".z"], z64.detach(), slack=2e-5, what=name + " z")
    assert_fp32_parity(ld.detach().cpu(), g[name + ".ld"], ld64.detach(), slack=2e-5, what=name + " log_det")
    assert abs(loss.item() - float(g[name + ".loss"])) <= 2e-5 and abs(loss.item() - l64.item()) <= 2e-5
    for (k, p), (_, p64) in zip(gpu.named_parameters(), m64.named_parameters()):
        _gclose(p.grad, g[name + ".grad." + k], what=k, ref32=p64.grad)
        _gclose(p.grad, p64.grad, what=k + " (float64)", ref32=g[name + ".grad." + k])


@pytest.mark.parametrize("name", ["spline", "maf", "iaf"])
def test_figure_model_adam_steps_vs_reference(cuda_device, name):
    g = load_golden("g16_fig_models.npz")
    x = torch.from_numpy(g["x"])

    def train(m, xx):
        _, lr = _build(name)
        opt = torch.optim.Adam(m.parameters(), lr=lr)
        losses = []
        for _ in range(3):
            z, ld = m.inverse(xx)
            loss = _loss(z, ld)
            opt.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(m.parameters(), 5.0)
            opt.step()
            losses.append(loss.item())
        return np.asarray(losses)

    m64 = _load(_build(name)[0], g, name + ".init.").double().train()
    l64 = train(m64, x.double())
    m = _load(_build(name)[0], g, name + ".init.").to(cuda_device).train()
    nfs_amd.reset_stats()
    losses = train(m, x.to(cuda_device))
    assert nfs_amd.STATS["torch"] == 0, nfs_amd.STATS
    ref = g[name + ".losses3"]
    ok = (np.abs(losses - ref) <= 5e-5) | (np.abs(losses - l64) <= 1e-4)
    assert ok.all(), (losses.tolist(), ref.tolist(), l64.tolist())
    final = ({k: torch.from_numpy(g[name + ".step3." + k]) for k in m.state_dict() if name + ".step3." + k in g}
             if np.abs(losses - ref).max() <= 5e-5 else m64.state_dict())
    for k, v in m.state_dict().items():
        if k.endswith("num_batches_tracked") or k not in final:
            continue
        a, b = v.detach().double().cpu(), final[k].double().cpu()
        assert ((a - b).abs() <= 2e-4 * (1 + b.abs())).all(), f"{name} {k}: {(a - b).abs().max().item():.3e}"
