"""GPU: the reference's remaining constructor options under autograd, against the reference's own
outputs, gradients and running statistics (G17, tests/golden/make_golden.py:g17) and float64
autograd of the same module (the reference's fp32 distance from float64 is the yardstick, as in
test_gpu_fig_models.py):

  iafbn   2x InverseAutoregressiveFlow(5, 32, use_batch_norm=True), TRAIN mode, density step: the
          sequential IAF.inverse is the reference's d MADE calls, each normalising with the batch
          statistics of its own partial vector and updating the running statistics
          (inverse_autoregressive_flow.py:65-103, made.py:93-106)
  mafbn   MaskedAutoregressiveFlow(5, 32, use_batch_norm=True), TRAIN mode, forward (sampling,
          sequential: masked_autoregressive_flow.py:46-78) under L = sum(y wy) + sum(ld wl)

Every call is HIP (STATS["torch"] == 0): the d train-mode MADE calls run on the any-shape path
(csrc/nfx_generic.hip: masked GEMMs, batch moments, running update, normalisation) with the
element step kernel, and the backward runs call by call in reverse
(_MadeAffineFlow._generic_seq_train_backward).
"""
import copy

import numpy as np
import pytest
import torch

import nfs_amd
from conftest import load_golden

pytestmark = pytest.mark.gpu


def _load(module, g, prefix):
    sd = module.state_dict()
    module.load_state_dict({k: (v if k.endswith("num_batches_tracked") else torch.from_numpy(np.array(g[prefix + k])))
                            for k, v in sd.items()})
    return module


def _gclose(a, b, what, ref32, frac=2e-4):
    """max|a - b| <= max(frac * max|b|, 4 * max|ref32 - b|)."""
    a, b, r = (torch.as_tensor(np.asarray(t.detach().cpu() if torch.is_tensor(t) else t)).double() for t in (a, b, ref32))
    err = (a - b).abs().max().item()
    bound = max(frac * max(b.abs().max().item(), 1e-30), 4 * (r - b).abs().max().item())
    assert err <= bound, f"{what}: max err {err:.3e} > {bound:.3e}"


def _loss(z, ld):
    return -(-0.5 * (z.pow(2).sum(1) + z.shape[1] * np.log(2 * np.pi)) + ld).mean()


def test_iaf_batchnorm_train_step_vs_reference(cuda_device):
    g = load_golden("g17_options.npz")
    m = nfs_amd.NormalizingFlowModel([nfs_amd.InverseAutoregressiveFlow(5, 32, use_batch_norm=True) for _ in range(2)])
    m = _load(m, g, "iafbn.init.").train()
    m64 = copy.deepcopy(m).double().train()
    gpu = m.to(cuda_device)
    x = torch.from_numpy(g["iafbn.x"])
    nfs_amd.reset_stats()
    z, ld = gpu.inverse(x.to(cuda_device))
    loss = _loss(z, ld)
    loss.backward()
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] >= 4, nfs_amd.STATS
    z64, ld64 = m64.inverse(x.double())
    l64 = _loss(z64, ld64)
    l64.backward()
    _gclose(z, g["iafbn.z"], "z", z64, frac=2e-5)
    _gclose(ld, g["iafbn.ld"], "ld", ld64, frac=2e-5)
    assert abs(loss.item() - float(g["iafbn.loss"])) <= 2e-5 and abs(loss.item() - l64.item()) <= 2e-5
    for (k, p), (_, p64) in zip(gpu.named_parameters(), m64.named_parameters()):
        _gclose(p.grad, g["iafbn.grad." + k], what=k, ref32=p64.grad)
        _gclose(p.grad, p64.grad, what=k + " (float64)", ref32=g["iafbn.grad." + k])
    n = 0
    for k, v in gpu.state_dict().items():
        if k.endswith(("running_mean", "running_var")):
            np.testing.assert_allclose(v.cpu().numpy(), g["iafbn.after." + k], rtol=1e-5, atol=1e-6, err_msg=k)
            n += 1
        elif k.endswith("num_batches_tracked"):
            assert int(v) == 5, (k, int(v))  # one update per MADE call: d = 5 calls per forward
    assert n == 12


def test_maf_batchnorm_train_sampling_vs_reference(cuda_device):
    g = load_golden("g17_options.npz")
    f = _load(nfs_amd.MaskedAutoregressiveFlow(5, 32, use_batch_norm=True), g, "mafbn.init.").train()
    f64 = copy.deepcopy(f).double().train()
    gpu = f.to(cuda_device)
    x = torch.from_numpy(g["mafbn.x"])
    wy, wl = torch.from_numpy(g["mafbn.wy"]), torch.from_numpy(g["mafbn.wl"])
    nfs_amd.reset_stats()
    xr = x.to(cuda_device).requires_grad_(True)
    y, ld = gpu.forward(xr)
    ((y * wy.to(cuda_device)).sum() + (ld * wl.to(cuda_device)).sum()).backward()
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] >= 2, nfs_amd.STATS
    x64 = x.double().requires_grad_(True)
    y64, ld64 = f64.forward(x64)
    ((y64 * wy.double()).sum() + (ld64 * wl.double()).sum()).backward()
    _gclose(y, g["mafbn.fwd.y"], "y", y64, frac=2e-5)
    _gclose(ld, g["mafbn.fwd.ld"], "ld", ld64, frac=2e-5)
    _gclose(xr.grad, g["mafbn.fwd.gx"], "dL/dx", x64.grad)
    for (k, p), (_, p64) in zip(gpu.named_parameters(), f64.named_parameters()):
        _gclose(p.grad, g["mafbn.fwd.grad." + k], what=k, ref32=p64.grad)
    for k, v in gpu.state_dict().items():
        if k.endswith(("running_mean", "running_var")):
            np.testing.assert_allclose(v.cpu().numpy(), g["mafbn.fwd.after." + k], rtol=1e-5, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("dname", ["fwd", "inv"])
def test_spline_per_dimension_bounds_vs_reference(cuda_device, dname):
    """spldm: SplineCouplingLayer(3, 32, mask = 0, K = 6) with per-dimension data_min / data_max
    tensors (spline_coupling_layer.py:78-94; the only mask the reference runs them with, see
    make_golden.py:g17), eval, both directions under autograd, on the any-shape path with the
    bounds (nfx_spline_rescale + nfx_spline_elem_*_bounded)."""
    g = load_golden("g17_options.npz")
    dmin, dmax = torch.from_numpy(g["spldm.data_min"]), torch.from_numpy(g["spldm.data_max"])
    f = nfs_amd.SplineCouplingLayer(3, 32, torch.zeros(3), num_bins=6, data_min=dmin, data_max=dmax)
    f = _load(f, g, "spldm.init.").eval()
    f64 = copy.deepcopy(f).double()
    f64.data_min, f64.data_max = dmin.double(), dmax.double()
    gpu = f.to(cuda_device)
    gpu.data_min, gpu.data_max = dmin.to(cuda_device), dmax.to(cuda_device)
    x = torch.from_numpy(g["spldm.x"])
    wy, wl = torch.from_numpy(g["spldm.wy"]), torch.from_numpy(g["spldm.wl"])
    nfs_amd.reset_stats()
    xr = x.to(cuda_device).requires_grad_(True)
    y, ld = (gpu.forward if dname == "fwd" else gpu.inverse)(xr)
    ((y * wy.to(cuda_device)).sum() + (ld * wl.to(cuda_device)).sum()).backward()
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] == 2, nfs_amd.STATS
    x64 = x.double().requires_grad_(True)
    y64, ld64 = (f64.forward if dname == "fwd" else f64.inverse)(x64)
    ((y64 * wy.double()).sum() + (ld64 * wl.double()).sum()).backward()
    pre = f"spldm.{dname}."
    _gclose(y, g[pre + "y"], "y", y64, frac=2e-5)
    _gclose(ld, g[pre + "ld"], "ld", ld64, frac=2e-5)
    _gclose(xr.grad, g[pre + "gx"], "dL/dx", x64.grad)
    for (k, p), (_, p64) in zip(gpu.named_parameters(), f64.named_parameters()):
        _gclose(p.grad, g[pre + "grad." + k], what=k, ref32=p64.grad)
