"""Train-mode CouplingLayer on the gfx950 kernels (csrc/nfx_affine_train.hip) vs the reference.

In train mode the conditioner BatchNorm1d normalises with batch statistics and updates its running
statistics (coupling_layer.py:18-35 under model.train(); the reference trains this way:
README.md:107-117, plots/_common.py:194-211). Checked here:
  * against the reference itself (G11, tests/golden/make_golden.py): RealNVP(2,8,64) inverse,
    NLL, every parameter gradient and the running statistics after the step; 5 Adam steps; a
    d=4 layer in both directions (padded kernel width, weighted y / log-det loss, dL/dx);
  * against float64 autograd of the same module on ragged and larger batches, d = 1..8,
    H = 16..64, both directions.
Tolerances: outputs |d| <= 2e-5 (1 + |ref|); gradients |d| <= 2e-4 max|ref| per tensor (the
kernels reduce over the batch in fp32 per lane, fp64 across waves; the biases that feed a
BatchNorm have an exactly-zero gradient and only carry summation noise < 2e-5 of the largest
gradient); running statistics 1e-6; NLL 1e-5.
"""
import copy

import numpy as np
import pytest
import torch

import nfs_amd
import oracle
from conftest import assert_fp32_parity, load_golden, oracle_sd
from nfs_amd.flows.coupling import CouplingLayer

pytestmark = pytest.mark.gpu


def _load(module, g, prefix):
    sd = module.state_dict()
    new = {}
    for k, v in sd.items():
        if k.endswith("num_batches_tracked"):
            new[k] = v
        else:
            new[k] = torch.from_numpy(np.array(g[prefix + k]))
    module.load_state_dict(new)
    return module


def _close(a, b, rel=2e-5, what=""):
    a = a.detach().double().cpu()
    b = torch.as_tensor(np.asarray(b)).double() if not torch.is_tensor(b) else b.detach().double().cpu()
    err = ((a - b).abs() / (1 + b.abs())).max().item() if a.numel() else 0.0
    assert err <= rel, f"{what}: max rel err {err:.3e} > {rel:.1e}"


PRE_BN_BIAS = ("net.0.bias", "net.3.bias")


def _t64(v):
    return v.detach().double().cpu() if torch.is_tensor(v) else torch.as_tensor(np.asarray(v)).double()


def _gclose(a, b, frac=2e-4, what="", gmax=None, ref32=None, ref_factor=4.0):
    """Gradient tensors: max|a - b| <= max(frac * max|b|, 4 * max|ref32 - b|), i.e. within frac of
    the tensor's scale or as close as the reference's own fp32 result (ref32, when b is the
    float64 evaluation). The biases of the Linear layers that feed a BatchNorm (PRE_BN_BIAS)
    have a gradient of exactly 0 in exact arithmetic (the batch mean removes them): there both
    sides hold summation noise (amplified by 1/sqrt(var + eps) for a zero-variance feature),
    bounded by 2e-5 of the largest gradient of the layer (`gmax`) or the reference's fp32 noise."""
    a, b = _t64(a), _t64(b)
    ref_err = (_t64(ref32) - b).abs().max().item() if ref32 is not None else 0.0
    if any(w.endswith(PRE_BN_BIAS) for w in what.split(" ")) and gmax is not None:
        bound = max(2e-5 * gmax, ref_factor * ref_err)
        assert (a - b).abs().max().item() <= bound, f"{what}: {a.abs().max().item():.3e} not ~0 (bound {bound:.3e})"
        return
    scale = max(b.abs().max().item(), 1e-30)
    err = (a - b).abs().max().item()
    assert err <= max(frac * scale, ref_factor * ref_err), f"{what}: max err {err:.3e} of max|ref| {scale:.3e} (ref32 err {ref_err:.3e})"


def _oracle_train64(g, prefix, x):
    """Float64 evaluation of the reference math (the oracle, train mode) + NLL gradients."""
    sd = {k: v.double() if v.is_floating_point() else v for k, v in oracle_sd(g, prefix).items()}
    for k, v in sd.items():
        if v.is_floating_point() and not k.endswith(("running_mean", "running_var", "mask")):
            v.requires_grad_(True)
    z, ld = oracle.flow_model(sd, oracle.realnvp_spec(8, training=True), x.double(), -1)
    loss = -(-0.5 * (z.pow(2).sum(1) + 2 * np.log(2 * np.pi)) + ld).mean()
    loss.backward()
    return z.detach(), ld.detach(), loss.item(), {k: v.grad for k, v in sd.items() if v.requires_grad}


def test_realnvp_train_step_vs_reference(cuda_device):
    g = load_golden("g11_train.npz")
    m = _load(nfs_amd.RealNVP(2, 8, 64), g, "rn.init.").to(cuda_device).train()
    x = torch.from_numpy(g["rn.x"]).to(cuda_device)
    nfs_amd.reset_stats()
    z, ld = m.inverse(x)
    loss = -(-0.5 * (z.pow(2).sum(1) + 2 * np.log(2 * np.pi)) + ld).mean()
    loss.backward()
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] >= 16, nfs_amd.STATS
    # per-sample outputs through 8 layers are ill-conditioned for a few rows (z ~ 1e3): judged
    # against the float64 evaluation with the reference's own fp32 error as the yardstick
    z64, ld64, loss64, g64 = _oracle_train64(g, "rn.init.", torch.from_numpy(g["rn.x"]))
    assert_fp32_parity(z.detach().cpu(), g["rn.z"], z64, slack=2e-5, floor=2e-4, what="z")
    assert_fp32_parity(ld.detach().cpu(), g["rn.ld"], ld64, slack=2e-5, floor=2e-4, what="log_det")
    assert abs(loss.item() - float(g["rn.loss"])) <= 1e-5 and abs(loss.item() - loss64) <= 2e-5
    gmax = max(float(np.abs(g["rn.grad." + k]).max()) for k, _ in m.named_parameters())
    for k, p in m.named_parameters():
        _gclose(p.grad, g["rn.grad." + k], what=k, gmax=gmax)
        _gclose(p.grad, g64[k], what=k + " (float64)", gmax=gmax, ref32=g["rn.grad." + k])
    for k, v in m.state_dict().items():
        if k.endswith(("running_mean", "running_var")):
            _close(v, g["rn.after." + k], rel=1e-6, what=k)
        if k.endswith("num_batches_tracked"):
            assert int(v) == 1, k


def test_realnvp_adam_steps_vs_reference(cuda_device):
    g = load_golden("g11_train.npz")
    m = _load(nfs_amd.RealNVP(2, 8, 64), g, "rn.init.").to(cuda_device).train()
    x = torch.from_numpy(g["rn.x"]).to(cuda_device)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    losses = []
    for _ in range(5):
        z, ld = m.inverse(x)
        loss = -(-0.5 * (z.pow(2).sum(1) + 2 * np.log(2 * np.pi)) + ld).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    np.testing.assert_allclose(losses, g["rn.adam_losses"], rtol=2e-5, atol=2e-5)
    for k, v in m.state_dict().items():
        # Linear biases feeding a BatchNorm have zero gradient up to rounding noise, which
        # Adam's normalisation turns into +-lr steps on both sides: they do not affect the
        # function (the batch mean removes them) and are not compared, nor is the running mean
        # of the BatchNorm they feed (it tracks those biases).
        if k.endswith(("num_batches_tracked", "net.0.bias", "net.3.bias", "running_mean")):
            continue
        # Adam normalises every update element-wise, so fp32 noise in small gradient entries
        # becomes O(lr) parameter noise: 2e-4 relative after 5 steps at lr 1e-3
        _close(v, g["rn.adam5." + k], rel=2e-4, what=k)


def test_layer_d4_both_directions_vs_reference(cuda_device):
    g = load_golden("g11_train.npz")
    layer = CouplingLayer(4, 16, torch.tensor([1.0, 0.0, 1.0, 0.0]))
    layer = _load(layer, g, "c4.init.").to(cuda_device).train()
    xc = torch.from_numpy(g["c4.x"]).to(cuda_device)
    wy = torch.from_numpy(g["c4.wy"]).to(cuda_device)
    wl = torch.from_numpy(g["c4.wl"]).to(cuda_device)
    for name, fn in (("inv", layer.inverse), ("fwd", layer.forward)):
        layer.zero_grad()
        xr = xc.clone().requires_grad_(True)
        y, ld = fn(xr)
        ((y * wy).sum() + (ld * wl).sum()).backward()
        _close(y, g[f"c4.{name}.y"], what=f"{name} y")
        _close(ld, g[f"c4.{name}.ld"], what=f"{name} ld")
        _gclose(xr.grad, g[f"c4.{name}.gx"], what=f"{name} gx")
        gmax = max(float(np.abs(g[f"c4.{name}.grad.{k}"]).max()) for k, _ in layer.named_parameters())
        for k, p in layer.named_parameters():
            _gclose(p.grad, g[f"c4.{name}.grad.{k}"], what=f"{name} {k}", gmax=gmax)
    for k, v in layer.state_dict().items():
        if k.endswith(("running_mean", "running_var")):
            _close(v, g["c4.after." + k], rel=1e-6, what=k)


def _perturbed_layer(d, H, seed, mask_even=True):
    torch.manual_seed(seed)
    mask = torch.zeros(d)
    if mask_even:
        mask[: d // 2] = 1
    else:
        mask[d // 2:] = 1
    layer = CouplingLayer(d, H, mask)
    gen = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in layer.parameters():
            p.add_(0.2 * torch.randn(p.shape, generator=gen))
        for bn in layer._batchnorms():
            bn.running_mean.copy_(0.1 * torch.randn(bn.running_mean.shape, generator=gen))
            bn.running_var.copy_(0.5 + torch.rand(bn.running_var.shape, generator=gen))
    return layer


@pytest.mark.parametrize("d,H,B,direction", [
    (2, 64, 2, -1), (2, 64, 31, -1), (2, 64, 1000, 1), (2, 64, 65537, -1),
    (1, 32, 500, -1), (3, 16, 777, 1), (5, 48, 4097, -1), (8, 64, 3000, 1), (2, 20, 129, -1),
])
def test_layer_vs_float64_autograd(cuda_device, d, H, B, direction):
    layer = _perturbed_layer(d, H, 100 + d * 7 + H, mask_even=(B % 2 == 0))
    ref = copy.deepcopy(layer).double().train()
    ref32 = copy.deepcopy(layer).train()
    gpu = layer.to(cuda_device).train()
    gen = torch.Generator().manual_seed(B)
    x = (torch.randn(B, d, generator=gen) * 1.3 + 0.2)
    wy = torch.randn(B, d, generator=gen)
    wl = torch.randn(B, generator=gen)
    xr = x.double().requires_grad_(True)
    yr, ldr = ref.forward(xr) if direction > 0 else ref.inverse(xr)
    ((yr * wy.double()).sum() + (ldr * wl.double()).sum()).backward()
    y32, ld32 = ref32.forward(x) if direction > 0 else ref32.inverse(x)
    ((y32 * wy).sum() + (ld32 * wl).sum()).backward()
    nfs_amd.reset_stats()
    xg = x.to(cuda_device).requires_grad_(True)
    yg, ldg = gpu.forward(xg) if direction > 0 else gpu.inverse(xg)
    ((yg * wy.to(cuda_device)).sum() + (ldg * wl.to(cuda_device)).sum()).backward()
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] == 2, nfs_amd.STATS
    _close(yg, yr, what="y")
    _close(ldg, ldr, what="log_det")
    _gclose(xg.grad, xr.grad, what="dL/dx")
    gmax = max(p.grad.abs().max().item() for p in ref.parameters())
    for (k, pg), (_, pr), (_, p32) in zip(gpu.named_parameters(), ref.named_parameters(), ref32.named_parameters()):
        # B < 8: BatchNorm over a handful of samples is ill-conditioned (x^ ~ +-1, the BN backward
        # nearly cancels); the kernel is then held to 8x the reference's own fp32 error
        _gclose(pg.grad, pr.grad, what=k, gmax=gmax, ref32=p32.grad, ref_factor=8.0 if B < 8 else 4.0)
    for (k, bg), (_, br) in zip(gpu.named_buffers(), ref.named_buffers()):
        if k.endswith(("running_mean", "running_var")):
            _close(bg, br, rel=1e-6, what=k)
        if k.endswith("num_batches_tracked"):
            assert int(bg) == int(br) == 1


def test_no_grad_train_forward_updates_running_stats(cuda_device):
    """Under no_grad in train mode BatchNorm still uses (and records) batch statistics."""
    layer = _perturbed_layer(2, 64, 7)
    ref = copy.deepcopy(layer).double().train()
    gpu = layer.to(cuda_device).train()
    x = torch.randn(5000, 2, generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        yr, ldr = ref.inverse(x.double())
        yg, ldg = gpu.inverse(x.to(cuda_device))
    _close(yg, yr, what="y")
    _close(ldg, ldr, what="log_det")
    for (k, bg), (_, br) in zip(gpu.named_buffers(), ref.named_buffers()):
        if k.endswith(("running_mean", "running_var")):
            _close(bg, br, rel=1e-6, what=k)


def test_eval_after_train_uses_running_stats(cuda_device):
    """model.eval() after HIP training steps -> the eval kernel sees the updated running stats
    (the pack cache notices the in-kernel running-statistics writes)."""
    layer = _perturbed_layer(2, 32, 9)
    gpu = layer.to(cuda_device)
    x = torch.randn(3000, 2, device=cuda_device)
    gpu.eval()
    with torch.no_grad():
        y0, _ = gpu.inverse(x)
    gpu.train()
    with torch.no_grad():
        gpu.inverse(x * 2.0 + 1.0)
    gpu.eval()
    ref = copy.deepcopy(gpu).cpu().double()
    with torch.no_grad():
        y1, _ = gpu.inverse(x)
        yr, _ = ref.inverse(x.double().cpu())
    _close(y1, yr, what="eval after train")
    assert (y1 - y0).abs().max().item() > 1e-4  # the running statistics did change


@pytest.mark.parametrize("d,H,B,direction", [
    (2, 64, 1, -1), (2, 64, 1000, 1), (2, 64, 65537, -1), (1, 32, 500, -1), (3, 16, 777, 1),
    (5, 48, 4097, -1), (8, 64, 3000, 1), (2, 20, 129, -1),
])
def test_eval_mode_backward_vs_float64_autograd(cuda_device, d, H, B, direction):
    """Eval-mode CouplingLayer under autograd (running-statistics BatchNorm, coupling_layer.py:
    40-96 with model.eval()): the fused train-mode backward kernels with the running statistics
    (nfx_affine_eval_stats, n < 0 triples), no recompute through ATen; gamma/beta gradients
    included, running statistics untouched."""
    layer = _perturbed_layer(d, H, 300 + d * 5 + H, mask_even=(B % 2 == 1))
    ref = copy.deepcopy(layer).double().eval()
    ref32 = copy.deepcopy(layer).eval()
    gpu = layer.to(cuda_device).eval()
    before = {k: v.clone() for k, v in gpu.named_buffers()}
    gen = torch.Generator().manual_seed(B + 11)
    x = (torch.randn(B, d, generator=gen) * 1.3 + 0.2)
    wy = torch.randn(B, d, generator=gen)
    wl = torch.randn(B, generator=gen)
    xr = x.double().requires_grad_(True)
    yr, ldr = ref.forward(xr) if direction > 0 else ref.inverse(xr)
    ((yr * wy.double()).sum() + (ldr * wl.double()).sum()).backward()
    y32, ld32 = ref32.forward(x) if direction > 0 else ref32.inverse(x)
    ((y32 * wy).sum() + (ld32 * wl).sum()).backward()
    nfs_amd.reset_stats()
    xg = x.to(cuda_device).requires_grad_(True)
    yg, ldg = gpu.forward(xg) if direction > 0 else gpu.inverse(xg)
    ((yg * wy.to(cuda_device)).sum() + (ldg * wl.to(cuda_device)).sum()).backward()
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] == 2, nfs_amd.STATS
    _close(yg, yr, what="y")
    _close(ldg, ldr, what="log_det")
    _gclose(xg.grad, xr.grad, what="dL/dx", ref32=None)
    for (k, pg), (_, pr), (_, p32) in zip(gpu.named_parameters(), ref.named_parameters(), ref32.named_parameters()):
        _gclose(pg.grad, pr.grad, what=k + " (eval)", ref32=p32.grad)
    for k, v in gpu.named_buffers():
        assert torch.equal(v, before[k]), f"eval backward changed buffer {k}"


def test_eval_mode_realnvp_step_matches_float64(cuda_device):
    """A full RealNVP(2,8,64) NLL step in eval mode: 8 HIP forwards + 8 fused eval backwards."""
    g = load_golden("g11_train.npz")
    m = _load(nfs_amd.RealNVP(2, 8, 64), g, "rn.init.")
    ref = copy.deepcopy(m).double().eval()
    gpu = m.to(cuda_device).eval()
    x = torch.from_numpy(g["rn.x"])
    zr, ldr = ref.inverse(x.double())
    lr = -(-0.5 * (zr.pow(2).sum(1) + 2 * np.log(2 * np.pi)) + ldr).mean()
    lr.backward()
    nfs_amd.reset_stats()
    z, ld = gpu.inverse(x.to(cuda_device))
    loss = -(-0.5 * (z.pow(2).sum(1) + 2 * np.log(2 * np.pi)) + ld).mean()
    loss.backward()
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] == 16, nfs_amd.STATS
    assert abs(loss.item() - lr.item()) <= 1e-5
    for (k, pg), (_, pr) in zip(gpu.named_parameters(), ref.named_parameters()):
        _gclose(pg.grad, pr.grad, frac=5e-4, what=k + " (eval step)")
