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


def _close_or_ref(a, b64, b32, rel=2e-5, what=""):
    """Outputs: max |a - b64| / (1 + |b64|) <= max(rel, 4x the reference's own fp32 error) — at
    H = 128 the batch-statistics chain is a little worse conditioned than the fixed 2e-5."""
    a, b64, b32 = (t.detach().double().cpu() for t in (a, b64, b32))
    err = ((a - b64).abs() / (1 + b64.abs())).max().item() if a.numel() else 0.0
    err32 = ((b32 - b64).abs() / (1 + b64.abs())).max().item() if a.numel() else 0.0
    assert err <= max(rel, 4 * err32), f"{what}: max rel err {err:.3e} > max({rel:.1e}, 4 x fp32 ref {err32:.3e})"


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
    # wide hidden layers (affine_trainw_kernel: one net per workgroup, wave per hidden tile)
    (2, 128, 2000, -1), (2, 128, 3, 1), (4, 96, 777, 1), (8, 128, 3000, -1), (2, 128, 65537, 1),
    (3, 100, 513, -1), (6, 72, 1000, 1),
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
    _close_or_ref(yg, yr, y32, what="y")
    _close_or_ref(ldg, ldr, ld32, what="log_det")
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


@pytest.mark.parametrize("d,H,B,direction", [(2, 64, 65537, -1), (5, 48, 4097, 1), (1, 32, 31, -1), (8, 64, 3000, 1)])
def test_recompute_path_vs_float64_autograd(cuda_device, monkeypatch, d, H, B, direction):
    """The default train-mode path (above) keeps the raw layer-2 pre-activations in the STATS2
    pass and reads them in OUTK, BWD1K and the one-net-per-workgroup BWD2K. NFX_TRAIN_KEEP=0
    selects the round-4 passes that recompute layers 1-2 instead (eval-layout forward, BatchNorm
    folded into the weights): held to the same float64 bar. (The two fp32 paths are not compared
    with each other directly: a ReLU input within rounding of 0 flips one sample's gradient.)"""
    monkeypatch.setenv("NFX_TRAIN_KEEP", "0")
    test_layer_vs_float64_autograd(cuda_device, d, H, B, direction)


def test_keep_budget_falls_back_to_recompute(cuda_device, monkeypatch):
    """A layer keeps its layer-2 pre-activations only within 1/32 of HBM (coupling._keep_budget);
    past it the forward keeps nothing and the backward recomputes (same float64 bar)."""
    from nfs_amd.flows import coupling as cp
    layer = _perturbed_layer(2, 64, 5).to(cuda_device).train()
    x = torch.randn(1000, 2, device=cuda_device)
    assert layer._train_forward(x, -1, keep=True)[2]._nfx_h2 is not None
    monkeypatch.setattr(cp, "_keep_budget", lambda dev: 0)
    assert layer._train_forward(x, -1, keep=True)[2]._nfx_h2 is None
    test_layer_vs_float64_autograd(cuda_device, 2, 64, 1000, 1)


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
    (2, 128, 1, -1), (2, 128, 2000, 1), (8, 128, 3000, -1), (5, 96, 4097, 1), (2, 128, 65537, -1),
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


def _fig_loss(z, ld):
    return -(-0.5 * (z.pow(2).sum(1) + 2 * np.log(2 * np.pi)) + ld).mean()


def test_figure_model_train_step_vs_reference(cuda_device):
    """The reference's benchmark-figure model, RealNVP(2, 10, 128) (plots/_common.py:161), in its
    training step (plots/_common.py:194-211: train-mode BatchNorm, full batch of 2,000 two-moons
    points) against the reference's own outputs, loss, gradients and running statistics (G15),
    and against float64 autograd: every layer runs the wide train-mode kernels (H = 128), no ATen."""
    g = load_golden("g15_fig_train.npz")
    m = _load(nfs_amd.RealNVP(2, 10, 128), g, "fig.init.")
    ref64 = copy.deepcopy(m).double().train()
    gpu = m.to(cuda_device).train()
    x = torch.from_numpy(g["fig.x"])
    nfs_amd.reset_stats()
    z, ld = gpu.inverse(x.to(cuda_device))
    loss = _fig_loss(z, ld)
    loss.backward()
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] == 20, nfs_amd.STATS
    z64, ld64 = ref64.inverse(x.double())
    l64 = _fig_loss(z64, ld64)
    l64.backward()
    assert_fp32_parity(z.detach().cpu(), g["fig.z"], z64.detach(), slack=2e-5, what="fig z")
    assert_fp32_parity(ld.detach().cpu(), g["fig.ld"], ld64.detach(), slack=2e-5, what="fig log_det")
    assert abs(loss.item() - float(g["fig.loss"])) <= 1e-5 and abs(loss.item() - l64.item()) <= 2e-5
    gmax = max(float(np.abs(g["fig.grad." + k]).max()) for k, _ in gpu.named_parameters())
    for (k, p), (_, p64) in zip(gpu.named_parameters(), ref64.named_parameters()):
        # vs the reference's fp32 gradients, with the reference's own distance from float64 as
        # the yardstick (through 10 train-mode layers a few BatchNorm sums are 4e-4 off exact)
        _gclose(p.grad, g["fig.grad." + k], what=k, gmax=gmax, ref32=p64.grad)
        _gclose(p.grad, p64.grad, what=k + " (float64)", gmax=gmax, ref32=g["fig.grad." + k])
    for k, v in gpu.state_dict().items():
        if k.endswith(("running_mean", "running_var")):
            _close(v, g["fig.after." + k], rel=1e-6, what=k)


def _fig_train(m, x, steps, dtype=None):
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    losses = []
    for _ in range(steps):
        z, ld = m.inverse(x)
        loss = _fig_loss(z, ld)
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 5.0)
        opt.step()
        losses.append(loss.item())
    return opt, losses


def test_figure_model_five_adam_steps_vs_reference(cuda_device):
    """Five full steps of the reference's figure training loop (Adam lr 1e-3, clip_grad_norm_ 5.0,
    plots/_common.py:194-211) on the HIP path. The trajectory is ill-conditioned in fp32: Adam
    normalises every update element-wise, so rounding noise in near-zero gradient entries becomes
    +-lr parameter steps, and the reference's own fp32 loss at step 3 is 3.8e-3 off its float64
    trajectory (one ulp of weight jitter moves it as much). Each loss must be within 5e-5 of the
    reference's (G15) or 1e-4 of the float64 trajectory, and the final parameters within 2e-4
    (relative) of the trajectory the losses followed."""
    g = load_golden("g15_fig_train.npz")
    x = torch.from_numpy(g["fig.x"])
    m64 = _load(nfs_amd.RealNVP(2, 10, 128), g, "fig.init.").double().train()
    _, l64 = _fig_train(m64, x.double(), 5)
    ref = g["fig.losses5"]
    m = _load(nfs_amd.RealNVP(2, 10, 128), g, "fig.init.").to(cuda_device).train()
    nfs_amd.reset_stats()
    _, losses = _fig_train(m, x.to(cuda_device), 5)
    assert nfs_amd.STATS["torch"] == 0, nfs_amd.STATS
    losses = np.asarray(losses)
    ok = (np.abs(losses - ref) <= 5e-5) | (np.abs(losses - np.asarray(l64)) <= 1e-4)
    assert ok.all(), (losses.tolist(), ref.tolist(), l64)
    final = {k: torch.from_numpy(g["fig.step5." + k]) for k in m.state_dict() if "fig.step5." + k in g} \
        if np.abs(losses - ref).max() <= 5e-5 else m64.state_dict()
    for k, v in m.state_dict().items():
        # as test_realnvp_adam_steps_vs_reference: biases feeding a BatchNorm (zero gradient up to
        # rounding noise, which Adam turns into +-lr steps) and the running means that track
        # them are not compared
        if k.endswith(("num_batches_tracked", "net.0.bias", "net.3.bias", "running_mean")):
            continue
        _close(v, final[k], rel=2e-4, what=k)


def test_figure_model_graphed_step_equals_eager(cuda_device):
    """The figure model's training step captured as one hipGraph (nfs_amd.GraphedTrainStep: 10
    wide train-mode layers forward + fused backward, clip_grad_norm_, capturable Adam) replays
    the eager step bit for bit (every reduction has a fixed order)."""
    g = load_golden("g15_fig_train.npz")
    x = torch.from_numpy(g["fig.x"]).to(cuda_device)
    a = _load(nfs_amd.RealNVP(2, 10, 128), g, "fig.init.").to(cuda_device).train()
    b = copy.deepcopy(a)
    opt_a = torch.optim.Adam(a.parameters(), lr=1e-3, capturable=True)
    opt_b = torch.optim.Adam(b.parameters(), lr=1e-3, capturable=True)
    la = []
    for _ in range(5):
        z, ld = a.inverse(x)
        loss = _fig_loss(z, ld)
        opt_a.zero_grad(set_to_none=True)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(list(a.parameters()), 5.0)
        opt_a.step()
        la.append(loss.item())
    nfs_amd.reset_stats()
    step = nfs_amd.GraphedTrainStep(b, x, opt_b, warmup=1, clip_grad_norm=5.0,
                                    loss_fn=lambda mod, xx: _fig_loss(*mod.inverse(xx)))
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] > 0, nfs_amd.STATS
    lb = [step().item() for _ in range(4)]
    assert la[1:] == lb, (la, lb)
    for (k, pa), (_, pb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert torch.equal(pa, pb), k
