"""GPU: the sampling pass with its base draw fused in (Flow.sample,
src/flows/flow/flow.py:40-54; the reference's throughput loop, plots/_common.py:264-274).

nfx_affine_chain_sample / nfx_spline_chain_sample draw z ~ N(0, I) on the device (Philox4x32-10 +
Box-Muller in the chain kernel's prologue) and run the forward chain in the same launch. Checked: x and log_det equal the
plain chain's forward(z) on the returned z bit for bit; every call (and every replay of a
captured graph) draws afresh; the same generator state reproduces the same draw; the draws are
standard normal (moments, Kolmogorov-Smirnov distance, no correlation between dimensions or
between consecutive samples).
"""
import math

import pytest
import torch

import nfs_amd

pytestmark = pytest.mark.gpu


def _realnvp(d, n_layers, H, seed):
    torch.manual_seed(seed)
    m = nfs_amd.RealNVP(d, n_layers, H)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.1 * torch.randn(p.shape, generator=g))
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.running_mean.copy_(0.1 * torch.randn(mod.running_mean.shape, generator=g))
                mod.running_var.copy_(0.5 + torch.rand(mod.running_var.shape, generator=g))
    return m


@pytest.mark.parametrize("d,L,H", [(2, 10, 128), (2, 8, 64), (4, 4, 32), (8, 6, 96)])
@pytest.mark.parametrize("n", [1, 33, 4000, 65536])
def test_fused_sample_equals_forward_of_its_draw(cuda_device, d, L, H, n):
    m = _realnvp(d, L, H, 3 * d + L).to(cuda_device).eval()
    assert m.sample_fused_ok(n, cuda_device)
    nfs_amd.reset_stats()
    with torch.no_grad():
        x, ld, z = m.sample_fused(n, cuda_device)
        assert nfs_amd.STATS["hip"] == 1 and nfs_amd.STATS["torch"] == 0
        xr, ldr = m.forward(z)
    assert z.shape == (n, d) and torch.isfinite(z).all()
    assert torch.equal(x, xr) and torch.equal(ld, ldr)


def test_fused_sample_fresh_and_reproducible(cuda_device):
    m = _realnvp(2, 8, 64, 1).to(cuda_device).eval()
    with torch.no_grad():
        _, _, z1 = m.sample_fused(4000, cuda_device)
        z1 = z1.clone()
        _, _, z2 = m.sample_fused(4000, cuda_device)
    assert not torch.equal(z1, z2)
    assert (z1 == z2).float().mean().item() < 1e-3
    dev = torch.device(cuda_device)
    seed, state = m.flow._nfx_rng[dev]
    state.zero_()  # the generator state back to its start: the first draw again
    with torch.no_grad():
        _, _, z3 = m.sample_fused(4000, cuda_device)
    assert torch.equal(z3, z1)


def test_fused_draw_is_standard_normal(cuda_device):
    m = _realnvp(2, 4, 32, 2).to(cuda_device).eval()
    zs = []
    with torch.no_grad():
        for _ in range(8):
            zs.append(m.sample_fused(65536, cuda_device)[2].double().cpu())
    z = torch.cat(zs)  # 524,288 x 2
    v = z.reshape(-1)
    assert abs(v.mean().item()) < 4 / math.sqrt(v.numel())
    assert abs(v.std().item() - 1) < 0.005
    assert abs(((v ** 4).mean() - 3).item()) < 0.03  # kurtosis of N(0, 1)
    s = v.sort().values
    cdf = 0.5 * (1 + torch.erf(s / math.sqrt(2)))
    emp = torch.arange(1, s.numel() + 1, dtype=torch.float64) / s.numel()
    ks = (cdf - emp).abs().max().item()
    assert ks < 1.63 / math.sqrt(s.numel()) * 1.5, ks  # ~1% KS level, with margin
    c = torch.corrcoef(torch.stack([z[:, 0], z[:, 1], torch.roll(z[:, 0], 1)]))
    assert c[0, 1].abs().item() < 0.01 and c[0, 2].abs().item() < 0.01


def test_graphed_fused_sampling(cuda_device):
    """GraphedFlow(mode="sample") on a RealNVP holds the fused kernel: each replay draws afresh
    (the generator state advances on the device), x = forward(z) bit for bit."""
    m = _realnvp(2, 10, 128, 4).to(cuda_device).eval()
    g = nfs_amd.GraphedFlow(m, torch.empty(4000, 2, device=cuda_device), mode="sample")
    assert g.fused_draw and g.launches == 1
    x1 = g()[0].clone()
    z1 = g.static_in.clone()
    x2 = g()[0].clone()
    z2 = g.static_in.clone()
    assert not torch.equal(z1, z2)
    with torch.no_grad():
        assert torch.equal(m.forward(z2)[0], x2)
        assert torch.equal(m.forward(z1)[0], x1)


def test_fused_sample_limits(cuda_device):
    m = _realnvp(2, 4, 32, 5).to(cuda_device)
    assert not m.sample_fused_ok(1 << 17, cuda_device)   # above the small-batch chain
    m.train()
    assert not m.sample_fused_ok(100, cuda_device)       # train-mode BatchNorm: not a fixed map
    with pytest.raises(NotImplementedError):
        m.sample_fused(100, cuda_device)


def _spline(n_layers, H, seed):
    torch.manual_seed(seed)
    m = nfs_amd.RealNVPSpline(2, n_layers, H)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.1 * torch.randn(p.shape, generator=g))
    return m


@pytest.mark.parametrize("L,H", [(8, 64), (4, 32)])
@pytest.mark.parametrize("n", [1, 4000, 300_001])
def test_fused_spline_sample_equals_forward_of_its_draw(cuda_device, L, H, n):
    """RealNVPSpline (K = 10): the spline chain draws z itself; x, log_det = forward(z) bit for
    bit, fresh draws per call, any batch (the streaming spline chain)."""
    m = _spline(L, H, L + H).to(cuda_device).eval()
    assert m.sample_fused_ok(n, cuda_device)
    nfs_amd.reset_stats()
    with torch.no_grad():
        x, ld, z = m.sample_fused(n, cuda_device)
        assert nfs_amd.STATS["hip"] == 1 and nfs_amd.STATS["torch"] == 0
        z = z.clone()
        xr, ldr = m.forward(z)
        _, _, z2 = m.sample_fused(n, cuda_device)
    assert torch.isfinite(z).all()
    assert torch.equal(x, xr) and torch.equal(ld, ldr)
    if n > 1:
        assert not torch.equal(z, z2)
        assert abs(z.mean().item()) < 6 / math.sqrt(z.numel()) + 1e-3 and abs(z.std().item() - 1) < 0.05


def test_graphed_fused_spline_sampling(cuda_device):
    m = _spline(8, 64, 9).to(cuda_device).eval()
    g = nfs_amd.GraphedFlow(m, torch.empty(4000, 2, device=cuda_device), mode="sample")
    assert g.fused_draw and g.launches == 1
    x1 = g()[0].clone()
    z1 = g.static_in.clone()
    g()
    z2 = g.static_in.clone()
    assert not torch.equal(z1, z2)
    with torch.no_grad():
        assert torch.equal(m.forward(z1)[0], x1)
