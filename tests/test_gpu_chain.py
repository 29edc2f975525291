"""GPU: the one-launch coupling chain (nfx_affine_chain, csrc/nfx_affine_chain.hip).

A run of eval-mode CouplingLayers (RealNVP / NormalizingFlowModel / SequentialFlow) at small and
medium batch sizes runs as ONE kernel that keeps each workgroup's rows and running log-det in LDS
through every layer. Its per-layer arithmetic is the small-batch kernel's, so it must equal the
per-layer launches under nfx_affine_kernel_policy(NFX_AFFINE_SMALL) BIT FOR BIT (y, log-det, fused
log_prob and the float64 NLL sums), and match the reference's fixtures (G2) and the oracle within
SURVEY §8(c)'s tolerances.
"""
import numpy as np
import pytest
import torch

import nfs_amd
import oracle
from conftest import load_golden, state_dict_from
from nfs_amd import _lib
from nfs_amd.flows import coupling as _cp

pytestmark = pytest.mark.gpu


def _model(d, H, nl, seed):
    torch.manual_seed(seed)
    layers = []
    for i in range(nl):
        mask = torch.zeros(d)
        mask[(i % 2)::2] = 1
        layers.append(nfs_amd.CouplingLayer(d, H, mask))
    m = nfs_amd.NormalizingFlowModel(layers)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.1 * torch.randn(p.shape, generator=g))
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.running_mean.copy_(0.1 * torch.randn(mod.running_mean.shape, generator=g))
                mod.running_var.copy_(0.5 + torch.rand(mod.running_var.shape, generator=g))
    return m


def _per_layer(fn):
    """Run fn with the chain disabled and the per-layer small-batch kernel forced."""
    old_max, _cp.CHAIN_MAX_B = _cp.CHAIN_MAX_B, 0
    L = _lib.lib()
    old_pol = L.nfx_affine_kernel_policy(_lib.NFX_AFFINE_SMALL)
    try:
        return fn()
    finally:
        _cp.CHAIN_MAX_B = old_max
        L.nfx_affine_kernel_policy(old_pol)


@pytest.mark.parametrize("d,H,nl,B", [(2, 64, 8, 1), (2, 64, 8, 31), (2, 128, 10, 4000), (2, 32, 3, 65536),
                                      (4, 96, 5, 1000), (8, 128, 4, 777), (2, 128, 1, 64), (8, 16, 12, 4097)])
def test_chain_equals_per_layer_bitwise(cuda_device, d, H, nl, B):
    m = _model(d, H, nl, d * 100 + H + nl).to(cuda_device).eval()
    x = torch.randn(B, d, device=cuda_device, generator=torch.Generator(device=cuda_device).manual_seed(B))
    x[0, 0] = float("nan") if B > 4 else x[0, 0]
    with torch.no_grad():
        nfs_amd.reset_stats()
        zc, ldc = m.inverse(x)
        xc, lfc = m.forward(x)
        lpc, sc = m.log_prob(x, return_sums=True)
        assert nfs_amd.STATS["hip"] == 3 and nfs_amd.STATS["torch"] == 0, nfs_amd.STATS  # one launch each
        zp, ldp = _per_layer(lambda: m.inverse(x))
        xp, lfp = _per_layer(lambda: m.forward(x))
        lpp, sp = _per_layer(lambda: m.log_prob(x, return_sums=True))
    for a, b, what in ((zc, zp, "z"), (ldc, ldp, "ld"), (xc, xp, "x"), (lfc, lfp, "fwd ld"), (lpc, lpp, "logp"),
                       (sc, sp, "sums")):
        assert torch.equal(torch.nan_to_num(a, nan=7.0), torch.nan_to_num(b, nan=7.0)), what
        assert torch.equal(torch.isnan(a), torch.isnan(b)), what


def test_chain_realnvp_vs_reference(cuda_device):
    """G2 (the reference's own RealNVP(2,8,64) outputs, incl. edge rows 0, +-1e-6, +-1e3, 1e10):
    the chain path at the fixture's 4,096 rows."""
    g = load_golden("g2_realnvp.npz")
    m = nfs_amd.RealNVP(2, 8, 64)
    m.load_state_dict(state_dict_from(g, "", m))
    m = m.to(cuda_device).eval()
    x = torch.from_numpy(g["x"]).to(cuda_device)
    z = torch.from_numpy(g["z"]).to(cuda_device)
    assert _cp.chain_ok(list(m.flow.flows), x)
    with torch.no_grad():
        zi, ldi = m.inverse(x)
        xf, ldf = m.forward(z)
    for a, ref, tol in ((zi, g["inv_z"], 1e-5), (xf, g["fwd_x"], 1e-5)):
        a, ref = a.cpu().numpy().astype(np.float64), ref.astype(np.float64)
        assert (np.abs(a - ref) <= tol * (1 + np.abs(ref))).all()
    assert np.abs(ldi.cpu().numpy() - g["inv_ld"]).max() <= 1e-4
    assert np.abs(ldf.cpu().numpy() - g["fwd_ld"]).max() <= 1e-4


def test_chain_sequential_flow_and_graph(cuda_device):
    """SequentialFlow (zeros(B) accumulator, sequential_flow.py:15-34) and a captured sampling
    graph (GraphedFlow mode='sample') take the chain; both equal the per-layer composition."""
    torch.manual_seed(5)
    masks = [torch.tensor([1.0, 0.0]), torch.tensor([0.0, 1.0])]
    sf = nfs_amd.SequentialFlow([nfs_amd.CouplingLayer(2, 128, masks[i % 2]) for i in range(10)])
    with torch.no_grad():
        for p in sf.parameters():
            p.add_(0.1 * torch.randn_like(p))
    sf = sf.to(cuda_device).eval()
    x = torch.randn(4000, 2, device=cuda_device)
    with torch.no_grad():
        nfs_amd.reset_stats()
        y, ld = sf.forward(x)
        assert nfs_amd.STATS["hip"] == 1, nfs_amd.STATS
        yp, ldp = _per_layer(lambda: sf.forward(x))
    assert torch.equal(y, yp) and torch.equal(ld, ldp)
    m = nfs_amd.RealNVP(2, 10, 128).to(cuda_device).eval()
    gf = nfs_amd.GraphedFlow(m.flow, x, mode="forward")
    with torch.no_grad():
        ye, lde = m.forward(x)
        yg = gf()
    yg = yg[0] if isinstance(yg, tuple) else yg
    assert torch.equal(yg, ye)


def _policy(pol, fn, chain=True):
    """Run fn under nfx_affine_kernel_policy(pol), with the one-launch chains on or off."""
    L = _lib.lib()
    old_max = _cp.CHAIN_MAX_B
    if not chain:
        _cp.CHAIN_MAX_B = 0
    old_pol = L.nfx_affine_kernel_policy(pol)
    try:
        return fn()
    finally:
        _cp.CHAIN_MAX_B = old_max
        L.nfx_affine_kernel_policy(old_pol)


@pytest.mark.parametrize("d,H,nl,B", [(2, 64, 8, 125000), (2, 64, 8, 1), (2, 64, 2, 65), (2, 32, 3, 70001),
                                      (4, 64, 5, 200003), (8, 64, 4, 600001), (8, 16, 6, 9999),
                                      (2, 64, 8, 2_000_001)])
def test_streaming_chain_equals_per_layer_bitwise(cuda_device, d, H, nl, B):
    """The streaming chain (csrc/nfx_affine_schain.hip: rows in LDS through every layer, the next
    layer's weights DMA'd during the current one) runs the per-layer streaming kernel's arithmetic:
    y, log-det and logp equal the per-layer streaming launches bit for bit; the float64 NLL sums
    (summed in another order) to 1e-12. B = 2,000,001 at d = 2 and 600,001 at d = 8 take more than
    one LDS slice per workgroup; B = 1 and 65 leave most workgroups without rows."""
    S = _lib.NFX_AFFINE_STREAMING
    m = _model(d, H, nl, d * 1000 + H + nl).to(cuda_device).eval()
    x = torch.randn(B, d, device=cuda_device, generator=torch.Generator(device=cuda_device).manual_seed(B))
    if B > 4:
        x[0, 0] = float("nan")
        x[1, -1] = float("inf")
        x[2] = 1e10
    assert _policy(S, lambda: _cp.chain_ok(list(m.flows), x))
    with torch.no_grad():
        nfs_amd.reset_stats()
        zc, ldc = _policy(S, lambda: m.inverse(x))
        xc, lfc = _policy(S, lambda: m.forward(x))
        lpc, sc = _policy(S, lambda: m.log_prob(x, return_sums=True))
        assert nfs_amd.STATS["hip"] == 3 and nfs_amd.STATS["torch"] == 0, nfs_amd.STATS  # one launch each
        zp, ldp = _policy(S, lambda: m.inverse(x), chain=False)
        xp, lfp = _policy(S, lambda: m.forward(x), chain=False)
        lpp, sp = _policy(S, lambda: m.log_prob(x, return_sums=True), chain=False)
    for a, b, what in ((zc, zp, "z"), (ldc, ldp, "ld"), (xc, xp, "x"), (lfc, lfp, "fwd ld"), (lpc, lpp, "logp")):
        assert torch.equal(torch.nan_to_num(a, nan=7.0), torch.nan_to_num(b, nan=7.0)), what
        assert torch.equal(torch.isnan(a), torch.isnan(b)), what
    assert float(sc[1]) == float(sp[1]) == B
    a, b = float(sc[0]), float(sp[0])
    assert a == b or abs(a - b) <= 1e-12 * max(1.0, abs(b)), (sc, sp)  # (-inf when a row's logp is -inf)


def test_streaming_chain_realnvp_vs_reference(cuda_device):
    """G2 through the streaming chain (policy forced) and the G8 full-scale cfg2 NLL at 1M rows
    through the default (AUTO) route, which is the streaming chain at that batch."""
    g = load_golden("g2_realnvp.npz")
    m = nfs_amd.RealNVP(2, 8, 64)
    m.load_state_dict(state_dict_from(g, "", m))
    m = m.to(cuda_device).eval()
    x = torch.from_numpy(g["x"]).to(cuda_device)
    with torch.no_grad():
        zi, ldi = _policy(_lib.NFX_AFFINE_STREAMING, lambda: m.inverse(x))
    a, ref = zi.cpu().numpy().astype(np.float64), g["inv_z"].astype(np.float64)
    assert (np.abs(a - ref) <= 1e-5 * (1 + np.abs(ref))).all()
    assert np.abs(ldi.cpu().numpy() - g["inv_ld"]).max() <= 1e-4
