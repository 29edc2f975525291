"""GPU: the one-launch spline coupling chain (nfx_spline_chain, csrc/nfx_spline_schain_kernel.h).

A run of eval-mode SplineCouplingLayers at d = 2 (cfg3, RealNVPSpline) runs as ONE kernel: one
workgroup per CU carries its rows and running log-det in LDS through every layer, with the
per-layer kernel's arithmetic (spline_unit_apply: the same operations in the same order). It must
equal the per-layer launches BIT FOR BIT (y, log-det, fused log_prob; the float64 NLL sums, summed
in another order, to 1e-12) and match the reference's fixtures (G3) within SURVEY §8(c)'s
tolerances.
"""
import numpy as np
import pytest
import torch

import nfs_amd
from conftest import load_golden, state_dict_from
from nfs_amd.flows import spline as _sp

pytestmark = pytest.mark.gpu


def _model(H, K, nl, seed, bound=5.0):
    torch.manual_seed(seed)
    layers = []
    for i in range(nl):
        mask = torch.zeros(2)
        mask[i % 2] = 1
        layers.append(nfs_amd.SplineCouplingLayer(2, H, mask, num_bins=K, bound=bound))
    m = nfs_amd.NormalizingFlowModel(layers)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.3 * torch.randn(p.shape, generator=g))
    return m


def _per_layer(fn):
    old, _sp.CHAIN_ENABLED = _sp.CHAIN_ENABLED, False
    try:
        return fn()
    finally:
        _sp.CHAIN_ENABLED = old


@pytest.mark.parametrize("H,K,nl,B", [(64, 8, 8, 125000), (64, 10, 8, 4000), (64, 8, 2, 1), (32, 2, 3, 65),
                                      (64, 11, 4, 70001), (16, 5, 6, 9999), (64, 8, 8, 2_000_001)])
def test_spline_chain_equals_per_layer_bitwise(cuda_device, H, K, nl, B):
    """B = 2,000,001 takes more than one LDS slice per workgroup; B = 1 and 65 leave most
    workgroups without rows; rows on knots, outside +-bound and non-finite inputs included."""
    m = _model(H, K, nl, H * 100 + K * 10 + nl).to(cuda_device).eval()
    x = 2.5 * torch.randn(B, 2, device=cuda_device, generator=torch.Generator(device=cuda_device).manual_seed(B))
    if B > 8:
        x[0, 0] = float("nan")
        x[1, 1] = float("inf")
        x[2] = 1e10
        x[3] = torch.tensor([5.0, -5.0])
        x[4] = torch.tensor([-5.0, 5.0 + 1e-6])
    assert _sp.chain_ok(list(m.flows), x)
    with torch.no_grad():
        nfs_amd.reset_stats()
        zc, ldc = m.inverse(x)
        xc, lfc = m.forward(x)
        lpc, sc = m.log_prob(x, return_sums=True)
        assert nfs_amd.STATS["hip"] == 3 and nfs_amd.STATS["torch"] == 0, nfs_amd.STATS  # one launch each
        zp, ldp = _per_layer(lambda: m.inverse(x))
        xp, lfp = _per_layer(lambda: m.forward(x))
        lpp, sp = _per_layer(lambda: m.log_prob(x, return_sums=True))
    for a, b, what in ((zc, zp, "z"), (ldc, ldp, "ld"), (xc, xp, "x"), (lfc, lfp, "fwd ld"), (lpc, lpp, "logp")):
        assert torch.equal(torch.nan_to_num(a, nan=7.0), torch.nan_to_num(b, nan=7.0)), what
        assert torch.equal(torch.isnan(a), torch.isnan(b)), what
    assert float(sc[1]) == float(sp[1]) == B
    a, b = float(sc[0]), float(sp[0])
    assert a == b or abs(a - b) <= 1e-12 * max(1.0, abs(b)), (sc, sp)  # (-inf when a row's logp is -inf)


def test_spline_chain_sequential_flow(cuda_device):
    """SequentialFlow of SplineCouplingLayers takes the chain too (zeros(B) accumulator)."""
    m = _model(64, 8, 4, 3)
    sf = nfs_amd.SequentialFlow(list(m.flows)).to(cuda_device).eval()
    x = torch.randn(3000, 2, device=cuda_device)
    with torch.no_grad():
        nfs_amd.reset_stats()
        y, ld = sf.forward(x)
        assert nfs_amd.STATS["hip"] == 1, nfs_amd.STATS
        yp, ldp = _per_layer(lambda: sf.forward(x))
    assert torch.equal(y, yp) and torch.equal(ld, ldp)


@pytest.mark.parametrize("tag", ["k8.", "k10."])
def test_spline_chain_vs_per_layer_on_reference_models(cuda_device, tag):
    """G3's models (the reference's own 8x SplineCouplingLayer(2,64,K=8) and RealNVPSpline(2,8,64)
    K=10 weights and rows, incl. knots, +-bound, outside it and 1e10): chain == per-layer bit for
    bit. (test_gpu_spline.py::test_spline_model_vs_reference checks the same models, now routed
    through the chain, against the reference's outputs.)"""
    from test_gpu_spline import load_model
    m, g = load_model(tag, cuda_device)
    x = torch.from_numpy(g["x"]).to(cuda_device)
    z = torch.from_numpy(g["z"]).to(cuda_device)
    flows = list(m.flows) if tag == "k8." else list(m.flow.flows)
    assert _sp.chain_ok(flows, x)
    with torch.no_grad():
        got = m.inverse(x) + m.forward(z)
        ref = _per_layer(lambda: m.inverse(x) + m.forward(z))
    for a, b in zip(got, ref):
        assert torch.equal(torch.nan_to_num(a, nan=7.0), torch.nan_to_num(b, nan=7.0))
