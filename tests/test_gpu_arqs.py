"""GPU parity of the ARQS kernel (csrc/nfx_arqs*.hip) through the C-ABI.

ARQS (src/flows/spline/arqs.py:7-114) chains d MADE evaluations and unit-interval splines per
sample; a different fp32 summation order in the MADE moves the spline parameters by ulps, which
the spline can amplify, so parity uses the fp32 error model of conftest.assert_fp32_parity:
the kernel must be as close to the float64 evaluation of the reference math (the oracle run in
double) as the reference's own fp32 output is (golden fixtures g10, or the fp32 oracle).
"""
import copy

import numpy as np
import pytest
import torch

import nfs_amd
import oracle
from conftest import assert_fp32_parity, fp32_jitter, load_golden, oracle_sd, state_dict_from

pytestmark = pytest.mark.gpu

CASES = ["a1", "a3", "a5", "a4bn", "a10"]


def _case(g, name):
    d, H, K, bn, lo, hi = g[name + ".meta"]
    rng = {} if np.isnan(lo) else {"data_min": float(lo), "data_max": float(hi)}
    return int(d), int(H), int(K), bool(bn), rng


def _module(g, name, dev):
    d, H, K, bn, rng = _case(g, name)
    m = nfs_amd.ARQS(d, hidden_dim=H, num_bins=K, use_batch_norm=bn, **rng)
    m.load_state_dict(state_dict_from(g, name + ".", m))
    return m.to(dev).eval()


def _oracle64(g, name, x, direction):
    d, H, K, bn, rng = _case(g, name)
    sd = {k: v.double() for k, v in oracle_sd(g, name + ".").items()}
    with torch.no_grad():
        return oracle.arqs(sd, "", x.double(), direction, K=K, batch_norm=bn, **rng)


@pytest.mark.parametrize("name", CASES)
def test_arqs_vs_reference(cuda_device, name):
    g = load_golden("g10_arqs.npz")
    m = _module(g, name, cuda_device)
    x = torch.from_numpy(g[name + ".x"])
    nfs_amd.reset_stats()
    with torch.no_grad():
        yf, lf = m.forward(x.to(cuda_device))
        yi, li = m.inverse(x.to(cuda_device))
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] == 2, nfs_amd.STATS
    for direction, key, y, ld in ((1, "fwd", yf, lf), (-1, "inv", yi, li)):
        y64, l64 = _oracle64(g, name, x, direction)
        d, H, K, bn, rng = _case(g, name)
        sd = oracle_sd(g, name + ".")
        sy, sl = fp32_jitter(lambda s, v: oracle.arqs(s, "", v, direction, K=K, batch_norm=bn, **rng), x, sd=sd)
        assert_fp32_parity(y.cpu(), g[f"{name}.{key}_y"], y64, what=f"{name} {key} y", sens=sy)
        assert_fp32_parity(ld.cpu(), g[f"{name}.{key}_ld"], l64, what=f"{name} {key} ld", sens=sl)


@pytest.mark.parametrize("B", [1, 31, 33, 1000, 4099])
def test_arqs_ragged_batches_vs_oracle(cuda_device, B):
    g = load_golden("g10_arqs.npz")
    name = "a5"
    m = _module(g, name, cuda_device)
    d, H, K, bn, rng = _case(g, name)
    x = torch.rand(B, d, generator=torch.Generator().manual_seed(B))
    sd = oracle_sd(g, name + ".")
    for direction in (1, -1):
        with torch.no_grad():
            y, ld = (m.forward if direction > 0 else m.inverse)(x.to(cuda_device))
            y32, l32 = oracle.arqs(sd, "", x, direction, K=K, batch_norm=bn, **rng)
        y64, l64 = _oracle64(g, name, x, direction)
        sy, sl = fp32_jitter(lambda s, v: oracle.arqs(s, "", v, direction, K=K, batch_norm=bn, **rng), x, sd=sd)
        assert_fp32_parity(y.cpu(), y32, y64, what=f"B={B} dir={direction} y", sens=sy)
        assert_fp32_parity(ld.cpu(), l32, l64, what=f"B={B} dir={direction} ld", sens=sl)


def test_arqs_samples_independent_and_empty(cuda_device):
    """Per-sample independence at a large batch: a 1,000-row slice equals the same rows of a
    200k-row launch bit for bit (size-independent property); B = 0 is a no-op."""
    g = load_golden("g10_arqs.npz")
    m = _module(g, "a10", cuda_device)
    x = 1.2 * torch.randn(200_000, 10, device=cuda_device)
    with torch.no_grad():
        y, ld = m.inverse(x)
        ys, lds = m.inverse(x[123_000:124_000].contiguous())
        ye, le = m.forward(torch.empty(0, 10, device=cuda_device))
    assert torch.equal(y[123_000:124_000], ys) and torch.equal(ld[123_000:124_000], lds)
    assert torch.isfinite(y).all() and torch.isfinite(ld).all()
    assert ye.shape == (0, 10) and le.shape == (0,)


def test_arqs_nonfinite_inputs_match_reference_pattern(cuda_device):
    """NaN/inf inputs: the reference has no guards in ARQS, so a NaN coordinate poisons the
    later MADE calls through 0*NaN in the masked weights; the kernel's NaN pattern must agree."""
    g = load_golden("g10_arqs.npz")
    name = "a3"
    m = _module(g, name, cuda_device)
    d, H, K, bn, rng = _case(g, name)
    x = torch.rand(8, d, generator=torch.Generator().manual_seed(5))
    x[1, 0] = float("nan")
    x[2, 1] = float("nan")
    x[3, 2] = float("inf")
    x[4, 0] = float("-inf")
    sd = oracle_sd(g, name + ".")
    for direction in (1, -1):
        with torch.no_grad():
            y, ld = (m.forward if direction > 0 else m.inverse)(x.to(cuda_device))
            yr, lr = oracle.arqs(sd, "", x, direction, K=K, batch_norm=bn, **rng)
        assert np.array_equal(np.isnan(y.cpu().numpy()), np.isnan(yr.numpy())), (y, yr)
        assert np.array_equal(np.isnan(ld.cpu().numpy()), np.isnan(lr.numpy())), (ld, lr)


def test_arqs_in_flow_model_and_autograd(cuda_device):
    """ARQS inside NormalizingFlowModel (log_prob through the chain) and autograd through the
    HIP forward and the HIP reverse-sweep backward (nfx_arqs_step) against the CPU composite."""
    g = load_golden("g10_arqs.npz")
    a = _module(g, "a4bn", "cpu")
    b = copy.deepcopy(a)
    model = nfs_amd.NormalizingFlowModel([a, nfs_amd.MaskedAutoregressiveFlow(4, 32), b]).eval()
    x = torch.rand(300, 4, generator=torch.Generator().manual_seed(9))
    with torch.no_grad():
        lp_cpu = model.log_prob(x)
    mg = copy.deepcopy(model).to(cuda_device)
    nfs_amd.reset_stats()
    with torch.no_grad():
        lp = mg.log_prob(x.to(cuda_device))
    assert nfs_amd.STATS["torch"] == 0
    assert ((lp.cpu() - lp_cpu).abs() <= 1e-3 * (1 + lp_cpu.abs())).all()

    layer = _module(g, "a3", cuda_device)
    xc = torch.rand(64, 3, generator=torch.Generator().manual_seed(10))
    xg = xc.to(cuda_device).requires_grad_(True)
    y, ld = layer.forward(xg)
    (y.sum() + ld.sum()).backward()
    cpu = _module(g, "a3", "cpu")
    xr = xc.clone().requires_grad_(True)
    yr, lr = cpu.forward(xr)
    (yr.sum() + lr.sum()).backward()
    np.testing.assert_allclose(xg.grad.cpu().numpy(), xr.grad.numpy(), rtol=1e-3, atol=1e-3)
