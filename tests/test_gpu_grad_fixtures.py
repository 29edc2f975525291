"""GPU: fused backward kernels against gradients captured from the REFERENCE itself (G14, G15).

G14 (tests/golden/make_golden.py:g14): dL/dx and every parameter gradient of
L = sum(y * wy) + sum(ld * wl) through the reference's own MaskedAutoregressiveFlow /
InverseAutoregressiveFlow (both directions; the sequential ones differentiated through all d
MADE calls: masked_autoregressive_flow.py:18-78, inverse_autoregressive_flow.py:30-103) and
SplineCouplingLayer K=8 / K=10 (spline_coupling_layer.py:96-309), in both directions.

Tolerance. The reference's gradients are fp32 autograd sums over the batch; the kernels sum in
another (MFMA) order. Each gradient tensor must satisfy
    max |g - g_ref| <= 2e-5 (1 + max |g_ref|) + 2 max |g_ref - g64|
g64 = float64 autograd of the same module (the exact gradient): within the fixed tolerance of
the reference, widened only by the reference's OWN measured distance from exact arithmetic
(spline inputs next to a knot are ill-conditioned; see test_gpu_spline_backward.py).
Outputs y / ld: MADE |dy| <= 2e-5 (1 + |ref|), |dld| <= 2e-4 (d = 784: + 1e-6 of max |ld|);
spline outputs by conftest.assert_fp32_parity.
"""
import copy

import numpy as np
import pytest
import torch

import nfs_amd
import oracle
from conftest import assert_fp32_parity, fp32_jitter, load_golden, oracle_sd, state_dict_from
from nfs_amd.flows.flow import STATS

pytestmark = pytest.mark.gpu


def _g14_module(name):
    if name.startswith("maf"):
        d, H = {"maf10": (10, 32), "maf63": (63, 64)}[name]
        return nfs_amd.MaskedAutoregressiveFlow(d, H)
    if name.startswith("iaf"):
        d, H = {"iaf10": (10, 32), "iaf784": (784, 64)}[name]
        return nfs_amd.InverseAutoregressiveFlow(d, H)
    if name == "sp8":
        return nfs_amd.SplineCouplingLayer(2, 64, torch.tensor([1.0, 0.0]), num_bins=8)
    return nfs_amd.SplineCouplingLayer(3, 32, torch.tensor([0.0, 1.0, 0.0]), num_bins=10)


def _run(m, x, wy, wl, dname):
    x = x.clone().requires_grad_(True)
    for p in m.parameters():
        p.grad = None
    y, ld = m.inverse(x) if dname == "inv" else m.forward(x)
    ((y * wy).sum() + (ld * wl).sum()).backward()
    return y.detach(), ld.detach(), x.grad, {k: p.grad for k, p in m.named_parameters()}


def _grad_close(g, ref, g64, what):
    g, ref, g64 = (np.asarray(t.detach().cpu().double() if torch.is_tensor(t) else t, np.float64) for t in (g, ref, g64))
    bound = 2e-5 * (1 + np.abs(ref).max()) + 2 * np.abs(ref - g64).max()
    err = np.abs(g - ref).max()
    assert err <= bound, f"{what}: max |g - g_ref| {err:.3g} > {bound:.3g} (reference vs float64 {np.abs(ref - g64).max():.3g})"


@pytest.mark.parametrize("name", ["maf10", "iaf10", "maf63", "iaf784", "sp8", "sp10"])
@pytest.mark.parametrize("dname", ["inv", "fwd"])
def test_backward_vs_reference_gradients_g14(cuda_device, name, dname):
    g = load_golden("g14_grads.npz")
    m = _g14_module(name)
    m.load_state_dict(state_dict_from(g, name + ".init.", m))
    m.eval()
    m64 = copy.deepcopy(m).double()
    x, wy, wl = (torch.from_numpy(g[f"{name}.{k}"]) for k in ("x", "wy", "wl"))
    _, _, gx64, gp64 = _run(m64, x.double(), wy.double(), wl.double(), dname)
    mg = m.to(cuda_device)
    STATS["hip"] = STATS["torch"] = 0
    y, ld, gx, gp = _run(mg, x.to(cuda_device), wy.to(cuda_device), wl.to(cuda_device), dname)
    assert STATS["torch"] == 0 and STATS["hip"] == 2, STATS  # fused forward + fused backward
    yr, ldr = g[f"{name}.{dname}.y"], g[f"{name}.{dname}.ld"]
    if name.startswith("sp"):  # RQ spline outputs: the fp32 error model of conftest
        K = 8 if name == "sp8" else 10
        sd = oracle_sd(g, name + ".init.")
        sd64 = {k: v.double() for k, v in sd.items()}
        direction = -1 if dname == "inv" else 1
        with torch.no_grad():
            y64, l64 = oracle.spline_coupling(sd64, "", x.double(), direction, K=K)
        ens = fp32_jitter(lambda s, v: oracle.spline_coupling(s, "", v, direction, K=K), x, sd=sd)
        assert_fp32_parity(y.cpu(), yr, y64, what=f"{name} {dname} y", sens=ens[0])
        assert_fp32_parity(ld.cpu(), ldr, l64, what=f"{name} {dname} ld", sens=ens[1])
    else:
        assert (np.abs(y.cpu().numpy().astype(np.float64) - yr) <= 2e-5 * (1 + np.abs(yr))).all()
        ltol = 1e-6 * np.abs(ldr).max() + 2e-4 if name == "iaf784" else 2e-4
        assert np.abs(ld.cpu().numpy().astype(np.float64) - ldr).max() <= ltol
    _grad_close(gx, g[f"{name}.{dname}.gx"], gx64, "dL/dx")
    for k in gp64:
        _grad_close(gp[k], g[f"{name}.{dname}.grad.{k}"], gp64[k], k)
