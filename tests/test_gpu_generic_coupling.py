"""GPU: CouplingLayer (RealNVP) on the any-shape path (csrc/nfx_generic.hip) — the conditioner
one nn.Linear at a time on fp32 MFMA, BatchNorm1d by its own kernels (running statistics in
eval; batch moments, SyncBN merge and running update in train), the affine element map and
adjoint — for layers beyond the fused kernel families (d > 8 or H > 128 in training, d > 64 or
H > 128 in eval).

* Forced onto the fused shapes (coupling.FORCE_GENERIC) it must pass the fused path's own
  reference tests: G11 (RealNVP(2,8,64) train step: z, NLL, every gradient, running statistics;
  a d = 4 layer both directions), G15 (the figure model RealNVP(2,10,128) train step), the
  eval-mode RealNVP step, and the G2 eval outputs — same tolerances as test_gpu_affine_train.py
  / test_gpu_affine.py.
* Beyond the fused families, against float64 autograd (train and eval mode) and the oracle
  (eval outputs), with the tolerances of test_gpu_affine_train.py (outputs of wide layers held to
  4x the reference's own fp32 error, _close_or_ref).
"""
import copy

import numpy as np
import pytest
import torch

import nfs_amd
import oracle
import test_gpu_affine_train as T
from conftest import load_golden, state_dict_from
from nfs_amd.flows import coupling as _cp
from nfs_amd.flows.flow import STATS

pytestmark = pytest.mark.gpu


@pytest.fixture
def force_generic():
    old = _cp.FORCE_GENERIC
    _cp.FORCE_GENERIC = True
    yield
    _cp.FORCE_GENERIC = old


def test_generic_g11_train_step(cuda_device, force_generic):
    T.test_realnvp_train_step_vs_reference(cuda_device)


def test_generic_g11_adam_steps(cuda_device, force_generic):
    T.test_realnvp_adam_steps_vs_reference(cuda_device)


def test_generic_g11_d4_layer(cuda_device, force_generic):
    T.test_layer_d4_both_directions_vs_reference(cuda_device)


def test_generic_g15_figure_model_step(cuda_device, force_generic):
    T.test_figure_model_train_step_vs_reference(cuda_device)


def test_generic_eval_realnvp_step(cuda_device, force_generic):
    T.test_eval_mode_realnvp_step_matches_float64(cuda_device)


def test_generic_g2_eval_outputs(cuda_device, force_generic):
    """The reference's RealNVP(2,8,64) eval outputs (G2, incl. edge rows) on the any-shape path."""
    from test_gpu_affine import realnvp_from_golden
    m, g = realnvp_from_golden(cuda_device)
    STATS["hip"] = STATS["torch"] = 0
    with torch.no_grad():
        zi, ldi = m.inverse(torch.from_numpy(g["x"]).to(cuda_device))
        xf, ldf = m.forward(torch.from_numpy(g["z"]).to(cuda_device))
    assert STATS["torch"] == 0 and STATS["hip"] == 16, STATS
    for a, ref in ((zi, g["inv_z"]), (xf, g["fwd_x"])):
        a, ref = a.cpu().numpy().astype(np.float64), ref.astype(np.float64)
        assert (np.abs(a - ref) <= 1e-5 * (1 + np.abs(ref))).all()
    assert np.abs(ldi.cpu().numpy() - g["inv_ld"]).max() <= 1e-4
    assert np.abs(ldf.cpu().numpy() - g["fwd_ld"]).max() <= 1e-4


@pytest.mark.parametrize("d,H,B,direction", [(12, 64, 1000, -1), (16, 32, 777, 1), (2, 256, 2000, -1),
                                             (10, 160, 513, 1), (80, 48, 300, -1)])
def test_generic_train_layer_vs_float64(cuda_device, d, H, B, direction):
    """Train mode beyond the fused train kernels (d > 8 or H > 128)."""
    assert not T._perturbed_layer(d, H, 0)._fused_train()
    T.test_layer_vs_float64_autograd(cuda_device, d, H, B, direction)


@pytest.mark.parametrize("d,H,B,direction", [(12, 64, 1000, 1), (2, 256, 2000, -1), (70, 40, 257, -1)])
def test_generic_eval_backward_vs_float64(cuda_device, d, H, B, direction):
    """Eval mode under autograd beyond the fused backward (d > 8 or H > 128); wide layers' fp32
    outputs are held to the reference's own fp32 error (T._close_or_ref), as in train mode."""
    layer = T._perturbed_layer(d, H, 300 + d * 5 + H, mask_even=(B % 2 == 1))
    assert not layer._fused_train()
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
    x32 = x.clone().requires_grad_(True)
    y32, ld32 = ref32.forward(x32) if direction > 0 else ref32.inverse(x32)
    ((y32 * wy).sum() + (ld32 * wl).sum()).backward()
    STATS["hip"] = STATS["torch"] = 0
    xg = x.to(cuda_device).requires_grad_(True)
    yg, ldg = gpu.forward(xg) if direction > 0 else gpu.inverse(xg)
    ((yg * wy.to(cuda_device)).sum() + (ldg * wl.to(cuda_device)).sum()).backward()
    assert STATS["torch"] == 0 and STATS["hip"] == 2, STATS
    T._close_or_ref(yg, yr, y32, what="y")
    T._close_or_ref(ldg, ldr, ld32, what="log_det")
    T._gclose(xg.grad, xr.grad, what="dL/dx", ref32=x32.grad)
    for (k, pg), (_, pr), (_, p32) in zip(gpu.named_parameters(), ref.named_parameters(), ref32.named_parameters()):
        T._gclose(pg.grad, pr.grad, what=k + " (eval)", ref32=p32.grad)
    for k, v in gpu.named_buffers():
        assert torch.equal(v, before[k]), f"eval backward changed buffer {k}"


@pytest.mark.parametrize("d,H", [(80, 32), (4, 256), (66, 200)])
def test_generic_eval_outputs_vs_oracle(cuda_device, d, H):
    """Eval outputs beyond the fused eval kernels (d > 64 or H > 128) against the oracle."""
    layer = T._perturbed_layer(d, H, 5 * d + H).eval()
    assert not layer._fused_family()
    sd = {k: v.clone() for k, v in layer.state_dict().items()}
    x = torch.randn(600, d, generator=torch.Generator().manual_seed(d))
    x[0, 0] = float("inf")
    gpu = layer.to(cuda_device)
    for direction in (1, -1):
        STATS["hip"] = STATS["torch"] = 0
        with torch.no_grad():
            yg, lg = (gpu.forward if direction > 0 else gpu.inverse)(x.to(cuda_device))
            y64, l64 = oracle.coupling({k: v.double() for k, v in sd.items()}, "", x.double(), direction)
            y32, l32 = oracle.coupling(sd, "", x, direction)
        assert STATS["hip"] == 1 and STATS["torch"] == 0, STATS
        # the oracle in float64, with the reference's own fp32 error as the yardstick
        T._close_or_ref(yg, y64, y32, what=f"y dir={direction}")
        T._close_or_ref(lg, l64, l32, rel=1e-4, what=f"ld dir={direction}")
