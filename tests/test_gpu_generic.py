"""GPU: the any-shape path (csrc/nfx_generic.hip) — nn.Linear on fp32 MFMA and the spline
coupling's element kernels, for layers beyond the fused kernel families.

* nfx_linear_*: forward (x * scale) W^T + b (+ ReLU), data gradient (masked by the ReLU feeding
  the layer, times a scale, accumulated) and weight/bias gradients (split over the batch, fixed
  order) against float64 torch on the same inputs. Tolerance: an fp32 dot product of length n
  carries at most ~n ulp of sum |a_i b_i|; checked as |C - C64| <= 1e-5 (|A||B|) + 1e-30 per
  element (|A||B| = the absolute-value product, the conditioning of each entry).
* SplineCouplingLayer on the any-shape path — eval beyond the fused eval family (H = 256,
  d = 80) against the CPU oracle with the fp32 parity model of conftest; gradients beyond the
  fused backward family (H = 128, several transformed dims at H = 64, d = 12) against float64
  autograd with the error model of test_gpu_spline_backward.py; and forced onto the fused shapes
  (spline.FORCE_GENERIC) against the reference's own gradients (G14) and the fused kernels.
* MAF / IAF on the any-shape path — forced onto the reference's fixtures (G5 both directions,
  G9, the G14 gradients of the parallel directions), H > 256 against the oracle (both
  directions; the sequential ones as the reference's d MADE calls), eval BatchNorm at H = 288,
  and H = 320 gradients against float64 autograd (MADE tolerances of test_gpu_made.py /
  test_gpu_grad_fixtures.py).
"""
import copy

import numpy as np
import pytest
import torch
import torch.nn as nn

import nfs_amd
import oracle
from conftest import assert_fp32_parity, fp32_jitter, load_golden, oracle_sd, state_dict_from
from nfs_amd.flows import generic as G
from nfs_amd.flows import spline as _sp
from nfs_amd.flows.flow import STATS
from test_gpu_spline_backward import _check, _grads, _ill_rows_checked, _layer

pytestmark = pytest.mark.gpu


def _close(c, c64, conditioning, what):
    c = c.double().cpu()
    err = (c - c64).abs()
    bound = 1e-5 * conditioning + 1e-30
    worst = (err - bound).max().item()
    assert worst <= 0, f"{what}: max excess {worst:.3g} (max err {err.max().item():.3g})"


@pytest.mark.parametrize("M,K,N", [(1000, 2, 64), (4097, 64, 64), (300, 128, 232), (70001, 128, 128),
                                   (5, 3, 1), (1, 96, 33), (2048, 784, 64),
                                   # the thin weight gradient (min(N, K) <= 8): x thin, gy thin, both
                                   (100003, 8, 256), (3000, 96, 5), (777, 200, 8), (65, 7, 3)])
def test_linear_kernels_vs_float64(cuda_device, M, K, N):
    g = torch.Generator().manual_seed(M + K + N)
    lin = nn.Linear(K, N)
    x = torch.randn(M, K, generator=g)
    s = (torch.rand(K, generator=g) > 0.3).float()
    gy = torch.randn(M, N, generator=g)
    act = torch.relu(torch.randn(M, K, generator=g))
    base = torch.randn(M, K, generator=g)
    w64, b64, x64, s64 = lin.weight.double(), lin.bias.double(), x.double(), s.double()
    linc = copy.deepcopy(lin).to(cuda_device)
    dx, ds, dgy, dact = (t.to(cuda_device) for t in (x, s, gy, act))
    # forward, with and without the ReLU and the input scale
    for relu, scale in ((False, None), (True, ds)):
        y = G.linear_forward(dx, linc, scale, relu=relu)
        xs = x64 * s64 if scale is not None else x64
        y64 = xs @ w64.T + b64
        if relu:
            y64 = torch.relu(y64)
        _close(y, y64, xs.abs() @ w64.abs().T + b64.abs(), f"forward relu={relu}")
    # data gradient: masked by act > 0, times s, accumulated into `base`
    out = base.to(cuda_device).clone()
    G.linear_backward_data(dgy, linc, act=dact, out_scale=ds, out=out)
    gx64 = base.double() + torch.where(act.double() > 0, (gy.double() @ w64) * s64, torch.zeros(()))
    _close(out, gx64, base.double().abs() + (gy.double().abs() @ w64.abs()), "backward data")
    gx = G.linear_backward_data(dgy, linc)
    _close(gx, gy.double() @ w64, gy.double().abs() @ w64.abs(), "backward data (plain)")
    # weight and bias gradients (input scaled by s)
    gw, gb = G.linear_backward_weight(dgy, dx, linc, ds)
    xs = x64 * s64
    _close(gw, gy.double().T @ xs, gy.double().abs().T @ xs.abs(), "weight grad")
    _close(gb, gy.double().sum(0), gy.double().abs().sum(0), "bias grad")


@pytest.mark.parametrize("K,N", [(128, 128), (2, 256), (256, 3)])
def test_linear_weight_grad_deterministic(cuda_device, K, N):
    """Split-K partials (MFMA and thin paths) are summed in a fixed order: bitwise identical on repeat."""
    lin = nn.Linear(K, N).to(cuda_device)
    x = torch.randn(300000, K, device=cuda_device)
    gy = torch.randn(300000, N, device=cuda_device)
    a = G.linear_backward_weight(gy, x, lin)
    b = G.linear_backward_weight(gy, x, lin)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def sd64(sd):
    return {k: v.double() for k, v in sd.items()}


@pytest.mark.parametrize("d,H,K,mask", [(2, 256, 8, [1, 0]), (4, 320, 5, [0, 1, 0, 1]),
                                        (80, 32, 4, [(i % 3 == 0) * 1.0 for i in range(80)])])
def test_generic_spline_eval_vs_oracle(cuda_device, d, H, K, mask):
    """Eval beyond the fused eval family (H > 128 or d > 64) runs the any-shape path."""
    torch.manual_seed(d * 100 + H + K)
    layer = nfs_amd.SplineCouplingLayer(d, H, torch.tensor(mask, dtype=torch.float32), num_bins=K)
    with torch.no_grad():
        for p in layer.parameters():
            p.add_(0.1 * torch.randn_like(p))
    x = torch.randn(1000, d) * 2.5
    x[0, 0] = float("nan")
    sd = {k: v.clone() for k, v in layer.state_dict().items()}
    layer = layer.to(cuda_device).eval()
    assert not layer._fused_family()
    for direction in (1, -1):
        STATS["hip"] = STATS["torch"] = 0
        with torch.no_grad():
            yg, lg = (layer.forward if direction > 0 else layer.inverse)(x.to(cuda_device))
        assert STATS["hip"] == 1 and STATS["torch"] == 0, STATS
        with torch.no_grad():
            yr, lr = oracle.spline_coupling(sd, "", x, direction, K=K)
            y64, l64 = oracle.spline_coupling(sd64(sd), "", x.double(), direction, K=K)
        sy, sl = fp32_jitter(lambda s, v: oracle.spline_coupling(s, "", v, direction, K=K), x, sd=sd, k=4,
                             n_perm=4, n_wjit=4)
        assert_fp32_parity(yg.cpu(), yr, y64, what=f"y dir={direction}", sens=sy)
        assert_fp32_parity(lg.cpu(), lr, l64, what=f"ld dir={direction}", sens=sl)


GRAD_CASES = [
    # d, H, K, mask, B — all beyond the fused backward (H > 64, or > 1 transformed dim at H = 64,
    # or d > 8)
    (2, 128, 10, [1, 0], 4096),        # RealNVPSpline(2, *, 128)
    (4, 64, 8, [1, 0, 1, 0], 2000),    # two transformed dims at H = 64
    (3, 128, 5, [0, 1, 0], 777),
    (12, 48, 4, [(i % 2) * 1.0 for i in range(12)], 513),
    (2, 256, 8, [0, 1], 300),
]


@pytest.mark.parametrize("direction", [1, -1])
@pytest.mark.parametrize("d,H,K,mask,B", GRAD_CASES)
def test_generic_spline_backward_vs_float64_autograd(cuda_device, d, H, K, mask, B, direction):
    f = _layer(d, H, K, mask, d * 1000 + H * 10 + K, scale=0.1)
    assert not f._fused_backward_ok()
    f64 = copy.deepcopy(f).double()
    g = torch.Generator().manual_seed(B + K)
    x = 2.0 * torch.randn(B, d, generator=g)
    if B >= 8:
        x[:4] *= 4.0
    gy = torch.randn(B, d, generator=g)
    gld = torch.randn(B, generator=g)
    fg = copy.deepcopy(f).to(cuda_device)
    ill = _ill_rows_checked(f, f64, fg, x, gy, gld, direction, cuda_device)
    gy[ill] = 0.0
    gld[ill] = 0.0
    gx64, gp64, _, _ = _grads(f64, x.double(), gy.double(), gld.double(), direction)
    gx32, gp32, _, _ = _grads(f, x, gy, gld, direction)
    STATS["hip"] = STATS["torch"] = 0
    gx, gp, _, _ = _grads(fg, x.to(cuda_device), gy.to(cuda_device), gld.to(cuda_device), direction)
    assert STATS["hip"] == 2 and STATS["torch"] == 0, STATS  # HIP forward + HIP backward
    _check(gx, gx32, gx64, "dL/dx")
    for (n, _), a, b, c in zip(f.named_parameters(), gp, gp32, gp64):
        _check(a, b, c, n)


@pytest.fixture
def force_generic():
    old = _sp.FORCE_GENERIC
    _sp.FORCE_GENERIC = True
    yield
    _sp.FORCE_GENERIC = old


@pytest.mark.parametrize("name", ["sp8", "sp10"])
@pytest.mark.parametrize("dname", ["inv", "fwd"])
def test_generic_spline_vs_reference_gradients_g14(cuda_device, force_generic, name, dname):
    """The any-shape path forced onto G14's layers: the reference's own fp32 gradients."""
    from test_gpu_grad_fixtures import _g14_module, _grad_close, _run
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
    assert STATS["torch"] == 0 and STATS["hip"] == 2, STATS
    K = 8 if name == "sp8" else 10
    sd = oracle_sd(g, name + ".init.")
    direction = -1 if dname == "inv" else 1
    with torch.no_grad():
        y64, l64 = oracle.spline_coupling(sd64(sd), "", x.double(), direction, K=K)
    ens = fp32_jitter(lambda s, v: oracle.spline_coupling(s, "", v, direction, K=K), x, sd=sd)
    assert_fp32_parity(y.cpu(), g[f"{name}.{dname}.y"], y64, what=f"{name} {dname} y", sens=ens[0])
    assert_fp32_parity(ld.cpu(), g[f"{name}.{dname}.ld"], l64, what=f"{name} {dname} ld", sens=ens[1])
    _grad_close(gx, g[f"{name}.{dname}.gx"], gx64, "dL/dx")
    for k in gp64:
        _grad_close(gp[k], g[f"{name}.{dname}.grad.{k}"], gp64[k], k)


def test_realnvp_spline_h128_training_step(cuda_device):
    """loss = -log_prob(x).mean(); backward through RealNVPSpline(2, 6, 128) (K = 10): every
    layer's forward and backward on HIP (fused eval kernel forward, any-shape backward), loss
    and gradients vs the float64 model."""
    from test_gpu_spline_backward import _ill_rows, _model_grads
    torch.manual_seed(5)
    model = nfs_amd.RealNVPSpline(2, 6, 128)
    g = torch.Generator().manual_seed(6)
    with torch.no_grad():
        for p in model.parameters():
            p.add_(0.1 * torch.randn(p.shape, generator=g))
    ref64 = copy.deepcopy(model).double()
    ref32 = copy.deepcopy(model)
    data = torch.randn(2000, 2, generator=g) * torch.tensor([1.5, 0.7])
    model = model.to(cuda_device).train()
    w = torch.ones(2000)
    loss64, gx64, _ = _model_grads(ref64, data.double(), w.double())
    _, gx32, _ = _model_grads(ref32, data, w)
    STATS["hip"] = STATS["torch"] = 0
    loss, gx, _ = _model_grads(model, data.to(cuda_device), w.to(cuda_device))
    assert STATS["torch"] == 0 and STATS["hip"] >= 12, STATS
    assert abs(loss.item() - loss64.item()) <= 1e-5 * (1 + abs(loss64.item()))
    ill = _ill_rows(gx, gx32, gx64, data.shape[0])
    w[ill] = 0.0
    _, gx64, gp64 = _model_grads(ref64, data.double(), w.double())
    _, gx32, gp32 = _model_grads(ref32, data, w)
    _, gx, gp = _model_grads(model, data.to(cuda_device), w.to(cuda_device))
    _check(gx, gx32, gx64, "dL/dx")
    for (n, _), a, b, c in zip(model.named_parameters(), gp, gp32, gp64):
        _check(a, b, c, n)


# ---- MADE flows (MAF / IAF) on the any-shape path ---------------------------------------------
from test_gpu_made import assert_ld, assert_y  # noqa: E402
from nfs_amd.flows import autoregressive as _ar  # noqa: E402


@pytest.fixture
def force_generic_made():
    old = _ar.FORCE_GENERIC
    _ar.FORCE_GENERIC = True
    yield
    _ar.FORCE_GENERIC = old


def test_generic_made_vs_reference_g5_g9(cuda_device, force_generic_made):
    """Forced onto the reference's MAF(63, 64) x5 (G5, both directions — the sequential one as
    the reference's d MADE calls) and its small MAF/IAF fixtures (G9)."""
    g = load_golden("g5_maf63.npz")
    m = nfs_amd.NormalizingFlowModel([nfs_amd.MaskedAutoregressiveFlow(63, 64) for _ in range(5)])
    m.load_state_dict(state_dict_from(g, "", m))
    m = m.to(cuda_device).eval()
    STATS["hip"] = STATS["torch"] = 0
    with torch.no_grad():
        z, ld = m.inverse(torch.from_numpy(g["x"]).to(cuda_device))
        x, lf = m.forward(torch.from_numpy(g["z"][:256]).to(cuda_device))
    assert STATS["torch"] == 0
    assert_y(z.cpu(), g["inv_z"])
    assert_ld(ld.cpu(), g["inv_ld"])
    assert_y(x.cpu(), g["fwd_x"][:256])
    assert_ld(lf.cpu(), g["fwd_ld"][:256])
    g9 = load_golden("g9_small.npz")
    for name, cls in (("maf4", nfs_amd.MaskedAutoregressiveFlow), ("iaf10", nfs_amd.InverseAutoregressiveFlow),
                      ("maf2", nfs_amd.MaskedAutoregressiveFlow), ("iaf3", nfs_amd.InverseAutoregressiveFlow)):
        sd = oracle_sd(g9, name + ".")
        f = cls(sd["conditioner.net.0.weight"].shape[1], sd["conditioner.net.0.weight"].shape[0])
        f.load_state_dict(state_dict_from(g9, name + ".", f))
        f = f.to(cuda_device).eval()
        xx = torch.from_numpy(g9[name + ".x"]).to(cuda_device)
        with torch.no_grad():
            yf, lf = f.forward(xx)
            yi, li = f.inverse(xx)
        assert_y(yf.cpu(), g9[name + ".fwd_y"])
        assert_ld(lf.cpu(), g9[name + ".fwd_ld"])
        assert_y(yi.cpu(), g9[name + ".inv_y"])
        assert_ld(li.cpu(), g9[name + ".inv_ld"])


@pytest.mark.parametrize("d,H,B", [(5, 320, 100), (40, 512, 257), (2, 300, 64), (300, 264, 33)])
def test_generic_made_wide_vs_oracle(cuda_device, d, H, B):
    """H > 256 (beyond nfx_made_big.hip): the any-shape path, both flows, both directions."""
    torch.manual_seed(d * 31 + H)
    for cls, fn in ((nfs_amd.MaskedAutoregressiveFlow, oracle.maf), (nfs_amd.InverseAutoregressiveFlow, oracle.iaf)):
        f = cls(d, H)
        with torch.no_grad():
            for p in f.parameters():
                p.add_(0.05 * torch.randn_like(p))
        sd = {k: v.clone() for k, v in f.state_dict().items()}
        f = f.to(cuda_device).eval()
        assert not f._fused_family()
        x = torch.randn(B, d)
        x[0, 0] = float("inf")
        for direction in (1, -1):
            STATS["hip"] = STATS["torch"] = 0
            with torch.no_grad():
                yg, lg = (f.forward if direction > 0 else f.inverse)(x.to(cuda_device))
                yr, lr = fn(sd, "", x, direction)
            assert STATS["hip"] == 1 and STATS["torch"] == 0, STATS
            yr = np.asarray(yr, np.float64)
            assert np.array_equal(np.isnan(yg.cpu().numpy()), np.isnan(yr))
            fin = np.isfinite(yr)
            assert_y(yg.cpu().numpy()[fin], yr[fin])
            assert_ld(lg.cpu(), lr, 5e-4)


def test_generic_made_batchnorm_eval_wide(cuda_device):
    """MADE(use_batch_norm=True), eval, H = 288: BatchNorm folded into the GEMM epilogue."""
    torch.manual_seed(19)
    f = nfs_amd.MaskedAutoregressiveFlow(12, 288, use_batch_norm=True)
    with torch.no_grad():
        for m in f.modules():
            if isinstance(m, torch.nn.BatchNorm1d):
                m.running_mean.normal_(0, 0.1)
                m.running_var.uniform_(0.5, 1.5)
                m.weight.normal_(1, 0.1)
                m.bias.normal_(0, 0.1)
    f.eval()
    x = torch.randn(300, 12)
    with torch.no_grad():
        zc, lc = f.inverse(x)
        xc, lfc = f.forward(x)
    f = f.to(cuda_device)
    with torch.no_grad():
        zg, lg = f.inverse(x.to(cuda_device))
        xg, lfg = f.forward(x.to(cuda_device))
    assert_y(zg.cpu(), zc)
    assert_ld(lg.cpu(), lc)
    assert_y(xg.cpu(), xc)
    assert_ld(lfg.cpu(), lfc)


@pytest.mark.parametrize("name", ["maf10", "iaf10", "maf63", "iaf784"])
@pytest.mark.parametrize("dname", ["inv", "fwd"])
def test_generic_made_vs_reference_gradients_g14(cuda_device, force_generic_made, name, dname):
    """Both directions on the any-shape path — parallel: element adjoint + MADE backward GEMMs;
    sequential: the triangular adjoint solve through the MADE — against the reference's own fp32
    gradients (G14; its sequential ones are autograd through all d MADE calls)."""
    from test_gpu_grad_fixtures import _g14_module, _grad_close, _run
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
    assert STATS["torch"] == 0 and STATS["hip"] == 2, STATS
    yr, ldr = g[f"{name}.{dname}.y"], g[f"{name}.{dname}.ld"]
    assert (np.abs(y.cpu().numpy().astype(np.float64) - yr) <= 2e-5 * (1 + np.abs(yr))).all()
    ltol = 1e-6 * np.abs(ldr).max() + 2e-4 if name == "iaf784" else 2e-4
    assert np.abs(ld.cpu().numpy().astype(np.float64) - ldr).max() <= ltol
    _grad_close(gx, g[f"{name}.{dname}.gx"], gx64, "dL/dx")
    for k in gp64:
        _grad_close(gp[k], g[f"{name}.{dname}.grad.{k}"], gp64[k], k)


@pytest.mark.parametrize("cls", ["maf", "iaf"])
@pytest.mark.parametrize("dname", ["inv", "fwd"])
def test_generic_made_wide_backward_vs_float64(cuda_device, cls, dname):
    """H = 320 (beyond the fused backward's H <= 128), both directions, vs float64 autograd."""
    from test_gpu_grad_fixtures import _grad_close, _run
    torch.manual_seed(23)
    f = (nfs_amd.MaskedAutoregressiveFlow if cls == "maf" else nfs_amd.InverseAutoregressiveFlow)(24, 320)
    with torch.no_grad():
        for p in f.parameters():
            p.add_(0.03 * torch.randn_like(p))
    g = torch.Generator().manual_seed(29)
    x, wy, wl = torch.randn(3000, 24, generator=g), torch.randn(3000, 24, generator=g), torch.randn(3000, generator=g)
    y32, l32, gx32, gp32 = _run(f, x, wy, wl, dname)
    _, _, gx64, gp64 = _run(copy.deepcopy(f).double(), x.double(), wy.double(), wl.double(), dname)
    fg = copy.deepcopy(f).to(cuda_device)
    STATS["hip"] = STATS["torch"] = 0
    y, ld, gx, gp = _run(fg, x.to(cuda_device), wy.to(cuda_device), wl.to(cuda_device), dname)
    assert STATS["torch"] == 0 and STATS["hip"] == 2, STATS
    assert_y(y.cpu(), y32)
    assert_ld(ld.cpu(), l32)
    _grad_close(gx, gx32, gx64, "dL/dx")
    for k in gp64:
        _grad_close(gp[k], gp32[k], gp64[k], k)


# ---- ARQS on the any-shape path: eval beyond H = 128 and the backward --------------------------
from nfs_amd.flows import arqs as _aq  # noqa: E402


def _arqs(d, H, K, seed, scale=0.05):
    torch.manual_seed(seed)
    f = nfs_amd.ARQS(d, hidden_dim=H, num_bins=K)
    with torch.no_grad():
        for p in f.parameters():
            p.add_(scale * torch.randn_like(p))
    return f


@pytest.mark.parametrize("d,H,K", [(3, 160, 8), (5, 256, 4), (2, 300, 11)])
def test_generic_arqs_eval_vs_oracle(cuda_device, d, H, K):
    """H > 128 (beyond nfx_arqs.hip): the reference's d steps, MADE on MFMA, vs the oracle."""
    f = _arqs(d, H, K, d * 10 + H + K)
    sd = {k: v.clone() for k, v in f.state_dict().items()}
    x = torch.rand(500, d, generator=torch.Generator().manual_seed(d))
    fg = f.to(cuda_device).eval()
    assert not fg._fused_family()
    for direction in (1, -1):
        STATS["hip"] = STATS["torch"] = 0
        with torch.no_grad():
            yg, lg = (fg.forward if direction > 0 else fg.inverse)(x.to(cuda_device))
        assert STATS["hip"] == 1 and STATS["torch"] == 0, STATS
        yr, lr = oracle.arqs(sd, "", x, direction, K=K)
        assert_y(yg.cpu(), yr, 1e-4)
        assert_ld(lg.cpu(), lr, 1e-3)


@pytest.mark.parametrize("d,H,K,direction", [(2, 32, 8, 1), (2, 32, 8, -1), (4, 64, 5, 1), (4, 64, 5, -1),
                                             (3, 160, 10, -1), (6, 48, 3, 1)])
def test_arqs_backward_vs_float64_autograd(cuda_device, d, H, K, direction):
    """dL/dx and every parameter gradient of L = <wy, y> + <wl, ld> through ARQS (reverse mode
    through the reference's d steps, nfx_arqs_step mode 1), against float64 autograd of the same
    module, with the reference's own fp32 error as the yardstick (test_gpu_grad_fixtures
    tolerance: max |g - g64| <= 2e-5 (1 + max|g64|) + 4 max|g32 - g64|)."""
    f = _arqs(d, H, K, 7 * d + H + K)
    g = torch.Generator().manual_seed(d + K)
    x = 0.05 + 0.9 * torch.rand(700, d, generator=g)
    wy, wl = torch.randn(700, d, generator=g), torch.randn(700, generator=g)

    def run(m, xx, wyy, wll):
        xx = xx.clone().requires_grad_(True)
        for p in m.parameters():
            p.grad = None
        y, ld = m.forward(xx) if direction > 0 else m.inverse(xx)
        ((y * wyy).sum() + (ld * wll).sum()).backward()
        return y.detach(), ld.detach(), xx.grad, [p.grad for p in m.parameters()]

    y64, l64, gx64, gp64 = run(copy.deepcopy(f).double(), x.double(), wy.double(), wl.double())
    y32, l32, gx32, gp32 = run(copy.deepcopy(f), x, wy, wl)
    fg = copy.deepcopy(f).to(cuda_device)
    STATS["hip"] = STATS["torch"] = 0
    yg, lg, gxg, gpg = run(fg, x.to(cuda_device), wy.to(cuda_device), wl.to(cuda_device))
    assert STATS["hip"] == 2 and STATS["torch"] == 0, STATS
    assert_y(yg.cpu(), y64, 1e-4)
    assert_ld(lg.cpu(), l64, 1e-3)

    def close(a, b32, b64, what):
        a, b32, b64 = a.double().cpu(), b32.double(), b64.double()
        bound = 2e-5 * (1 + b64.abs().max().item()) + 4 * (b32 - b64).abs().max().item()
        err = (a - b64).abs().max().item()
        assert err <= bound, f"{what}: max err {err:.3g} > {bound:.3g}"

    close(gxg, gx32, gx64, "dL/dx")
    for (n, _), a, b, c in zip(f.named_parameters(), gpg, gp32, gp64):
        close(a, b, c, n)


@pytest.mark.parametrize("name", ["a1", "a3", "a5", "a4bn", "a10"])
def test_generic_arqs_vs_reference_g10(cuda_device, name):
    """The any-shape ARQS steps (mode 0, also the backward's recompute) forced onto the
    reference's ARQS fixtures (G10): outputs and log-dets under the fused kernel's parity test
    (a10 carries scalar data_min/data_max: the any-shape path rescales with nfx_arqs_bounds)."""
    from test_gpu_arqs import test_arqs_vs_reference
    old = _aq.FORCE_GENERIC
    _aq.FORCE_GENERIC = True
    try:
        test_arqs_vs_reference(cuda_device, name)
    finally:
        _aq.FORCE_GENERIC = old


# ---- MADE with BatchNorm1d (use_batch_norm=True) under autograd --------------------------------
def _made_bn(cls, d, H, seed):
    torch.manual_seed(seed)
    f = cls(d, H, use_batch_norm=True)
    with torch.no_grad():
        for p in f.parameters():
            p.add_(0.03 * torch.randn_like(p))
        for m in f.modules():
            if isinstance(m, torch.nn.BatchNorm1d):
                m.running_mean.normal_(0, 0.1)
                m.running_var.uniform_(0.5, 1.5)
                m.weight.normal_(1, 0.1)
                m.bias.normal_(0, 0.1)
    return f


@pytest.mark.parametrize("cls", ["maf", "iaf"])
@pytest.mark.parametrize("dname", ["inv", "fwd"])
@pytest.mark.parametrize("d,H", [(12, 32), (5, 288)])
@pytest.mark.parametrize("mode", ["eval", "train"])
def test_generic_made_batchnorm_backward_vs_float64(cuda_device, cls, dname, d, H, mode):
    """MADE(use_batch_norm=True) under autograd. eval: running-statistics BatchNorm, both
    directions (the sequential ones by the triangular adjoint through the BatchNorm'ed MADE);
    train: batch-statistics BatchNorm with the running update, both directions (the sequential
    ones as the reference's d MADE calls, each with its own batch statistics and running update,
    differentiated call by call). Against float64 autograd of the same module (outputs, dL/dx,
    every parameter gradient, running statistics after the step)."""
    from test_gpu_grad_fixtures import _grad_close, _run
    klass = nfs_amd.MaskedAutoregressiveFlow if cls == "maf" else nfs_amd.InverseAutoregressiveFlow
    f = _made_bn(klass, d, H, d * 7 + H)
    f = f.train() if mode == "train" else f.eval()
    g = torch.Generator().manual_seed(d + H)
    x, wy, wl = torch.randn(1500, d, generator=g), torch.randn(1500, d, generator=g), torch.randn(1500, generator=g)
    f64, f32 = copy.deepcopy(f).double(), copy.deepcopy(f)
    _, _, gx64, gp64 = _run(f64, x.double(), wy.double(), wl.double(), dname)
    y32, l32, gx32, gp32 = _run(f32, x, wy, wl, dname)
    fg = copy.deepcopy(f).to(cuda_device)
    STATS["hip"] = STATS["torch"] = 0
    y, ld, gx, gp = _run(fg, x.to(cuda_device), wy.to(cuda_device), wl.to(cuda_device), dname)
    assert STATS["torch"] == 0 and STATS["hip"] == 2, STATS
    assert_y(y.cpu(), y32, 5e-5)
    assert_ld(ld.cpu(), l32, 5e-4)
    _grad_close(gx, gx32, gx64, "dL/dx")
    gmax = max(float(v.abs().max()) for v in gp64.values())
    for k in gp64:
        if mode == "train" and k.endswith(("net.0.bias", "net.3.bias", "net.6.bias")):
            # a Linear bias feeding a train-mode BatchNorm has an exactly-zero gradient (the
            # batch mean removes it): both sides are summation noise, bounded as in
            # test_gpu_affine_train._gclose by 2e-5 of the largest gradient or 4x the
            # reference's own fp32 noise
            err = float((gp[k].double().cpu() - gp64[k]).abs().max())
            bound = max(2e-5 * gmax, 4 * float((gp32[k].double() - gp64[k]).abs().max()))
            assert err <= bound, f"{k}: {err:.3g} not ~0 (bound {bound:.3g})"
            continue
        _grad_close(gp[k], gp32[k], gp64[k], k)
    for (k, bg), (_, b64) in zip(fg.named_buffers(), f64.named_buffers()):
        if k.endswith(("running_mean", "running_var")):
            assert np.abs(bg.cpu().double().numpy() - b64.numpy()).max() <= 1e-6 * (1 + np.abs(b64.numpy()).max()), k
