"""GPU parity of the fused RQ-spline coupling kernel (csrc/nfx_spline*.hip) and the unit-interval
RQS kernel (nfx_rqs_unit) against the reference's golden outputs and the CPU oracle.

Parity (conftest.assert_fp32_parity): every element within SURVEY §8(c)'s fixed tolerance of the
reference's fp32 result (|dy| <= 1e-5 (1+|ref|), |dld| <= 1e-4), except at most 2 % (5 % for the
stress-weight shapes test) whose bound is widened by 8x their MEASURED fp32 conditioning — the
spline's softmax/exp/log chain and the citardauq root are ill-conditioned next to steep knots,
where the reference's own fp32 log-det is up to ~1e-3 off float64 (conditioning = max of that
error and the spread of one-ulp-jittered fp32 oracle runs, conftest.fp32_jitter). NLL: <= 1e-5.
"""
import numpy as np
import pytest
import torch

import nfs_amd
import oracle
from conftest import assert_fp32_parity, fp32_jitter, golden_json, load_golden, oracle_sd, state_dict_from

pytestmark = pytest.mark.gpu

N_REGULAR = 4048


def assert_y(y, ref, tol=2e-5, skip=None):
    y, ref = np.asarray(y, np.float64), np.asarray(ref, np.float64)
    err = np.abs(y - ref) / (1 + np.abs(ref))
    assert err.max() <= tol, f"max rel err {err.max():.3g} at {np.unravel_index(err.argmax(), err.shape)}"


def assert_ld(ld, ref, tol=2e-4):
    d = np.abs(np.asarray(ld, np.float64) - np.asarray(ref, np.float64))
    assert d.max() <= tol, f"max |dld| {d.max():.3g} at {d.argmax()}"


def k8_model(K=8):
    layers = []
    for i in range(8):
        mask = torch.zeros(2)
        mask[(0 if i % 2 == 0 else 1)] = 1
        layers.append(nfs_amd.SplineCouplingLayer(2, 64, mask, num_bins=K))
    return nfs_amd.NormalizingFlowModel(layers)


def sd64(sd):
    return {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}


def load_model(tag, dev):
    g = load_golden("g3_spline.npz")
    m = k8_model() if tag == "k8." else nfs_amd.RealNVPSpline(2, 8, 64)
    m.load_state_dict(state_dict_from(g, tag, m))
    return m.to(dev).eval(), g


@pytest.mark.parametrize("tag", ["k8.", "k10."])
def test_spline_model_vs_reference(cuda_device, tag):
    m, g = load_model(tag, cuda_device)
    x = torch.from_numpy(g["x"]).to(cuda_device)
    z = torch.from_numpy(g["z"]).to(cuda_device)
    nfs_amd.reset_stats()
    with torch.no_grad():
        zi, ldi = m.inverse(x)
        xf, ldf = m.forward(z)
        lp = m.log_prob(x)
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] >= 3  # one chain launch per call
    K = 8 if tag == "k8." else 10
    spec = [("spline", f"{'flow.' if K == 10 else ''}flows.{i}.", {"K": K}) for i in range(8)]
    sd = sd64(oracle_sd(g, tag))
    with torch.no_grad():
        z64, l64 = oracle.flow_model(sd, spec, torch.from_numpy(g["x"]).double(), -1)
        x64, lf64 = oracle.flow_model(sd, spec, torch.from_numpy(g["z"]).double(), 1)
    sd32 = oracle_sd(g, tag)
    si = fp32_jitter(lambda s, v: oracle.flow_model(s, spec, v, -1), torch.from_numpy(g["x"]), sd=sd32)
    sf = fp32_jitter(lambda s, v: oracle.flow_model(s, spec, v, 1), torch.from_numpy(g["z"]), sd=sd32)
    assert_fp32_parity(zi.cpu(), g[tag + "inv_z"], z64, what="inv z", sens=si[0])
    assert_fp32_parity(ldi.cpu(), g[tag + "inv_ld"], l64, what="inv ld", sens=si[1])
    assert_fp32_parity(xf.cpu(), g[tag + "fwd_x"], x64, what="fwd x", sens=sf[0])
    assert_fp32_parity(ldf.cpu(), g[tag + "fwd_ld"], lf64, what="fwd ld", sens=sf[1])
    ref_lp = g[tag + "log_prob"].astype(np.float64)
    nll = -float(lp[:N_REGULAR].double().mean())
    assert abs(nll - (-ref_lp[:N_REGULAR].mean())) <= 1e-5


@pytest.mark.parametrize("name", ["spl_alt", "spl_half", "spl_d3"])
def test_small_spline_layers(cuda_device, name):
    """d in {3,4}, H=16, K=10 — the reference's own test shapes (n_t = 1 or 2 dims)."""
    g = load_golden("g9_small.npz")
    sd = oracle_sd(g, name + ".")
    d = sd["mask"].numel()
    layer = nfs_amd.SplineCouplingLayer(d, 16, sd["mask"].clone())
    layer.load_state_dict(state_dict_from(g, name + ".", layer))
    layer = layer.to(cuda_device).eval()
    x = torch.from_numpy(g[name + ".x"]).to(cuda_device)
    with torch.no_grad():
        yf, lf = layer.forward(x)
        yi, li = layer.inverse(x)
        xd = x.cpu().double()
        yf64, lf64 = oracle.spline_coupling(sd64(sd), "", xd, 1)
        yi64, li64 = oracle.spline_coupling(sd64(sd), "", xd, -1)
    sf = fp32_jitter(lambda s, v: oracle.spline_coupling(s, "", v, 1), x.cpu(), sd=sd)
    si = fp32_jitter(lambda s, v: oracle.spline_coupling(s, "", v, -1), x.cpu(), sd=sd)
    assert_fp32_parity(yf.cpu(), g[name + ".fwd_y"], yf64, what="fwd y", sens=sf[0])
    assert_fp32_parity(lf.cpu(), g[name + ".fwd_ld"], lf64, what="fwd ld", sens=sf[1])
    assert_fp32_parity(yi.cpu(), g[name + ".inv_y"], yi64, what="inv y", sens=si[0])
    assert_fp32_parity(li.cpu(), g[name + ".inv_ld"], li64, what="inv ld", sens=si[1])


@pytest.mark.parametrize("K", [2, 3, 5, 11])
@pytest.mark.parametrize("H", [16, 32, 96, 128])
def test_spline_layer_shapes_vs_oracle(cuda_device, K, H):
    torch.manual_seed(K * 1000 + H)
    d = 3
    mask = torch.tensor([0.0, 1.0, 0.0])
    layer = nfs_amd.SplineCouplingLayer(d, H, mask, num_bins=K)
    with torch.no_grad():
        for p in layer.parameters():
            p.add_(0.2 * torch.randn_like(p))
    x = torch.randn(777, d) * 2.5
    sd = {k: v.clone() for k, v in layer.state_dict().items()}
    layer = layer.to(cuda_device).eval()
    for direction in (1, -1):
        with torch.no_grad():
            yg, lg = (layer.forward if direction > 0 else layer.inverse)(x.to(cuda_device))
            yr, lr = oracle.spline_coupling(sd, "", x, direction, K=K)
            y64, l64 = oracle.spline_coupling(sd64(sd), "", x.double(), direction, K=K)
        sy, sl = fp32_jitter(lambda s, v: oracle.spline_coupling(s, "", v, direction, K=K), x, sd=sd)
        # stress weights (0.2 perturbation, K up to 11): log-dets next to steep knots are
        # ill-conditioned; they must match a valid fp32 evaluation (input jitter, hidden order)
        assert_fp32_parity(yg.cpu(), yr, y64, what=f"y dir={direction}", sens=sy)
        assert_fp32_parity(lg.cpu(), lr, l64, what=f"ld dir={direction}", sens=sl)


def test_spline_rescale_and_edges(cuda_device):
    """data_min/data_max rescale (:78-94), inputs outside [-B, B], exact knots and non-finite."""
    torch.manual_seed(5)
    mask = torch.tensor([1.0, 0.0])
    layer = nfs_amd.SplineCouplingLayer(2, 32, mask, num_bins=6, data_min=-3.0, data_max=4.0)
    with torch.no_grad():
        for p in layer.parameters():
            p.add_(0.3 * torch.randn_like(p))
    x = torch.randn(500, 2) * 3
    x[:8, 1] = torch.tensor([-3.0, 4.0, 10.0, -10.0, float("inf"), float("nan"), 0.5, 1e30])
    x[8, 0] = float("inf")
    sd = {k: v.clone() for k, v in layer.state_dict().items()}
    layer = layer.to(cuda_device).eval()
    for direction in (1, -1):
        with torch.no_grad():
            yg, lg = (layer.forward if direction > 0 else layer.inverse)(x.to(cuda_device))
            yr, lr = oracle.spline_coupling(sd, "", x, direction, K=6, data_min=-3.0, data_max=4.0)
            y64, l64 = oracle.spline_coupling(sd64(sd), "", x.double(), direction, K=6, data_min=-3.0, data_max=4.0)
        assert np.array_equal(np.isfinite(yg.cpu().numpy()), np.isfinite(yr.numpy()))
        sy, sl = fp32_jitter(lambda s, v: oracle.spline_coupling(s, "", v, direction, K=6, data_min=-3.0,
                                                                data_max=4.0), x, sd=sd)
        assert_fp32_parity(yg.cpu(), yr, y64, what=f"y dir={direction}", sens=sy)
        assert_fp32_parity(lg.cpu(), lr, l64, what=f"ld dir={direction}", sens=sl)


def test_rqs_unit_vs_reference(cuda_device):
    g = load_golden("g4_rqs_unit.npz")
    args = [torch.from_numpy(g[k]).to(cuda_device) for k in ("x", "uw", "uh", "ud")]
    nfs_amd.reset_stats()
    yf, lf = nfs_amd.rational_quadratic_spline(*args, inverse=False)
    yi, li = nfs_amd.rational_quadratic_spline(*args, inverse=True)
    assert nfs_amd.STATS["hip"] == 2 and nfs_amd.STATS["torch"] == 0
    a64 = [torch.from_numpy(g[k]).double() for k in ("x", "uw", "uh", "ud")]
    yf64, lf64 = oracle.rqs_unit(*a64, inverse=False)
    yi64, li64 = oracle.rqs_unit(*a64, inverse=True)
    a32 = [torch.from_numpy(g[k]) for k in ("x", "uw", "uh", "ud")]
    sf = fp32_jitter(lambda *v: oracle.rqs_unit(*v, inverse=False), *a32)
    si = fp32_jitter(lambda *v: oracle.rqs_unit(*v, inverse=True), *a32)
    assert_fp32_parity(yf.cpu(), g["fwd_y"], yf64, what="fwd y", sens=sf[0])
    assert_fp32_parity(lf.cpu(), g["fwd_ld"], lf64, what="fwd ld", sens=sf[1])
    assert_fp32_parity(yi.cpu(), g["inv_y"], yi64, what="inv y", sens=si[0])
    assert_fp32_parity(li.cpu(), g["inv_ld"], li64, what="inv ld", sens=si[1])


def test_full_scale_nll_cfg3(cuda_device):
    """BASELINE cfg3 at full size: 8x Spline(2,64,K=8), B=1M, NLL vs the reference (G8)."""
    meta = golden_json("g8_full_nll.json")["cfg3_spline_k8_d2_B1M"]
    x = torch.randn(meta["B"], meta["d"], generator=torch.Generator().manual_seed(meta["seed"]))
    assert abs(float(x.double().sum()) - meta["input_sum_f64"]) < 1e-6
    m, _ = load_model("k8.", cuda_device)
    nll = m.nll(x.to(cuda_device))
    assert abs(nll - meta["nll_f64"]) <= 1e-5, (nll, meta["nll_f64"])


@pytest.mark.parametrize("K", [8, 10])
def test_spline_extreme_logits_vs_oracle(cuda_device, K):
    """Spline logits the reference handles without NaN: a -inf width/height/derivative logit
    (softmax weight 0, softplus 0), a spread of ~95 (exp of the minimum is subnormal in torch
    and flushed by the kernel's exp; min_bin_width/min_derivative absorb it) and a spread of
    ~300 (exp underflows to 0 in both). The kernel's exp_safe must reproduce all of them."""
    torch.manual_seed(K)
    mask = torch.tensor([1.0, 0.0])
    layer = nfs_amd.SplineCouplingLayer(2, 32, mask, num_bins=K)
    with torch.no_grad():
        for p in layer.parameters():
            p.add_(0.2 * torch.randn_like(p))
        P = 3 * K - 1
        b = layer.param_net[4].bias
        b[P + 0] = float("-inf")        # width logit 0 of the transformed dim 1
        b[P + 1] = 95.0                 # spread ~95 against the others
        b[P + K + 2] = -300.0           # height logit far below the rest
        b[P + K + 3] = float("-inf")
        b[P + 2 * K] = float("-inf")    # derivative logit: softplus(-inf) = 0
        b[P + 2 * K + 1] = -120.0       # softplus(-120) subnormal -> min_derivative
    x = torch.randn(2000, 2) * 2.5
    sd = {k: v.clone() for k, v in layer.state_dict().items()}
    layer = layer.to(cuda_device).eval()
    for direction in (1, -1):
        with torch.no_grad():
            yg, lg = (layer.forward if direction > 0 else layer.inverse)(x.to(cuda_device))
            yr, lr = oracle.spline_coupling(sd, "", x, direction, K=K)
            y64, l64 = oracle.spline_coupling(sd64(sd), "", x.double(), direction, K=K)
        assert torch.isfinite(yr).all() and torch.isfinite(lr).all()
        assert torch.isfinite(yg).all() and torch.isfinite(lg).all()
        sy, sl = fp32_jitter(lambda s, v: oracle.spline_coupling(s, "", v, direction, K=K), x, sd=sd)
        assert_fp32_parity(yg.cpu(), yr, y64, what=f"y dir={direction}", sens=sy)
        assert_fp32_parity(lg.cpu(), lr, l64, what=f"ld dir={direction}", sens=sl)


def _rqs_grads(fn, args, wy, wl, inverse):
    xs = [a.clone().requires_grad_(True) for a in args]
    y, ld = fn(*xs, inverse=inverse)
    ((y * wy).sum() + (ld * wl).sum()).backward()
    return y.detach(), ld.detach(), [t.grad for t in xs]


@pytest.mark.parametrize("inverse", [False, True])
def test_rqs_unit_backward_vs_float64(cuda_device, inverse):
    """The stand-alone rational_quadratic_spline under autograd on the GPU (nfx_rqs_unit +
    nfx_rqs_unit_backward): dL/d(inputs, widths, heights, derivatives) for L = sum(y wy) +
    sum(ld wl) on the reference's G4 inputs, against float64 autograd of the composite
    (rational_quadratic_spline.py:4-104), within 4x the fp32 composite's own distance from it
    (+ 2e-5 relative); every call HIP."""
    from nfs_amd.flows.spline import _rqs_unit_torch
    g = load_golden("g4_rqs_unit.npz")
    a32 = [torch.from_numpy(g[k]) for k in ("x", "uw", "uh", "ud")]
    gen = torch.Generator().manual_seed(44)
    wy, wl = torch.randn(a32[0].shape, generator=gen), torch.randn(a32[0].shape, generator=gen)

    def comp(*v, inverse):
        return _rqs_unit_torch(*v, inverse, 1e-3, 1e-3, 1e-3)

    _, _, g64 = _rqs_grads(comp, [a.double() for a in a32], wy.double(), wl.double(), inverse)
    _, _, g32 = _rqs_grads(comp, a32, wy, wl, inverse)
    nfs_amd.reset_stats()
    y, ld, gg = _rqs_grads(nfs_amd.rational_quadratic_spline, [a.to(cuda_device) for a in a32], wy.to(cuda_device),
                           wl.to(cuda_device), inverse)
    assert nfs_amd.STATS["hip"] == 2 and nfs_amd.STATS["torch"] == 0, nfs_amd.STATS
    yk, lk = ("inv_y", "inv_ld") if inverse else ("fwd_y", "fwd_ld")
    np.testing.assert_array_equal(y.cpu().numpy(), nfs_amd.rational_quadratic_spline(
        *[a.to(cuda_device) for a in a32], inverse=inverse)[0].cpu().numpy())
    assert np.allclose(y.cpu().numpy(), g[yk], rtol=1e-5, atol=1e-5, equal_nan=True)
    assert np.allclose(ld.cpu().numpy(), g[lk], rtol=1e-4, atol=1e-4, equal_nan=True)
    for name, a, b32, b64 in zip(("dL/dx", "dL/dwidths", "dL/dheights", "dL/dderivatives"), gg, g32, g64):
        a, b32, b64 = a.double().cpu(), b32.double(), b64.double()
        fin = torch.isfinite(b64)
        assert torch.equal(torch.isfinite(a), fin), f"{name}: non-finite pattern differs"
        bound = 2e-5 * (1 + b64[fin].abs().max().item()) + 4 * (b32 - b64)[fin].abs().max().item()
        err = (a - b64)[fin].abs().max().item()
        assert err <= bound, f"{name}: max err {err:.3g} > {bound:.3g}"


def test_rqs_unit_nd_and_unsupported(cuda_device):
    """N-d inputs run the same kernels elementwise (equal to the flattened call bit for bit, both
    passes); GPU calls outside the kernels raise instead of running eager PyTorch."""
    gen = torch.Generator().manual_seed(45)
    B, d, K = 300, 3, 7
    x = torch.rand(B, d, generator=gen)
    uw, uh, ud = (torch.randn(B, d, K, generator=gen), torch.randn(B, d, K, generator=gen),
                  torch.randn(B, d, K - 1, generator=gen))
    dev = [t.to(cuda_device) for t in (x, uw, uh, ud)]
    flat = [dev[0].reshape(-1), dev[1].reshape(-1, K), dev[2].reshape(-1, K), dev[3].reshape(-1, K - 1)]
    nfs_amd.reset_stats()
    for inverse in (False, True):
        y, ld = nfs_amd.rational_quadratic_spline(*dev, inverse=inverse)
        yf, lf = nfs_amd.rational_quadratic_spline(*flat, inverse=inverse)
        assert y.shape == (B, d) and ld.shape == (B, d)
        assert torch.equal(y.reshape(-1), yf) and torch.equal(ld.reshape(-1), lf)
        wy = torch.randn(B, d, generator=gen).to(cuda_device)
        _, _, gn = _rqs_grads(nfs_amd.rational_quadratic_spline, dev, wy, wy, inverse)
        _, _, gfl = _rqs_grads(nfs_amd.rational_quadratic_spline, flat, wy.reshape(-1), wy.reshape(-1), inverse)
        for a, b in zip(gn, gfl):
            assert torch.equal(a.reshape(b.shape), b)
    assert nfs_amd.STATS["torch"] == 0
    with pytest.raises(NotImplementedError):
        nfs_amd.rational_quadratic_spline(*[t.double() for t in dev])
    with pytest.raises(NotImplementedError):
        nfs_amd.rational_quadratic_spline(dev[0], *(torch.randn(B, d, k).to(cuda_device) for k in (17, 17, 16)))
    with pytest.raises(ValueError):
        nfs_amd.rational_quadratic_spline(dev[0], dev[1][:1], dev[2], dev[3])
