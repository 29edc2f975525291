"""GPU parity of the fused affine-coupling kernel (csrc/nfx_affine*.hip) through the C-ABI.

Checks against (a) the reference's own outputs (golden fixtures, tests/golden/) and (b) the CPU
oracle on the same seeded inputs, including ragged batches, B=0 and non-finite inputs.
Both kernels are exercised: the small-batch one (a workgroup per 32 samples) and the
streaming one, forced through nfx_affine_kernel_policy by the `affine_kernel` fixture.
Tolerances: per-sample z/x |d| <= 1e-5 * (1 + |ref|); log-det <= 1e-4 (d=2);
NLL <= 1e-5 absolute.
"""
import numpy as np
import pytest
import torch

import nfs_amd
import oracle
from conftest import golden_json, load_golden, oracle_sd, state_dict_from

pytestmark = pytest.mark.gpu


def assert_y(y, ref, tol=1e-5):
    y, ref = np.asarray(y, np.float64), np.asarray(ref, np.float64)
    err = np.abs(y - ref) / (1 + np.abs(ref))
    assert err.max() <= tol, f"max rel err {err.max():.3g} at {np.unravel_index(err.argmax(), err.shape)}"


def assert_ld(ld, ref, tol=1e-4):
    d = np.abs(np.asarray(ld, np.float64) - np.asarray(ref, np.float64))
    assert d.max() <= tol, f"max |dld| {d.max():.3g} at {d.argmax()}"


def assert_lp(lp, ref):
    """log p = -0.5|z|^2 + ...: huge for the 1e3/1e10 edge rows, so the bound is relative there."""
    lp, ref = np.asarray(lp, np.float64), np.asarray(ref, np.float64)
    bad = np.abs(lp - ref) > 1e-4 + 2e-5 * np.abs(ref)
    assert not bad.any(), f"log_prob mismatch at {np.flatnonzero(bad)[:5]}: {lp[bad][:5]} vs {ref[bad][:5]}"


@pytest.fixture(params=["small", "streaming"])
def affine_kernel(request):
    """Route every affine-coupling launch of the test to one kernel, restore afterwards."""
    L = nfs_amd._lib
    prev = L.lib().nfx_affine_kernel_policy(L.NFX_AFFINE_SMALL if request.param == "small" else L.NFX_AFFINE_STREAMING)
    yield request.param
    L.lib().nfx_affine_kernel_policy(prev)


N_REGULAR = 4048  # g2/g3 rows before the 45 edge rows (|x| up to 1e10)


def realnvp_from_golden(dev, name="g2_realnvp.npz"):
    g = load_golden(name)
    m = nfs_amd.RealNVP(2, 8, 64)
    m.load_state_dict(state_dict_from(g, "", m))
    return m.to(dev).eval(), g


def test_layer0_inverse_forward(cuda_device, affine_kernel):
    m, g = realnvp_from_golden(cuda_device)
    layer = m.flow.flows[0]
    nfs_amd.reset_stats()
    with torch.no_grad():
        zi, ldi = layer.inverse(torch.from_numpy(g["x"]).to(cuda_device))
        xf, ldf = layer.forward(torch.from_numpy(g["z"]).to(cuda_device))
    assert nfs_amd.STATS["hip"] == 2 and nfs_amd.STATS["torch"] == 0
    assert_y(zi.cpu(), g["l0_inv_z"])
    assert_ld(ldi.cpu(), g["l0_inv_ld"])
    assert_y(xf.cpu(), g["l0_fwd_x"])
    assert_ld(ldf.cpu(), g["l0_fwd_ld"])


def test_realnvp_model_vs_reference(cuda_device, affine_kernel):
    m, g = realnvp_from_golden(cuda_device)
    x = torch.from_numpy(g["x"]).to(cuda_device)
    z = torch.from_numpy(g["z"]).to(cuda_device)
    nfs_amd.reset_stats()
    with torch.no_grad():
        zi, ldi = m.inverse(x)
        xf, ldf = m.forward(z)
        lp, sums = m.log_prob(x, return_sums=True)
    assert nfs_amd.STATS["torch"] == 0
    assert_y(zi.cpu(), g["inv_z"])
    assert_ld(ldi.cpu(), g["inv_ld"])
    assert_y(xf.cpu(), g["fwd_x"])
    assert_ld(ldf.cpu(), g["fwd_ld"])
    assert_lp(lp.cpu(), g["log_prob"])
    assert float(sums[1]) == x.shape[0]
    nll = -float(lp[:N_REGULAR].double().mean())
    assert abs(nll - (-g["log_prob"][:N_REGULAR].astype(np.float64).mean())) <= 1e-5


def test_moons_config1(cuda_device, affine_kernel):
    """Config 1 (two-moons 5k, trained RealNVP) log_prob / NLL vs the reference."""
    m, g = realnvp_from_golden(cuda_device, "g7_moons.npz")
    with torch.no_grad():
        lp = m.log_prob(torch.from_numpy(g["x"]).to(cuda_device))
    assert_lp(lp.cpu(), g["log_prob"])
    assert abs(-float(lp.double().mean()) - float(g["nll_f64"])) <= 1e-5


@pytest.mark.parametrize("name", ["cpl_alt", "cpl_half", "cpl_d3", "cpl_d1"])
def test_small_coupling_layers(cuda_device, affine_kernel, name):
    """d in {1,3,4}, H=16 (padded to one 32-row MFMA tile) as in the reference's own tests."""
    g = load_golden("g9_small.npz")
    sd = oracle_sd(g, name + ".")
    d = sd["mask"].numel()
    layer = nfs_amd.CouplingLayer(d, 16, sd["mask"].clone())
    layer.load_state_dict(state_dict_from(g, name + ".", layer))
    layer = layer.to(cuda_device).eval()
    x = torch.from_numpy(g[name + ".x"]).to(cuda_device)
    with torch.no_grad():
        yf, lf = layer.forward(x)
        yi, li = layer.inverse(x)
    assert_y(yf.cpu(), g[name + ".fwd_y"])
    assert_ld(lf.cpu(), g[name + ".fwd_ld"])
    assert_y(yi.cpu(), g[name + ".inv_y"])
    assert_ld(li.cpu(), g[name + ".inv_ld"])


@pytest.mark.parametrize("B", [1, 31, 63, 64, 65, 1000, 4097])
def test_ragged_batches_vs_oracle(cuda_device, affine_kernel, B):
    m, _ = realnvp_from_golden(cuda_device)
    x = torch.randn(B, 2, generator=torch.Generator().manual_seed(B)) * 1.5
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    with torch.no_grad():
        zi, ldi = m.inverse(x.to(cuda_device))
        zr, ldr = oracle.flow_model(sd, oracle.realnvp_spec(8), x, -1)
        xf, ldf = m.forward(x.to(cuda_device))
        xr, lfr = oracle.flow_model(sd, oracle.realnvp_spec(8), x, 1)
    assert_y(zi.cpu(), zr)
    assert_ld(ldi.cpu(), ldr)
    assert_y(xf.cpu(), xr)
    assert_ld(ldf.cpu(), lfr)


def test_empty_batch(cuda_device, affine_kernel):
    m, _ = realnvp_from_golden(cuda_device)
    with torch.no_grad():
        z, ld = m.inverse(torch.empty(0, 2, device=cuda_device))
        lp, sums = m.log_prob(torch.empty(0, 2, device=cuda_device), return_sums=True)
    assert z.shape == (0, 2) and ld.shape == (0,) and lp.shape == (0,)
    assert float(sums[1]) == 0.0


def test_nonfinite_inputs_follow_reference_guards(cuda_device, affine_kernel):
    """inf/NaN inputs: the reference's clamp (NaN-propagating), 0*inf=NaN masking and the
    NaN/Inf -> 0 guards must come out identical (single layer, so no float drift)."""
    m, _ = realnvp_from_golden(cuda_device)
    layer = m.flow.flows[0]
    inf, nan = float("inf"), float("nan")
    x = torch.tensor([[inf, 0.5], [0.5, inf], [-inf, 1.0], [nan, 0.1], [0.2, nan], [1e38, 1e38],
                      [3e38, -3e38], [0.0, 0.0]], dtype=torch.float32)
    sd = {k: v.detach().cpu() for k, v in layer.state_dict().items()}
    for direction in (1, -1):
        with torch.no_grad():
            yg, lg = (layer.forward if direction > 0 else layer.inverse)(x.to(cuda_device))
            yr, lr = oracle.coupling(sd, "", x, direction)
        yg, lg = yg.cpu().numpy(), lg.cpu().numpy()
        assert np.array_equal(np.isfinite(yg), np.isfinite(yr.numpy()))
        assert_y(yg, yr.numpy())
        assert_ld(lg, lr.numpy())


def test_autograd_through_hip_forward(cuda_device):
    """Eval-mode gradients: HIP forward + composite backward == CPU composite gradients."""
    m, _ = realnvp_from_golden(cuda_device)
    layer = m.flow.flows[1]
    x = torch.randn(256, 2, generator=torch.Generator().manual_seed(3))
    xg = x.to(cuda_device).requires_grad_(True)
    y, ld = layer.inverse(xg)
    (y.sum() + ld.sum()).backward()
    cpu_layer = nfs_amd.CouplingLayer(2, 64, layer.mask.cpu().clone())
    cpu_layer.load_state_dict({k: v.cpu() for k, v in layer.state_dict().items()})
    cpu_layer.eval()
    xc = x.clone().requires_grad_(True)
    yc, lc = cpu_layer.inverse(xc)
    (yc.sum() + lc.sum()).backward()
    np.testing.assert_allclose(xg.grad.cpu().numpy(), xc.grad.numpy(), rtol=1e-4, atol=1e-4)
    for (n, p), (_, q) in zip(layer.named_parameters(), cpu_layer.named_parameters()):
        np.testing.assert_allclose(p.grad.cpu().numpy(), q.grad.numpy(), rtol=1e-3, atol=1e-3, err_msg=n)


def test_weight_update_invalidates_pack(cuda_device):
    m, _ = realnvp_from_golden(cuda_device)
    layer = m.flow.flows[0]
    x = torch.randn(128, 2, device=cuda_device)
    with torch.no_grad():
        y0, _ = layer.inverse(x)
        layer.s_net[6].weight.mul_(0.5)
        y1, _ = layer.inverse(x)
        sd = {k: v.detach().cpu() for k, v in layer.state_dict().items()}
        yr, _ = oracle.coupling(sd, "", x.cpu(), -1)
    assert not torch.equal(y0, y1)
    assert_y(y1.cpu(), yr)


def test_full_scale_nll_cfg2(cuda_device):
    """BASELINE cfg2 at its full size: RealNVP(2,8,64), B=1M, NLL vs the reference (G8)."""
    meta = golden_json("g8_full_nll.json")["cfg2_realnvp_d2_B1M"]
    x = torch.randn(meta["B"], meta["d"], generator=torch.Generator().manual_seed(meta["seed"]))
    assert abs(float(x.double().sum()) - meta["input_sum_f64"]) < 1e-6
    m, _ = realnvp_from_golden(cuda_device)
    nll = m.nll(x.to(cuda_device))
    assert abs(nll - meta["nll_f64"]) <= 1e-5, (nll, meta["nll_f64"])


@pytest.mark.parametrize("d,H,B", [(2, 64, 4000), (2, 128, 777), (3, 96, 1000), (8, 32, 513), (1, 16, 65)])
def test_small_and_streaming_kernels_agree(cuda_device, d, H, B):
    """Both kernels compute the same layer: equal up to the output-layer summation order."""
    torch.manual_seed(d * 1000 + H)
    mask = torch.zeros(d)
    mask[::2] = 1
    layer = nfs_amd.CouplingLayer(d, H, mask)
    with torch.no_grad():
        for p in layer.parameters():
            p.add_(0.1 * torch.randn(p.shape))
    layer = layer.to(cuda_device).eval()
    x = torch.randn(B, d, device=cuda_device)
    L = nfs_amd._lib
    f = L.lib().nfx_affine_kernel_policy
    prev = f(-1)
    out = {}
    try:
        for name, pol in (("small", L.NFX_AFFINE_SMALL), ("streaming", L.NFX_AFFINE_STREAMING)):
            f(pol)
            with torch.no_grad():
                out[name] = layer.forward(x) + layer.inverse(x)
    finally:
        f(prev)
    for a, b in zip(out["small"], out["streaming"]):
        assert ((a - b).abs() <= 2e-6 * (1 + b.abs())).all(), (a - b).abs().max().item()


@pytest.mark.parametrize("B", [1_000_037, 999_999])
def test_streaming_half_chunk_tail_vs_oracle(cuda_device, B):
    """Streaming kernel at a batch where every wave runs F >= 1 whole 64-sample chunks AND the
    leftover chunks are split into 32-sample half chunks (2R <= nwaves): the tail region
    [F*nwaves*64, B) lies inside the last 2^18 rows, which are checked per element against the
    oracle in both directions, and the whole batch against the small-batch kernel, including
    the fused log_prob (LOGP) variant."""
    m, _ = realnvp_from_golden(cuda_device)
    x = torch.randn(B, 2, generator=torch.Generator().manual_seed(B)) * 1.5
    L = nfs_amd._lib
    f = L.lib().nfx_affine_kernel_policy
    prev = f(L.NFX_AFFINE_STREAMING)
    try:
        with torch.no_grad():
            xs = x.to(cuda_device)
            zi, ldi = m.inverse(xs)
            xf, ldf = m.forward(xs)
            lp = m.log_prob(xs)
        f(L.NFX_AFFINE_SMALL)
        with torch.no_grad():
            zi2, ldi2 = m.inverse(xs)
            xf2, ldf2 = m.forward(xs)
            lp2 = m.log_prob(xs)
    finally:
        f(prev)
    for a, b in ((zi, zi2), (xf, xf2)):
        assert ((a - b).abs() <= 2e-6 * (1 + b.abs())).all(), (a - b).abs().max().item()
    for a, b in ((ldi, ldi2), (ldf, ldf2), (lp, lp2)):
        assert ((a - b).abs() <= 2e-5 + 2e-6 * b.abs()).all(), (a - b).abs().max().item()
    tail = slice(B - (1 << 18), B)
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    with torch.no_grad():
        zr, ldr = oracle.flow_model(sd, oracle.realnvp_spec(8), x[tail], -1)
        xr, lfr = oracle.flow_model(sd, oracle.realnvp_spec(8), x[tail], 1)
        lpr = oracle.gauss_log_prob(zr, ldr)
    assert_y(zi[tail].cpu(), zr)
    assert_ld(ldi[tail].cpu(), ldr)
    assert_y(xf[tail].cpu(), xr)
    assert_ld(ldf[tail].cpu(), lfr)
    assert_lp(lp[tail].cpu(), lpr)


def _policy_run(pol, fn):
    L = nfs_amd._lib
    f = L.lib().nfx_affine_kernel_policy
    prev = f(pol)
    try:
        with torch.no_grad():
            return fn()
    finally:
        f(prev)


def test_split_mfma_layer2_accuracy_and_bias(cuda_device):
    """The streaming kernels run layer 2 of each net as six bf16 piece products per fp32
    multiply-add (csrc/nfx_affine_kernel.h affine_net_split, round 6). Against the fp32 chain of
    the small-batch kernel on the G2 RealNVP at 1M rows: per element within 2e-6 (1 + |ref|)
    (the bound two fp32 orderings meet too), and no systematic shift — the mean log p agrees to
    2e-8 (all-truncation pieces measured 4e-8, the shipped split 5e-9; profiles/r06_split/)."""
    m, _ = realnvp_from_golden(cuda_device)
    x = (torch.randn(1 << 20, 2, generator=torch.Generator().manual_seed(1234)) * 1.5).to(cuda_device)
    L = nfs_amd._lib
    zs, lds = _policy_run(L.NFX_AFFINE_STREAMING, lambda: m.inverse(x))
    lps = _policy_run(L.NFX_AFFINE_STREAMING, lambda: m.log_prob(x)).double()
    zf, ldf = _policy_run(L.NFX_AFFINE_SMALL, lambda: m.inverse(x))
    lpf = _policy_run(L.NFX_AFFINE_SMALL, lambda: m.log_prob(x)).double()
    assert ((zs - zf).abs() <= 2e-6 * (1 + zf.abs())).all()
    assert (lds - ldf).abs().max().item() <= 1e-5
    assert abs((lps - lpf).mean().item()) <= 2e-8


def test_split_mfma_fallback_is_per_tile(cuda_device):
    """A 32-row tile holding a non-finite or huge masked input runs the fp32 nets (the reference's
    inf / NaN propagation); the choice is per 32-aligned tile, so every other tile's rows — the
    other tile of the same 64-row unit included — are bit-identical to a clean batch, and the
    tile's finite rows stay within the oracle's tolerance."""
    m, _ = realnvp_from_golden(cuda_device)
    layer = m.flow.flows[0]
    B = 1 << 17
    x = torch.randn(B, 2, generator=torch.Generator().manual_seed(7)).to(cuda_device)
    xb = x.clone()
    xb[40, 0] = float("inf")   # tile 1 (rows 32..63) of unit 0
    xb[100, 1] = 3e38          # tile 3 (rows 96..127), huge but finite
    L = nfs_amd._lib
    for fn in (layer.forward, layer.inverse):
        y0, l0 = _policy_run(L.NFX_AFFINE_STREAMING, lambda: fn(x))
        y1, l1 = _policy_run(L.NFX_AFFINE_STREAMING, lambda: fn(xb))
        keep = torch.ones(B, dtype=torch.bool, device=cuda_device)
        keep[32:64] = False
        keep[96:128] = False
        assert torch.equal(y0[keep], y1[keep]) and torch.equal(l0[keep], l1[keep])
        # the fallback tiles' clean rows: the fp32 nets, within the parity tolerance of the clean run
        for lo, bad in ((32, 40), (96, 100)):
            rows = [r for r in range(lo, lo + 32) if r != bad]
            assert ((y1[rows] - y0[rows]).abs() <= 1e-5 * (1 + y0[rows].abs())).all()
        ys, ls = _policy_run(L.NFX_AFFINE_SMALL, lambda: fn(xb))
        assert torch.equal(torch.isnan(y1), torch.isnan(ys)) and torch.equal(torch.isinf(y1), torch.isinf(ys))
        assert torch.equal(torch.isnan(l1), torch.isnan(ls))
