"""GPU: fused Gaussian log_prob epilogue in the last inverse layer (nfx_*_logprob).

NormalizingFlowModel.log_prob runs the last layer of the inverse chain through its
`*_logprob` entry point when it has one (affine coupling, spline coupling, MAF inverse with
d <= 64 or H <= 64, the sequential IAF inverse with H <= 64)
and through nfx_gauss_logprob otherwise. Both evaluate
    logp = -0.5 * (fp32(d log 2pi) + sum_j z_j^2) + log_det
with the same sequential fp32 sum, so the fused per-sample logp must be BIT-identical to
inverse() + nfx_gauss_logprob; the float64 [sum, B] partials differ only by summation grouping
(|rel| <= 1e-12). Parity of inverse()/log_prob against the reference itself is covered in
test_gpu_affine.py / test_gpu_spline.py / test_gpu_made.py.
"""
import pytest
import torch

import nfs_amd
from nfs_amd.models.normalizing_flow_model import gauss_logprob

pytestmark = pytest.mark.gpu


def _perturb(m, sigma, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(sigma * torch.randn(p.shape, generator=g))
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.running_mean.copy_(0.1 * torch.randn(mod.running_mean.shape, generator=g))
                mod.running_var.copy_(0.5 + torch.rand(mod.running_var.shape, generator=g))
    return m


def _alt_mask(d, i):
    m = torch.zeros(d)
    m[(i % 2)::2] = 1
    return m


def _model(kind):
    torch.manual_seed(7)
    if kind == "realnvp":
        return _perturb(nfs_amd.RealNVP(2, 4, 64), 0.1, 1), 2, True
    if kind == "realnvp_bn_between":
        return _perturb(nfs_amd.RealNVP(2, 4, 64, batch_norm_between_layers=True), 0.1, 2), 2, True
    if kind == "affine_d5_h96":
        fl = [nfs_amd.CouplingLayer(5, 96, _alt_mask(5, i)) for i in range(3)]
        return _perturb(nfs_amd.NormalizingFlowModel(fl), 0.1, 3), 5, True
    if kind == "spline_k5":
        fl = [nfs_amd.SplineCouplingLayer(3, 64, _alt_mask(3, i), num_bins=5) for i in range(3)]
        return _perturb(nfs_amd.NormalizingFlowModel(fl), 0.1, 4), 3, True
    if kind == "maf63":
        fl = [nfs_amd.MaskedAutoregressiveFlow(63, 64) for _ in range(2)]
        return _perturb(nfs_amd.NormalizingFlowModel(fl), 0.02, 5), 63, True
    if kind == "maf80_wide":
        fl = [nfs_amd.MaskedAutoregressiveFlow(80, 64) for _ in range(2)]
        return _perturb(nfs_amd.NormalizingFlowModel(fl), 0.02, 6), 80, True
    if kind == "maf100_h128_chunked":
        fl = [nfs_amd.MaskedAutoregressiveFlow(100, 128) for _ in range(2)]
        return _perturb(nfs_amd.NormalizingFlowModel(fl), 0.02, 8), 100, False
    if kind == "iaf10_sequential":
        fl = [nfs_amd.InverseAutoregressiveFlow(10, 32) for _ in range(2)]
        return _perturb(nfs_amd.NormalizingFlowModel(fl), 0.02, 7), 10, True
    if kind == "iaf150_sequential":
        fl = [nfs_amd.InverseAutoregressiveFlow(150, 64) for _ in range(2)]
        return _perturb(nfs_amd.NormalizingFlowModel(fl), 0.02, 9), 150, True
    if kind == "maf40_h256":
        fl = [nfs_amd.MaskedAutoregressiveFlow(40, 256) for _ in range(2)]
        return _perturb(nfs_amd.NormalizingFlowModel(fl), 0.02, 11), 40, False
    if kind == "iaf90_h192_sequential":
        fl = [nfs_amd.InverseAutoregressiveFlow(90, 192) for _ in range(2)]
        return _perturb(nfs_amd.NormalizingFlowModel(fl), 0.02, 12), 90, False
    if kind == "iaf20_h96_sequential":
        fl = [nfs_amd.InverseAutoregressiveFlow(20, 96) for _ in range(2)]
        return _perturb(nfs_amd.NormalizingFlowModel(fl), 0.02, 10), 20, False
    raise ValueError(kind)


KINDS = ["realnvp", "realnvp_bn_between", "affine_d5_h96", "spline_k5", "maf63",
         "maf80_wide", "maf100_h128_chunked", "iaf10_sequential", "iaf150_sequential",
         "iaf20_h96_sequential", "maf40_h256", "iaf90_h192_sequential"]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("B", [0, 1, 77, 4099, 300_001])
def test_fused_logprob_matches_unfused(cuda_device, kind, B):
    if kind.startswith("iaf") and B > 4099:
        pytest.skip("sequential IAF inverse: small batches only")
    m, d, fused_expected = _model(kind)
    m = m.to(cuda_device).eval()
    g = torch.Generator().manual_seed(100 + B)
    x = (1.5 * torch.randn(B, d, generator=g)).to(cuda_device)
    with torch.no_grad():
        lp, sums = m.log_prob(x, return_sums=True)
        z, ld = m.inverse(x)
        lp_ref, sums_ref = gauss_logprob(z, ld)
        torch.cuda.synchronize()
    assert lp.shape == (B,) and sums.dtype == torch.float64
    bad = (lp != lp_ref).nonzero().flatten().tolist()
    assert not bad, (len(bad), bad[:16], lp[bad[:4]].tolist(), lp_ref[bad[:4]].tolist())
    s, sr = sums.cpu(), sums_ref.cpu()
    assert s[1].item() == B
    assert abs(s[0].item() - sr[0].item()) <= 1e-12 * max(1.0, abs(sr[0].item()))
    if B:
        assert abs(s[0].item() - lp.double().sum().item()) <= 1e-9 * max(1.0, abs(s[0].item()))


@pytest.mark.parametrize("kind", ["iaf150_sequential", "maf63"])
def test_repeat_calls_bit_identical(cuda_device, kind):
    # The sequential kernel stages weight blocks by LDS-DMA into a double buffer: repeated calls
    # (fused and unfused, different grids for B and B + 32) must give identical rows.
    m, d, _ = _model(kind)
    m = m.to(cuda_device).eval()
    g = torch.Generator().manual_seed(5)
    x = (1.5 * torch.randn(4099 + 32, d, generator=g)).to(cuda_device)
    with torch.no_grad():
        z0, ld0 = m.inverse(x[:4099])
        lp0 = m.log_prob(x[:4099])
        for it in range(8):
            xb = x if it % 2 else x[:4099]
            z, ld = m.inverse(xb)
            lp = m.log_prob(xb)
            for a, b, name in ((z[:4099], z0, "z"), (ld[:4099], ld0, "ld"), (lp[:4099], lp0, "lp")):
                bad = (a != b).reshape(4099, -1).any(dim=1).nonzero().flatten().tolist()
                assert not bad, (it, name, len(bad), bad[:16])


@pytest.mark.parametrize("kind", KINDS)
def test_fused_path_taken(cuda_device, kind):
    """Layers with a fused variant skip the separate Gaussian pass (one launch fewer)."""
    m, d, fused_expected = _model(kind)
    m = m.to(cuda_device).eval()
    x = torch.randn(1000, d, device=cuda_device)
    with torch.no_grad():
        logp, sums = torch.empty(1000, device=cuda_device), torch.empty(2, device=cuda_device, dtype=torch.float64)
        ws = torch.empty(1 << 16, device=cuda_device, dtype=torch.uint8)  # (any content, ABI 3)
        chain = getattr(m, "flow", m)  # RealNVP wraps a NormalizingFlowModel
        _, _, fused = chain._hip_chain(x, -1, logprob=(logp, sums, ws))
    assert fused == fused_expected


def test_fused_logprob_nonfinite_rows(cuda_device):
    """Non-finite inputs go through the reference guards first (z, log-det zeroed), so the
    fused and unfused logp agree on them too."""
    m, d, _ = _model("realnvp")
    m = m.to(cuda_device).eval()
    x = torch.randn(256, 2)
    x[3, 0] = float("nan")
    x[10, 1] = float("inf")
    x[20] = 1e10
    x = x.to(cuda_device)
    with torch.no_grad():
        lp = m.log_prob(x)
        z, ld = m.inverse(x)
        lp_ref, _ = gauss_logprob(z, ld)
    assert torch.equal(lp.isnan(), lp_ref.isnan())
    ok = ~lp.isnan()
    assert torch.equal(lp[ok], lp_ref[ok])


@pytest.mark.parametrize("kind", ["realnvp", "spline_k5", "maf63", "iaf10_sequential"])
def test_graphed_flow_matches_eager(cuda_device, kind):
    """A captured HIP graph of the whole pass replays to the eager result bit for bit, and a
    weight update after capture is refused under strict=True."""
    m, d, _ = _model(kind)
    m = m.to(cuda_device).eval()
    x = torch.randn(3000, d, device=cuda_device)
    g = nfs_amd.GraphedFlow(m, x, mode="log_prob")
    gf = nfs_amd.GraphedFlow(m, x, mode="forward")
    with torch.no_grad():
        lp, sums = m.log_prob(x, return_sums=True)
        y, ld = m.forward(x)
    x2 = torch.randn(3000, d, device=cuda_device)
    with torch.no_grad():
        lp2 = m.log_prob(x2)
    glp, gsums = g()
    assert torch.equal(glp, lp) and torch.equal(gsums, sums)
    gy, gld = gf()
    assert torch.equal(gy, y) and torch.equal(gld, ld)
    assert torch.equal(g(x2)[0], lp2)
    with torch.no_grad():
        next(m.parameters()).add_(1e-3)
    with pytest.raises(RuntimeError):
        g()


def test_graphed_sampling(cuda_device):
    """GraphedFlow(mode="sample") — on-device z ~ N(0, I) + forward in one graph launch
    (§8(f) item 3): every replay draws fresh z, the output equals the eager forward of that z
    bit for bit, and the draws are standard normal."""
    m, d, _ = _model("realnvp")
    m = m.to(cuda_device).eval()
    g = nfs_amd.GraphedFlow(m, torch.empty(4000, d, device=cuda_device), mode="sample")
    x1, ld1 = g()
    z1 = g.static_in.clone()
    x1 = x1.clone()
    x2, _ = g()
    z2 = g.static_in.clone()
    assert not torch.equal(z1, z2)
    with torch.no_grad():
        y, ld = m.forward(z2)
    assert torch.equal(x2, y)
    zs = torch.cat([z1, z2])
    assert abs(zs.mean().item()) < 0.05 and abs(zs.std().item() - 1) < 0.05
    with pytest.raises(ValueError):
        g(z1)


@pytest.mark.parametrize("kind", ["realnvp", "maf63", "iaf150_sequential"])
def test_concurrent_streams_own_workspaces(cuda_device, kind):
    """Two log_prob calls issued on two streams at once (different inputs) and two captured
    graphs replayed on two streams: each uses its own workspace (per-stream cache, the graphs'
    own), so every NLL partial equals its serial value bit for bit (a shared arrival counter /
    partials array would let the launches corrupt each other's sums)."""
    m, d, _ = _model(kind)
    m = m.to(cuda_device).eval()
    B1, B2 = (300_001, 200_003) if not kind.startswith("iaf") else (4099, 3001)
    g = torch.Generator().manual_seed(5)
    xa = torch.randn(B1, d, generator=g).to(cuda_device)
    xb = torch.randn(B2, d, generator=g).to(cuda_device)
    with torch.no_grad():
        la, sa = m.log_prob(xa, return_sums=True)
        lb, sb = m.log_prob(xb, return_sums=True)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(4):
        s1.wait_stream(torch.cuda.current_stream())
        s2.wait_stream(torch.cuda.current_stream())
        with torch.no_grad():
            with torch.cuda.stream(s1):
                la2, sa2 = m.log_prob(xa, return_sums=True)
            with torch.cuda.stream(s2):
                lb2, sb2 = m.log_prob(xb, return_sums=True)
        torch.cuda.synchronize()
        assert torch.equal(sa2, sa) and torch.equal(sb2, sb)
        assert torch.equal(la2, la) and torch.equal(lb2, lb)
    ga = nfs_amd.GraphedFlow(m, xa, mode="log_prob")
    gb = nfs_amd.GraphedFlow(m, xb, mode="log_prob")
    assert ga.workspace.data_ptr() != gb.workspace.data_ptr()
    for _ in range(4):
        s1.wait_stream(torch.cuda.current_stream())
        s2.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s1):
            ra = ga()
        with torch.cuda.stream(s2):
            rb = gb()
        torch.cuda.synchronize()
        assert torch.equal(ra[1], sa) and torch.equal(rb[1], sb)


def test_log_prob_caller_workspace(cuda_device):
    """log_prob(x, workspace=...) runs on a caller-owned workspace (and rejects one that is too
    small)."""
    from nfs_amd.models.normalizing_flow_model import new_gauss_workspace
    m, d, _ = _model("spline_k5")
    m = m.to(cuda_device).eval()
    x = torch.randn(5000, d, device=cuda_device)
    ws = new_gauss_workspace(5000, cuda_device)
    with torch.no_grad():
        lp, s = m.log_prob(x, return_sums=True)
        lp2, s2 = m.log_prob(x, return_sums=True, workspace=ws)
        with pytest.raises(ValueError):
            m.log_prob(x, return_sums=True, workspace=ws[:8])
    assert torch.equal(lp, lp2) and torch.equal(s, s2)


@pytest.mark.parametrize("kind", ["realnvp", "maf63", "iaf10_sequential"])
def test_log_prob_autograd_gauss_adjoint(cuda_device, kind):
    """loss = -log_prob(x).mean() under autograd on the GPU: the base log-density is the HIP
    epilogue with its HIP adjoint (nfx_gauss_logprob_backward). The loss, dL/dx and every
    parameter gradient agree with float64 autograd of the same model within 4x the fp32
    composite's own distance from it (+ 2e-5 of the gradient's scale); every call HIP, and logp
    equals the eval path's bit for bit."""
    import copy
    model, d, _ = _model(kind)
    model = model.eval()
    g = torch.Generator().manual_seed(31)
    x = torch.randn(3000, d, generator=g) * 0.8

    def run(m, xx):
        xx = xx.clone().requires_grad_(True)
        logp = m.log_prob(xx)
        loss = -logp.mean()
        loss.backward()
        return logp.detach(), xx.grad, [p.grad for p in m.parameters()]

    l64, gx64, gp64 = run(copy.deepcopy(model).double(), x.double())
    l32, gx32, gp32 = run(copy.deepcopy(model), x)
    gm = copy.deepcopy(model).to(cuda_device)
    nfs_amd.reset_stats()
    lg, gxg, gpg = run(gm, x.to(cuda_device))
    assert nfs_amd.STATS["torch"] == 0, nfs_amd.STATS
    with torch.no_grad():
        assert torch.equal(lg, gm.log_prob(x.to(cuda_device)))

    def close(a, b32, b64, what):
        a, b32, b64 = a.double().cpu(), b32.double(), b64.double()
        bound = 2e-5 * (1 + b64.abs().max().item()) + 4 * (b32 - b64).abs().max().item()
        err = (a - b64).abs().max().item()
        assert err <= bound, f"{what}: max err {err:.3g} > {bound:.3g}"

    close(lg, l32, l64, "logp")
    close(gxg, gx32, gx64, "dL/dx")
    for (n, _), a, b, c in zip(model.named_parameters(), gpg, gp32, gp64):
        close(a, b, c, n)


def test_last_kernel_names_dispatch(cuda_device):
    """nfx_last_kernel names the kernel an entry point dispatched (bench.py labels its roofline
    with it): a RealNVP log_prob at 100k rows runs the streaming chain, at 4k the small-batch
    chain; an IAF(784, 64) log_prob at 1Ki the push kernel."""
    from nfs_amd import _lib
    model = nfs_amd.RealNVP(2, 4, 64).to(cuda_device).eval()
    with torch.no_grad():
        model.log_prob(torch.randn(100_000, 2, device=cuda_device))
        assert _lib.last_kernel() == "affine_schain_kernel"
        model.log_prob(torch.randn(4_000, 2, device=cuda_device))
        assert _lib.last_kernel() == "affine_chain_kernel"
        iaf = nfs_amd.NormalizingFlowModel([nfs_amd.InverseAutoregressiveFlow(784, 64)]).to(cuda_device).eval()
        iaf.log_prob(torch.randn(1024, 784, device=cuda_device))
        assert _lib.last_kernel() == "made_seqp_kernel"


@pytest.mark.parametrize("kind", KINDS + ["iaf784_push", "iaf784_seqs"])
def test_garbage_workspace_gives_serial_sums(cuda_device, kind):
    """ABI 3: the log_prob workspace needs no zero-fill. A workspace filled with 0xFF, zeros, or
    an arrival word holding another tag with a count, gives the serial [sum log p, B] and logp bit
    for bit, call after call, for every fused epilogue and the separate Gaussian pass."""
    from nfs_amd.models.normalizing_flow_model import new_gauss_workspace
    if kind.startswith("iaf784"):
        torch.manual_seed(9)
        m = _perturb(nfs_amd.NormalizingFlowModel([nfs_amd.InverseAutoregressiveFlow(784, 64)]), 0.01, 9)
        d = 784
        B = 1024 if kind == "iaf784_push" else 8192
    else:
        m, d, _ = _model(kind)
        B = 4099 if kind.startswith("iaf") else 70_001
    m = m.to(cuda_device).eval()
    x = torch.randn(B, d, generator=torch.Generator().manual_seed(3)).to(cuda_device)
    ws0 = new_gauss_workspace(B, cuda_device)
    ws0.zero_()
    with torch.no_grad():
        lp, s = m.log_prob(x, return_sums=True, workspace=ws0)
        wsf = new_gauss_workspace(B, cuda_device)
        for fill in ("ff", "midcount", "zero", "ff"):
            if fill == "ff":
                wsf.fill_(0xFF)
            elif fill == "zero":  # the ABI-2 convention: a foreign word for ABI 3, claimed once
                wsf.zero_()
            else:  # arrival word (after the 4096 float64 partials): another launch's tag, count 3
                wsf.zero_()
                w = wsf.view(torch.int64)
                w[4096] = (0x123456789 << 16) | 3
            for _ in range(2):
                lp2, s2 = m.log_prob(x, return_sums=True, workspace=wsf)
                torch.cuda.synchronize()
                assert torch.equal(s2, s), (fill, s2.tolist(), s.tolist())
                assert torch.equal(lp2, lp)
