"""GPU: fused backward of the MAF density direction (nfx_made_affine_backward, §8(f) item 1).

Gradients (dL/dx and every MADE parameter) of L = <gz, z> + <gld, log_det> through
MaskedAutoregressiveFlow.inverse, against autograd of the same module evaluated in float64 on
the CPU (the reference's ops, masked_autoregressive_flow.py:18-44). The fp32 kernel must be as
close to the float64 gradients as the fp32 composite is (checked side by side), within
  per element |g - g64| <= 1e-5 * (1 + |g64|) for dL/dx, and
  max |g - g64| <= 2e-5 * (1 + max |g64|) for the parameter gradients (sums over the batch).
"""
import copy

import pytest
import torch

import nfs_amd
from nfs_amd.flows.flow import STATS

pytestmark = pytest.mark.gpu


def _maf(d, H, seed):
    torch.manual_seed(seed)
    f = nfs_amd.MaskedAutoregressiveFlow(d, H)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in f.parameters():
            p.add_(0.1 * torch.randn(p.shape, generator=g))
    return f


def _grads(f, x, gz, gld):
    x = x.clone().requires_grad_(True)
    for p in f.parameters():
        p.grad = None
    z, ld = f.inverse(x)
    ((z * gz).sum() + (ld * gld).sum()).backward()
    return x.grad, [p.grad for p in f.parameters()]


def _check(g, ref, tol):
    g, ref = g.double().cpu(), ref.double().cpu()
    err = (g - ref).abs().max().item()
    assert err <= tol * (1 + ref.abs().max().item()), (err, ref.abs().max().item())


@pytest.mark.parametrize("d,H,B", [(5, 16, 1), (5, 16, 77), (33, 32, 1000), (63, 64, 2048), (64, 64, 300),
                                   (2, 64, 500)])
def test_made_backward_vs_float64_autograd(cuda_device, d, H, B):
    f = _maf(d, H, d * 100 + H)
    f64 = copy.deepcopy(f).double()
    x = torch.randn(B, d)
    x[: min(B, 3)] *= 4.0  # some rows saturate the alpha clamp
    gz = torch.randn(B, d)
    gld = torch.randn(B)
    gx64, gp64 = _grads(f64, x.double(), gz.double(), gld.double())
    fg = f.to(cuda_device).train()  # train(): parameters require grad; no BatchNorm in this MADE
    STATS["hip"] = 0
    gx, gp = _grads(fg, x.to(cuda_device), gz.to(cuda_device), gld.to(cuda_device))
    assert STATS["hip"] >= 2  # fused forward + fused backward
    assert ((gx.double().cpu() - gx64).abs() <= 1e-5 * (1 + gx64.abs())).all()
    for g, r in zip(gp, gp64):
        _check(g, r, 2e-5)


def test_made_backward_logdet_clamp_and_training_step(cuda_device):
    """A saturated log-det (|sum alpha| > 100 is impossible at |alpha| <= 3 for d < 34, so use
    d = 63 with large alphas) blocks the log-det gradient exactly like torch.clamp; then one
    full training step through NormalizingFlowModel matches the composite backward."""
    d, H = 63, 64
    f = _maf(d, H, 7)
    with torch.no_grad():
        f.conditioner.linears()[-1].bias[d:] += 5.0  # every alpha clamps at +3 -> ld = -189 -> clamp
    f64 = copy.deepcopy(f).double()
    x = torch.randn(256, d)
    gz, gld = torch.randn(256, d), torch.randn(256)
    gx64, gp64 = _grads(f64, x.double(), gz.double(), gld.double())
    gx, gp = _grads(f.to(cuda_device), x.to(cuda_device), gz.to(cuda_device), gld.to(cuda_device))
    assert ((gx.double().cpu() - gx64).abs() <= 1e-5 * (1 + gx64.abs())).all()
    for g, r in zip(gp, gp64):
        _check(g, r, 2e-5)

    torch.manual_seed(1)
    model = nfs_amd.NormalizingFlowModel([_maf(d, H, 20 + i) for i in range(3)])
    ref = copy.deepcopy(model).double()
    data = torch.randn(1024, d)
    loss64 = -ref.log_prob(data.double()).mean()
    loss64.backward()
    model = model.to(cuda_device).train()
    loss = -model.log_prob(data.to(cuda_device)).mean()
    loss.backward()
    assert abs(loss.item() - loss64.item()) <= 1e-5 * (1 + abs(loss64.item()))
    for p, p64 in zip(model.parameters(), ref.parameters()):
        _check(p.grad, p64.grad, 2e-5)


# ---- every MADE direction under autograd (IAF density / sampling, MAF sampling) ---------------
def _flow(cls, d, H, seed, sigma=0.1):
    torch.manual_seed(seed)
    f = cls(d, H)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for p in f.parameters():
            p.add_(sigma * torch.randn(p.shape, generator=g))
    return f


def _dir_grads(f, x, gy, gld, direction):
    x = x.clone().requires_grad_(True)
    for p in f.parameters():
        p.grad = None
    y, ld = f.forward(x) if direction > 0 else f.inverse(x)
    ((y * gy).sum() + (ld * gld).sum()).backward()
    return y.detach(), x.grad, [p.grad for p in f.parameters()]


def _close_or_ref(g, g64, g32, tol, what):
    """|g - g64| <= max(tol * (1 + max|g64|), 4 * |g32 - g64|max): within tol of the float64
    gradient's scale, or as close as the reference's own fp32 composite."""
    g, g64, g32 = g.double().cpu(), g64.double().cpu(), g32.double().cpu()
    err = (g - g64).abs().max().item()
    ref_err = (g32 - g64).abs().max().item()
    bound = max(tol * (1 + g64.abs().max().item()), 4 * ref_err)
    assert err <= bound, f"{what}: err {err:.3e} > {bound:.3e} (fp32 composite err {ref_err:.3e})"


@pytest.mark.parametrize("kind,direction,d,H,B", [
    ("iaf", -1, 5, 16, 1), ("iaf", -1, 20, 32, 300), ("iaf", -1, 100, 64, 64), ("iaf", -1, 10, 96, 200),
    ("iaf", -1, 7, 128, 100), ("iaf", -1, 784, 64, 6),
    ("maf", 1, 5, 16, 77), ("maf", 1, 20, 64, 300), ("maf", 1, 9, 128, 65),
    ("iaf", 1, 5, 16, 1), ("iaf", 1, 33, 32, 1000), ("iaf", 1, 63, 64, 2048), ("iaf", 1, 2, 64, 500),
    # general-shape parallel kernel (made_bwdw_kernel): d > 64 or H > 64
    ("maf", -1, 100, 64, 300), ("maf", -1, 20, 128, 257), ("maf", -1, 63, 96, 513), ("iaf", 1, 784, 64, 100),
    ("iaf", 1, 65, 32, 31), ("maf", -1, 130, 128, 64),
])
def test_all_directions_backward_vs_float64_autograd(cuda_device, kind, direction, d, H, B):
    """Fused backward of each MADE direction (nfx_made_affine_backward for the parallel ones,
    nfx_made_seq_backward's reverse sweep for the sequential ones, nfx_made_backward_weights for
    the parameters) against autograd through the reference ops in float64, side by side with
    the fp32 composite: inverse_autoregressive_flow.py:30-103, masked_autoregressive_flow.py:46-78."""
    cls = nfs_amd.InverseAutoregressiveFlow if kind == "iaf" else nfs_amd.MaskedAutoregressiveFlow
    f = _flow(cls, d, H, d * 31 + H + (direction > 0))
    f64 = copy.deepcopy(f).double()
    f32 = copy.deepcopy(f)
    gen = torch.Generator().manual_seed(B + d)
    x = torch.randn(B, d, generator=gen)
    if B > 3:
        x[:3] *= 6.0  # saturate clamps on a few rows
    gy = torch.randn(B, d, generator=gen)
    gld = torch.randn(B, generator=gen)
    y64, gx64, gp64 = _dir_grads(f64, x.double(), gy.double(), gld.double(), direction)
    _, gx32, gp32 = _dir_grads(f32, x, gy, gld, direction)
    fg = f.to(cuda_device)
    STATS["hip"] = 0
    STATS["torch"] = 0
    y, gx, gp = _dir_grads(fg, x.to(cuda_device), gy.to(cuda_device), gld.to(cuda_device), direction)
    assert STATS["hip"] == 2 and STATS["torch"] == 0, STATS  # fused forward + fused backward
    assert ((y.double().cpu() - y64).abs() <= 2e-5 * (1 + y64.abs())).all()
    _close_or_ref(gx, gx64, gx32, 2e-5, "dL/dx")
    for (k, _), g, r, r32 in zip(f.named_parameters(), gp, gp64, gp32):
        _close_or_ref(g, r, r32, 2e-5, k)


@pytest.mark.parametrize("policy", ["wave", "segment"])
@pytest.mark.parametrize("kind,direction,d,H,B", [
    ("iaf", -1, 2, 64, 2000), ("iaf", -1, 5, 16, 1), ("iaf", -1, 20, 32, 300), ("iaf", -1, 100, 48, 64),
    ("iaf", -1, 784, 64, 6), ("maf", 1, 2, 64, 2000), ("maf", 1, 5, 16, 77), ("maf", 1, 63, 64, 300),
])
def test_sequential_backward_both_kernels(cuda_device, kind, direction, d, H, B, policy):
    """The sequential directions' backward on both kernels (nfx_made_seq_policy): the
    lane-per-sample reverse sweep (made_seq_bwd_kernel) and the wave-per-sample one
    (made_seqw_bwd_kernel, H <= 64), against float64 autograd side by side with the fp32
    composite; d = 2, H = 64, B = 2,000 is the reference's IAF / MAF figure-model layer."""
    from nfs_amd import _lib
    L = _lib.lib()
    old = L.nfx_made_seq_policy(_lib.NFX_MADE_SEQ_WAVE if policy == "wave" else _lib.NFX_MADE_SEQ_SEGMENT)
    try:
        test_all_directions_backward_vs_float64_autograd(cuda_device, kind, direction, d, H, B)
    finally:
        L.nfx_made_seq_policy(old)


def test_iaf_density_training_step(cuda_device):
    """NormalizingFlowModel of IAF layers trained on the density direction (the reference's
    IAF.inverse under -log_prob): loss and every gradient match float64 autograd."""
    torch.manual_seed(3)
    flows = [_flow(nfs_amd.InverseAutoregressiveFlow, 12, 32, 50 + k) for k in range(3)]
    model = nfs_amd.NormalizingFlowModel(flows)
    m64 = copy.deepcopy(model).double()
    x = torch.randn(512, 12, generator=torch.Generator().manual_seed(9))
    l64 = -m64.log_prob(x.double()).mean()
    l64.backward()
    mg = model.to(cuda_device)
    STATS["torch"] = 0
    loss = -mg.log_prob(x.to(cuda_device)).mean()
    loss.backward()
    assert STATS["torch"] == 0, STATS
    assert abs(loss.item() - l64.item()) <= 1e-5 * (1 + abs(l64.item()))
    for (k, p), (_, p64) in zip(mg.named_parameters(), m64.named_parameters()):
        _check(p.grad, p64.grad, 5e-5)


@pytest.mark.parametrize("cls", [nfs_amd.MaskedAutoregressiveFlow, nfs_amd.InverseAutoregressiveFlow])
def test_wide_hidden_training_step(cuda_device, cls):
    """H = 256 (outside the fused backward kernels' H <= 128): the forward runs nfx_made_big.hip,
    autograd recomputes through the layer's composite; loss and gradients match float64."""
    torch.manual_seed(5)
    flows = [_flow(cls, 10, 256, 70 + k) for k in range(2)]
    model = nfs_amd.NormalizingFlowModel(flows)
    m64 = copy.deepcopy(model).double()
    x = torch.randn(300, 10, generator=torch.Generator().manual_seed(4))
    l64 = -m64.log_prob(x.double()).mean()
    l64.backward()
    mg = model.to(cuda_device)
    loss = -mg.log_prob(x.to(cuda_device)).mean()
    loss.backward()
    assert abs(loss.item() - l64.item()) <= 1e-5 * (1 + abs(l64.item()))
    for (k, p), (_, p64) in zip(mg.named_parameters(), m64.named_parameters()):
        _check(p.grad, p64.grad, 5e-5)


def test_made_weight_grad_nonfinite_pattern(cuda_device):
    """The weight-gradient contraction skips output tiles whose 32x32 mask block is all zero
    (round 6). Where the reference's (δ·aᵀ) ⊙ mask is NaN there (0 x inf: a non-finite upstream
    gradient reaches a δ row), the kernel must give NaN too: every parameter gradient has the
    composite's NaN / inf pattern, and equal values elsewhere within the parity bar."""
    d, H, B = 63, 64, 512
    f = _maf(d, H, 11)
    x = torch.randn(B, d)
    gz, gld = torch.randn(B, d), torch.randn(B)
    gz[7, 20] = float("inf")
    gxc, gpc = _grads(copy.deepcopy(f), x, gz, gld)
    gx, gp = _grads(f.to(cuda_device).train(), x.to(cuda_device), gz.to(cuda_device), gld.to(cuda_device))
    for g, r in zip(gp, gpc):
        g = g.cpu()
        assert torch.equal(g.isnan(), r.isnan()), (int(g.isnan().sum()), int(r.isnan().sum()))
        assert torch.equal(g.isinf(), r.isinf())
        fin = r.isfinite()
        if fin.any():
            _check(g[fin], r[fin], 2e-5)


@pytest.mark.parametrize("B", [1000, 4099])
def test_made_backward_weights_abi_nonfinite_factors(cuda_device, B):
    """nfx_made_backward_weights on synthetic factors against float64 (δ·aᵀ) ⊙ mask and Σ δ:
    a non-finite INPUT row entry (column flags of the skipped masked tiles) and a NaN δ entry
    (row flags) give the reference's NaN / inf pattern; every finite entry within 2e-5 of the
    float64 value's scale."""
    from nfs_amd import _lib
    import ctypes
    L = _lib.lib()
    d, H = 63, 64
    f = _maf(d, H, 5)
    masks = [lin.mask.detach().float() for lin in f.conditioner.linears()]
    g = torch.Generator().manual_seed(B)
    rows = 2 * d + 3 * H + 3 * (H + 1) + (d + 1)
    fac = torch.randn(rows, B, generator=g)
    o = {"D4": 0, "D3": 2 * d, "D2": 2 * d + H, "D1": 2 * d + 2 * H, "H3": 2 * d + 3 * H,
         "H2": 2 * d + 4 * H + 1, "H1": 2 * d + 5 * H + 2, "X1": 2 * d + 6 * H + 3}
    fac[o["X1"] + 40, 5] = float("inf")   # input 40 of layer 1: a column of W1's tiles
    fac[o["D2"] + 3, 7] = float("nan")    # δ row 3 of layer 2
    pairs = [("D1", H, "X1", d), ("D2", H, "H1", H), ("D3", H, "H2", H), ("D4", 2 * d, "H3", H)]
    want = []
    for (dn, m, an, n), mk in zip(pairs, masks):
        D = fac[o[dn]:o[dn] + m].double()
        A = fac[o[an]:o[an] + n].double()
        want += [(D @ A.T) * mk.double(), D.sum(1)]
    assert L.nfx_made_backward_factor_floats(B, d, H) >= fac.numel()
    dev = cuda_device
    facd = torch.zeros(L.nfx_made_backward_factor_floats(B, d, H), device=dev)
    facd[:fac.numel()] = fac.reshape(-1).to(dev)
    grads = torch.empty(L.nfx_made_param_floats(d, H), device=dev)
    ws = torch.empty(max(1, L.nfx_made_wgrad_workspace_bytes(B, d, H)), device=dev, dtype=torch.uint8)
    md = [m.to(dev).contiguous() for m in masks]
    mp = (ctypes.c_void_p * 4)(*[m.data_ptr() for m in md])
    _lib.check(L.nfx_made_backward_weights(_lib.ptr(facd), B, d, H, mp, _lib.ptr(grads), _lib.ptr(ws),
                                           _lib.stream_of(facd)), "nfx_made_backward_weights")
    got, off = [], 0
    gc = grads.cpu()
    for w in want:
        got.append(gc[off:off + w.numel()].view_as(w))
        off += w.numel()
    for gv, wv in zip(got, want):
        assert torch.equal(gv.isnan(), wv.isnan()), (int(gv.isnan().sum()), int(wv.isnan().sum()))
        assert torch.equal(gv.isinf(), wv.isinf())
        fin = wv.isfinite()
        err = (gv.double()[fin] - wv[fin]).abs().max().item()
        assert err <= 2e-5 * (1 + wv[fin].abs().max().item()), err
