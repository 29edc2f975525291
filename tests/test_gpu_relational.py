"""GPU: the reference's relational acceptance suite (tests/correctness/) run on the HIP path.

Mirrors:
* test_invertibility.py:131-161 — forward(inverse(x)) round trip and log_det_fwd + log_det_inv = 0
  (tolerance 1e-5, 1e-3 for MAF/IAF as the reference states), on the kernels, eval mode, with
  trained-looking (perturbed) weights and between-layer BatchNorm.
* test_logdet_autodiff.py — kernel log-det vs log|det J| of the layer map, J by autograd on a
  float64 copy of the same module (rel 1e-4 / abs 1e-4, the reference's tolerance).
* test_autoregressive_mask_correctness.py — the Jacobian is triangular; here checked on the
  kernels themselves, bit for bit: perturbing input j leaves every output i < j unchanged.
* test_distribution_preservation.py — 200 Adam steps on N(0, I) data on the HIP path (train-mode
  coupling kernels + fused backward, fused MAF backward), test NLL < 3.0 on the reference's seed
  and within the oracle's own per-seed bound on the others, sample mean/covariance within the
  reference's bounds (median over three seeds: the outcome is chaotic).
"""
import copy
import json
import os

import pytest
import torch

import nfs_amd

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

pytestmark = pytest.mark.gpu


def _mask(dim, kind):
    m = torch.zeros(dim)
    if kind == "alternating":
        m[::2] = 1
    else:
        m[: dim // 2] = 1
    return m


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


def _flows(dim, H=32):
    """The reference's flow list (test_invertibility.py:31-59, test_logdet_autodiff.py:31-52)."""
    return {
        "coupling_alt": nfs_amd.CouplingLayer(dim, H, _mask(dim, "alternating")),
        "coupling_half": nfs_amd.CouplingLayer(dim, H, _mask(dim, "half")),
        "spline_alt": nfs_amd.SplineCouplingLayer(dim, H, _mask(dim, "alternating"), num_bins=8),
        "spline_half": nfs_amd.SplineCouplingLayer(dim, H, _mask(dim, "half"), num_bins=8),
        "maf": nfs_amd.MaskedAutoregressiveFlow(dim, H),
        "iaf": nfs_amd.InverseAutoregressiveFlow(dim, H),
        "arqs": nfs_amd.ARQS(dim, H, num_bins=8),
        "realnvp_bn": nfs_amd.RealNVP(dim, 4, H, batch_norm_between_layers=True),
        "realnvp_spline_bn": nfs_amd.RealNVPSpline(dim, 2, H, batch_norm_between_layers=True),
        "mixed": nfs_amd.NormalizingFlowModel([
            nfs_amd.CouplingLayer(dim, H, _mask(dim, "alternating")),
            nfs_amd.MaskedAutoregressiveFlow(dim, H),
            nfs_amd.CouplingLayer(dim, H, _mask(dim, "half"))]),
    }


AUTOREG = ("maf", "iaf")


# ARQS is left out: the reference's inverse conditions on z where its forward conditions on x
# (arqs.py:54 vs :92), so ARQS.inverse is not the inverse of ARQS.forward (g10 fixtures).
@pytest.mark.parametrize("name", [n for n in _flows(4).keys() if n != "arqs"])
def test_invertibility_and_logdet_symmetry(cuda_device, name):
    torch.manual_seed(456)
    f = _perturb(_flows(4)[name], 0.05 if name in AUTOREG else 0.1, 7).to(cuda_device).eval()
    z = torch.randn(512, 4, device=cuda_device)
    nfs_amd.reset_stats()
    with torch.no_grad():
        x, ld_fwd = f.forward(z)
        z2, ld_inv = f.inverse(x)
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] > 0, nfs_amd.STATS
    # the reference's tolerances (test_invertibility.py:154): 1e-3 for MAF/IAF, 1e-5 otherwise
    tol = 1e-3 if name in AUTOREG else 1e-5
    err = (ld_fwd + ld_inv).abs().max().item()
    assert err < tol, err
    assert ((z2 - z).abs() / (1 + z.abs())).max().item() < 1e-4


@pytest.mark.parametrize("name", ["coupling_alt", "spline_half", "maf", "iaf", "realnvp_bn", "mixed"])
@pytest.mark.parametrize("dim", [2, 3])
def test_logdet_matches_autodiff_jacobian(cuda_device, name, dim):
    torch.manual_seed(0)
    f = _perturb(_flows(dim)[name], 0.05 if name in AUTOREG else 0.1, 11).eval()
    f64 = copy.deepcopy(f).double()
    fg = f.to(cuda_device)
    x = torch.randn(16, dim)
    with torch.no_grad():
        _, ld = fg.forward(x.to(cuda_device))
    ld = ld.double().cpu()
    for i in range(x.shape[0]):
        J = torch.autograd.functional.jacobian(lambda t: f64.forward(t.unsqueeze(0))[0].squeeze(0), x[i].double())
        ref = torch.linalg.slogdet(J)[1]
        assert abs(ld[i].item() - ref.item()) <= 1e-4 + 1e-4 * abs(ref.item()), (i, ld[i].item(), ref.item())


@pytest.mark.parametrize("cls,direction", [("maf", -1), ("maf", 1), ("iaf", 1), ("iaf", -1), ("arqs", 1),
                                           ("arqs", -1)])
@pytest.mark.parametrize("d", [3, 5, 10, 63, 100])
def test_autoregressive_structure_bitwise(cuda_device, cls, direction, d):
    """Output i of the kernel depends only on inputs <= i (inputs < i for the conditioner):
    moving input j must leave outputs 0..j-1 bit-identical."""
    torch.manual_seed(d)
    f = _perturb(_flows(d, 32)[cls], 0.05, d).to(cuda_device).eval()
    x = torch.randn(64, d, device=cuda_device)
    if cls == "arqs":
        x = torch.rand(64, d, device=cuda_device) * 0.5  # inside the unit interval after +0.75
    run = f.inverse if direction < 0 else f.forward
    with torch.no_grad():
        y0, _ = run(x)
        for j in sorted({0, 1, d // 2, d - 1}):
            xp = x.clone()
            xp[:, j] += 0.75
            y1, _ = run(xp)
            assert torch.equal(y0[:, :j], y1[:, :j]), (j, (y0[:, :j] - y1[:, :j]).abs().max().item())
            assert not torch.equal(y0[:, j:], y1[:, j:])


def _train(flow, data, steps=200, lr=1e-3):
    opt = torch.optim.Adam(flow.parameters(), lr=lr)
    for _ in range(steps):
        opt.zero_grad()
        loss = -flow.log_prob(data).mean()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(flow.parameters(), max_norm=1.0)
        opt.step()
        if not torch.isfinite(loss) or loss.item() < 0.5:
            break
    return flow


def _oracle_nll_bounds():
    """Per (model, seed) NLL bounds from the ORACLE's own runs of this protocol
    (tests/golden/relational_oracle.jsonl, tools/relational_seeds_oracle.py: the reference
    arithmetic on CPU, fp32 and float64, same seeds, same initial weights and data): the larger of
    the oracle's two values for that seed plus that model's largest fp32-vs-float64 gap over its
    seeds (at least 0.01) — how far the reference's own arithmetic moves the 200-step result."""
    rows = [json.loads(ln) for ln in open(os.path.join(GOLDEN, "relational_oracle.jsonl"))]
    by = {}
    for r in rows:
        by.setdefault((r["kind"], r["seed"]), {})[r["dtype"]] = r["nll"]
    gap = {}
    for (k, _), v in by.items():
        gap[k] = max(gap.get(k, 0.01), abs(v["float32"] - v["float64"]))
    bounds = {key: max(v.values()) + gap[key[0]] for key, v in by.items()}
    f32 = {key: v["float32"] for key, v in by.items()}
    return bounds, f32


@pytest.mark.parametrize("kind", ["realnvp", "maf2", "mixed"])
def test_distribution_preservation_training(cuda_device, kind):
    """tests/correctness/test_distribution_preservation.py: train on N(0, I) samples, then the
    model's samples must have mean ~0 and covariance ~I. 200 Adam steps from a fresh init are
    chaotic for the train-mode BatchNorm models: the reference arithmetic itself (the oracle on
    CPU, tests/golden/relational_oracle.jsonl) ends seed 0 at NLL 3.35 in fp32 and 2.85 in float64,
    seed 7 at 3.63 / 2.92, and reaches ||cov - I|| = 1.04 (seed 2, fp32). The reference's mean /
    covariance thresholds are therefore applied to the median over three seeds; its NLL < 3 to
    its own seed (42, the only one its test runs); every seed's NLL must stay within the oracle's
    own per-seed bound (_oracle_nll_bounds), and their mean within 0.1 of the oracle's fp32 mean over
the same seeds. The GPU values per seed on both train paths are in
    profiles/r06_relational_seeds/ (tools/relational_seeds.py)."""
    bounds, oracle32 = _oracle_nll_bounds()
    nlls = []
    dim, H = 2, 32
    covs, means = [], []
    for seed in (42, 0, 1):
        torch.manual_seed(seed)
        if kind == "realnvp":
            f = nfs_amd.RealNVP(dim, 4, H)
        elif kind == "maf2":
            f = nfs_amd.NormalizingFlowModel([nfs_amd.MaskedAutoregressiveFlow(dim, H) for _ in range(2)])
        else:
            f = nfs_amd.NormalizingFlowModel([nfs_amd.CouplingLayer(dim, H, _mask(dim, "alternating")),
                                              nfs_amd.MaskedAutoregressiveFlow(dim, H),
                                              nfs_amd.CouplingLayer(dim, H, _mask(dim, "half"))])
        f = f.to(cuda_device).train()
        base = torch.distributions.MultivariateNormal(torch.zeros(dim), torch.eye(dim))
        train = base.sample((1000,)).to(cuda_device)
        test = base.sample((500,)).to(cuda_device)
        _train(f, train)
        f.eval()
        with torch.no_grad():
            nll = -f.log_prob(test)
            assert torch.isfinite(nll).all()
            assert nll.mean().item() < bounds[(kind, seed)], (seed, nll.mean().item(), bounds[(kind, seed)])
            if seed == 42:
                assert nll.mean().item() < 3.0, nll.mean().item()  # the reference's own bar
            nlls.append(nll.mean().item())
            xs, _ = f.forward(torch.randn(1000, dim, device=cuda_device))
        means.append(torch.norm(xs.mean(0)).item())
        covs.append(torch.norm(torch.cov(xs.T) - torch.eye(dim, device=cuda_device)).item())
    assert sorted(means)[1] < 0.3, means
    assert sorted(covs)[1] < 0.5, covs
    # and over the three seeds the kernels do no worse than the reference arithmetic in fp32
    ref = sum(oracle32[(kind, sd)] for sd in (42, 0, 1)) / 3
    assert sum(nlls) / 3 <= ref + 0.1, (nlls, ref)
