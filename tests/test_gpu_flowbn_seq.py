"""GPU parity of the between-layer BatchNorm (csrc/nfx_flowbn.hip) and of the SequentialFlow chain
against the reference's own outputs (G12, G13 from tests/golden/make_golden.py).

* NormalizingFlowModel(batch_norm_between_layers=True) (normalizing_flow_model.py:25-128): eval
  both directions + log_prob, the train-mode forward (running statistics updated from the batch
  moments, then the affine with the updated statistics), and gradients through the HIP backward
  of the between-layer affine vs float64 autograd.
* SequentialFlow (sequential_flow.py:15-34): a RealNVP-style chain of CouplingLayers (the
  examples/visualization_demo.py shape) and a mixed coupling/spline/MAF/IAF d=5 chain.
Tolerances: per-sample |dz| <= 1e-5 (1+|ref|) (2e-5 with MADE layers), |dld| <= 1e-4
(d=2) / 2e-4; chains containing RQ splines use the fp32 error model of conftest.assert_fp32_parity
against the float64 oracle, like tests/test_gpu_spline.py.
"""
import numpy as np
import pytest
import torch

import nfs_amd
import oracle
from conftest import assert_fp32_parity, fp32_jitter, load_golden, oracle_sd, state_dict_from

pytestmark = pytest.mark.gpu


def rel_close(a, ref, tol):
    a, ref = np.asarray(a, np.float64), np.asarray(ref, np.float64)
    err = np.abs(a - ref) / (1 + np.abs(ref))
    assert err.max() <= tol, f"max rel err {err.max():.3g} at {np.unravel_index(err.argmax(), err.shape)}"


def abs_close(a, ref, tol):
    d = np.abs(np.asarray(a, np.float64) - np.asarray(ref, np.float64))
    assert d.max() <= tol, f"max abs err {d.max():.3g} at {d.argmax()}"


def g12_model(name):
    if name == "rn":
        return nfs_amd.RealNVP(2, 8, 64, batch_norm_between_layers=True)
    if name == "rs":
        return nfs_amd.RealNVPSpline(2, 8, 64, batch_norm_between_layers=True)
    return nfs_amd.NormalizingFlowModel([nfs_amd.MaskedAutoregressiveFlow(10, 16) for _ in range(3)],
                                        batch_norm_between_layers=True)


G12_SPEC = {
    "rn": (lambda tr: oracle.realnvp_spec(8, training=tr), "flow.batch_norms."),
    "rs": (lambda tr: oracle.spline_model_spec(8), "flow.batch_norms."),
    "maf": (lambda tr: oracle.maf_spec(3), "batch_norms."),
}


def load_g12(name, dev):
    g = load_golden("g12_flowbn.npz")
    m = g12_model(name)
    sd = {k: v for k, v in state_dict_from(g, name + ".", m).items()}
    m.load_state_dict(sd)
    return m.to(dev).eval(), g


def sd64(sd):
    return {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in sd.items()}


@pytest.mark.parametrize("name", ["rn", "rs", "maf"])
def test_between_layer_bn_eval_vs_reference(cuda_device, name):
    m, g = load_g12(name, cuda_device)
    x = torch.from_numpy(g[f"{name}.x"]).to(cuda_device)
    z = torch.from_numpy(g[f"{name}.z"]).to(cuda_device)
    nfs_amd.reset_stats()
    with torch.no_grad():
        zi, ldi = m.inverse(x)
        xf, ldf = m.forward(z)
        lp = (m.flow if hasattr(m, "flow") else m).log_prob(x)
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] > 0, nfs_amd.STATS
    ref = {k: g[f"{name}.{k}"] for k in ("inv_z", "inv_ld", "fwd_x", "fwd_ld", "log_prob")}
    if name == "rs":
        spec_fn, bnp = G12_SPEC[name]
        sd = sd64(oracle_sd(g, name + "."))
        with torch.no_grad():
            z64, l64 = oracle.flow_model(sd, spec_fn(False), x.cpu().double(), -1, bn_prefix=bnp)
            x64, lf64 = oracle.flow_model(sd, spec_fn(False), z.cpu().double(), 1, bn_prefix=bnp)
        sd32 = {k: v for k, v in oracle_sd(g, name + ".").items() if not k.startswith("after_train.")}
        si = fp32_jitter(lambda s, v: oracle.flow_model(s, spec_fn(False), v, -1, bn_prefix=bnp), x.cpu(), sd=sd32)
        sf = fp32_jitter(lambda s, v: oracle.flow_model(s, spec_fn(False), v, 1, bn_prefix=bnp), z.cpu(), sd=sd32)
        assert_fp32_parity(zi.cpu(), ref["inv_z"], z64, what="inv z", sens=si[0], rows=x.cpu())
        assert_fp32_parity(ldi.cpu(), ref["inv_ld"], l64, what="inv ld", sens=si[1], rows=x.cpu())
        assert_fp32_parity(xf.cpu(), ref["fwd_x"], x64, what="fwd x", sens=sf[0])
        assert_fp32_parity(ldf.cpu(), ref["fwd_ld"], lf64, what="fwd ld", sens=sf[1])
        nll_ref = -float(torch.from_numpy(ref["log_prob"][:2000]).double().mean())  # 24 edge rows at the end
        assert abs(-float(lp[:2000].double().mean()) - nll_ref) <= 1e-5
        return
    ytol, ltol = (1e-5, 1e-4) if name == "rn" else (2e-5, 2e-4)
    rel_close(zi.cpu(), ref["inv_z"], ytol)
    abs_close(ldi.cpu(), ref["inv_ld"], ltol)
    rel_close(xf.cpu(), ref["fwd_x"], ytol)
    abs_close(ldf.cpu(), ref["fwd_ld"], ltol)
    # log p = -0.5|z|^2 + ...: ~1e20 for the 1e10 edge rows, so the bound is relative there
    lpd = np.abs(lp.cpu().numpy().astype(np.float64) - ref["log_prob"].astype(np.float64))
    assert (lpd <= ltol + 2e-5 * np.abs(ref["log_prob"])).all(), lpd.max()
    n_reg = 2000 if name == "rn" else lp.shape[0]  # rn: 24 edge rows (|x| up to 1e10) at the end
    nll_ref = -float(torch.from_numpy(ref["log_prob"][:n_reg]).double().mean())
    assert abs(-float(lp[:n_reg].double().mean()) - nll_ref) <= 1e-5


@pytest.mark.parametrize("name", ["rn", "rs", "maf"])
def test_between_layer_bn_train_forward_updates_running_stats(cuda_device, name):
    """Train mode (normalizing_flow_model.py:74-79): every between-layer BatchNorm folds the batch
    moments of its input into the running statistics, then applies the affine with them."""
    m, g = load_g12(name, cuda_device)
    m.train()
    z = torch.from_numpy(g[f"{name}.z"]).to(cuda_device)
    nfs_amd.reset_stats()
    with torch.no_grad():
        xt, ldt = m.forward(z)
    assert nfs_amd.STATS["torch"] == 0, nfs_amd.STATS
    after = state_dict_from(g, f"{name}.after_train.", g12_model(name))
    for k, v in m.state_dict().items():
        if "batch_norms" in k and ("running_mean" in k or "running_var" in k):
            rel_close(v.cpu(), after[k], 1e-6 if name != "rn" else 1e-5)
    if name in ("rs", "rn"):  # 8-layer chains: spline conditioning / train-mode batch statistics
        spec_fn, bnp = G12_SPEC[name]
        sd = sd64(oracle_sd(g, name + "."))
        sd = {k: v for k, v in sd.items() if not k.startswith("after_train.")}
        with torch.no_grad():
            x64, l64 = oracle.flow_model(sd, spec_fn(True), z.cpu().double(), 1, bn_prefix=bnp, training=True)
        sd32 = {k: v for k, v in oracle_sd(g, name + ".").items() if not k.startswith("after_train.")}

        def fwd_train(s, v):  # a fresh copy per call: train mode updates the running stats in place
            s2 = {k: t.clone() for k, t in s.items()}
            return oracle.flow_model(s2, spec_fn(True), v, 1, bn_prefix=bnp, training=True)

        st = fp32_jitter(fwd_train, z.cpu(), sd=sd32)
        assert_fp32_parity(xt.cpu(), g[f"{name}.train_fwd_x"], x64, what="train fwd x", sens=st[0])
        assert_fp32_parity(ldt.cpu(), g[f"{name}.train_fwd_ld"], l64, what="train fwd ld", sens=st[1])
        return
    ytol, ltol = (2e-5, 2e-4)
    rel_close(xt.cpu(), g[f"{name}.train_fwd_x"], ytol)
    abs_close(ldt.cpu(), g[f"{name}.train_fwd_ld"], ltol)


@pytest.mark.parametrize("name,direction", [("maf", -1), ("maf", 1), ("rs", -1), ("rs", 1)])
def test_between_layer_bn_gradients_vs_float64(cuda_device, name, direction):
    """Autograd through the HIP between-layer affine (nfx_flowbn_backward) and the layers' fused
    backward kernels vs float64 autograd of the same module on the CPU composite path."""
    m, g = load_g12(name, cuda_device)
    x = torch.from_numpy(g[f"{name}.x" if direction < 0 else f"{name}.z"])[:500]
    w = torch.randn(x.shape, generator=torch.Generator().manual_seed(3))
    m64 = g12_model(name).double()
    m64.load_state_dict({k: (v.double() if v.is_floating_point() else v) for k, v in m.state_dict().items()})
    m64.eval()

    def run(model, xx, ww):
        xx = xx.clone().requires_grad_(True)
        y, ld = model.inverse(xx) if direction < 0 else model.forward(xx)
        loss = (y * ww).sum() + ld.sum()
        loss.backward()
        return xx.grad, {k: p.grad for k, p in model.named_parameters()}

    nfs_amd.reset_stats()
    gx, gp = run(m, x.to(cuda_device), w.to(cuda_device))
    stats = dict(nfs_amd.STATS)
    gx64, gp64 = run(m64, x.double(), w.double())
    # every layer backward is a fused kernel (HipFlowFunction counts a composite recompute as
    # a torch call), incl. the sequential MAF sampling direction (made_seq_bwd_kernel)
    assert stats["torch"] == 0, stats
    scale = float(gx64.abs().max())
    rel = float((gx.cpu().double() - gx64).abs().max()) / max(scale, 1e-12)
    assert rel <= (2e-4 if name == "rs" else 2e-5), f"dL/dx rel err {rel:.3g}"
    for k in gp64:
        if "batch_norms" not in k or gp64[k] is None:  # the last BatchNorm is never applied
            assert gp64[k] is None or gp[k] is not None, k
            continue
        a, b = gp[k].cpu().double(), gp64[k]
        err = float((a - b).abs().max()) / max(float(b.abs().max()), 1e-12)
        assert err <= (2e-4 if name == "rs" else 2e-5), f"{k}: rel err {err:.3g}"


G13_SPECS = {
    "s2": [("coupling", f"flows.{i}.", {}) for i in range(4)],
    "s5": [("coupling", "flows.0.", {}), ("spline", "flows.1.", {"K": 8}), ("maf", "flows.2.", {}),
           ("iaf", "flows.3.", {})],
}


def g13_model(name):
    def alt(dim, even):
        mask = torch.zeros(dim)
        mask[(0 if even else 1)::2] = 1
        return mask

    if name == "s2":
        return nfs_amd.SequentialFlow([nfs_amd.CouplingLayer(2, 32, alt(2, i % 2 == 0)) for i in range(4)])
    return nfs_amd.SequentialFlow([nfs_amd.CouplingLayer(5, 32, alt(5, True)),
                                   nfs_amd.SplineCouplingLayer(5, 32, alt(5, False), num_bins=8),
                                   nfs_amd.MaskedAutoregressiveFlow(5, 16),
                                   nfs_amd.InverseAutoregressiveFlow(5, 16)])


@pytest.mark.parametrize("name", ["s2", "s5"])
def test_sequential_flow_vs_reference(cuda_device, name):
    g = load_golden("g13_sequential.npz")
    m = g13_model(name)
    m.load_state_dict(state_dict_from(g, name + ".", m))
    m = m.to(cuda_device).eval()
    x = torch.from_numpy(g[f"{name}.x"]).to(cuda_device)
    z = torch.from_numpy(g[f"{name}.z"]).to(cuda_device)
    nfs_amd.reset_stats()
    with torch.no_grad():
        zi, ldi = m.inverse(x)
        xf, ldf = m.forward(z)
    # s2 (4 CouplingLayers) runs as one nfx_affine_chain launch per direction; s5 layer by layer
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] == (2 if name == "s2" else 8), nfs_amd.STATS
    if name == "s2":
        rel_close(zi.cpu(), g[f"{name}.inv_z"], 1e-5)
        abs_close(ldi.cpu(), g[f"{name}.inv_ld"], 1e-4)
        rel_close(xf.cpu(), g[f"{name}.fwd_x"], 1e-5)
        abs_close(ldf.cpu(), g[f"{name}.fwd_ld"], 1e-4)
    else:
        sd = sd64(oracle_sd(g, name + "."))
        with torch.no_grad():
            z64, l64 = oracle.sequential_flow(sd, G13_SPECS[name], x.cpu().double(), -1)
            x64, lf64 = oracle.sequential_flow(sd, G13_SPECS[name], z.cpu().double(), 1)
        sd32 = oracle_sd(g, name + ".")
        si = fp32_jitter(lambda s, v: oracle.sequential_flow(s, G13_SPECS[name], v, -1), x.cpu(), sd=sd32)
        sf = fp32_jitter(lambda s, v: oracle.sequential_flow(s, G13_SPECS[name], v, 1), z.cpu(), sd=sd32)
        assert_fp32_parity(zi.cpu(), g[f"{name}.inv_z"], z64, what="inv z", sens=si[0], rows=x.cpu())
        assert_fp32_parity(ldi.cpu(), g[f"{name}.inv_ld"], l64, what="inv ld", sens=si[1], rows=x.cpu())
        assert_fp32_parity(xf.cpu(), g[f"{name}.fwd_x"], x64, what="fwd x", sens=sf[0])
        assert_fp32_parity(ldf.cpu(), g[f"{name}.fwd_ld"], lf64, what="fwd ld", sens=sf[1])
    # the in-place chain equals the reference's per-layer composition bit for bit (the one-launch
    # coupling chain computes each layer as the per-layer small-batch kernel does)
    from nfs_amd import _lib
    old = _lib.lib().nfx_affine_kernel_policy(_lib.NFX_AFFINE_SMALL)
    try:
        with torch.no_grad():
            cur, tot = x, torch.zeros(x.shape[0], device=cuda_device)
            for f in reversed(m.flows):
                cur, ld = f.inverse(cur)
                tot += ld
    finally:
        _lib.lib().nfx_affine_kernel_policy(old)
    assert torch.equal(cur, zi) and torch.equal(tot, ldi)


def test_sequential_flow_gradients(cuda_device):
    """Gradients through a SequentialFlow on the GPU (per-layer HIP forward + fused backward)."""
    g = load_golden("g13_sequential.npz")
    m = g13_model("s2")
    m.load_state_dict(state_dict_from(g, "s2.", m))
    m64 = g13_model("s2").double()
    m64.load_state_dict({k: (v.double() if v.is_floating_point() else v) for k, v in m.state_dict().items()})
    m, m64 = m.to(cuda_device).eval(), m64.eval()
    x = torch.from_numpy(g["s2.x"])[:300]
    xg = x.to(cuda_device).requires_grad_(True)
    y, ld = m.inverse(xg)
    (y.pow(2).sum() - ld.sum()).backward()
    x64 = x.double().requires_grad_(True)
    y64, ld64 = m64.inverse(x64)
    (y64.pow(2).sum() - ld64.sum()).backward()
    rel = float((xg.grad.cpu().double() - x64.grad).abs().max()) / float(x64.grad.abs().max())
    assert rel <= 2e-5, rel
