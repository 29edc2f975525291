"""Pin the oracle (oracle/flows_ref.py) against golden vectors produced by the reference itself
(tests/golden/make_golden.py). The oracle restates the reference op for op on the same ATen CPU
kernels, so agreement is (near-)bitwise; tolerances below allow a few ulp."""
import numpy as np
import pytest
import torch

import oracle
from conftest import load_golden, oracle_sd

T = dict(rtol=1e-6, atol=1e-6)


def close(a, b, **kw):
    kw = kw or T
    np.testing.assert_allclose(np.asarray(a), np.asarray(b), **kw)


@pytest.mark.parametrize("dH", [(1, 8), (2, 64), (3, 16), (3, 32), (4, 16), (5, 16), (10, 16),
                                (63, 64), (154, 64), (784, 64)])
def test_made_masks_bit_exact(dH):
    d, H = dH
    g = load_golden("g1_made_masks.npz")
    assert oracle.made_degrees(d, H) == g[f"d{d}_h{H}_deg"].tolist()
    m1, mhh, m2 = oracle.made_masks(d, H)
    assert np.array_equal(m1.numpy(), g[f"d{d}_h{H}_m1"])
    assert np.array_equal(mhh.numpy(), g[f"d{d}_h{H}_mhh"])
    assert np.array_equal(m2.numpy(), g[f"d{d}_h{H}_m2"])


def test_made_degrees_linspace_sweep():
    """The float64 restatement equals numpy.linspace flooring over a wide (d, H) sweep, where
    the integer form i*(d-1)//(H-1) is known to fail."""
    for d in range(3, 800, 7):
        for H in (8, 16, 32, 48, 64, 100, 128, 256):
            ref = np.floor(np.linspace(0, d - 1, H)).astype(int).tolist()
            assert oracle.made_degrees(d, H) == ref, (d, H)


def test_realnvp_g2():
    g = load_golden("g2_realnvp.npz")
    sd = oracle_sd(g)
    x, z = torch.from_numpy(g["x"]), torch.from_numpy(g["z"])
    spec = oracle.realnvp_spec(8)
    with torch.no_grad():
        zi, ldi = oracle.flow_model(sd, spec, x, -1)
        xf, ldf = oracle.flow_model(sd, spec, z, 1)
        lp = oracle.gauss_log_prob(zi, ldi)
    close(zi, g["inv_z"])
    close(ldi, g["inv_ld"])
    close(xf, g["fwd_x"])
    close(ldf, g["fwd_ld"])
    close(lp, g["log_prob"])
    assert abs(oracle.nll_f64(lp) - float(g["nll_f64"])) < 1e-9
    y0, l0 = oracle.coupling(sd, "flow.flows.0.", x, -1)
    close(y0, g["l0_inv_z"])
    close(l0, g["l0_inv_ld"])


@pytest.mark.parametrize("tag,K", [("k8.", 8), ("k10.", 10)])
def test_spline_g3(tag, K):
    g = load_golden("g3_spline.npz")
    sd = oracle_sd(g, tag)
    x, z = torch.from_numpy(g["x"]), torch.from_numpy(g["z"])
    spec = [("spline", f"{'flow.' if K == 10 else ''}flows.{i}.", {"K": K}) for i in range(8)]
    with torch.no_grad():
        zi, ldi = oracle.flow_model(sd, spec, x, -1)
        xf, ldf = oracle.flow_model(sd, spec, z, 1)
    close(zi, g[tag + "inv_z"])
    close(ldi, g[tag + "inv_ld"], rtol=1e-6, atol=2e-6)
    close(xf, g[tag + "fwd_x"])
    close(ldf, g[tag + "fwd_ld"], rtol=1e-6, atol=2e-6)


def test_rqs_unit_g4():
    g = load_golden("g4_rqs_unit.npz")
    x, uw, uh, ud = (torch.from_numpy(g[k]) for k in ("x", "uw", "uh", "ud"))
    yf, lf = oracle.rqs_unit(x, uw, uh, ud, inverse=False)
    yi, li = oracle.rqs_unit(x, uw, uh, ud, inverse=True)
    close(yf, g["fwd_y"])
    close(lf, g["fwd_ld"])
    np.testing.assert_array_equal(np.isnan(yi.numpy()), np.isnan(g["inv_y"]))
    close(np.nan_to_num(yi.numpy()), np.nan_to_num(g["inv_y"]))
    close(np.nan_to_num(li.numpy()), np.nan_to_num(g["inv_ld"]))


def test_maf63_g5():
    g = load_golden("g5_maf63.npz")
    sd = oracle_sd(g)
    x, z = torch.from_numpy(g["x"]), torch.from_numpy(g["z"])
    spec = oracle.maf_spec(5)
    with torch.no_grad():
        zi, ldi = oracle.flow_model(sd, spec, x, -1)
        xf, ldf = oracle.flow_model(sd, spec, z, 1)
    close(zi, g["inv_z"], rtol=1e-5, atol=1e-5)
    close(ldi, g["inv_ld"], rtol=1e-5, atol=1e-4)
    close(xf, g["fwd_x"], rtol=1e-5, atol=1e-5)
    close(ldf, g["fwd_ld"], rtol=1e-5, atol=1e-4)


def test_iaf784_g6():
    g = load_golden("g6_iaf784.npz")
    sd = oracle_sd(g)
    z, x = torch.from_numpy(g["z"]), torch.from_numpy(g["x"])
    with torch.no_grad():
        xf, ldf = oracle.iaf(sd, "", z, 1)
        zi, ldi = oracle.iaf(sd, "", x, -1)
    close(xf, g["fwd_x"], rtol=1e-5, atol=1e-5)
    close(ldf, g["fwd_ld"], rtol=1e-5, atol=1e-4)
    close(zi, g["inv_z"], rtol=1e-5, atol=1e-5)
    close(ldi, g["inv_ld"], rtol=1e-5, atol=1e-4)


def test_moons_g7():
    g = load_golden("g7_moons.npz")
    sd = oracle_sd(g)
    x = torch.from_numpy(g["x"])
    with torch.no_grad():
        zi, ldi = oracle.flow_model(sd, oracle.realnvp_spec(8), x, -1)
        lp = oracle.gauss_log_prob(zi, ldi)
    close(lp, g["log_prob"], rtol=1e-5, atol=1e-5)
    assert abs(oracle.nll_f64(lp) - float(g["nll_f64"])) < 1e-6
    assert g["train_curve"][-1] < g["train_curve"][0]


SMALL = [("cpl_alt", "coupling"), ("cpl_half", "coupling"), ("cpl_d3", "coupling"),
         ("cpl_d1", "coupling"), ("spl_alt", "spline"), ("spl_half", "spline"),
         ("spl_d3", "spline"), ("maf4", "maf"), ("iaf4", "iaf"), ("maf10", "maf"),
         ("iaf10", "iaf"), ("maf2", "maf"), ("iaf3", "iaf")]


@pytest.mark.parametrize("name,kind", SMALL)
def test_small_layers_g9(name, kind):
    g = load_golden("g9_small.npz")
    sd = oracle_sd(g, name + ".")
    x = torch.from_numpy(g[name + ".x"])
    fn = {"coupling": oracle.coupling, "spline": oracle.spline_coupling, "maf": oracle.maf, "iaf": oracle.iaf}[kind]
    with torch.no_grad():
        yf, lf = fn(sd, "", x, 1)
        yi, li = fn(sd, "", x, -1)
    close(yf, g[name + ".fwd_y"], rtol=1e-5, atol=1e-5)
    close(lf, g[name + ".fwd_ld"], rtol=1e-5, atol=1e-5)
    close(yi, g[name + ".inv_y"], rtol=1e-5, atol=1e-5)
    close(li, g[name + ".inv_ld"], rtol=1e-5, atol=1e-5)


ARQS_CASES = ["a1", "a3", "a5", "a4bn", "a10"]


def arqs_case(g, name):
    d, H, K, bn, lo, hi = g[name + ".meta"]
    rng = {} if np.isnan(lo) else {"data_min": float(lo), "data_max": float(hi)}
    return int(d), int(H), int(K), bool(bn), rng


@pytest.mark.parametrize("name", ARQS_CASES)
def test_arqs_g10(name):
    """ARQS (arqs.py:44-114): the oracle's sequential restatement vs the reference."""
    g = load_golden("g10_arqs.npz")
    d, H, K, bn, rng = arqs_case(g, name)
    sd = oracle_sd(g, name + ".")
    x = torch.from_numpy(g[name + ".x"])
    for direction, key in ((1, "fwd"), (-1, "inv")):
        with torch.no_grad():
            y, ld = oracle.arqs(sd, "", x, direction, K=K, batch_norm=bn, **rng)
        close(y, g[f"{name}.{key}_y"], rtol=1e-5, atol=1e-6)
        close(ld, g[f"{name}.{key}_ld"], rtol=1e-5, atol=1e-5)


def test_train_mode_g11():
    """Train-mode BatchNorm (batch statistics + running-statistics update) and the NLL gradients
    of RealNVP(2,8,64) through the oracle vs the reference (G11), and a d=4 layer both ways."""
    g = load_golden("g11_train.npz")
    sd = oracle_sd(g, "rn.init.")
    for k, v in sd.items():
        if v.is_floating_point() and not k.endswith(("running_mean", "running_var", "mask")):
            v.requires_grad_(True)
    x = torch.from_numpy(g["rn.x"])
    z, ld = oracle.flow_model(sd, oracle.realnvp_spec(8, training=True), x, -1)
    loss = -oracle.gauss_log_prob(z, ld).mean()
    loss.backward()
    close(z.detach(), g["rn.z"], rtol=1e-5, atol=1e-5)
    close(ld.detach(), g["rn.ld"], rtol=1e-5, atol=1e-5)
    assert abs(loss.item() - float(g["rn.loss"])) < 1e-5
    for k, v in sd.items():
        if v.requires_grad:
            ref = g["rn.grad." + k]
            close(v.grad, ref, rtol=1e-4, atol=1e-4 * max(1.0, float(np.abs(ref).max())))
        elif k.endswith(("running_mean", "running_var")):
            close(v, g["rn.after." + k], rtol=1e-6, atol=1e-7)
    sd4 = oracle_sd(g, "c4.init.")
    for name, direction in (("inv", -1), ("fwd", 1)):
        params = {k: v.clone().requires_grad_(True) if v.is_floating_point() and not k.endswith(
            ("running_mean", "running_var", "mask")) else v for k, v in sd4.items()}
        xr = torch.from_numpy(g["c4.x"]).clone().requires_grad_(True)
        y, l4 = oracle.coupling(params, "", xr, direction, training=True)
        ((y * torch.from_numpy(g["c4.wy"])).sum() + (l4 * torch.from_numpy(g["c4.wl"])).sum()).backward()
        close(y.detach(), g[f"c4.{name}.y"], rtol=1e-5, atol=1e-5)
        close(l4.detach(), g[f"c4.{name}.ld"], rtol=1e-5, atol=1e-5)
        close(xr.grad, g[f"c4.{name}.gx"], rtol=1e-4, atol=1e-4)
        sd4 = params  # running statistics carry over to the second call, as in the reference
    for k in sd4:
        if k.endswith(("running_mean", "running_var")):
            close(sd4[k], g["c4.after." + k], rtol=1e-6, atol=1e-7)


G12_CASES = {
    "rn": (lambda tr: oracle.realnvp_spec(8, training=tr), "flow.batch_norms."),
    "rs": (lambda tr: oracle.spline_model_spec(8), "flow.batch_norms."),
    "maf": (lambda tr: oracle.maf_spec(3), "batch_norms."),
}


@pytest.mark.parametrize("name", sorted(G12_CASES))
def test_between_layer_batchnorm_g12(name):
    """NormalizingFlowModel(batch_norm_between_layers=True) (normalizing_flow_model.py:25-128):
    eval both directions + log_prob, and the train-mode forward's running-stat update."""
    g = load_golden("g12_flowbn.npz")
    sd = oracle_sd(g, name + ".")
    sd = {k: v for k, v in sd.items() if not k.startswith("after_train.")}
    spec_fn, bnp = G12_CASES[name]
    x, z = torch.from_numpy(g[f"{name}.x"]), torch.from_numpy(g[f"{name}.z"])
    with torch.no_grad():
        zi, ldi = oracle.flow_model(sd, spec_fn(False), x, -1, bn_prefix=bnp)
        xf, ldf = oracle.flow_model(sd, spec_fn(False), z, 1, bn_prefix=bnp)
        lp = oracle.gauss_log_prob(zi, ldi)
    tol = dict(rtol=1e-6, atol=2e-6)
    close(zi, g[f"{name}.inv_z"], **tol)
    close(ldi, g[f"{name}.inv_ld"], **tol)
    close(xf, g[f"{name}.fwd_x"], **tol)
    close(ldf, g[f"{name}.fwd_ld"], **tol)
    close(lp, g[f"{name}.log_prob"], **tol)
    sdt = {k: v.clone() for k, v in sd.items()}
    with torch.no_grad():
        xt, ldt = oracle.flow_model(sdt, spec_fn(True), z, 1, bn_prefix=bnp, training=True)
    close(xt, g[f"{name}.train_fwd_x"], **tol)
    close(ldt, g[f"{name}.train_fwd_ld"], **tol)
    after = oracle_sd(g, f"{name}.after_train.")
    for k, v in after.items():
        close(sdt[k], v, **tol)


G13_SPECS = {
    "s2": [("coupling", f"flows.{i}.", {}) for i in range(4)],
    "s5": [("coupling", "flows.0.", {}), ("spline", "flows.1.", {"K": 8}), ("maf", "flows.2.", {}),
           ("iaf", "flows.3.", {})],
}


@pytest.mark.parametrize("name", sorted(G13_SPECS))
def test_sequential_flow_g13(name):
    """SequentialFlow (sequential_flow.py:15-34): zeros(B) accumulator."""
    g = load_golden("g13_sequential.npz")
    sd = oracle_sd(g, name + ".")
    x, z = torch.from_numpy(g[f"{name}.x"]), torch.from_numpy(g[f"{name}.z"])
    with torch.no_grad():
        zi, ldi = oracle.sequential_flow(sd, G13_SPECS[name], x, -1)
        xf, ldf = oracle.sequential_flow(sd, G13_SPECS[name], z, 1)
    tol = dict(rtol=1e-6, atol=2e-6)
    close(zi, g[f"{name}.inv_z"], **tol)
    close(ldi, g[f"{name}.inv_ld"], **tol)
    close(xf, g[f"{name}.fwd_x"], **tol)
    close(ldf, g[f"{name}.fwd_ld"], **tol)


G14_CASES = {"maf10": ("maf", {}), "iaf10": ("iaf", {}), "maf63": ("maf", {}), "iaf784": ("iaf", {}),
             "sp8": ("spline", {"K": 8}), "sp10": ("spline", {"K": 10})}


@pytest.mark.parametrize("name", list(G14_CASES))
@pytest.mark.parametrize("dname", ["inv", "fwd"])
def test_gradients_g14(name, dname):
    """The oracle under autograd reproduces the reference's own gradients (G14: dL/dx and every
    parameter gradient of sum(y*wy) + sum(ld*wl), masked_autoregressive_flow.py:18-78,
    inverse_autoregressive_flow.py:30-103, spline_coupling_layer.py:96-309)."""
    g = load_golden("g14_grads.npz")
    kind, kw = G14_CASES[name]
    sd = oracle_sd(g, name + ".init.")
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items() if not k.endswith("mask")}
    sd.update(params)
    x = torch.from_numpy(g[f"{name}.x"]).clone().requires_grad_(True)
    fn = {"maf": oracle.maf, "iaf": oracle.iaf, "spline": oracle.spline_coupling}[kind]
    y, ld = fn(sd, "", x, -1 if dname == "inv" else 1, **kw)
    ((y * torch.from_numpy(g[f"{name}.wy"])).sum() + (ld * torch.from_numpy(g[f"{name}.wl"])).sum()).backward()
    close(y.detach(), g[f"{name}.{dname}.y"], rtol=1e-6, atol=1e-6)
    close(ld.detach(), g[f"{name}.{dname}.ld"], rtol=1e-6, atol=1e-5)
    ref_gx = g[f"{name}.{dname}.gx"]
    assert np.abs(x.grad.numpy() - ref_gx).max() <= 1e-5 * (1 + np.abs(ref_gx).max())
    n = 0
    for k, p in params.items():
        ref = g[f"{name}.{dname}.grad.{k}"]
        assert np.abs(p.grad.numpy() - ref).max() <= 1e-5 * (1 + np.abs(ref).max()), k
        n += 1
    assert n >= 6


@pytest.mark.parametrize("name", ["spline", "maf", "iaf"])
def test_figure_models_g16(name):
    """The oracle's training step of the reference's other benchmark-figure models
    (plots/_common.py:157-169, 194-211) reproduces the reference's own z, log-det, loss and raw
    gradients (G16) in float32 on 2,000 two-moons points."""
    g = load_golden("g16_fig_models.npz")
    spec = oracle.spline_model_spec(8) if name == "spline" else [(name, f"flows.{i}.", {}) for i in range(6)]
    sd = oracle_sd(g, name + ".init.")
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items() if not k.endswith("mask")}
    sd.update(params)
    x = torch.from_numpy(g["x"])
    z, ld = oracle.flow_model(sd, spec, x, -1)
    loss = -oracle.gauss_log_prob(z, ld).mean()
    loss.backward()
    close(z.detach(), g[name + ".z"], rtol=2e-5, atol=2e-5)
    close(ld.detach(), g[name + ".ld"], rtol=2e-5, atol=2e-5)
    assert abs(loss.item() - float(g[name + ".loss"])) <= 1e-5
    n = 0
    for k, p in params.items():
        ref = g[name + ".grad." + k]
        assert np.abs(p.grad.numpy() - ref).max() <= 1e-4 * (1 + np.abs(ref).max()), k
        n += 1
    assert n == 48


def _g17_layer_spec(name):
    if name == "mafbn":
        return "maf", {"batch_norm": True, "training": True}
    if name == "arqsbn":
        return "arqs", {"K": 5, "batch_norm": True, "training": True}
    return "spline", {"K": 6}


@pytest.mark.parametrize("case", ["iafbn", "mafbn.fwd", "arqsbn.fwd", "arqsbn.inv", "spldm.fwd", "spldm.inv"])
def test_options_g17(case):
    """G17 (the reference's remaining constructor options under autograd): the oracle reproduces
    the reference's outputs, gradients and running statistics — train-mode use_batch_norm=True in
    the sequential MADE directions (d calls, each with its own batch statistics), ARQS with a
    train-mode BatchNorm MADE, and per-dimension data_min/data_max spline bounds."""
    g = load_golden("g17_options.npz")
    if case == "iafbn":
        sd = oracle_sd(g, "iafbn.init.")
        params = {k: v.clone().requires_grad_(True) for k, v in sd.items()
                  if not k.endswith(("mask", "running_mean", "running_var"))}
        sd.update(params)
        spec = [("iaf", f"flows.{i}.", {"batch_norm": True, "training": True}) for i in range(2)]
        x = torch.from_numpy(g["iafbn.x"])
        z, ld = oracle.flow_model(sd, spec, x, -1)
        loss = -oracle.gauss_log_prob(z, ld).mean()
        loss.backward()
        close(z.detach(), g["iafbn.z"], rtol=2e-5, atol=2e-5)
        close(ld.detach(), g["iafbn.ld"], rtol=2e-5, atol=2e-5)
        assert abs(loss.item() - float(g["iafbn.loss"])) <= 1e-5
        grads = {k: p.grad for k, p in params.items()}
        gpre, after = "iafbn.grad.", "iafbn.after."
    else:
        name, dname = case.split(".")
        kind, kw = _g17_layer_spec(name)
        sd = oracle_sd(g, name + ".init.")
        params = {k: v.clone().requires_grad_(True) for k, v in sd.items()
                  if not k.endswith(("mask", "running_mean", "running_var"))}
        sd.update(params)
        if name == "spldm":
            kw = dict(kw, data_min=torch.from_numpy(g["spldm.data_min"]), data_max=torch.from_numpy(g["spldm.data_max"]))
        x = torch.from_numpy(g[name + ".x"]).clone().requires_grad_(True)
        y, ld = getattr(oracle, {"maf": "maf", "arqs": "arqs", "spline": "spline_coupling"}[kind])(
            sd, "", x, 1 if dname == "fwd" else -1, **kw)
        ((y * torch.from_numpy(g[name + ".wy"])).sum() + (ld * torch.from_numpy(g[name + ".wl"])).sum()).backward()
        close(y.detach(), g[f"{case}.y"], rtol=2e-5, atol=2e-5)
        close(ld.detach(), g[f"{case}.ld"], rtol=2e-5, atol=2e-5)
        ref = g[f"{case}.gx"]
        assert np.abs(x.grad.numpy() - ref).max() <= 1e-4 * (1 + np.abs(ref).max())
        grads = {k: p.grad for k, p in params.items()}
        gpre, after = f"{case}.grad.", f"{case}.after."
    n = 0
    for k, gr in grads.items():
        ref = g[gpre + k]
        assert gr is not None, k
        assert np.abs(gr.numpy() - ref).max() <= 1e-4 * (1 + np.abs(ref).max()), k
        n += 1
    assert n > 0
    for k in g:  # running statistics after the step(s): updated once per MADE call
        if k.startswith(after):
            close(sd[k[len(after):]], g[k], rtol=1e-5, atol=1e-6)


def test_relational_oracle_fixture_reproduces():
    """tests/golden/relational_oracle.jsonl (the per-seed bounds of
    test_gpu_relational.py::test_distribution_preservation_training) is the oracle's own output:
    re-run the cheapest entry (maf2, seed 42, fp32: 200 Adam steps through oracle/flows_ref.py)."""
    import json
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tools"))
    import relational_seeds_oracle as rso
    rows = [json.loads(ln) for ln in open(os.path.join(root, "tests", "golden", "relational_oracle.jsonl"))]
    want = next(r for r in rows if r["kind"] == "maf2" and r["seed"] == 42 and r["dtype"] == "float32")
    got = rso.run(42, torch.float32, "maf2")
    assert got["steps"] == want["steps"] and abs(got["nll"] - want["nll"]) <= 2e-4, (got, want)
