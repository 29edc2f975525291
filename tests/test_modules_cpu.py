"""Host-side checks of the drop-in modules (no GPU): state_dict keys, constructor semantics and
the composite (CPU / fp64 / autograd) path against the reference's golden outputs."""
import numpy as np
import pytest
import torch

import nfs_amd
from conftest import load_golden, oracle_sd, state_dict_from


def test_realnvp_state_dict_keys_match_reference():
    g = load_golden("g2_realnvp.npz")
    m = nfs_amd.RealNVP(2, 8, 64)
    keys = {k for k, v in m.state_dict().items() if v.dtype != torch.int64}
    assert keys == set(k for k in g if k.startswith("flow."))


def test_spline_and_maf_state_dict_keys():
    g = load_golden("g3_spline.npz")
    m = nfs_amd.RealNVPSpline(2, 8, 64)
    assert {"k10." + k for k in m.state_dict()} == {k for k in g if k.startswith("k10.flow.")}
    g5 = load_golden("g5_maf63.npz")
    m5 = nfs_amd.NormalizingFlowModel([nfs_amd.MaskedAutoregressiveFlow(63, 64) for _ in range(5)])
    assert set(m5.state_dict()) == {k for k in g5 if k.startswith("flows.")}


def test_odd_layers_rejected():
    with pytest.raises(AssertionError):
        nfs_amd.RealNVP(2, 3, 8)
    with pytest.raises(AssertionError):
        nfs_amd.RealNVPSpline(2, 5, 8)


@pytest.mark.parametrize("dH", [(1, 8), (2, 64), (3, 16), (4, 16), (10, 16), (63, 64), (154, 64), (784, 64)])
def test_product_made_masks_match_reference(dH):
    d, H = dH
    g = load_golden("g1_made_masks.npz")
    made = nfs_amd.MADE(d, H)
    assert made.m[0].tolist() == g[f"d{d}_h{H}_deg"].tolist()
    assert np.array_equal(made.masks[0].numpy().astype(np.uint8), g[f"d{d}_h{H}_m1"])
    assert np.array_equal(made.masks[1].numpy().astype(np.uint8), g[f"d{d}_h{H}_mhh"])
    assert np.array_equal(made.masks[2].numpy().astype(np.uint8), g[f"d{d}_h{H}_m2"])


def test_realnvp_composite_matches_reference():
    g = load_golden("g2_realnvp.npz")
    m = nfs_amd.RealNVP(2, 8, 64)
    m.load_state_dict(state_dict_from(g, "", m))
    m.eval()
    with torch.no_grad():
        z, ld = m.inverse(torch.from_numpy(g["x"]))
        lp = m.log_prob(torch.from_numpy(g["x"]))
    np.testing.assert_allclose(z.numpy(), g["inv_z"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(ld.numpy(), g["inv_ld"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(lp.numpy(), g["log_prob"], rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("tag,K", [("k8.", 8), ("k10.", 10)])
def test_spline_composite_matches_reference(tag, K):
    g = load_golden("g3_spline.npz")
    if K == 10:
        m = nfs_amd.RealNVPSpline(2, 8, 64)
    else:
        layers = []
        for i in range(8):
            mask = torch.zeros(2)
            mask[(0 if i % 2 == 0 else 1)] = 1
            layers.append(nfs_amd.SplineCouplingLayer(2, 64, mask, num_bins=8))
        m = nfs_amd.NormalizingFlowModel(layers)
    m.load_state_dict(state_dict_from(g, tag, m))
    m.eval()
    with torch.no_grad():
        z, ld = m.inverse(torch.from_numpy(g["x"]))
        x, lf = m.forward(torch.from_numpy(g["z"]))
    np.testing.assert_allclose(z.numpy(), g[tag + "inv_z"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(ld.numpy(), g[tag + "inv_ld"], rtol=1e-6, atol=2e-6)
    np.testing.assert_allclose(x.numpy(), g[tag + "fwd_x"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(lf.numpy(), g[tag + "fwd_ld"], rtol=1e-6, atol=2e-6)


def test_maf_composite_matches_reference():
    g = load_golden("g5_maf63.npz")
    m = nfs_amd.NormalizingFlowModel([nfs_amd.MaskedAutoregressiveFlow(63, 64) for _ in range(5)])
    m.load_state_dict(state_dict_from(g, "", m))
    m.eval()
    with torch.no_grad():
        z, ld = m.inverse(torch.from_numpy(g["x"]))
        x, lf = m.forward(torch.from_numpy(g["z"]))
    np.testing.assert_allclose(z.numpy(), g["inv_z"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ld.numpy(), g["inv_ld"], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(x.numpy(), g["fwd_x"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(lf.numpy(), g["fwd_ld"], rtol=1e-5, atol=1e-4)


def test_rqs_unit_composite_matches_reference():
    g = load_golden("g4_rqs_unit.npz")
    args = [torch.from_numpy(g[k]) for k in ("x", "uw", "uh", "ud")]
    y, l = nfs_amd.rational_quadratic_spline(*args, inverse=False)
    np.testing.assert_allclose(y.numpy(), g["fwd_y"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(l.numpy(), g["fwd_ld"], rtol=1e-6, atol=1e-6)
    y, l = nfs_amd.rational_quadratic_spline(*args, inverse=True)
    np.testing.assert_allclose(np.nan_to_num(y.numpy()), np.nan_to_num(g["inv_y"]), rtol=1e-6, atol=1e-6)


def test_relational_invertibility_and_logdet_symmetry():
    """Reference tests/correctness/test_invertibility.py:131-161 on the product modules (CPU)."""
    torch.manual_seed(456)
    d, H = 4, 16
    mask = torch.zeros(d)
    mask[::2] = 1
    flows = [nfs_amd.CouplingLayer(d, H, mask), nfs_amd.SplineCouplingLayer(d, H, mask),
             nfs_amd.MaskedAutoregressiveFlow(d, H), nfs_amd.InverseAutoregressiveFlow(d, H),
             nfs_amd.RealNVP(d, 2, H, batch_norm_between_layers=True)]
    for f in flows:
        z = torch.randn(8, d)
        x, lf = f.forward(z)
        zr, li = f.inverse(x)
        tol = 1e-3 if isinstance(f, (nfs_amd.MaskedAutoregressiveFlow, nfs_amd.InverseAutoregressiveFlow)) else 1e-5
        assert float((lf + li).abs().max()) < tol, type(f).__name__
        assert float((zr - z).abs().max()) < 1e-3, type(f).__name__


def test_gradcheck_float64_coupling():
    """Reference tests/correctness/test_gradcheck.py:143-162 style (float64 composite path)."""
    torch.manual_seed(0)
    mask = torch.tensor([1.0, 0.0, 1.0])
    f = nfs_amd.CouplingLayer(3, 8, mask).double().eval()
    with torch.no_grad():
        f.s_net[6].weight.normal_(0, 0.1)
        f.b_net[6].weight.normal_(0, 0.1)
    x = torch.randn(4, 3, dtype=torch.float64, requires_grad=True)
    assert torch.autograd.gradcheck(lambda t: f.inverse(t)[0], (x,), eps=1e-6, atol=1e-4, rtol=1e-3)
    assert torch.autograd.gradcheck(lambda t: f.inverse(t)[1], (x,), eps=1e-6, atol=1e-4, rtol=1e-3)


@pytest.mark.parametrize("name", ["a1", "a3", "a5", "a4bn", "a10"])
def test_arqs_composite_matches_reference(name):
    """nfs_amd.ARQS (constructor, state_dict keys, composite path) vs the reference's outputs."""
    g = load_golden("g10_arqs.npz")
    d, H, K, bn, lo, hi = g[name + ".meta"]
    kw = {} if np.isnan(lo) else {"data_min": float(lo), "data_max": float(hi)}
    m = nfs_amd.ARQS(int(d), hidden_dim=int(H), num_bins=int(K), use_batch_norm=bool(bn), **kw)
    ours = {k for k in m.state_dict() if not k.endswith("num_batches_tracked")}
    assert ours == {k[len(name) + 1:] for k in g if k.startswith(name + ".conditioner.")}
    m.load_state_dict(state_dict_from(g, name + ".", m))
    m.eval()
    x = torch.from_numpy(g[name + ".x"])
    with torch.no_grad():
        yf, lf = m.forward(x)
        yi, li = m.inverse(x)
    for got, key in ((yf, "fwd_y"), (lf, "fwd_ld"), (yi, "inv_y"), (li, "inv_ld")):
        np.testing.assert_allclose(got.numpy(), g[f"{name}.{key}"], rtol=1e-5, atol=1e-5, err_msg=key)


def _g12_model(name):
    if name == "rn":
        return nfs_amd.RealNVP(2, 8, 64, batch_norm_between_layers=True)
    if name == "rs":
        return nfs_amd.RealNVPSpline(2, 8, 64, batch_norm_between_layers=True)
    return nfs_amd.NormalizingFlowModel([nfs_amd.MaskedAutoregressiveFlow(10, 16) for _ in range(3)],
                                        batch_norm_between_layers=True)


@pytest.mark.parametrize("name", ["rn", "rs", "maf"])
def test_between_layer_batchnorm_composite_matches_reference(name):
    """NormalizingFlowModel(batch_norm_between_layers=True) on the CPU composite path vs G12:
    state_dict keys, eval both directions, and the train-mode forward's running statistics."""
    g = load_golden("g12_flowbn.npz")
    m = _g12_model(name)
    keys = {k for k, v in m.state_dict().items() if v.dtype != torch.int64}
    assert {name + "." + k for k in keys} == {k for k in g if k.startswith(name + ".") and
                                              not k.startswith(name + ".after_train.") and
                                              k.count(".") > 1 and not k.split(".", 1)[1] in
                                              ("x", "z", "inv_z", "inv_ld", "fwd_x", "fwd_ld", "log_prob",
                                               "nll_f64", "train_fwd_x", "train_fwd_ld")}
    m.load_state_dict(state_dict_from(g, name + ".", m))
    m.eval()
    tol = dict(rtol=1e-6, atol=2e-6)
    with torch.no_grad():
        z, ld = m.inverse(torch.from_numpy(g[f"{name}.x"]))
        x, ldf = m.forward(torch.from_numpy(g[f"{name}.z"]))
    np.testing.assert_allclose(z.numpy(), g[f"{name}.inv_z"], **tol)
    np.testing.assert_allclose(ld.numpy(), g[f"{name}.inv_ld"], **tol)
    np.testing.assert_allclose(x.numpy(), g[f"{name}.fwd_x"], **tol)
    np.testing.assert_allclose(ldf.numpy(), g[f"{name}.fwd_ld"], **tol)
    m.train()
    with torch.no_grad():
        xt, ldt = m.forward(torch.from_numpy(g[f"{name}.z"]))
    np.testing.assert_allclose(xt.numpy(), g[f"{name}.train_fwd_x"], **tol)
    np.testing.assert_allclose(ldt.numpy(), g[f"{name}.train_fwd_ld"], **tol)
    after = state_dict_from(g, f"{name}.after_train.", _g12_model(name))
    for k, v in m.state_dict().items():
        if v.is_floating_point():
            np.testing.assert_allclose(v.numpy(), after[k].numpy(), **tol)


def test_sequential_flow_composite_matches_reference():
    """SequentialFlow (sequential_flow.py:5-34) of mixed layers on the CPU composite path vs G13."""
    g = load_golden("g13_sequential.npz")

    def alt(dim, even):
        mask = torch.zeros(dim)
        mask[(0 if even else 1)::2] = 1
        return mask

    models = {"s2": nfs_amd.SequentialFlow([nfs_amd.CouplingLayer(2, 32, alt(2, i % 2 == 0)) for i in range(4)]),
              "s5": nfs_amd.SequentialFlow([nfs_amd.CouplingLayer(5, 32, alt(5, True)),
                                            nfs_amd.SplineCouplingLayer(5, 32, alt(5, False), num_bins=8),
                                            nfs_amd.MaskedAutoregressiveFlow(5, 16),
                                            nfs_amd.InverseAutoregressiveFlow(5, 16)])}
    with pytest.raises(ValueError):
        nfs_amd.SequentialFlow(models["s2"].flows[0])
    for name, m in models.items():
        m.load_state_dict(state_dict_from(g, name + ".", m))
        m.eval()
        with torch.no_grad():
            z, ld = m.inverse(torch.from_numpy(g[f"{name}.x"]))
            x, ldf = m.forward(torch.from_numpy(g[f"{name}.z"]))
        tol = dict(rtol=1e-6, atol=2e-6)
        np.testing.assert_allclose(z.numpy(), g[f"{name}.inv_z"], **tol)
        np.testing.assert_allclose(ld.numpy(), g[f"{name}.inv_ld"], **tol)
        np.testing.assert_allclose(x.numpy(), g[f"{name}.fwd_x"], **tol)
        np.testing.assert_allclose(ldf.numpy(), g[f"{name}.fwd_ld"], **tol)
