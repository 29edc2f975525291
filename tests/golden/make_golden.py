"""Generate the golden parity fixtures from the REFERENCE implementation itself.

Runs only in the build container (needs /root/reference; never on the GPU box):

    python tests/golden/make_golden.py [--skip-full]

It imports itxtx/normalizing-flows-study from /root/reference (a stub `torchdiffeq` module is
injected in-process because the continuous-flow package imports it at package import time; no
hot-path code calls it), builds the reference modules with fixed seeds, perturbs their weights so
no layer is the identity, runs them on seeded inputs, and writes plain arrays:

  g1_made_masks.npz   MADE degrees/masks (uint8) for the (d, H) pairs of SURVEY §8(c) G1
  g2_realnvp.npz      RealNVP(2,8,64) eval: inverse/forward/log_prob on 4,096 rows (+ edge rows)
  g3_spline.npz       8x SplineCouplingLayer(2,64,K=8) and RealNVPSpline(2,8,64) (K=10)
  g4_rqs_unit.npz     rational_quadratic_spline, N=4,096, K=8, both directions
  g5_maf63.npz        5x MAF(63,64): inverse 1,024 rows, forward 128 rows
  g6_iaf784.npz       IAF(784,64): forward 64 rows, inverse 16 rows
  g7_moons.npz        config 1: two-moons 5k, RealNVP(2,8,64) trained 45 steps, eval log_prob/NLL
  g9_small.npz        d=4/H=16 layers of the reference's own tests (+ MAF/IAF d=10)
  g10_arqs.npz        ARQS (src/flows/spline/arqs.py) forward/inverse: d in {1,3,5,10}, H up to
                      128, K in {2,5,8,11}, scalar data_min/data_max, eval BatchNorm in MADE
  g11_train.npz       TRAIN-mode coupling layers (batch-statistics BatchNorm, coupling_layer.py:18-35):
                      RealNVP(2,8,64) inverse + NLL backward (grads, running stats) and 5 Adam steps
                      on two-moons (README.md:107-117); CouplingLayer(4,16) both directions
  g12_flowbn.npz      between-layer BatchNorm (normalizing_flow_model.py:67-128): RealNVP(2,8,64,True),
                      RealNVPSpline(2,8,64,True) and 3x MAF(10,16) with BatchNorm between layers, eval
                      both directions + log_prob, and a train-mode forward (running-stat update)
  g13_sequential.npz  SequentialFlow (sequential_flow.py:5-34): 4 CouplingLayers d=2 as in
                      examples/visualization_demo.py:26-36, and a mixed d=5 chain
  g14_grads.npz       gradients (dL/dx + every parameter) through the reference's own MAF(10,32),
                      IAF(10,32), MAF(63,64), IAF(784,64) (both directions, the sequential ones through
                      all d MADE calls) and SplineCouplingLayer K=8 (d=2, H=64) / K=10 (d=3, H=32)
  g15_fig_train.npz   the benchmark-figure model RealNVP(2,10,128) (plots/_common.py:161) trained as
                      plots/_common.py:194-211: train-mode step on 2,000 two-moons points (z, ld, loss,
                      gradients, running stats) and 5 Adam + clip steps (losses, final state)
  g16_fig_models.npz  the other benchmark-figure models (plots/_common.py:157-169): RealNVPSpline(2,8,64),
                      6x MAF(2,64), 6x IAF(2,64): first train step (z, ld, loss, gradients) and 3 Adam +
                      clip steps (losses, final state) on 2,000 two-moons points
  g17_options.npz     the remaining constructor options under autograd: train-mode use_batch_norm=True
                      in IAF density (2-layer model step) and MAF sampling, ARQS with BatchNorm in train
                      mode (both directions), SplineCouplingLayer with per-dimension data_min/data_max
  g18_arqs_bounds.npz ARQS with data_min/data_max (per-dimension tensors and python floats), eval,
                      both directions under autograd: y, ld, dL/dx, every parameter gradient
  g8_full_nll.json    oracle NLL scalars (float64) at the full BASELINE batch sizes (+ cfg5: IAF(784,64)
                      inverse NLL at B=8192 and forward checksums at B=524288)

Each npz holds the module's state_dict arrays under their reference keys (prefixed per case),
inputs and expected outputs. Nothing pickled; load with numpy.load(allow_pickle=False).
"""
import argparse
import json
import os
import sys
import time
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("NFS_REFERENCE", "/root/reference")


def import_reference():
    stub = types.ModuleType("torchdiffeq")

    def odeint(*a, **k):
        raise RuntimeError("torchdiffeq is not installed (stub for the reference import)")

    stub.odeint = odeint
    sys.modules.setdefault("torchdiffeq", stub)
    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import src.flows as flows  # noqa: F401
    import src.models as models  # noqa: F401
    return sys.modules["src.flows"], sys.modules["src.models"]


def perturb(module, sigma, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in module.named_parameters():
            p.add_(sigma * torch.randn(p.shape, generator=g))
        for name, mod in module.named_modules():
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.running_mean.copy_(0.1 * torch.randn(mod.running_mean.shape, generator=g))
                mod.running_var.copy_(0.5 + torch.rand(mod.running_var.shape, generator=g))


def sd_arrays(module, prefix):
    out = {}
    for k, v in module.state_dict().items():
        if v.dtype == torch.int64:  # num_batches_tracked
            continue
        out[prefix + k] = v.detach().cpu().numpy().copy()  # train mode mutates buffers in place
    return out


def edge_rows(d):
    vals = [0.0, 1e-6, -1e-6, 1e3, -1e3, 1e10, -1e10, 5.0, -5.0, 4.9999, -4.9999, 5.0001, -5.0001, 10.0, -10.0]
    rows = []
    for v in vals:
        rows.append([v] * d)
        r = [0.3] * d
        r[0] = v
        rows.append(r)
        r = [-0.7] * d
        r[-1] = v
        rows.append(r)
    return torch.tensor(rows, dtype=torch.float32)


def mvn_logp(z, ld):
    from torch.distributions import MultivariateNormal
    d = z.shape[1]
    base = MultivariateNormal(torch.zeros(d), torch.eye(d))
    return base.log_prob(z) + ld


def run_model(model, x_inv, z_fwd):
    with torch.no_grad():
        zi, ldi = model.inverse(x_inv)
        xf, ldf = model.forward(z_fwd)
        lp = mvn_logp(zi, ldi)
    return {"inv_z": zi.numpy(), "inv_ld": ldi.numpy(), "fwd_x": xf.numpy(), "fwd_ld": ldf.numpy(),
            "log_prob": lp.numpy(), "nll_f64": np.float64(-lp.double().mean().item())}


def g1(flows):
    MADE = flows.MADE
    out = {}
    for d, H in [(1, 8), (2, 64), (3, 16), (3, 32), (4, 16), (5, 16), (10, 16), (63, 64), (154, 64), (784, 64)]:
        m = MADE(d, H)
        out[f"d{d}_h{H}_deg"] = np.asarray(m.m[0], dtype=np.int32)
        out[f"d{d}_h{H}_m1"] = m.masks[0].numpy().astype(np.uint8)
        out[f"d{d}_h{H}_mhh"] = m.masks[1].numpy().astype(np.uint8)
        out[f"d{d}_h{H}_m2"] = m.masks[2].numpy().astype(np.uint8)
    np.savez_compressed(os.path.join(HERE, "g1_made_masks.npz"), **out)


def moons(n, noise, rs):
    from sklearn.datasets import make_moons
    X, _ = make_moons(n_samples=n, noise=noise, random_state=rs)
    return torch.FloatTensor(X)


def g2(models):
    torch.manual_seed(0)
    m = models.RealNVP(2, 8, 64)
    perturb(m, 0.1, 1)
    m.eval()
    g = torch.Generator().manual_seed(2)
    x = torch.cat([moons(2048, 0.05, 42), torch.randn(2000, 2, generator=g), edge_rows(2)])
    z = torch.randn(4096, 2, generator=g)
    out = sd_arrays(m, "")
    out.update({"x": x.numpy(), "z": z.numpy()})
    out.update(run_model(m, x, z))
    with torch.no_grad():
        l0 = m.flow.flows[0]
        zi, ldi = l0.inverse(x)
        xf, ldf = l0.forward(z)
    out.update({"l0_inv_z": zi.numpy(), "l0_inv_ld": ldi.numpy(), "l0_fwd_x": xf.numpy(), "l0_fwd_ld": ldf.numpy()})
    np.savez_compressed(os.path.join(HERE, "g2_realnvp.npz"), **out)
    return m


def spline_stack(flows, models, d, H, K, n_layers, seed):
    torch.manual_seed(seed)
    layers = []
    for i in range(n_layers):
        mask = torch.zeros(d)
        if i % 2 == 0:
            mask[:d // 2] = 1
        else:
            mask[d // 2:] = 1
        layers.append(flows.SplineCouplingLayer(d, H, mask, num_bins=K))
    return models.NormalizingFlowModel(layers)


def g3(flows, models):
    m = spline_stack(flows, models, 2, 64, 8, 8, 10)
    perturb(m, 0.1, 11)
    m.eval()
    g = torch.Generator().manual_seed(12)
    x = torch.cat([moons(2048, 0.05, 42), torch.randn(2000, 2, generator=g) * 2.0, edge_rows(2)])
    z = torch.randn(4096, 2, generator=g)
    out = sd_arrays(m, "k8.")
    out.update({"x": x.numpy(), "z": z.numpy()})
    out.update({"k8." + k: v for k, v in run_model(m, x, z).items()})
    torch.manual_seed(13)
    m10 = models.RealNVPSpline(2, 8, 64)
    perturb(m10, 0.1, 14)
    m10.eval()
    out.update(sd_arrays(m10, "k10."))
    out.update({"k10." + k: v for k, v in run_model(m10, x, z).items()})
    np.savez_compressed(os.path.join(HERE, "g3_spline.npz"), **out)
    return m


def g4(flows):
    rqs = flows.rational_quadratic_spline
    g = torch.Generator().manual_seed(20)
    N, K = 4096, 8
    uw = 1.5 * torch.randn(N, K, generator=g)
    uh = 1.5 * torch.randn(N, K, generator=g)
    ud = 1.5 * torch.randn(N, K - 1, generator=g)
    x = torch.rand(N, generator=g) * 1.4 - 0.2
    x[:8] = torch.tensor([0.0, 1.0, 0.5, -0.1, 1.1, 1e-7, 1 - 1e-7, 2.0])
    yf, lf = rqs(x, uw, uh, ud, inverse=False)
    yi, li = rqs(x, uw, uh, ud, inverse=True)
    np.savez_compressed(os.path.join(HERE, "g4_rqs_unit.npz"), x=x.numpy(), uw=uw.numpy(), uh=uh.numpy(),
                        ud=ud.numpy(), fwd_y=yf.numpy(), fwd_ld=lf.numpy(), inv_y=yi.numpy(), inv_ld=li.numpy())


def maf_stack(flows, models, d, H, n, seed):
    torch.manual_seed(seed)
    return models.NormalizingFlowModel([flows.MaskedAutoregressiveFlow(d, H) for _ in range(n)])


def g5(flows, models):
    m = maf_stack(flows, models, 63, 64, 5, 30)
    perturb(m, 0.02, 31)
    m.eval()
    g = torch.Generator().manual_seed(32)
    x = torch.randn(1024, 63, generator=g)
    z = torch.randn(128, 63, generator=g)
    out = sd_arrays(m, "")
    out.update({"x": x.numpy(), "z": z.numpy()})
    with torch.no_grad():
        zi, ldi = m.inverse(x)
        xf, ldf = m.forward(z)
        lp = mvn_logp(zi, ldi)
    out.update({"inv_z": zi.numpy(), "inv_ld": ldi.numpy(), "fwd_x": xf.numpy(), "fwd_ld": ldf.numpy(),
                "log_prob": lp.numpy(), "nll_f64": np.float64(-lp.double().mean().item())})
    np.savez_compressed(os.path.join(HERE, "g5_maf63.npz"), **out)
    return m


def g6(flows):
    torch.manual_seed(40)
    f = flows.InverseAutoregressiveFlow(784, 64)
    perturb(f, 0.01, 41)
    f.eval()
    g = torch.Generator().manual_seed(42)
    z = torch.randn(64, 784, generator=g)
    x = torch.randn(16, 784, generator=g)
    with torch.no_grad():
        xf, ldf = f.forward(z)
        zi, ldi = f.inverse(x)
    out = sd_arrays(f, "")
    out.update({"z": z.numpy(), "x": x.numpy(), "fwd_x": xf.numpy(), "fwd_ld": ldf.numpy(),
                "inv_z": zi.numpy(), "inv_ld": ldi.numpy()})
    np.savez_compressed(os.path.join(HERE, "g6_iaf784.npz"), **out)
    return f


def g7(models, src_utils):
    data = src_utils.get_two_moons_data(n_samples=5000, noise=0.05)
    from torch.distributions import MultivariateNormal
    base = MultivariateNormal(torch.zeros(2), torch.eye(2))
    torch.manual_seed(0)
    m = models.RealNVP(data_dim=2, n_layers=8, hidden_dim=64)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    curve = []
    for epoch in range(45):  # README.md:111-117 quickstart loop; stopped at 45 steps, before the
        # reference's train-mode-BN run diverges (NLL 1.16 at step 40, a 2e13 spike at step 50, 9.0 by step 300)
        z, log_det = m.inverse(data)
        loss = -(base.log_prob(z) + log_det).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        curve.append(loss.item())
    m.eval()
    with torch.no_grad():
        z, ld = m.inverse(data)
        lp = base.log_prob(z) + ld
    out = sd_arrays(m, "")
    out.update({"x": data.numpy(), "inv_z": z.numpy(), "inv_ld": ld.numpy(), "log_prob": lp.numpy(),
                "nll_f64": np.float64(-lp.double().mean().item()), "train_curve": np.asarray(curve, np.float32)})
    np.savez_compressed(os.path.join(HERE, "g7_moons.npz"), **out)


def g9(flows, models):
    """Small layers exactly as the reference's own correctness tests build them (d=4, H=16)."""
    def create_mask(dim, kind):
        mask = torch.zeros(dim)
        if kind == "alternating":
            mask[::2] = 1
        else:
            mask[:dim // 2] = 1
        return mask

    out = {}
    g = torch.Generator().manual_seed(50)
    cases = [
        ("cpl_alt", lambda: flows.CouplingLayer(4, 16, create_mask(4, "alternating")), 0.1),
        ("cpl_half", lambda: flows.CouplingLayer(4, 16, create_mask(4, "half")), 0.1),
        ("cpl_d3", lambda: flows.CouplingLayer(3, 16, create_mask(3, "alternating")), 0.1),
        ("cpl_d1", lambda: flows.CouplingLayer(1, 16, create_mask(1, "alternating")), 0.1),
        ("spl_alt", lambda: flows.SplineCouplingLayer(4, 16, create_mask(4, "alternating")), 0.1),
        ("spl_half", lambda: flows.SplineCouplingLayer(4, 16, create_mask(4, "half")), 0.1),
        ("spl_d3", lambda: flows.SplineCouplingLayer(3, 16, create_mask(3, "alternating")), 0.1),
        ("maf4", lambda: flows.MaskedAutoregressiveFlow(4, 16), 0.05),
        ("iaf4", lambda: flows.InverseAutoregressiveFlow(4, 16), 0.05),
        ("maf10", lambda: flows.MaskedAutoregressiveFlow(10, 16), 0.05),
        ("iaf10", lambda: flows.InverseAutoregressiveFlow(10, 16), 0.05),
        ("maf2", lambda: flows.MaskedAutoregressiveFlow(2, 64), 0.05),
        ("iaf3", lambda: flows.InverseAutoregressiveFlow(3, 32), 0.05),
    ]
    for i, (name, ctor, sigma) in enumerate(cases):
        torch.manual_seed(100 + i)
        f = ctor()
        perturb(f, sigma, 200 + i)
        f.eval()
        d = f.data_dim
        x = torch.cat([torch.randn(61, d, generator=g), torch.zeros(1, d), torch.full((1, d), 3.0),
                       torch.full((1, d), -6.0)])
        with torch.no_grad():
            yf, lf = f.forward(x)
            yi, li = f.inverse(x)
        out.update(sd_arrays(f, name + "."))
        out.update({name + ".x": x.numpy(), name + ".fwd_y": yf.numpy(), name + ".fwd_ld": lf.numpy(),
                    name + ".inv_y": yi.numpy(), name + ".inv_ld": li.numpy()})
    np.savez_compressed(os.path.join(HERE, "g9_small.npz"), **out)


def g10(flows):
    """ARQS: the sequential unit-interval spline flow with a MADE(d, H, 3K-1) conditioner."""
    out = {}
    cases = [  # name, dim, hidden, K, data range, use_batch_norm, rows
        ("a1", 1, 16, 2, None, False, 64),
        ("a3", 3, 16, 8, None, False, 512),
        ("a5", 5, 128, 8, None, False, 256),
        ("a4bn", 4, 32, 11, None, True, 256),
        ("a10", 10, 64, 5, (-3.0, 3.0), False, 256),
    ]
    for i, (name, d, H, K, rng, bn, n) in enumerate(cases):
        torch.manual_seed(100 + i)
        kw = {"data_min": rng[0], "data_max": rng[1]} if rng else {}
        m = flows.ARQS(d, hidden_dim=H, num_bins=K, use_batch_norm=bn, **kw)
        perturb(m, 0.3, 200 + i)
        m.eval()
        g = torch.Generator().manual_seed(300 + i)
        if rng:
            x = torch.randn(n, d, generator=g) * 1.2
        else:
            x = torch.rand(n, d, generator=g)
            x[:4] = torch.tensor([0.0, 1.0, 0.5, 1e-7])[:, None].expand(4, d)
            x[4:6] = torch.tensor([-0.25, 1.25])[:, None].expand(2, d)  # clamped by the spline
        with torch.no_grad():
            xf, ldf = m.forward(x)
            zi, ldi = m.inverse(x)
            zr, ldr = m.inverse(xf)
        out.update(sd_arrays(m, name + "."))
        out.update({f"{name}.x": x.numpy(), f"{name}.fwd_y": xf.numpy(), f"{name}.fwd_ld": ldf.numpy(),
                    f"{name}.inv_y": zi.numpy(), f"{name}.inv_ld": ldi.numpy(),
                    f"{name}.rt_y": zr.numpy(), f"{name}.rt_ld": ldr.numpy(),
                    f"{name}.meta": np.array([d, H, K, int(bn), rng[0] if rng else np.nan,
                                              rng[1] if rng else np.nan], dtype=np.float64)})
    np.savez_compressed(os.path.join(HERE, "g10_arqs.npz"), **out)


def g11(flows, models):
    """Train mode: BatchNorm1d normalises with batch statistics and updates running stats."""
    from torch.distributions import MultivariateNormal
    out = {}
    torch.manual_seed(50)
    m = models.RealNVP(2, 8, 64)
    perturb(m, 0.03, 51)
    m.train()
    out.update(sd_arrays(m, "rn.init."))
    x = torch.cat([moons(1900, 0.05, 42), torch.randn(100, 2, generator=torch.Generator().manual_seed(52))])
    out["rn.x"] = x.numpy()
    base = MultivariateNormal(torch.zeros(2), torch.eye(2))
    z, ld = m.inverse(x)
    loss = -(base.log_prob(z) + ld).mean()
    loss.backward()
    out.update({"rn.z": z.detach().numpy(), "rn.ld": ld.detach().numpy(), "rn.loss": np.float64(loss.item())})
    for k, p in m.named_parameters():
        out["rn.grad." + k] = p.grad.numpy()
    out.update(sd_arrays(m, "rn.after."))
    # 5 full-batch Adam steps from the same initial state (README.md:107-117)
    torch.manual_seed(50)
    m = models.RealNVP(2, 8, 64)
    perturb(m, 0.03, 51)
    m.train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    losses = []
    for _ in range(5):
        z, ld = m.inverse(x)
        loss = -(base.log_prob(z) + ld).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    out["rn.adam_losses"] = np.asarray(losses, dtype=np.float64)
    out.update(sd_arrays(m, "rn.adam5."))
    # single layer, d = 4 (padded kernel width), both directions, loss with weights on y and ld
    torch.manual_seed(53)
    mask = torch.tensor([1.0, 0.0, 1.0, 0.0])
    layer = flows.CouplingLayer(4, 16, mask)
    perturb(layer, 0.2, 54)
    layer.train()
    out.update(sd_arrays(layer, "c4.init."))
    g = torch.Generator().manual_seed(55)
    xc = torch.randn(333, 4, generator=g) * 1.5
    wy = torch.randn(333, 4, generator=g)
    wl = torch.randn(333, generator=g)
    out.update({"c4.x": xc.numpy(), "c4.wy": wy.numpy(), "c4.wl": wl.numpy()})
    for name, fn in (("inv", layer.inverse), ("fwd", layer.forward)):
        layer.zero_grad()
        xr = xc.clone().requires_grad_(True)
        y, ldc = fn(xr)
        ((y * wy).sum() + (ldc * wl).sum()).backward()
        out[f"c4.{name}.y"] = y.detach().numpy()
        out[f"c4.{name}.ld"] = ldc.detach().numpy()
        out[f"c4.{name}.gx"] = xr.grad.numpy()
        for k, p in layer.named_parameters():
            out[f"c4.{name}.grad.{k}"] = p.grad.numpy()
    out.update(sd_arrays(layer, "c4.after."))  # running stats after the two calls
    np.savez_compressed(os.path.join(HERE, "g11_train.npz"), **out)


def g12(flows, models):
    """Between-layer BatchNorm: invertible affine with running stats, scalar log-det."""
    out = {}
    g = torch.Generator().manual_seed(60)
    x = torch.cat([moons(1000, 0.05, 42), torch.randn(1000, 2, generator=g) * 1.5, edge_rows(2)[:24]])
    z = torch.randn(1024, 2, generator=g)
    cases = [("rn", lambda: models.RealNVP(2, 8, 64, batch_norm_between_layers=True), 0.1, x, z),
             ("rs", lambda: models.RealNVPSpline(2, 8, 64, batch_norm_between_layers=True), 0.1, x, z),
             ("maf", lambda: models.NormalizingFlowModel([flows.MaskedAutoregressiveFlow(10, 16) for _ in range(3)],
                                                         batch_norm_between_layers=True), 0.05,
              torch.randn(512, 10, generator=g), torch.randn(256, 10, generator=g))]
    for i, (name, ctor, sigma, xi, zi) in enumerate(cases):
        torch.manual_seed(600 + i)
        m = ctor()
        perturb(m, sigma, 610 + i)
        bns = m.flow.batch_norms if hasattr(m, "flow") else m.batch_norms
        with torch.no_grad():  # gamma away from 1 so the log-det term is non-trivial
            for bn in bns:
                bn.weight.copy_(0.6 + 0.8 * torch.rand(bn.weight.shape, generator=g))
                bn.bias.copy_(0.2 * torch.randn(bn.bias.shape, generator=g))
        m.eval()
        out.update(sd_arrays(m, name + "."))
        out.update({f"{name}.x": xi.numpy(), f"{name}.z": zi.numpy()})
        out.update({f"{name}.{k}": v for k, v in run_model(m, xi, zi).items()})
        # train mode: forward(z) updates the between-layer running statistics (and, for RealNVP,
        # normalises the conditioner BatchNorms with batch statistics)
        m.train()
        with torch.no_grad():
            xt, ldt = m.forward(zi)
        out.update({f"{name}.train_fwd_x": xt.numpy(), f"{name}.train_fwd_ld": ldt.numpy()})
        out.update(sd_arrays(m, name + ".after_train."))
    np.savez_compressed(os.path.join(HERE, "g12_flowbn.npz"), **out)


def g13(flows):
    """SequentialFlow: zeros(B) accumulator, layers in order / reverse order."""
    SequentialFlow = flows.SequentialFlow
    out = {}
    g = torch.Generator().manual_seed(70)

    def alt(dim, even):
        mask = torch.zeros(dim)
        if even:
            mask[::2] = 1
        else:
            mask[1::2] = 1
        return mask

    torch.manual_seed(700)
    s2 = SequentialFlow([flows.CouplingLayer(2, 32, alt(2, i % 2 == 0)) for i in range(4)])
    torch.manual_seed(701)
    s5 = SequentialFlow([flows.CouplingLayer(5, 32, alt(5, True)),
                         flows.SplineCouplingLayer(5, 32, alt(5, False), num_bins=8),
                         flows.MaskedAutoregressiveFlow(5, 16),
                         flows.InverseAutoregressiveFlow(5, 16)])
    for name, m, d in (("s2", s2, 2), ("s5", s5, 5)):
        perturb(m, 0.1, 710 + d)
        m.eval()
        xi = torch.cat([torch.randn(500, d, generator=g) * 1.3, torch.zeros(1, d), torch.full((1, d), 4.0)])
        zi = torch.randn(300, d, generator=g)
        with torch.no_grad():
            zo, ldi = m.inverse(xi)
            xo, ldf = m.forward(zi)
        out.update(sd_arrays(m, name + "."))
        out.update({f"{name}.x": xi.numpy(), f"{name}.z": zi.numpy(), f"{name}.inv_z": zo.numpy(),
                    f"{name}.inv_ld": ldi.numpy(), f"{name}.fwd_x": xo.numpy(), f"{name}.fwd_ld": ldf.numpy()})
    np.savez_compressed(os.path.join(HERE, "g13_sequential.npz"), **out)


def g14(flows):
    """Gradients through the reference's own layers under autograd (loss = sum(y * wy) +
    sum(ld * wl), random weights wy, wl): MaskedAutoregressiveFlow and InverseAutoregressiveFlow in
    both directions (masked_autoregressive_flow.py:18-78, inverse_autoregressive_flow.py:30-103,
    the sequential directions differentiated through all d MADE calls) and SplineCouplingLayer
    (spline_coupling_layer.py:96-309), K = 8 and 10, both directions. Stores y, ld, dL/dx and
    every parameter gradient per case."""
    out = {}
    g = torch.Generator().manual_seed(140)
    cases = [
        ("maf10", lambda: flows.MaskedAutoregressiveFlow(10, 32), 0.1, 300, 1.0),
        ("iaf10", lambda: flows.InverseAutoregressiveFlow(10, 32), 0.1, 300, 1.0),
        ("maf63", lambda: flows.MaskedAutoregressiveFlow(63, 64), 0.02, 128, 1.0),
        ("iaf784", lambda: flows.InverseAutoregressiveFlow(784, 64), 0.01, 8, 1.0),
        ("sp8", lambda: flows.SplineCouplingLayer(2, 64, torch.tensor([1.0, 0.0]), num_bins=8), 0.1, 500, 2.5),
        ("sp10", lambda: flows.SplineCouplingLayer(3, 32, torch.tensor([0.0, 1.0, 0.0]), num_bins=10), 0.1, 500, 2.5),
    ]
    for i, (name, ctor, sigma, B, scale) in enumerate(cases):
        torch.manual_seed(1400 + i)
        m = ctor()
        perturb(m, sigma, 1410 + i)
        m.eval()
        out.update(sd_arrays(m, name + ".init."))
        d = m.dim if hasattr(m, "dim") else m.data_dim
        x = torch.randn(B, d, generator=g) * scale
        if name.startswith("sp"):
            x[:4, -1] = torch.tensor([6.0, -7.0, 4.999, -4.999])  # outside / at the spline bound
        wy = torch.randn(B, d, generator=g)
        wl = torch.randn(B, generator=g)
        out.update({f"{name}.x": x.numpy(), f"{name}.wy": wy.numpy(), f"{name}.wl": wl.numpy()})
        for dname, fn in (("inv", m.inverse), ("fwd", m.forward)):
            m.zero_grad()
            xr = x.clone().requires_grad_(True)
            y, ld = fn(xr)
            ((y * wy).sum() + (ld * wl).sum()).backward()
            out[f"{name}.{dname}.y"] = y.detach().numpy()
            out[f"{name}.{dname}.ld"] = ld.detach().numpy()
            out[f"{name}.{dname}.gx"] = xr.grad.numpy()
            for k, p in m.named_parameters():
                out[f"{name}.{dname}.grad.{k}"] = p.grad.numpy()
        print("g14", name, flush=True)
    np.savez_compressed(os.path.join(HERE, "g14_grads.npz"), **out)


def figure_moons(n, seed):
    """plots/_common.py:103-112 (two_moons: make_moons(noise=0.07) standardized, float32)."""
    from sklearn.datasets import make_moons
    x, _ = make_moons(n_samples=n, noise=0.07, random_state=seed)
    x = np.asarray(x, dtype=np.float32)
    return torch.from_numpy((x - x.mean(0)) / (x.std(0) + 1e-8))


def g15(models):
    """The reference's benchmark-figure model in training: RealNVP(2, 10, 128)
    (plots/_common.py:161), full-batch step on 2,000 two-moons points (NDATA, :183) in train mode
    with the loop of plots/_common.py:194-211 (Adam lr 1e-3, clip_grad_norm_ 5.0). Stores the
    first step's z, ld, loss and raw gradients (before the clip), the running statistics after it,
    and the losses + final state of 5 full steps."""
    from torch.distributions import MultivariateNormal
    out = {}
    x = figure_moons(2000, 0)
    out["fig.x"] = x.numpy()
    base = MultivariateNormal(torch.zeros(2), torch.eye(2))

    def fresh():
        torch.manual_seed(150)
        m = models.RealNVP(2, 10, 128)
        perturb(m, 0.03, 151)
        return m.train()

    m = fresh()
    out.update(sd_arrays(m, "fig.init."))
    z, ld = m.inverse(x)
    loss = -(base.log_prob(z) + ld).mean()
    loss.backward()
    out.update({"fig.z": z.detach().numpy(), "fig.ld": ld.detach().numpy(), "fig.loss": np.float64(loss.item())})
    for k, p in m.named_parameters():
        out["fig.grad." + k] = p.grad.numpy()
    out.update({k: v for k, v in sd_arrays(m, "fig.after.").items() if k.endswith(("running_mean", "running_var"))})
    m = fresh()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    losses = []
    for _ in range(5):
        z, ld = m.inverse(x)
        loss = -(base.log_prob(z) + ld).mean()
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 5.0)
        opt.step()
        losses.append(loss.item())
    out["fig.losses5"] = np.asarray(losses, dtype=np.float64)
    out.update(sd_arrays(m, "fig.step5."))
    np.savez_compressed(os.path.join(HERE, "g15_fig_train.npz"), **out)


def g16(flows, models):
    """The reference's other benchmark-figure models in training (plots/_common.py:157-169,
    179-183, 194-211): RealNVPSpline(2, 8, 64) (lr 5e-4), 6x MaskedAutoregressiveFlow(2, 64) and
    6x InverseAutoregressiveFlow(2, 64) in a NormalizingFlowModel (lr 1e-3), full batch on 2,000
    two-moons points. Per model: the first step's z, ld, loss and raw gradients, then the losses
    and final state of 3 Adam + clip_grad_norm_(5.0) steps."""
    from torch.distributions import MultivariateNormal
    out = {}
    x = figure_moons(2000, 0)
    out["x"] = x.numpy()
    base = MultivariateNormal(torch.zeros(2), torch.eye(2))
    builders = {
        "spline": (lambda: models.RealNVPSpline(2, 8, 64), 5e-4),
        "maf": (lambda: models.NormalizingFlowModel([flows.MaskedAutoregressiveFlow(2, 64) for _ in range(6)]), 1e-3),
        "iaf": (lambda: models.NormalizingFlowModel([flows.InverseAutoregressiveFlow(2, 64) for _ in range(6)]), 1e-3),
    }
    for seed, (name, (build, lr)) in enumerate(builders.items()):
        def fresh():
            torch.manual_seed(160 + seed)
            m = build()
            perturb(m, 0.03, 170 + seed)
            return m.train()

        m = fresh()
        out.update(sd_arrays(m, name + ".init."))
        z, ld = m.inverse(x)
        loss = -(base.log_prob(z) + ld).mean()
        loss.backward()
        out.update({name + ".z": z.detach().numpy(), name + ".ld": ld.detach().numpy(),
                    name + ".loss": np.float64(loss.item())})
        for k, p in m.named_parameters():
            out[name + ".grad." + k] = p.grad.numpy()
        m = fresh()
        opt = torch.optim.Adam(m.parameters(), lr=lr)
        losses = []
        for _ in range(3):
            z, ld = m.inverse(x)
            loss = -(base.log_prob(z) + ld).mean()
            opt.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(m.parameters(), 5.0)
            opt.step()
            losses.append(loss.item())
        out[name + ".losses3"] = np.asarray(losses, dtype=np.float64)
        out.update(sd_arrays(m, name + ".step3."))
    np.savez_compressed(os.path.join(HERE, "g16_fig_models.npz"), **out)


def g17(flows, models):
    """The reference's remaining constructor options under autograd:
      iafbn   NormalizingFlowModel of 2x InverseAutoregressiveFlow(5, 32, use_batch_norm=True) in
              TRAIN mode, density direction (the sequential IAF.inverse: d MADE calls, each with its
              own batch statistics, inverse_autoregressive_flow.py:65-103, made.py:93-106):
              z, ld, loss = -mean log_prob, every gradient, running statistics after the step
      mafbn   MaskedAutoregressiveFlow(5, 32, use_batch_norm=True), TRAIN mode, forward (sampling,
              sequential, masked_autoregressive_flow.py:46-78) under L = sum(y wy) + sum(ld wl)
      arqsbn  ARQS(4, 32, num_bins=5, use_batch_norm=True) (arqs.py:7-114), TRAIN mode, both
              directions under L (each direction on a fresh copy of the initial state)
      spldm   SplineCouplingLayer(3, 32, mask = 0, num_bins=6, data_min/data_max = per-dimension
              tensors) (spline_coupling_layer.py:78-91), eval, both directions under L
    Per case: y, ld, dL/dx, every parameter gradient and (train mode) the running statistics after."""
    from torch.distributions import MultivariateNormal
    out = {}
    g = torch.Generator().manual_seed(170)

    # iafbn: density training step through NormalizingFlowModel
    torch.manual_seed(1700)
    m = models.NormalizingFlowModel([flows.InverseAutoregressiveFlow(5, 32, use_batch_norm=True) for _ in range(2)])
    perturb(m, 0.1, 1701)
    m.train()
    out.update(sd_arrays(m, "iafbn.init."))
    x = torch.randn(256, 5, generator=g)
    out["iafbn.x"] = x.numpy()
    z, ld = m.inverse(x)
    base = MultivariateNormal(torch.zeros(5), torch.eye(5))
    loss = -(base.log_prob(z) + ld).mean()
    loss.backward()
    out.update({"iafbn.z": z.detach().numpy(), "iafbn.ld": ld.detach().numpy(), "iafbn.loss": np.float64(loss.item())})
    for k, p in m.named_parameters():
        out["iafbn.grad." + k] = p.grad.numpy()
    out.update({k: v for k, v in sd_arrays(m, "iafbn.after.").items() if k.endswith(("running_mean", "running_var"))})

    def layer_case(name, build, dirs, B, scale):
        torch.manual_seed(1710 + len(out) % 97)
        f = build()
        perturb(f, 0.1, 1720 + len(name))
        init = {k: v.detach().clone() for k, v in f.state_dict().items()}
        out.update(sd_arrays(f, name + ".init."))
        d = f.dim if hasattr(f, "dim") else f.data_dim
        xx = torch.randn(B, d, generator=g) * scale
        wy = torch.randn(B, d, generator=g)
        wl = torch.randn(B, generator=g)
        out.update({f"{name}.x": xx.numpy(), f"{name}.wy": wy.numpy(), f"{name}.wl": wl.numpy()})
        for dname in dirs:
            f.load_state_dict(init)
            f.zero_grad()
            xr = xx.clone().requires_grad_(True)
            y, ldd = (f.forward if dname == "fwd" else f.inverse)(xr)
            ((y * wy).sum() + (ldd * wl).sum()).backward()
            out[f"{name}.{dname}.y"] = y.detach().numpy()
            out[f"{name}.{dname}.ld"] = ldd.detach().numpy()
            out[f"{name}.{dname}.gx"] = xr.grad.numpy()
            for k, p in f.named_parameters():
                out[f"{name}.{dname}.grad.{k}"] = p.grad.numpy()
            out.update({k: v for k, v in sd_arrays(f, f"{name}.{dname}.after.").items()
                        if k.endswith(("running_mean", "running_var"))})

    layer_case("mafbn", lambda: flows.MaskedAutoregressiveFlow(5, 32, use_batch_norm=True).train(), ("fwd",), 200, 1.0)
    layer_case("arqsbn", lambda: flows.ARQS(4, 32, num_bins=5, use_batch_norm=True).train(), ("fwd", "inv"), 200, 0.3)
    dmin, dmax = torch.tensor([-3.0, -2.0, -4.0]), torch.tensor([3.0, 2.5, 1.0])
    out["spldm.data_min"], out["spldm.data_max"] = dmin.numpy(), dmax.numpy()
    # (per-dimension bounds only run in the reference when every dim is transformed: with a
    # conditioning dim, _rescale_from_spline broadcasts the [d] bounds against the [B, n_t] slice and
    # raises — spline_coupling_layer.py:94,122)
    layer_case("spldm", lambda: flows.SplineCouplingLayer(3, 32, torch.tensor([0.0, 0.0, 0.0]), num_bins=6,
                                                          data_min=dmin, data_max=dmax).eval(),
               ("fwd", "inv"), 300, 1.2)
    np.savez_compressed(os.path.join(HERE, "g17_options.npz"), **out)
    print("g17 written", flush=True)


def g18(flows):
    """ARQS with data bounds under autograd (arqs.py:28-42 rescale, :44-114 both
    directions): eval mode, loss L = sum(y wy) + sum(ld wl), each direction from the same state.
      arqsdm  ARQS(3, 32, num_bins=6, data_min/data_max = per-dimension tensors)
      arqssc  ARQS(4, 24, num_bins=5, data_min=-2.5, data_max=3.0) (python float bounds)
    Per case: y, ld, dL/dx and every parameter gradient."""
    out = {}
    g = torch.Generator().manual_seed(180)

    def case(name, build, B, scale):
        torch.manual_seed(1800 + len(name))
        f = build()
        perturb(f, 0.1, 1810 + len(name))
        f.eval()
        init = {k: v.detach().clone() for k, v in f.state_dict().items()}
        out.update(sd_arrays(f, name + ".init."))
        d = f.dim
        xx = torch.randn(B, d, generator=g) * scale
        wy = torch.randn(B, d, generator=g)
        wl = torch.randn(B, generator=g)
        out.update({f"{name}.x": xx.numpy(), f"{name}.wy": wy.numpy(), f"{name}.wl": wl.numpy()})
        for dname in ("fwd", "inv"):
            f.load_state_dict(init)
            f.zero_grad()
            xr = xx.clone().requires_grad_(True)
            y, ldd = (f.forward if dname == "fwd" else f.inverse)(xr)
            ((y * wy).sum() + (ldd * wl).sum()).backward()
            out[f"{name}.{dname}.y"] = y.detach().numpy()
            out[f"{name}.{dname}.ld"] = ldd.detach().numpy()
            out[f"{name}.{dname}.gx"] = xr.grad.numpy()
            for k, p in f.named_parameters():
                out[f"{name}.{dname}.grad.{k}"] = p.grad.numpy()

    dmin, dmax = torch.tensor([-3.0, -2.0, -4.0]), torch.tensor([3.0, 2.5, 1.0])
    out["arqsdm.data_min"], out["arqsdm.data_max"] = dmin.numpy(), dmax.numpy()
    case("arqsdm", lambda: flows.ARQS(3, 32, num_bins=6, data_min=dmin, data_max=dmax), 300, 1.2)
    out["arqssc.data_min"], out["arqssc.data_max"] = np.float64(-2.5), np.float64(3.0)
    case("arqssc", lambda: flows.ARQS(4, 24, num_bins=5, data_min=-2.5, data_max=3.0), 256, 1.0)
    np.savez_compressed(os.path.join(HERE, "g18_arqs_bounds.npz"), **out)
    print("g18 written", flush=True)


def g8_cfg5(f6):
    """cfg5 IAF(784,64) (G6 weights): inverse NLL at B=8192 (seed 1237) and forward checksums at
    B=524288 (seed 1238); merged into g8_full_nll.json."""
    torch.set_num_threads(8)
    path = os.path.join(HERE, "g8_full_nll.json")
    with open(path) as fh:
        res = json.load(fh)
    B, d = 8192, 784
    x = torch.randn(B, d, generator=torch.Generator().manual_seed(1237))
    t0 = time.time()
    tot = 0.0
    with torch.no_grad():
        for s in range(0, B, 1024):
            z, ld = f6.inverse(x[s:s + 1024])
            tot += mvn_logp(z, ld).double().sum().item()
    res["cfg5i_iaf_d784_B8192"] = {"B": B, "d": d, "seed": 1237, "input_sum_f64": float(x.double().sum()),
                                   "input_head": [float(v) for v in x.view(-1)[:8]], "nll_f64": -tot / B,
                                   "ref_seconds": time.time() - t0}
    print("cfg5i", res["cfg5i_iaf_d784_B8192"], flush=True)
    B = 524288
    z = torch.randn(B, d, generator=torch.Generator().manual_seed(1238))
    t0 = time.time()
    sx = sax = sld = 0.0
    with torch.no_grad():
        for s in range(0, B, 65536):
            xf, ldf = f6.forward(z[s:s + 65536])
            sx += xf.double().sum().item()
            sax += xf.double().abs().sum().item()
            sld += ldf.double().sum().item()
            if s == 0:
                head_x = [float(v) for v in xf[:4].reshape(-1)]
                head_ld = [float(v) for v in ldf[:64]]
    res["cfg5f_iaf_d784_B524288"] = {"B": B, "d": d, "seed": 1238, "input_sum_f64": float(z.double().sum()),
                                     "input_head": [float(v) for v in z.view(-1)[:8]], "out_sum_f64": sx,
                                     "out_abs_sum_f64": sax, "ld_sum_f64": sld, "out_head_rows4": head_x,
                                     "ld_head64": head_ld, "ref_seconds": time.time() - t0}
    print("cfg5f", {k: v for k, v in res["cfg5f_iaf_d784_B524288"].items() if "head" not in k}, flush=True)
    res["_meta"]["weights_cfg5"] = "g6_iaf784.npz"
    with open(path, "w") as fh:
        json.dump(res, fh, indent=1)


def g8(m2, m3, m5):
    """Full-scale NLL scalars (float64 mean of the reference's fp32 log_prob)."""
    torch.set_num_threads(8)
    res = {}

    def run(name, model, B, d, seed, chunk):
        x = torch.randn(B, d, generator=torch.Generator().manual_seed(seed))
        t0 = time.time()
        tot = 0.0
        with torch.no_grad():
            for s in range(0, B, chunk):
                z, ld = model.inverse(x[s:s + chunk])
                tot += mvn_logp(z, ld).double().sum().item()
        res[name] = {"B": B, "d": d, "seed": seed, "input_sum_f64": float(x.double().sum()),
                     "input_head": [float(v) for v in x.view(-1)[:8]], "nll_f64": -tot / B,
                     "ref_seconds": time.time() - t0}
        print(name, res[name], flush=True)

    run("cfg2_realnvp_d2_B1M", m2, 1_000_000, 2, 1234, 1_000_000)
    run("cfg3_spline_k8_d2_B1M", m3, 1_000_000, 2, 1235, 1_000_000)
    run("cfg4_maf_d63_B4M", m5, 4_000_000, 63, 1236, 500_000)
    res["_meta"] = {"torch": torch.__version__, "numpy": np.__version__,
                    "input": "torch.randn(B, d, generator=torch.Generator().manual_seed(seed)) on CPU",
                    "weights": "g2_realnvp.npz / g3_spline.npz (k8.) / g5_maf63.npz"}
    with open(os.path.join(HERE, "g8_full_nll.json"), "w") as f:
        json.dump(res, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-full", action="store_true")
    ap.add_argument("--only", default=None, help="write one fixture only, e.g. g10")
    a = ap.parse_args()
    flows, models = import_reference()
    if a.only == "g10":
        g10(flows)
        return
    if a.only == "g11":
        g11(flows, models)
        return
    if a.only == "g12":
        g12(flows, models)
        return
    if a.only == "g13":
        g13(flows)
        return
    if a.only == "g14":
        g14(flows)
        return
    if a.only == "g15":
        g15(models)
        return
    if a.only == "g16":
        g16(flows, models)
        return
    if a.only == "g17":
        g17(flows, models)
        return
    if a.only == "g18":
        g18(flows)
        return
    if a.only == "g8_cfg5":
        g8_cfg5(g6(flows))
        return
    import src.utils as src_utils
    g1(flows)
    m2 = g2(models)
    m3 = g3(flows, models)
    g4(flows)
    m5 = g5(flows, models)
    f6 = g6(flows)
    g7(models, src_utils)
    g9(flows, models)
    g10(flows)
    g12(flows, models)
    g13(flows)
    g14(flows)
    g15(models)
    g16(flows, models)
    g17(flows, models)
    g18(flows)
    if not a.skip_full:
        g8(m2, m3, m5)
        g8_cfg5(f6)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
