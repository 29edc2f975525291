"""GPU parity of the MADE-affine kernels (csrc/nfx_made*.hip): MAF.inverse / IAF.forward
(parallel, fp32 MFMA) and MAF.forward / IAF.inverse (sequential over d, one MADE evaluation
per sample) against the reference's golden outputs and the CPU oracle.

Tolerances: z/x |d| <= 2e-5 * (1 + |ref|); log-det <= 2e-4 (d = 63), 1e-3 (d = 784: a sum of
784 clamped alphas); NLL relative <= 1e-6 at cfg4.
"""
import numpy as np
import pytest
import torch

import nfs_amd
import oracle
from conftest import golden_json, load_golden, oracle_sd, state_dict_from

pytestmark = pytest.mark.gpu


_SEQ_POLICIES = {"wave": "NFX_MADE_SEQ_WAVE", "segment": "NFX_MADE_SEQ_SEGMENT", "push": "NFX_MADE_SEQ_PUSH"}


@pytest.fixture(params=["wave", "segment", "push"])
def seq_policy(request, cuda_device):
    """Run a test on every sequential-direction kernel (nfx_made_seq_policy): the wave-per-sample
    made_seqw_kernel, the segment-parallel made_seqs_kernel and the push-formulation
    made_seqp_kernel (d <= 1024; the wave kernel beyond)."""
    from nfs_amd import _lib
    L = _lib.lib()
    old = L.nfx_made_seq_policy(getattr(_lib, _SEQ_POLICIES[request.param]))
    yield request.param
    L.nfx_made_seq_policy(old)


def assert_y(y, ref, tol=2e-5):
    y, ref = np.asarray(y, np.float64), np.asarray(ref, np.float64)
    err = np.abs(y - ref) / (1 + np.abs(ref))
    assert err.max() <= tol, f"max rel err {err.max():.3g} at {np.unravel_index(err.argmax(), err.shape)}"


def assert_ld(ld, ref, tol=2e-4):
    d = np.abs(np.asarray(ld, np.float64) - np.asarray(ref, np.float64))
    assert d.max() <= tol, f"max |dld| {d.max():.3g} at {d.argmax()}"


def maf63(dev):
    g = load_golden("g5_maf63.npz")
    m = nfs_amd.NormalizingFlowModel([nfs_amd.MaskedAutoregressiveFlow(63, 64) for _ in range(5)])
    m.load_state_dict(state_dict_from(g, "", m))
    return m.to(dev).eval(), g


def test_maf63_inverse_parallel_vs_reference(cuda_device):
    m, g = maf63(cuda_device)
    nfs_amd.reset_stats()
    with torch.no_grad():
        z, ld = m.inverse(torch.from_numpy(g["x"]).to(cuda_device))
        lp = m.log_prob(torch.from_numpy(g["x"]).to(cuda_device))
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] >= 5
    assert_y(z.cpu(), g["inv_z"])
    assert_ld(ld.cpu(), g["inv_ld"])
    nll = -float(lp.double().mean())
    assert abs(nll - float(g["nll_f64"])) <= 1e-6 * abs(float(g["nll_f64"]))


def test_maf63_forward_sequential_vs_reference(cuda_device, seq_policy):
    m, g = maf63(cuda_device)
    with torch.no_grad():
        x, ld = m.forward(torch.from_numpy(g["z"]).to(cuda_device))
    assert_y(x.cpu(), g["fwd_x"])
    assert_ld(ld.cpu(), g["fwd_ld"])


def test_iaf784_vs_reference(cuda_device, seq_policy):
    g = load_golden("g6_iaf784.npz")
    f = nfs_amd.InverseAutoregressiveFlow(784, 64)
    f.load_state_dict(state_dict_from(g, "", f))
    f = f.to(cuda_device).eval()
    with torch.no_grad():
        x, ldf = f.forward(torch.from_numpy(g["z"]).to(cuda_device))
        z, ldi = f.inverse(torch.from_numpy(g["x"]).to(cuda_device))
    assert_y(x.cpu(), g["fwd_x"])
    assert_ld(ldf.cpu(), g["fwd_ld"], 1e-3)
    assert_y(z.cpu(), g["inv_z"])
    assert_ld(ldi.cpu(), g["inv_ld"], 1e-3)


@pytest.mark.parametrize("name,kind", [("maf4", "maf"), ("iaf4", "iaf"), ("maf10", "maf"),
                                       ("iaf10", "iaf"), ("maf2", "maf"), ("iaf3", "iaf")])
def test_small_made_flows(cuda_device, name, kind):
    g = load_golden("g9_small.npz")
    sd = oracle_sd(g, name + ".")
    d = sd["conditioner.net.0.weight"].shape[1]
    H = sd["conditioner.net.0.weight"].shape[0]
    cls = nfs_amd.MaskedAutoregressiveFlow if kind == "maf" else nfs_amd.InverseAutoregressiveFlow
    f = cls(d, H)
    f.load_state_dict(state_dict_from(g, name + ".", f))
    f = f.to(cuda_device).eval()
    x = torch.from_numpy(g[name + ".x"]).to(cuda_device)
    with torch.no_grad():
        yf, lf = f.forward(x)
        yi, li = f.inverse(x)
    assert_y(yf.cpu(), g[name + ".fwd_y"])
    assert_ld(lf.cpu(), g[name + ".fwd_ld"])
    assert_y(yi.cpu(), g[name + ".inv_y"])
    assert_ld(li.cpu(), g[name + ".inv_ld"])


@pytest.mark.parametrize("d,H,B", [(5, 16, 1), (33, 32, 65), (63, 96, 130), (100, 128, 257), (7, 64, 1000),
                                   (65, 64, 129), (100, 32, 700), (200, 64, 1500), (784, 64, 77),
                                   (300, 16, 33), (130, 48, 70), (129, 64, 35),
                                   # segments longer than a 64-step staged block (sequential kernel)
                                   (400, 4, 50), (1000, 8, 20), (777, 64, 9),
                                   # 128 < H <= 256: nfx_made_big.hip
                                   (5, 256, 70), (63, 160, 100), (100, 256, 65), (300, 256, 33), (2, 200, 40),
                                   (64, 129, 97)])
def test_made_shapes_vs_oracle(cuda_device, d, H, B, seq_policy):
    torch.manual_seed(d * 31 + H)
    for cls, fn in ((nfs_amd.MaskedAutoregressiveFlow, oracle.maf), (nfs_amd.InverseAutoregressiveFlow, oracle.iaf)):
        f = cls(d, H)
        with torch.no_grad():
            for p in f.parameters():
                p.add_(0.05 * torch.randn_like(p))
        sd = {k: v.clone() for k, v in f.state_dict().items()}
        f = f.to(cuda_device).eval()
        x = torch.randn(B, d)
        for direction in (1, -1):
            with torch.no_grad():
                yg, lg = (f.forward if direction > 0 else f.inverse)(x.to(cuda_device))
                yr, lr = fn(sd, "", x, direction)
            assert_y(yg.cpu(), yr)
            assert_ld(lg.cpu(), lr, 5e-4)


@pytest.mark.parametrize("d,H", [(6, 16), (100, 64), (40, 224)])
def test_made_nonfinite_inputs(cuda_device, d, H, seq_policy):
    """inf/NaN rows: parallel directions propagate 0*inf = NaN through the dense masked weights;
    sequential directions reproduce the reference's contamination of every later step."""
    torch.manual_seed(3)
    for cls, fn in ((nfs_amd.MaskedAutoregressiveFlow, oracle.maf), (nfs_amd.InverseAutoregressiveFlow, oracle.iaf)):
        f = cls(d, H)
        with torch.no_grad():
            for p in f.parameters():
                p.add_(0.1 * torch.randn_like(p))
        sd = {k: v.clone() for k, v in f.state_dict().items()}
        f = f.to(cuda_device).eval()
        x = torch.randn(8, d)
        x[0, 0] = float("inf")
        x[1, 3] = float("nan")
        x[2, d - 1] = -float("inf")
        x[3, :] = 1e30
        for direction in (1, -1):
            with torch.no_grad():
                yg, lg = (f.forward if direction > 0 else f.inverse)(x.to(cuda_device))
                yr, lr = fn(sd, "", x, direction)
            yg, yr = yg.cpu().numpy(), yr.numpy()
            assert np.array_equal(np.isnan(yg), np.isnan(yr)) and np.array_equal(np.isinf(yg), np.isinf(yr))
            fin = np.isfinite(yr)
            assert_y(yg[fin], yr[fin])
            assert_ld(lg.cpu(), lr)


def test_made_batchnorm_eval(cuda_device):
    """MADE(use_batch_norm=True) in eval mode: BatchNorm folded from running stats."""
    torch.manual_seed(9)
    f = nfs_amd.MaskedAutoregressiveFlow(12, 32, use_batch_norm=True)
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


def test_full_scale_nll_cfg4(cuda_device):
    """BASELINE cfg4 at full size on one GPU: 5x MAF(63,64), B=4M, NLL vs the reference (G8)."""
    meta = golden_json("g8_full_nll.json")["cfg4_maf_d63_B4M"]
    x = torch.randn(meta["B"], meta["d"], generator=torch.Generator().manual_seed(meta["seed"]))
    assert abs(float(x.double().sum()) - meta["input_sum_f64"]) < 1e-3
    m, _ = maf63(cuda_device)
    nll = m.nll(x.to(cuda_device))
    assert abs(nll - meta["nll_f64"]) <= 1e-6 * abs(meta["nll_f64"]), (nll, meta["nll_f64"])


def _iaf784(dev):
    g = load_golden("g6_iaf784.npz")
    f = nfs_amd.InverseAutoregressiveFlow(784, 64)
    f.load_state_dict(state_dict_from(g, "", f))
    return nfs_amd.NormalizingFlowModel([f]).to(dev).eval()


def test_full_scale_nll_cfg5i(cuda_device, seq_policy):
    """BASELINE cfg5 density direction at full size: IAF(784,64) log_prob through the sequential
    inverse (inverse_autoregressive_flow.py:65-103), B = 8192, NLL vs the reference (G8)."""
    meta = golden_json("g8_full_nll.json")["cfg5i_iaf_d784_B8192"]
    x = torch.randn(meta["B"], meta["d"], generator=torch.Generator().manual_seed(meta["seed"]))
    assert abs(float(x.double().sum()) - meta["input_sum_f64"]) < 1e-3
    m = _iaf784(cuda_device)
    nfs_amd.reset_stats()
    nll = m.nll(x.to(cuda_device))
    assert nfs_amd.STATS["torch"] == 0
    assert abs(nll - meta["nll_f64"]) <= 1e-6 * abs(meta["nll_f64"]), (nll, meta["nll_f64"])


def test_full_scale_forward_cfg5f(cuda_device):
    """BASELINE cfg5 sampling direction at full size: IAF(784,64).forward (parallel,
    inverse_autoregressive_flow.py:30-63), B = 524,288, vs the reference's checksums (G8): the
    float64 sums of x, |x| and log-det, and the first rows element by element."""
    meta = golden_json("g8_full_nll.json")["cfg5f_iaf_d784_B524288"]
    z = torch.randn(meta["B"], meta["d"], generator=torch.Generator().manual_seed(meta["seed"]))
    assert abs(float(z.double().sum()) - meta["input_sum_f64"]) < 1e-3
    m = _iaf784(cuda_device)
    with torch.no_grad():
        x, ld = m.forward(z.to(cuda_device))
        sx, sax, sld = (float(v) for v in (x.double().sum(), x.double().abs().sum(), ld.double().sum()))
    assert abs(sax - meta["out_abs_sum_f64"]) <= 1e-6 * meta["out_abs_sum_f64"], (sax, meta["out_abs_sum_f64"])
    assert abs(sx - meta["out_sum_f64"]) <= 1e-6 * meta["out_abs_sum_f64"], (sx, meta["out_sum_f64"])
    assert abs(sld - meta["ld_sum_f64"]) <= 1e-6 * meta["B"], (sld, meta["ld_sum_f64"])
    assert_y(x[:4].reshape(-1).cpu(), np.asarray(meta["out_head_rows4"]))
    assert_ld(ld[:64].cpu(), np.asarray(meta["ld_head64"]), 1e-3)


def _made_tables(packed, d, H):
    """nk extents + tsafe of the packed MADE image (mirror of MadeLayout, nfx_made_kernel.h)."""
    up4 = lambda v: (v + 3) & ~3
    HT = (H + 31) // 32
    Hp, NKC = 32 * HT, (d + 31) // 32
    NJ = NKC
    o = HT * 4 * NKC * 256 + HT * 32 + 2 * (HT * HT * 1024 + HT * 32) + NJ * 2 * HT * 1024 + NJ * 64
    o += up4(d * Hp) + Hp + 2 * (Hp * Hp + Hp) + up4(2 * d * Hp) + up4(2 * d) + 3 * Hp
    ints = packed.view(torch.int32).cpu()
    nk = [ints[o + i * HT:o + (i + 1) * HT].tolist() for i in range(3)] + [ints[o + 3 * HT:o + 3 * HT + NJ].tolist()]
    return nk, float(packed[o + 3 * HT + NJ].cpu())


def test_made_structural_zero_tables(cuda_device):
    """d=63, H=64 (cfg4): every 32x32 block above the MADE block diagonal is exactly zero."""
    f = nfs_amd.MaskedAutoregressiveFlow(63, 64).to(cuda_device).eval()
    with torch.no_grad():
        f.inverse(torch.randn(64, 63, device=cuda_device))
    packed = f._nfx_pack_cache[1]
    nk, tsafe = _made_tables(packed, 63, 64)
    assert nk == [[1, 2], [1, 2], [1, 2], [1, 2]], nk
    assert 1e30 < tsafe < 1e37


@pytest.mark.parametrize("d,H", [(5, 16), (33, 32), (63, 64), (64, 96), (40, 128), (2, 64),
                                 (100, 32), (200, 64), (784, 64)])
def test_made_block_skip_bit_identical(cuda_device, d, H):
    """Tiles whose inputs pass the finite/bound test skip structurally-zero blocks; a tile with
    one huge row runs the dense product. The other rows of that tile must come out bit-identical
    to the same rows computed on the skipping path (32-row tiles for d <= 64, 64-row chunks of
    the wide kernel above)."""
    torch.manual_seed(d * 1000 + H)
    for cls in (nfs_amd.MaskedAutoregressiveFlow, nfs_amd.InverseAutoregressiveFlow):
        f = cls(d, H)
        with torch.no_grad():
            for p in f.parameters():
                p.add_(0.1 * torch.randn_like(p))
        f = f.to(cuda_device).eval()
        x = torch.randn(96, d, device=cuda_device)
        xd = x.clone()
        xd[37, 0] = 1e38  # tile 1 (rows 32..63) -> dense path
        fwd = f.forward if cls is nfs_amd.InverseAutoregressiveFlow else f.inverse
        with torch.no_grad():
            y, ld = fwd(x)
            yd, ldd = fwd(xd)
        keep = torch.ones(96, dtype=torch.bool, device=cuda_device)
        keep[37] = False
        assert torch.equal(y[keep], yd[keep]) and torch.equal(ld[keep], ldd[keep])


@pytest.mark.parametrize("d,H", [(2, 64), (63, 64), (17, 128)])
def test_made_tile_spread_launch_bit_identical(cuda_device, d, H):
    """Below 4 tiles per CU the parallel direction launches the tile kernel with 1-3 waves per
    workgroup and the weights read through L2 instead of 8-wave workgroups staging them in LDS
    (csrc/nfx_made.hip, round 6): the per-tile arithmetic is the same, so rows computed in a
    small batch equal the same rows inside a full-size batch bit for bit (ragged tails too)."""
    torch.manual_seed(d * 7 + H)
    big = 4 * 256 * 32 + 77  # at least 4 tiles per CU on a 256-CU part: the 8-wave launch
    for cls in (nfs_amd.MaskedAutoregressiveFlow, nfs_amd.InverseAutoregressiveFlow):
        f = cls(d, H)
        with torch.no_grad():
            for p in f.parameters():
                p.add_(0.1 * torch.randn_like(p))
        f = f.to(cuda_device).eval()
        fwd = f.forward if cls is nfs_amd.InverseAutoregressiveFlow else f.inverse
        x = torch.randn(big, d, device=cuda_device)
        with torch.no_grad():
            yb, ldb = fwd(x)
            for B in (1, 31, 33, 4000, 20000):
                y, ld = fwd(x[:B].contiguous())
                assert torch.equal(y, yb[:B]) and torch.equal(ld, ldb[:B]), (cls.__name__, B)
