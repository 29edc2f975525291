"""GPU: a whole training step captured as one HIP graph (nfs_amd.GraphedTrainStep) computes the
same training run as the eager step, bit for bit (every kernel is deterministic: fixed-order
reductions), for the reference's full-batch RealNVP loop (README.md:107-117, train-mode
BatchNorm) and a MAF stack (fused MAF backward), and for wide models on the any-shape path
(RealNVP H = 256 with train-mode BatchNorm, RealNVPSpline H = 128, MAF H = 320)."""
import copy

import pytest
import torch

import nfs_amd

pytestmark = pytest.mark.gpu


def _data(n, seed):
    g = torch.Generator().manual_seed(seed)
    t = torch.rand(n, generator=g) * 3.14159
    x = torch.stack([torch.cos(t), torch.sin(t)], 1) + 0.05 * torch.randn(n, 2, generator=g)
    return x


# realnvp / maf: the fused train kernels; the *_wide kinds run the any-shape path
# (csrc/nfx_generic.hip: GEMM conditioner, BatchNorm moments / running update, element adjoints)
@pytest.mark.parametrize("kind", ["realnvp", "maf", "realnvp_wide", "spline_wide", "maf_wide"])
def test_graphed_train_step_equals_eager(cuda_device, kind):
    torch.manual_seed(3)
    if kind == "realnvp":
        m = nfs_amd.RealNVP(2, 8, 64)
    elif kind == "realnvp_wide":
        m = nfs_amd.RealNVP(2, 4, 256)
    elif kind == "spline_wide":
        m = nfs_amd.RealNVPSpline(2, 4, 128)
    elif kind == "maf_wide":
        m = nfs_amd.NormalizingFlowModel([nfs_amd.MaskedAutoregressiveFlow(2, 320) for _ in range(3)])
    else:
        m = nfs_amd.NormalizingFlowModel([nfs_amd.MaskedAutoregressiveFlow(2, 64) for _ in range(4)])
    a = copy.deepcopy(m).to(cuda_device).train()
    b = copy.deepcopy(m).to(cuda_device).train()
    x = _data(5000, 4).to(cuda_device)
    opt_a = torch.optim.Adam(a.parameters(), lr=1e-3, capturable=True)
    opt_b = torch.optim.Adam(b.parameters(), lr=1e-3, capturable=True)
    warm, steps = 3, 10
    la = []
    for _ in range(warm + steps):
        opt_a.zero_grad(set_to_none=True)
        loss = -a.log_prob(x).mean()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(list(a.parameters()), 5.0)
        opt_a.step()
        la.append(loss.item())
    nfs_amd.reset_stats()
    step = nfs_amd.GraphedTrainStep(b, x, opt_b, clip_grad_norm=5.0, warmup=warm)
    assert nfs_amd.STATS["torch"] == 0 and nfs_amd.STATS["hip"] > 0, nfs_amd.STATS
    lb = [step().item() for _ in range(steps)]
    assert la[warm:] == lb, (la[warm:], lb)
    for (k, pa), (_, pb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert torch.equal(pa, pb), k
