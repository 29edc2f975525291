"""tests/test_gpu_relational.py::test_distribution_preservation_training's protocol run through
the ORACLE (oracle/flows_ref.py, CPU autograd) for the 9 seeds of tools/relational_seeds.py:
NLL on the 500 test points, ||mean|| and ||cov - I|| of 1,000 samples, after up to 200 Adam steps
(lr 1e-3, clip 1.0) on 1,000 N(0, I) points — the reference's test_distribution_preservation.py:
134-157 recipe. The same seeds give the same initial weights and data as the GPU runs (both
initialise and sample on the CPU generator). fp32 and float64 trajectories, so the per-seed
spread of the reference arithmetic itself is on record (tests/golden/relational_oracle.jsonl is
this output; the GPU test derives its per-seed bounds from it):
    python tools/relational_seeds_oracle.py > tests/golden/relational_oracle.jsonl"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "normalizing-flows-study_amd"))
sys.path.insert(0, ROOT)
import nfs_amd  # noqa: E402
import oracle  # noqa: E402

NOT_PARAM = ("running_mean", "running_var", "num_batches_tracked")


def _mask(dim, kind):  # tests/test_gpu_relational.py _mask
    m = torch.zeros(dim)
    if kind == "alternating":
        m[::2] = 1
    else:
        m[: dim // 2] = 1
    return m


def model_and_specs(kind):
    """The test's three models (tests/test_gpu_relational.py::test_distribution_preservation_training)
    and their oracle specs (train mode, eval mode)."""
    if kind == "realnvp":
        return nfs_amd.RealNVP(2, 4, 32), oracle.realnvp_spec(4, training=True), oracle.realnvp_spec(4)
    if kind == "maf2":
        m = nfs_amd.NormalizingFlowModel([nfs_amd.MaskedAutoregressiveFlow(2, 32) for _ in range(2)])
        return m, oracle.maf_spec(2), oracle.maf_spec(2)
    m = nfs_amd.NormalizingFlowModel([nfs_amd.CouplingLayer(2, 32, _mask(2, "alternating")),
                                      nfs_amd.MaskedAutoregressiveFlow(2, 32),
                                      nfs_amd.CouplingLayer(2, 32, _mask(2, "half"))])
    sp = [("coupling", "flows.0.", {}), ("maf", "flows.1.", {}), ("coupling", "flows.2.", {})]
    return m, [(k, p, {"training": True} if k == "coupling" else {}) for k, p, _ in sp], sp


def run(seed, dtype, kind="realnvp"):
    torch.manual_seed(seed)
    m, spec_t, spec_e = model_and_specs(kind)
    base = torch.distributions.MultivariateNormal(torch.zeros(2), torch.eye(2))
    train = base.sample((1000,)).to(dtype)
    test = base.sample((500,)).to(dtype)
    sd = {k: v.detach().clone().to(dtype) if v.is_floating_point() else v.detach().clone()
          for k, v in m.state_dict().items()}
    params = [sd[k] for k, _ in m.named_parameters()]
    for p in params:
        p.requires_grad_(True)
    opt = torch.optim.Adam(params, lr=1e-3)
    steps = 0
    for _ in range(200):
        opt.zero_grad()
        z, ld = oracle.flow_model(sd, spec_t, train, -1)
        loss = -oracle.gauss_log_prob(z, ld).mean()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, max_norm=1.0)
        opt.step()
        steps += 1
        if not torch.isfinite(loss) or loss.item() < 0.5:
            break
    with torch.no_grad():
        z, ld = oracle.flow_model(sd, spec_e, test, -1)
        nll = -oracle.gauss_log_prob(z, ld).mean().item()
        xs, _ = oracle.flow_model(sd, spec_e, torch.randn(1000, 2, dtype=dtype), 1)
        cov = torch.norm(torch.cov(xs.T) - torch.eye(2, dtype=dtype)).item()
        mean = torch.norm(xs.mean(0)).item()
    return {"kind": kind, "seed": seed, "dtype": str(dtype).split(".")[1], "steps": steps, "nll": round(nll, 4),
            "mean": round(mean, 3), "cov": round(cov, 3)}


if __name__ == "__main__":
    # realnvp: the 9 seeds of tools/relational_seeds.py; maf2 / mixed: the test's seeds 42, 0, 1
    torch.set_num_threads(4)
    for kind, seeds in (("realnvp", (42, 0, 1, 2, 3, 4, 5, 6, 7)), ("maf2", (42, 0, 1)), ("mixed", (42, 0, 1))):
        for seed in seeds:
            for dt in (torch.float32, torch.float64):
                print(json.dumps({"path": "oracle", **run(seed, dt, kind)}), flush=True)
