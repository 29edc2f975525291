"""NLL / mean / covariance of tests/test_gpu_relational.py::test_distribution_preservation_training
per seed, with the kept-activation train path (NFX_TRAIN_KEEP=1) or the recompute path (0)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "normalizing-flows-study_amd"))
import nfs_amd  # noqa: E402


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


dev = torch.device("cuda:0")
for seed in (42, 0, 1, 2, 3, 4, 5, 6, 7):
    torch.manual_seed(seed)
    f = nfs_amd.RealNVP(2, 4, 32).to(dev).train()
    base = torch.distributions.MultivariateNormal(torch.zeros(2), torch.eye(2))
    train = base.sample((1000,)).to(dev)
    test = base.sample((500,)).to(dev)
    _train(f, train)
    f.eval()
    with torch.no_grad():
        nll = -f.log_prob(test)
        xs, _ = f.forward(torch.randn(1000, 2, device=dev))
    print(json.dumps({"keep": os.environ.get("NFX_TRAIN_KEEP", "1"), "seed": seed, "nll": round(nll.mean().item(), 4),
                      "mean": round(torch.norm(xs.mean(0)).item(), 3),
                      "cov": round(torch.norm(torch.cov(xs.T) - torch.eye(2, device=dev)).item(), 3)}), flush=True)
