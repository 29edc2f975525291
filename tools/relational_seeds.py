"""NLL / mean / covariance of tests/test_gpu_relational.py::test_distribution_preservation_training
per seed on the GPU, with the kept-activation train path (NFX_TRAIN_KEEP=1) or the recompute path
(0): realnvp over the 9 seeds, maf2 / mixed over the test's seeds 42, 0, 1 (the same models and
seeds as tools/relational_seeds_oracle.py, whose oracle values are tests/golden/relational_oracle.jsonl)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from relational_seeds_oracle import model_and_specs  # noqa: E402


def _train(flow, data, steps=200, lr=1e-3):
    opt = torch.optim.Adam(flow.parameters(), lr=lr)
    n = 0
    for _ in range(steps):
        opt.zero_grad()
        loss = -flow.log_prob(data).mean()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(flow.parameters(), max_norm=1.0)
        opt.step()
        n += 1
        if not torch.isfinite(loss) or loss.item() < 0.5:
            break
    return n


dev = torch.device("cuda:0")
for kind, seeds in (("realnvp", (42, 0, 1, 2, 3, 4, 5, 6, 7)), ("maf2", (42, 0, 1)), ("mixed", (42, 0, 1))):
    for seed in seeds:
        torch.manual_seed(seed)
        f = model_and_specs(kind)[0].to(dev).train()
        base = torch.distributions.MultivariateNormal(torch.zeros(2), torch.eye(2))
        train = base.sample((1000,)).to(dev)
        test = base.sample((500,)).to(dev)
        steps = _train(f, train)
        f.eval()
        with torch.no_grad():
            nll = -f.log_prob(test)
            xs, _ = f.forward(torch.randn(1000, 2, device=dev))
        print(json.dumps({"path": "gpu", "keep": os.environ.get("NFX_TRAIN_KEEP", "1"), "kind": kind, "seed": seed,
                          "steps": steps, "nll": round(nll.mean().item(), 4),
                          "mean": round(torch.norm(xs.mean(0)).item(), 3),
                          "cov": round(torch.norm(torch.cov(xs.T) - torch.eye(2, device=dev)).item(), 3)}), flush=True)
