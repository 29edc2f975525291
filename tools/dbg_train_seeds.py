"""Debug: distribution-preservation outcome over seeds, CPU fp32 composite vs GPU kernels."""
import copy
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(_ROOT, "normalizing-flows-study_amd"), _ROOT]
import torch  # noqa: E402
import nfs_amd  # noqa: E402


def run(f, train, dev):
    opt = torch.optim.Adam(f.parameters(), lr=1e-3)
    for _ in range(200):
        opt.zero_grad()
        loss = -f.log_prob(train).mean()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(f.parameters(), max_norm=1.0)
        opt.step()
    f.eval()
    z = torch.randn(20000, 2, generator=torch.Generator().manual_seed(5)).to(dev)
    with torch.no_grad():
        xs, _ = f.forward(z)
    return loss.item(), torch.norm(torch.cov(xs.T.double().cpu()) - torch.eye(2, dtype=torch.float64)).item()


devs = ["cpu"] + (["cuda:0"] if torch.cuda.is_available() else [])
for seed in range(8):
    torch.manual_seed(seed)
    f = nfs_amd.RealNVP(2, 4, 32)
    train = torch.randn(1000, 2)
    out = []
    for dev in devs:
        l, c = run(copy.deepcopy(f).to(dev).train(), train.to(dev), dev)
        out.append(f"{dev}: loss {l:.4f} cov {c:.3f}")
    print(seed, " | ".join(out), flush=True)
