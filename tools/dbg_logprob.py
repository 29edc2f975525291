"""Debug: where do fused and unfused log_prob differ (z, log-det or the Gaussian term)?"""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "normalizing-flows-study_amd"); sys.path.insert(0, ".")
import torch
from test_gpu_logprob import _model
from nfs_amd.models.normalizing_flow_model import gauss_logprob, gauss_workspace

dev = torch.device("cuda:0")
m, d, _ = _model(sys.argv[1] if len(sys.argv) > 1 else "affine_d5_h96")
m = m.to(dev).eval()
B = 77
g = torch.Generator().manual_seed(100 + B)
x = (1.5 * torch.randn(B, d, generator=g)).to(dev)
with torch.no_grad():
    logp = torch.empty(B, device=dev); sums = torch.empty(2, device=dev, dtype=torch.float64)
    z1, ld1, fused = m._hip_chain(x, -1, logprob=(logp, sums, gauss_workspace(B, dev)))
    z0, ld0 = m.inverse(x)
    lp0, _ = gauss_logprob(z0, ld0)
    lp1, _ = gauss_logprob(z1, ld1)
print("fused", fused, "z equal", torch.equal(z0, z1), "ld equal", torch.equal(ld0, ld1))
print("gauss(z1,ld1)==fused logp", torch.equal(lp1, logp), "max", (lp1 - logp).abs().max().item())
i = (lp1 - logp).abs().argmax().item()
zz = z1[i].cpu(); c = torch.tensor(d * 1.8378770664093453, dtype=torch.float64).float()
mm = zz[0] * zz[0]
for j in range(1, d): mm = mm + zz[j] * zz[j]
print("row", i, "z", zz.tolist(), "ld", ld1[i].item(), "fused", logp[i].item(), "gauss", lp1[i].item(),
      "host", (-0.5 * (mm + c) + ld1[i].cpu()).item())
