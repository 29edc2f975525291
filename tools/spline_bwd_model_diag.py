"""Diagnostics: RealNVPSpline(2,8,64) training-step gradients, HIP vs fp32 CPU reference vs float64."""
import copy
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normalizing-flows-study_amd"), os.path.join(ROOT, "tests")]
import nfs_amd  # noqa: E402
from test_gpu_spline_backward import _model_grads  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(3)
model = nfs_amd.RealNVPSpline(2, 8, 64)
g = torch.Generator().manual_seed(4)
with torch.no_grad():
    for p in model.parameters():
        p.add_(0.2 * torch.randn(p.shape, generator=g))
ref64 = copy.deepcopy(model).double()
ref32 = copy.deepcopy(model)
data = torch.randn(4096, 2, generator=g) * torch.tensor([1.5, 0.7])
model = model.to(dev).train()
w = torch.ones(4096)
_, gx64, _ = _model_grads(ref64, data.double(), w.double())
_, gx32, _ = _model_grads(ref32, data, w)
_, gx, _ = _model_grads(model, data.to(dev), w.to(dev))
e32 = (gx32.double() - gx64).abs() / (1 + gx64.abs())
eh = (gx.double().cpu() - gx64).abs() / (1 + gx64.abs())
print("gx rel err quantiles ref32:", [f"{float(e32.max(1).values.quantile(q)):.2e}" for q in (0.5, 0.9, 0.99, 0.999, 1.0)])
print("gx rel err quantiles hip  :", [f"{float(eh.max(1).values.quantile(q)):.2e}" for q in (0.5, 0.9, 0.99, 0.999, 1.0)])
top = eh.max(1).values.argsort(descending=True)[:8]
for r in top.tolist():
    print(f"  row {r} x {data[r].tolist()} hip {eh[r].max():.2e} ref {e32[r].max():.2e} gx64 {gx64[r].tolist()}")
for thr in (1e-4, 1e-5):
    ill = (e32 > thr).any(1) | (eh > thr).any(1)
    ww = w.clone()
    ww[ill] = 0
    _, _, gp64 = _model_grads(ref64, data.double(), ww.double())
    _, _, gp32 = _model_grads(ref32, data, ww)
    _, _, gp = _model_grads(model, data.to(dev), ww.to(dev))
    print(f"== excluding {int(ill.sum())} rows (thr {thr})")
    for (n, _), a, b, c in zip(model.named_parameters(), gp, gp32, gp64):
        a, b, c = a.double().cpu(), b.double(), c.double()
        print(f"  {n:36s} |g64| {c.abs().max():.2e} hip max {(a-c).abs().max():.2e} mean {(a-c).abs().mean():.2e}"
              f"  ref max {(b-c).abs().max():.2e} mean {(b-c).abs().mean():.2e}")
