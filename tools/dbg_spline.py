"""Debug helper: dump GPU spline outputs for offline error analysis (gpurun_out/dbg_spline.npz)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "normalizing-flows-study_amd")]
import nfs_amd  # noqa: E402

out = {}
dev = torch.device("cuda:0")
for K, H in [(5, 32), (11, 96), (3, 128)]:
    torch.manual_seed(K * 1000 + H)
    d = 3
    layer = nfs_amd.SplineCouplingLayer(d, H, torch.tensor([0.0, 1.0, 0.0]), num_bins=K)
    with torch.no_grad():
        for p in layer.parameters():
            p.add_(0.2 * torch.randn_like(p))
    x = torch.randn(777, d) * 2.5
    layer = layer.to(dev).eval()
    with torch.no_grad():
        for direction in (1, -1):
            y, l = (layer.forward if direction > 0 else layer.inverse)(x.to(dev))
            out[f"K{K}H{H}d{direction}_y"] = y.cpu().numpy()
            out[f"K{K}H{H}d{direction}_l"] = l.cpu().numpy()
g = np.load(os.path.join(ROOT, "tests/golden/g4_rqs_unit.npz"))
args = [torch.from_numpy(g[k]).to(dev) for k in ("x", "uw", "uh", "ud")]
y, l = nfs_amd.rational_quadratic_spline(*args, inverse=False)
out["rqs_fwd_y"], out["rqs_fwd_l"] = y.cpu().numpy(), l.cpu().numpy()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "dbg_spline.npz"), **out)
print("saved")
